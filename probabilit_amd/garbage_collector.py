"""Garbage collection of intermediate node samples (garbage_collector.py:5-71 of the reference).

Semantics are unchanged; what is freed is HBM: deleting `.samples_` drops the node's device
vector, so with gc_strategy=[] a deep DAG keeps only the vectors still needed downstream.
"""

import collections
from collections.abc import Collection


class GarbageCollector:
    """Reference-counts unsampled children; once a parent has none left its `.samples_` is
    deleted unless the parent is the sink or listed in `strategy`.

    strategy : None (keep everything) or a collection of nodes to keep besides the sink.
    """

    def __init__(self, strategy=None):
        if not (strategy is None or isinstance(strategy, Collection)):
            raise TypeError(f"`strategy` must be None or a collection, got: {strategy}")
        self.strategy = strategy

    def set_sink(self, sink):
        self.sink = sink
        if self.strategy is None:
            return self
        self._unsampled_children = collections.defaultdict(int)
        for node in self.sink.nodes():
            for parent in node.get_parents():
                self._unsampled_children[parent] += 1
        return self

    def decrement_and_delete(self, node):
        """Count `node` as sampled for each of its parents; return the parents freed."""
        if not hasattr(self, "sink"):
            raise ValueError("You must call 'set_sink' first.")
        if self.strategy is None:
            return []
        freed = []
        for parent in node.get_parents():
            self._unsampled_children[parent] -= 1
            count = self._unsampled_children[parent]
            if count == 0 and parent not in self.strategy:
                del parent.samples_
                freed.append(parent)
            assert count >= 0
        return freed

    def freed_by(self, order):
        """The parents decrement_and_delete would free over the nodes of `order`, with the
        same bookkeeping but nothing deleted and this collector's counts untouched -- for the
        fused evaluation (probabilit_amd.dag), which never materialises the freed nodes."""
        if not hasattr(self, "sink"):
            raise ValueError("You must call 'set_sink' first.")
        if self.strategy is None:
            return set()
        counts = collections.defaultdict(int, self._unsampled_children)
        freed = set()
        for node in order:
            for parent in node.get_parents():
                counts[parent] -= 1
                if counts[parent] == 0 and parent not in self.strategy:
                    freed.add(parent)
        return freed
