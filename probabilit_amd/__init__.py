"""probabilit_amd -- MI355X (gfx950) native drop-in for probabilit's Monte Carlo sampling path.

    import probabilit_amd as probabilit              # same names as `import probabilit`
    from probabilit_amd.modeling import Distribution, NoOp
    from probabilit_amd.correlation import ImanConover, nearest_correlation_matrix

All sampling runs in hand-written HIP kernels (libprobabilit_hip.so, C-ABI in
include/probabilit_hip.h); see DESIGN.md.
"""

import os as _os

# The step-4 lanes, the deferred counts' stream, torch's stream and (row-sharded runs) RCCL's
# stream and the exchange-issue stream run concurrently: more than HIP's default of 4 hardware
# queues per process, beyond which two streams share a queue and serialise (measured 1.5-4 ms per
# cfg3 step, profiles/r03).  Read when the HIP runtime initialises, i.e. at the first GPU call:
# effective when this package is imported before anything initialises HIP (import it before the
# first torch.cuda call); an explicit setting is kept.  Child processes inherit the variable.
def _hw_queues():
    import sys

    if "GPU_MAX_HW_QUEUES" in _os.environ:
        return
    _os.environ["GPU_MAX_HW_QUEUES"] = "8"
    torch = sys.modules.get("torch")  # never imported here: only asks whether HIP is already up
    if torch is not None and torch.cuda.is_initialized():
        import warnings

        warnings.warn("probabilit_amd was imported after the HIP runtime started: GPU_MAX_HW_QUEUES=8 has no "
                      "effect in this process, so its concurrent streams share HIP's default 4 hardware queues "
                      "(slower, same results); import probabilit_amd first or export GPU_MAX_HW_QUEUES=8",
                      RuntimeWarning, stacklevel=3)


_hw_queues()

from .modeling import (  # noqa: F401,E402
    Constant,
    CumulativeDistribution,
    DiscreteDistribution,
    Distribution,
    EmpiricalDistribution,
    Equal,
    MultivariateDistribution,
    scalar_transform,
)
from .distributions import PERT  # noqa: F401  (probabilit/__init__.py:11)


def plot(*variables, **kwargs):
    """probabilit.inspection.plot (a seaborn pairplot of sampled nodes) is UI, outside the
    sampling hot path this package accelerates: use the reference's plot
    on the `.samples_` arrays, which are plain numpy."""
    raise NotImplementedError("probabilit_amd does not provide plotting; call probabilit.inspection.plot "
                              "(seaborn) on the sampled nodes' .samples_ arrays")


__all__ = ["Distribution", "Constant", "EmpiricalDistribution", "CumulativeDistribution", "DiscreteDistribution",
           "Equal", "scalar_transform", "MultivariateDistribution", "PERT", "plot"]
__version__ = "0.1.0"
