"""Restatements of the quantile engines behind modeling.py:479-489 (TEST INFRASTRUCTURE ONLY).

PCG64 (numpy 2.2.6): 128-bit LCG, state' = state * M + inc, output = rotr64(hi ^ lo, state >> 122)
of the NEW state; next_double = (u64 >> 11) * 2^-53; next_uint32 buffers the high half.
numpy's Generator.shuffle draws j = random_interval(i) for i = n-1 .. 1 with masked
rejection sampling on 32-bit draws (64-bit when i > 2^32 - 1).

LatinHypercube._random_lhs (scipy:stats/_qmc.py): u = rng.uniform(size=(n, d)) (row-major),
then d independent shuffles of arange(1, n+1), q = (perm.T - u) / n.

Sobol' closed form: x_i = (shift ^ XOR_{b : bit b of gray(i)} sv[:, b]) * 2^-bits.
"""

import numpy as np

M128 = (1 << 128) - 1
M64 = (1 << 64) - 1
PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645


class PCG64:
    def __init__(self, state, inc):
        self.state, self.inc = state, inc
        self.has32, self.buf32 = False, 0

    @classmethod
    def from_numpy(cls, gen):
        st = gen.bit_generator.state
        g = cls(st["state"]["state"], st["state"]["inc"])
        g.has32, g.buf32 = bool(st["has_uint32"]), st["uinteger"]
        return g

    def next64(self):
        self.state = (self.state * PCG_MULT + self.inc) & M128
        hi, lo = self.state >> 64, self.state & M64
        rot = self.state >> 122
        x = hi ^ lo
        return ((x >> rot) | (x << ((-rot) & 63))) & M64

    def next32(self):
        if self.has32:
            self.has32 = False
            return self.buf32
        v = self.next64()
        self.has32, self.buf32 = True, v >> 32
        return v & 0xFFFFFFFF

    def next_double(self):
        return (self.next64() >> 11) * (1.0 / 9007199254740992.0)

    def random_interval(self, mx):
        if mx == 0:
            return 0
        mask = mx
        for s in (1, 2, 4, 8, 16, 32):
            mask |= mask >> s
        if mx <= 0xFFFFFFFF:
            while True:
                v = self.next32() & mask
                if v <= mx:
                    return v
        while True:
            v = self.next64() & mask
            if v <= mx:
                return v


def lhs_reference(gen_state, n, d):
    """(n, d) Latin hypercube exactly as scipy's LatinHypercube(d, rng).random(n), given the
    engine's PCG64 (state, inc) before the call.  Pure Python: keep n * d small."""
    g = PCG64(*gen_state)
    u = np.array([[g.next_double() for _ in range(d)] for _ in range(n)])
    perms = np.empty((d, n), dtype=np.int64)
    for k in range(d):
        p = list(range(1, n + 1))
        for i in range(n - 1, 0, -1):
            j = g.random_interval(i)
            p[i], p[j] = p[j], p[i]
        perms[k] = p
    return (perms.T - u) / n


def sobol_closed_form(sv, shift, n, bits=30, index0=0):
    """Points index0 .. index0+n-1 of the scrambled Sobol' sequence with direction matrix sv
    (d x bits) and digital shift (d,)."""
    idx = np.arange(index0, index0 + n, dtype=np.uint64)
    gray = idx ^ (idx >> np.uint64(1))
    x = np.broadcast_to(shift.astype(np.uint64), (n, sv.shape[0])).copy()
    for b in range(bits):
        on = ((gray >> np.uint64(b)) & np.uint64(1)).astype(bool)
        x[on] ^= sv[:, b].astype(np.uint64)
    return x.astype(np.float64) * (1.0 / 2 ** bits)
