"""Quantile sources for Node.sample (modeling.py:478-489), generated on the GPU.

    method=None     numpy's own streams bit for bit: RandomState (MT19937) for None / an int /
                    a RandomState, Generator (PCG64) for a Generator, as check_random_state
                    gives at modeling.py:484-486 (pbh_mt19937_random, pbh_pcg64_random:
                    device jump-ahead, the caller's generator advanced exactly as numpy does)
    method="lhs"    native Latin hypercube (default): per column a keyed Feistel bijection of
                    the strata plus a SplitMix64 jitter keyed by (seed, column, stratum), fused
                    into the ppf kernel (pbh_lhs_ppf);
                    with stream="reference": scipy's LatinHypercube stream bit for bit
                    (pbh_lhs_reference: device PCG64 uniforms + host Fisher-Yates shuffles)
    method="sobol"  scrambled Sobol', bit-exact with scipy.stats.qmc.Sobol (pbh_fill_sobol);
                    only the O(d * bits^2) engine setup (direction numbers, LMS scramble,
                    digital shift) runs on the host, consuming the numpy Generator exactly
                    as scipy does.
    method="halton" scrambled Halton, bit-exact with scipy.stats.qmc.Halton (pbh_fill_halton).

The native LHS design is statistically the same as scipy's but counter-based, so any row
range can be generated independently (row-sharding across GPUs, generator fused into the
inverse CDF); it is not scipy's PCG64 Fisher-Yates stream, which is sequential by
construction.  For that method bit-level parity with the reference holds at
Node.sample_from_quantiles (identical quantiles in give identical samples out), or end to end
with stream="reference".
"""

import ctypes
import functools
import numbers
import os
import warnings

import numpy as np

from . import _lib, device

MASK63 = (1 << 63) - 1


# ------------------------------------------------------------------ numpy bit-generator state
PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645
M128 = (1 << 128) - 1


def check_random_state(seed):
    """scipy._lib._util.check_random_state, which modeling.py:485 calls: None (or np.random) ->
    numpy's global RandomState, int -> a new RandomState(seed), Generator / RandomState -> itself."""
    if seed is None or seed is np.random:
        return np.random.mtrand._rand
    if isinstance(seed, (numbers.Integral, np.integer)):
        return np.random.RandomState(seed)
    if isinstance(seed, (np.random.RandomState, np.random.Generator)):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState instance")


def pcg64_advance(state, inc, k):
    """PCG64's 128-bit LCG state after k steps (host bookkeeping of the caller's Generator)."""
    acc_mult, acc_plus, cur_mult, cur_plus = 1, 0, PCG_MULT, inc
    while k:
        if k & 1:
            acc_mult = acc_mult * cur_mult & M128
            acc_plus = (acc_plus * cur_mult + cur_plus) & M128
        cur_plus = (cur_mult + 1) * cur_plus & M128
        cur_mult = cur_mult * cur_mult & M128
        k >>= 1
    return (acc_mult * state + acc_plus) & M128


def _u128_words(v):
    return np.array([v & ((1 << 64) - 1), v >> 64], dtype=np.uint64)


# ------------------------------------------------------------------ seeds
def seed_from(random_state):
    """A 64-bit seed for the native counter-based streams.

    int -> that int; None -> fresh OS entropy; np.random.Generator / RandomState -> one
    draw from it (so successive calls with one generator give different streams)."""
    if random_state is None:
        return int(np.random.SeedSequence().entropy) & ((1 << 64) - 1)
    if isinstance(random_state, (int, np.integer)):
        if random_state < 0:
            raise ValueError("Seed must be non-negative")
        return int(random_state) & ((1 << 64) - 1)
    if isinstance(random_state, np.random.Generator):
        return int(random_state.integers(0, MASK63, dtype=np.int64))
    if isinstance(random_state, np.random.RandomState):
        return int(random_state.randint(0, MASK63, dtype=np.int64))
    raise ValueError(f"{random_state!r} cannot be used to seed a numpy.random.Generator instance")


def engine_rng(rng):
    """The Generator a scipy QMC engine owns when built as `Engine(d=d, rng=rng)`
    (modeling.py:488): scipy's `_transition_to_rng` normalises the keyword with
    np.random.default_rng, and QMCEngine._initialize spawns an owned child from it
    (scipy:stats/_qmc.py)."""
    g = np.random.default_rng(rng)
    bg = g.bit_generator
    return np.random.Generator(type(bg)(bg.seed_seq.spawn(1)[0]))


# ------------------------------------------------------------------ Sobol' engine setup
_DIRECTION = {}


def _direction_numbers():
    """Joe & Kuo direction numbers as shipped by the pinned scipy (data file, read once)."""
    if not _DIRECTION:
        import scipy.stats

        path = os.path.join(os.path.dirname(scipy.stats.__file__), "_sobol_direction_numbers.npz")
        with np.load(path, allow_pickle=False) as z:
            _DIRECTION["poly"] = z["poly"].astype(np.int64)
            _DIRECTION["vinit"] = z["vinit"].astype(np.int64)
    return _DIRECTION["poly"], _DIRECTION["vinit"]


MAXDIM = 21201


def sobol_direction_matrix(d, bits=30):
    """Unscrambled direction matrix v (d x bits), Bratley & Fox recurrence."""
    return _direction_matrix(d, bits).copy()


@functools.lru_cache(maxsize=64)
def _direction_matrix(d, bits):
    poly, vinit = _direction_numbers()
    v = np.zeros((d, bits), dtype=np.uint64)
    if d == 0:
        return v.astype(np.uint32)
    v[0, :] = 1
    for k in range(1, d):
        p = int(poly[k])
        m = p.bit_length() - 1
        for j in range(m):
            v[k, j] = vinit[k, j]
        for j in range(m, bits):
            newv = int(v[k, j - m])
            pow2 = 1
            for i in range(m):
                pow2 <<= 1
                if (p >> (m - 1 - i)) & 1:
                    newv ^= pow2 * int(v[k, j - i - 1])
            v[k, j] = newv
    scale = np.array([1 << (bits - 1 - j) for j in range(bits)], dtype=np.uint64)
    return (v * scale[None, :]).astype(np.uint32 if bits <= 32 else np.uint64)


def _lms_scramble(sv, ltm, bits):
    """Linear matrix scramble: each direction number times a random lower-triangular binary
    matrix (unit diagonal) over GF(2), MSB first: bit (bits-1-p) of the result is the parity
    of row p of the matrix AND-ed with the number (scipy's _cscramble loop, as one GF(2)
    matrix product per dimension)."""
    ltm = ltm.astype(np.int64, copy=True)
    idx = np.arange(bits)
    ltm[:, idx, idx] = 1
    shifts = (bits - 1 - idx).astype(np.uint64)
    vb = ((sv.astype(np.uint64)[:, :, None] >> shifts[None, None, :]) & 1).astype(np.int64)  # (d, j, i) MSB first
    ob = np.einsum("kji,kpi->kjp", vb, ltm) & 1  # (d, j, p)
    return (ob.astype(np.uint64) << shifts[None, None, :]).sum(axis=2).astype(sv.dtype)


def sobol_setup(d, rng=None, bits=30, scramble=True):
    """(sv, shift) of scipy.stats.qmc.Sobol(d, rng=rng, bits=bits, scramble=scramble)."""
    if d > MAXDIM:
        raise ValueError(f"Maximum supported dimensionality is {MAXDIM}.")
    if bits > 32:
        raise NotImplementedError("native Sobol' supports bits <= 32")
    sv = sobol_direction_matrix(d, bits)
    if not scramble:
        return sv, np.zeros(d, dtype=np.uint32)
    g = engine_rng(rng)
    shift = np.dot(g.integers(0, 2, size=(d, bits), dtype=np.uint32),
                   2 ** np.arange(bits, dtype=np.uint32)).astype(np.uint32)
    ltm = np.tril(g.integers(0, 2, size=(d, bits, bits), dtype=np.uint32))
    return _lms_scramble(sv, ltm, bits).astype(np.uint32), shift


# ------------------------------------------------------------------ sources
class QuantileSource:
    """Yields the columns of an (n, d) quantile matrix in order (the iterator of
    modeling.py:510).  Each column is either a device vector with a stride or a fused
    generator descriptor understood by Distribution._sample."""

    def __init__(self, n, d):
        self.n, self.d, self._next = int(n), int(d), 0
        self.row0, self.rows = 0, int(n)  # the rows this process evaluates (all, unless sharded)

    def shard(self, row0, rows):
        """Restrict generation to rows [row0, row0 + rows) of the n-row design (row-sharded
        multi-GPU evaluation); generators are counter-addressed, so a shard is generated
        without the others."""
        self.row0, self.rows = int(row0), int(rows)
        return self

    def next_column(self):
        if self._next >= self.d:
            raise StopIteration("quantile columns exhausted")
        c = self._next
        self._next += 1
        return self.column(c)


class DeviceMatrixSource(QuantileSource):
    """User-supplied quantiles (numpy or device tensor), shape (n, d), any layout."""

    def __init__(self, quantiles):
        import torch

        if isinstance(quantiles, torch.Tensor):
            q = quantiles.to(device.device(), dtype=torch.float64)
        else:
            q = device.to_device(np.asarray(quantiles, dtype=np.float64))
        if q.dim() != 2:
            raise ValueError("quantiles must be a 2-D array of shape (samples, dimensions)")
        super().__init__(q.shape[0], q.shape[1])
        self.q = q

    def column(self, c):
        col = self.q[self.row0:self.row0 + self.rows, c]
        return ("vector", col, col.stride(0))


class MT19937Source(QuantileSource):
    """RandomState.random((n, d)) bit for bit (modeling.py:484-486 with random_state None, an
    int or a RandomState), generated on the device (pbh_mt19937_random) at the first column.
    The RandomState itself advances exactly as numpy's random() would (pbh_mt19937_advance),
    unless it is a throwaway instance made here from an int seed."""

    def __init__(self, n, d, rs, advance=True):
        super().__init__(n, d)
        st = rs.get_state(legacy=False)
        if st.get("bit_generator") != "MT19937":
            raise NotImplementedError(f"RandomState over {st.get('bit_generator')!r}: only MT19937 has a native stream")
        self.key = np.ascontiguousarray(st["state"]["key"], dtype=np.uint32)
        self.pos = int(st["state"]["pos"])
        self.q = None
        if advance:
            lib = _lib.load()
            ws = _workspace(lib.pbh_mt19937_workspace_size, 0, 0)
            key_out = np.empty(624, dtype=np.uint32)
            pos_out = ctypes.c_int32()
            _lib.check(lib.pbh_mt19937_advance(_lib.np_ptr(self.key), self.pos, 2 * self.n * self.d,
                                               _lib.np_ptr(key_out), ctypes.byref(pos_out), ws.data_ptr(),
                                               ws.numel(), device.stream()), "pbh_mt19937_advance")
            st["state"] = {"key": key_out, "pos": int(pos_out.value)}
            rs.set_state(st)

    def column(self, c):
        if self.q is None:
            lib = _lib.load()
            ws = _workspace(lib.pbh_mt19937_workspace_size, self.rows, self.d)
            self.q = device.empty((self.d, self.rows))
            _lib.check(lib.pbh_mt19937_random(_lib.np_ptr(self.key), self.pos, self.row0, self.rows, self.d,
                                              self.q.data_ptr(), max(self.rows, 1), ws.data_ptr(), ws.numel(),
                                              device.stream()), "pbh_mt19937_random")
        return ("vector", self.q[c], 1)


class PCG64Source(QuantileSource):
    """Generator(PCG64).random((n, d)) bit for bit (modeling.py:484-486 with a Generator),
    generated on the device (pbh_pcg64_random); the Generator advances by n * d draws."""

    def __init__(self, n, d, gen, advance=True):
        super().__init__(n, d)
        bg = gen.bit_generator
        if type(bg) is not np.random.PCG64:
            raise NotImplementedError(f"Generator over {type(bg).__name__}: only PCG64 has a native stream")
        st = bg.state
        self.state, self.inc = int(st["state"]["state"]), int(st["state"]["inc"])
        self.q = None
        if advance:  # Generator.random leaves the buffered 32-bit half untouched
            st["state"] = {"state": pcg64_advance(self.state, self.inc, self.n * self.d), "inc": self.inc}
            bg.state = st

    def column(self, c):
        if self.q is None:
            lib = _lib.load()
            ws = _workspace(lib.pbh_pcg64_workspace_size)
            self.q = device.empty((self.d, self.rows))
            s, inc = _u128_words(self.state), _u128_words(self.inc)
            _lib.check(lib.pbh_pcg64_random(_lib.np_ptr(s), _lib.np_ptr(inc), self.row0 * self.d, self.rows, self.d,
                                            self.q.data_ptr(), max(self.rows, 1), ws.data_ptr(), ws.numel(),
                                            device.stream()), "pbh_pcg64_random")
        return ("vector", self.q[c], 1)


def _workspace(size_fn, *args):
    need = ctypes.c_size_t()
    _lib.check(size_fn(*args, ctypes.byref(need)))
    return device.empty(max(int(need.value), 1), "uint8")


def pseudo_random_source(n, d, random_state):
    """modeling.py:484-486: check_random_state(random_state).random((size, d))."""
    rs = check_random_state(random_state)
    if isinstance(rs, np.random.Generator):
        return PCG64Source(n, d, rs)
    fresh = isinstance(random_state, (numbers.Integral, np.integer))
    return MT19937Source(n, d, rs, advance=not fresh)


class LHSSource(QuantileSource):
    def __init__(self, n, d, seed):
        super().__init__(n, d)
        self.seed = seed

    def column(self, c):
        return ("lhs", self.seed, self.n, c, self.row0)

    def materialize(self, c):
        out = device.empty(self.rows)
        lib = _lib.load()
        _lib.check(lib.pbh_fill_lhs(self.seed, self.n, self.row0, self.rows, c, 1, out.data_ptr(),
                                    max(self.rows, 1), device.stream()), "pbh_fill_lhs")
        return out


class ReferenceLHSSource(QuantileSource):
    """scipy.stats.qmc.LatinHypercube(d, rng=random_state).random(n) bit for bit: the
    reference's own LHS stream (modeling.py:480,488), opt-in with stream="reference".

    The engine's owned Generator is set up exactly as scipy does (engine_rng: a spawned child,
    which also advances a caller Generator's seed sequence as scipy would); pbh_lhs_reference
    draws the n x d uniforms and decodes the d Fisher-Yates shuffles -- one sequential stream by
    construction -- on the device (pbh_lhs_dev.hip).  The whole matrix is made at the first
    column; a row shard (multi-GPU) makes it on its own GPU and keeps its rows, since every row
    of a column depends on the whole shuffle."""

    def __init__(self, n, d, rng):
        super().__init__(n, d)
        if n >= 2 ** 31:
            raise NotImplementedError("the reference LHS stream is supported for n < 2**31")
        st = engine_rng(rng).bit_generator.state
        self.state, self.inc = int(st["state"]["state"]), int(st["state"]["inc"])
        self.has32, self.buf32 = int(st["has_uint32"]), int(st["uinteger"])
        self.q = None
        self.keep_strata = False  # set before the first column: keep each row's stratum as well
        self.strata = None

    def matrix(self):
        if self.q is None and self.n > 0 and self.d > 0:
            lib = _lib.load()
            ws = _workspace(lib.pbh_lhs_reference_workspace_size, self.n, self.d)
            self.q = device.empty((self.d, self.n))
            if self.keep_strata:
                self.strata = device.empty((self.d, self.n), "int32")
            s, inc = _u128_words(self.state), _u128_words(self.inc)
            _lib.check(lib.pbh_lhs_reference_strata(_lib.np_ptr(s), _lib.np_ptr(inc), self.has32, self.buf32, self.n,
                                                    self.d, self.q.data_ptr(), self.n,
                                                    self.strata.data_ptr() if self.strata is not None else None,
                                                    self.n, ws.data_ptr(), ws.numel(), device.stream()),
                       "pbh_lhs_reference")
            del ws
        return self.q

    def column(self, c):
        return ("vector", self.matrix()[c, self.row0:self.row0 + self.rows], 1)

    def strata_of(self, c):
        """Column c's strata (each row's rank - 1 in the whole column: int32 device vector), when
        kept (keep_strata) and this process holds every row; else None.  A monotone inverse CDF
        keeps these ranks, which lets Iman-Conover order the column without sorting it."""
        if self.strata is None or self.row0 != 0 or self.rows != self.n:
            return None
        return self.strata[c]


_DEFAULT_STREAM = os.environ.get("PBH_LHS_STREAM", "native")


def set_default_stream(stream):
    """Module default for Node.sample(method="lhs", stream=None): "native" (the counter-based
    design, fused into the inverse-CDF kernels; the default) or "reference" (scipy's
    LatinHypercube stream bit for bit).  The environment variable PBH_LHS_STREAM sets the
    initial value."""
    global _DEFAULT_STREAM
    if stream not in ("native", "reference"):
        raise ValueError(f"stream must be 'native' or 'reference', got {stream!r}")
    _DEFAULT_STREAM = stream


class SobolSource(QuantileSource):
    def __init__(self, n, d, rng, bits=30):
        super().__init__(n, d)
        if n > 2 ** bits:
            raise ValueError(f"At most 2**{bits}={2 ** bits} distinct points can be generated. "
                             f"0 points have been previously generated, then: n=0+{n}={n}. "
                             "Consider increasing `bits`.")
        if n > 1 and (n & (n - 1)) != 0:
            warnings.warn("The balance properties of Sobol' points require n to be a power of 2.", stacklevel=3)
        self.bits = bits
        self.sv, self.shift = sobol_setup(d, rng, bits)

    def column(self, c):
        """A lazy column: inverse-CDF nodes fuse the point generation into their kernel
        (pbh_sobol_ppf); other consumers call materialize(c)."""
        return ("sobol", self, c)

    def materialize(self, c):
        out = device.empty(self.rows)
        lib = _lib.load()
        sv = np.ascontiguousarray(self.sv, dtype=np.uint32)
        sh = np.ascontiguousarray(self.shift, dtype=np.uint32)
        _lib.check(lib.pbh_fill_sobol(_lib.np_ptr(sv), _lib.np_ptr(sh), self.d, self.bits, self.row0, self.rows, c,
                                      1, out.data_ptr(), max(self.rows, 1), device.stream()), "pbh_fill_sobol")
        return out


def first_primes(d):
    """The first d primes (scipy.stats._qmc.n_primes: the Halton bases)."""
    out, k = [], 2
    while len(out) < d:
        if all(k % p for p in out if p * p <= k):
            out.append(k)
        k += 1
    return out


def halton_setup(d, rng=None):
    """(bases, counts, perms) of scipy.stats.qmc.Halton(d, rng=rng): per dimension
    ceil(54 / log2(base)) - 1 shuffled copies of arange(base), drawn from the engine's owned
    Generator in dimension order (scipy:stats/_qmc.py _van_der_corput_permutations)."""
    import math

    g = engine_rng(rng)
    bases = first_primes(d)
    counts, perms = [], []
    for b in bases:
        count = math.ceil(54 / math.log2(b)) - 1
        p = np.repeat(np.arange(b)[None], count, axis=0)
        for row in p:
            g.shuffle(row)
        counts.append(count)
        perms.append(p.astype(np.int32).ravel())
    return (np.asarray(bases, dtype=np.int32), np.asarray(counts, dtype=np.int32),
            np.concatenate(perms) if perms else np.zeros(0, np.int32))


class HaltonSource(QuantileSource):
    """scipy.stats.qmc.Halton(d, rng=random_state).random(n) (modeling.py:481,488), bit-exact:
    engine setup (primes, digit permutations) on the host, the points on the device."""

    def __init__(self, n, d, rng):
        super().__init__(n, d)
        self.bases, self.counts, self.perms = halton_setup(d, rng)
        self.q = None

    def column(self, c):
        if self.q is None:
            lib = _lib.load()
            b, k, p = self.bases, self.counts, np.ascontiguousarray(self.perms)
            ws = _workspace(lib.pbh_halton_workspace_size, _lib.np_ptr(b), _lib.np_ptr(k), self.d)
            self.q = device.empty((self.d, self.rows))
            _lib.check(lib.pbh_fill_halton(_lib.np_ptr(b), _lib.np_ptr(k), _lib.np_ptr(p), self.d, self.row0, self.rows,
                                           0, self.d, self.q.data_ptr(), max(self.rows, 1), ws.data_ptr(),
                                           ws.numel(), device.stream()), "pbh_fill_halton")
        return ("vector", self.q[c], 1)


def make_source(method, n, d, random_state, stream=None):
    """The quantile source of Node.sample (modeling.py:478-489).  `stream` only matters for
    method="lhs": "native" (default) or "reference" (see set_default_stream)."""
    stream = _DEFAULT_STREAM if stream is None else stream
    if stream not in ("native", "reference"):
        raise ValueError(f"stream must be 'native' or 'reference', got {stream!r}")
    if method is None:
        return pseudo_random_source(n, d, random_state)
    m = method.lower().strip()
    if m == "lhs":
        if stream == "reference":
            return ReferenceLHSSource(n, d, random_state)
        return LHSSource(n, d, seed_from(random_state))
    if m == "sobol":
        return SobolSource(n, d, random_state)
    if m == "halton":
        return HaltonSource(n, d, random_state)
    raise KeyError(method)
