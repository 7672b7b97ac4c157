"""Drop-in for probabilit.correlation (src/probabilit/correlation.py @ 2025-09-19).

* `ImanConover` keeps the Correlator protocol of the reference (`correlator()`,
  `.set_target(C)`, `inst(X) -> Y` on (N, K) arrays; correlation.py:161-202, 288-425) and
  runs the transform on the GPU through pbh_iman_conover.  numpy inputs are uploaded and the
  result downloaded; torch device tensors stay on the device.
* `nearest_correlation_matrix` solves the same weighted problem as the reference's cvxpy /
  SCS formulation (correlation.py:59-150: minimise ||H o (X - G)||_F subject to diag(X) = 1
  and X - (10 eps / n) I >= 0) with a host ADMM on the K x K matrix (cvxpy is not a
  dependency).  It returns the optimum to ~1e-10, where SCS stops at its `eps`.
* `Cholesky` (correlation.py:205-285) and `decorrelate` (correlation.py:706-754): column
  means and the centered Gram on the device (pbh_column_sums, pbh_centered_gram), the K x K
  factors on the host, the N-sized row transform on the device (pbh_affine_rows).
"""

import ctypes

import numpy as np

from . import _lib, device


class CorrelatorError(Exception):
    pass


# ------------------------------------------------------------------ nearest correlation matrix
def _project_psd(A, floor):
    w, V = np.linalg.eigh((A + A.T) / 2.0)
    w = np.maximum(w, floor)
    return (V * w) @ V.T


def nearest_correlation_matrix(matrix, *, weights=None, eps=1e-6, verbose=False):
    """Nearest correlation matrix to `matrix` in the `weights`-weighted Frobenius norm.

    Same problem as correlation.py:59-150 (Qi & Sun's H-weighted formulation, eq. (3)):
    minimise ||H o (X - G)||_F  s.t.  diag(X) = 1,  X >= (10 eps / n) I.
    Solved by ADMM on the splitting X (PSD cone, shifted) = Y (unit diagonal, weighted
    least squares), which is exact at convergence; feasible inputs are returned as-is.
    """
    if not isinstance(matrix, np.ndarray):
        raise TypeError("Input argument `matrix` must be np.ndarray.")
    if not matrix.ndim == 2 and matrix.shape[0] == matrix.shape[1]:
        raise ValueError("Input argument `matrix` must be square.")
    G = np.array(matrix, dtype=float)
    H = np.ones_like(G) if weights is None else weights
    if not isinstance(H, np.ndarray):
        raise TypeError("Input argument `weights` must be np.ndarray.")
    if not (H.shape == G.shape):
        raise ValueError("Argument `weights` must have same shape as `matrix`.")
    n = G.shape[0]
    floor = (eps / n) * 10

    # already feasible (to rounding): the optimum is G itself, returned unchanged so that a
    # valid target reaches the correlator bit for bit (e.g. 0.9 * corrcoef(A) + 0.1 * I)
    if np.allclose(G, G.T, rtol=0, atol=1e-12) and np.allclose(np.diag(G), 1.0, rtol=0, atol=1e-12):
        if np.linalg.eigvalsh((G + G.T) / 2).min() >= floor:
            return G.copy()

    H2 = np.asarray(H, dtype=float) ** 2
    rho = max(float(np.mean(H2)), 1e-3)
    Y = (G + G.T) / 2.0
    np.fill_diagonal(Y, 1.0)
    U = np.zeros_like(G)
    X = Y
    for it in range(20000):
        X = _project_psd(Y - U, floor)
        Y_old = Y
        Y = (H2 * G + rho * (X + U)) / (H2 + rho)
        np.fill_diagonal(Y, 1.0)
        U = U + X - Y
        r = np.linalg.norm(X - Y)
        s = rho * np.linalg.norm(Y - Y_old)
        if verbose and it % 100 == 0:
            print(f"ncm admm it={it} primal={r:.3e} dual={s:.3e} rho={rho:.3e}")
        if r < 1e-12 * n and s < 1e-12 * n:
            break
        if r > 10 * s:  # residual balancing
            rho *= 2.0
            U /= 2.0
        elif s > 10 * r:
            rho /= 2.0
            U *= 2.0
    # exact unit diagonal while keeping the eigenvalue floor: project, rescale, re-project
    X = _project_psd(X, floor)
    d = np.sqrt(np.diag(X))
    X = X / d[:, None] / d[None, :]
    X = (X + X.T) / 2.0
    np.fill_diagonal(X, 1.0)
    is_symmetric = np.allclose(X, X.T)
    is_PD = np.linalg.eig(X)[0].min() > 0
    if not (is_symmetric and is_PD) and (eps > 1e-14):
        if verbose:
            print(f"Recursively calling solver with eps := {eps} / 10")
        return nearest_correlation_matrix(G, weights=H, eps=eps / 10, verbose=verbose)
    return X


def _is_positive_definite(X):
    try:
        np.linalg.cholesky(X)
        return True
    except np.linalg.LinAlgError:
        return False


# The device correlators hold K x K matrices and per-variable state in fixed workspaces
# (pbh_iman_conover, the Gram / affine kernels, the permutation climb): K <= 128 variables.
# The reference has no such limit; a larger K raises this ValueError instead of a native error.
MAX_VARIABLES = 128


def _check_k(K):
    if K > MAX_VARIABLES:
        raise ValueError(f"probabilit_amd correlates at most {MAX_VARIABLES} variables on the device; got {K}")


class Correlator:
    """Correlator protocol (correlation.py:161-202): set_target validates and factors C."""

    def set_target(self, correlation_matrix):
        if not isinstance(correlation_matrix, np.ndarray):
            raise TypeError("Input argument `correlation_matrix` must be NumPy array.")
        if not correlation_matrix.ndim == 2:
            raise ValueError("Correlation matrix must be square.")
        if not correlation_matrix.shape[0] == correlation_matrix.shape[1]:
            raise ValueError("Correlation matrix must be square.")
        if not np.allclose(np.diag(correlation_matrix), 1.0):
            raise ValueError("Correlation matrix must have 1.0 on diagonal.")
        if not np.allclose(correlation_matrix.T, correlation_matrix):
            raise ValueError("Correlation matrix must be symmetric.")
        if not _is_positive_definite(correlation_matrix):
            raise ValueError("Correlation matrix must be positive definite.")
        self.C = correlation_matrix.copy()
        self.P = np.linalg.cholesky(self.C)
        return self

    def _validate_X(self, X, check_rows_cols=True):
        if not (hasattr(self, "C") and hasattr(self, "P")):
            raise CorrelatorError("User must call `set_target` first.")
        import torch

        if not isinstance(X, (np.ndarray, torch.Tensor)):
            raise TypeError("Input argument `X` must be NumPy array.")
        if not X.ndim == 2:
            raise ValueError("Correlation matrix must be square.")
        N, K = X.shape
        if self.P.shape[0] != K:
            raise ValueError(f"Shape of `X` ({tuple(X.shape)}) does not match shape of correlation matrix "
                             f"({self.P.shape})")
        if check_rows_cols and N <= K:
            raise ValueError(f"The matrix X must have rows > columns. Got shape: {tuple(X.shape)}")
        _check_k(K)
        return N, K


def _as_block(X):
    """(N, K) numpy array or device tensor -> (K, N) contiguous device block, plus whether the
    caller passed a device tensor."""
    import torch

    on_device = isinstance(X, torch.Tensor)
    Xd = X.to(device.device(), torch.float64) if on_device else device.to_device(np.asarray(X, dtype=np.float64))
    return Xd.t().contiguous(), on_device


def _block_stats(block):
    """Column means (numpy's mean: sum / N) and centered Gram sum_r (x_r - m)(x_r - m)^T of a
    (K, N) device block, both as host arrays."""
    K, N = block.shape
    lib = _lib.load()
    nb = ctypes.c_size_t()
    _lib.check(lib.pbh_gram_workspace_size(K, ctypes.byref(nb)))
    ws = device.empty(max(int(nb.value), 1), "uint8")
    sums = device.zeros(K)
    _lib.check(lib.pbh_column_sums(block.data_ptr(), N, K, block.stride(0), sums.data_ptr(), ws.data_ptr(), nb.value,
                                   device.stream()), "pbh_column_sums")
    mean = device.to_host(sums) / N
    G = device.zeros((K, K))
    _lib.check(lib.pbh_centered_gram(block.data_ptr(), N, K, block.stride(0), device.to_device(mean).data_ptr(),
                                     G.data_ptr(), ws.data_ptr(), nb.value, device.stream()), "pbh_centered_gram")
    return mean, device.to_host(G)


def _affine_block(block, shift, scale, offset, M):
    """(K, N) device block -> Y (K, N): Y[:, r] = offset + ((X[:, r] - shift) / scale) @ M."""
    K, N = block.shape
    lib = _lib.load()
    nb = ctypes.c_size_t()
    _lib.check(lib.pbh_affine_workspace_size(K, ctypes.byref(nb)))
    ws = device.empty(int(nb.value), "uint8")
    Y = device.empty((K, N))
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (shift, scale, offset, M)]
    _lib.check(lib.pbh_affine_rows(block.data_ptr(), N, K, 1, block.stride(0), *[_lib.np_ptr(a) for a in arrs],
                                   Y.data_ptr(), 1, N, ws.data_ptr(), nb.value, device.stream()), "pbh_affine_rows")
    return Y


class Cholesky(Correlator):
    """Cholesky correlator (correlation.py:205-285): X_n = (X - mean) / std, remove the
    correlation of X_n with its own Cholesky factor, impose P, restore mean and std.  Does not
    preserve marginals (that is what ImanConover is for).

    Floating-point parity: the reference's covariance and products are BLAS calls whose
    summation order is library dependent, so the device result agrees to ~1e-12 relative,
    not bit for bit."""

    def set_target(self, correlation_matrix):
        super().set_target(correlation_matrix)
        return self

    def __call__(self, X):
        """Transform X of shape (N, K); returns a new array (or device tensor)."""
        self._validate_X(X)
        block, on_device = _as_block(X)
        Y = self._transform_device(block).t()
        return Y.contiguous() if on_device else device.to_host(Y)

    def _transform_device(self, block, ev=None, stats=None, n=None):
        """block: (K, rows) device tensor.  stats / n (row-sharded runs): the column means and
        centered Gram matrix over all n rows (distributed.block_stats); default: this block's."""
        import scipy.linalg

        K, N = block.shape
        if n is not None:
            N = n
        self._validate_X(block.T if n is None else np.lib.stride_tricks.as_strided(np.zeros(1), (N, K), (0, 0)))
        mean, G = _block_stats(block) if stats is None else stats
        std = np.sqrt(np.diag(G) / N)                        # np.std(X, axis=0)
        with np.errstate(divide="ignore", invalid="ignore"):
            cov = G / N / np.outer(std, std)                 # np.cov(X_n, rowvar=False, ddof=0)
        P = np.linalg.cholesky(cov)                          # :262
        transform = scipy.linalg.solve_triangular(P.T, self.P.T, lower=False)  # :284
        return _affine_block(block, mean, std, mean, transform * std)          # :285


def decorrelate(X, remove_variance=True):
    """Removes correlations (and optionally variances) from X of shape (N, K), keeping the
    mean (correlation.py:706-754): mean + (X - mean) @ inv(L).T with L = cholesky(cov(X)),
    or L / sqrt(var) when remove_variance is False."""
    import scipy.linalg

    _check_k(np.shape(X)[1])
    block, on_device = _as_block(X)
    K, N = block.shape
    mean, G = _block_stats(block)
    var = np.diag(G) / N                                     # np.var(X, axis=0, ddof=0)
    cov = G / (N - 1)                                        # np.cov(X, rowvar=False)
    L = np.linalg.cholesky(cov)
    if not remove_variance:
        L = L / np.sqrt(var)
    M = scipy.linalg.solve_triangular(L, np.eye(K), lower=True).T  # inv(L).T
    Y = _affine_block(block, mean, np.ones(K), mean, M).t()
    return Y.contiguous() if on_device else device.to_host(Y)


_NOT_PD_MSG = ("Rank data correlation not positive definite."
               "There are perfect correlations in the ranked data."
               "Supply more data (rows in X) or sample differently.")


class ImanConover(Correlator):
    """Iman-Conover rank-correlation induction (correlation.py:288-425) on the GPU.

    Steps 1-4 of the reference run in pbh_iman_conover: van der Waerden scores from
    'average' ranks, E = corrcoef(scores) with the positive-definiteness check, the
    forward substitution with cholesky(E) and the multiply by P^T, then every column of X
    re-ordered by the ranks of the correlated scores (marginals preserved)."""

    def set_target(self, correlation_matrix):
        super().set_target(correlation_matrix)
        return self

    def _run(self, X, n, k, x_rs, x_cs, Y, y_rs, y_cs, debug=None, columns=None, strata=None):
        lib = _lib.load()
        ws_bytes = ctypes.c_size_t()
        _lib.check(lib.pbh_ic_workspace_size(n, k, ctypes.byref(ws_bytes)))
        ws = device.empty(int(ws_bytes.value), "uint8")
        P = np.ascontiguousarray(self.P, dtype=np.float64)
        args = _lib.ICArgs()
        if columns is not None:
            arr = (_lib.ICColumn * k)(*columns)
            args.columns = ctypes.cast(arr, ctypes.POINTER(_lib.ICColumn))
        args.X, args.n, args.k, args.x_rs, args.x_cs = (X.data_ptr() if X is not None else None), n, k, x_rs, x_cs
        args.target_chol_host = P.ctypes.data
        args.Y, args.y_rs, args.y_cs = Y.data_ptr(), y_rs, y_cs
        args.ws, args.ws_bytes = ws.data_ptr(), ws_bytes.value
        if strata is not None and any(t is not None for t in strata):
            import torch

            for t in strata:
                if t is not None and (t.dtype != torch.int32 or t.numel() != n or not t.is_contiguous()):
                    raise ValueError("strata: contiguous int32 device vectors of n entries")
            sptr = (ctypes.c_void_p * k)(*[t.data_ptr() if t is not None else None for t in strata])
            args.strata = ctypes.cast(sptr, ctypes.c_void_p)
        if debug is not None:  # intermediates for parity tests; "idx" selects the gather form of step 4
            if "S" in debug:
                args.scores_out = debug["S"].data_ptr()
            if "CS" in debug:
                args.cscores_out = debug["CS"].data_ptr()
            if "idx" in debug:
                args.idx_out = debug["idx"].data_ptr()
            if "E" in debug:
                args.corr_host_out = debug["E"].ctypes.data
        status = lib.pbh_iman_conover(ctypes.byref(args), device.stream())
        if status in (_lib.ERR_NOT_PD, _lib.ERR_NONFINITE):
            raise ValueError(_NOT_PD_MSG)
        _lib.check(status, "pbh_iman_conover")
        del ws

    def __call__(self, X):
        """Transform X of shape (N, K); returns a new array (X is not modified)."""
        import torch

        N, K = self._validate_X(X)
        on_device = isinstance(X, torch.Tensor)
        Xd = X.to(device.device(), torch.float64) if on_device else device.to_device(np.asarray(X, dtype=np.float64))
        Xd = Xd.contiguous()
        Y = device.empty((N, K))
        self._run(Xd, N, K, K, 1, Y, K, 1)
        return Y if on_device else device.to_host(Y)

    def _transform_device(self, block, ev=None, strata=None, debug=None):
        """block: (K, N) contiguous device tensor of the correlated variables (DAG path).
        strata: optional list of K entries, each None or row j's known ranks - 1 (an int32
        device vector: an LHS column's strata, which a monotone inverse CDF keeps); step 1 then
        orders that column by a scatter instead of a sort, after checking it on the device."""
        K, N = block.shape
        self._validate_X(block.T)
        if strata is not None and len(strata) != K:
            raise ValueError(f"strata: {len(strata)} entries for {K} columns")
        Y = device.empty((K, N))
        self._run(block, N, K, 1, N, Y, 1, N, strata=strata, debug=debug)
        return Y

    def _transform_generated(self, columns, n, debug=None):
        """DAG fast path: K natively generated LHS columns (list of _lib.ICColumn) are
        generated, correlated and returned as a (K, N) device block without ever
        materialising the uncorrelated samples (see pbh_ic_column).  debug: optional dict of
        buffers for the intermediates (device (K, N) "S" / "CS", host (K, K) "E"), for the
        parity tests of the production step 4 (no "idx": that would select the gather form)."""
        K = len(columns)
        if not (hasattr(self, "C") and hasattr(self, "P")):
            raise CorrelatorError("User must call `set_target` first.")
        if self.P.shape[0] != K:
            raise ValueError(f"Shape of `X` ({(n, K)}) does not match shape of correlation matrix ({self.P.shape})")
        if n <= K:
            raise ValueError(f"The matrix X must have rows > columns. Got shape: {(n, K)}")
        _check_k(K)
        Y = device.empty((K, n))
        self._run(None, n, K, 1, n, Y, 1, n, columns=columns, debug=debug)
        return Y

    def _call_debug(self, X):
        """Transform plus the intermediates (scores, correlated scores, step-4 indices,
        rank correlation E) for parity tests."""
        N, K = self._validate_X(X)
        Xd = device.to_device(np.asarray(X, dtype=np.float64)).contiguous()
        Y = device.empty((N, K))
        dbg = {"S": device.empty((K, N)), "CS": device.empty((K, N)), "idx": device.empty((K, N), "int32"),
               "E": np.zeros((K, K))}
        self._run(Xd, N, K, K, 1, Y, K, 1, debug=dbg)
        return (device.to_host(Y), device.to_host(dbg["S"]).T, device.to_host(dbg["CS"]).T,
                device.to_host(dbg["idx"]).T, dbg["E"])


def rankdata(x):
    """scipy.stats.rankdata(x, method='average') of a 1-D array, on the device."""
    import torch

    on_device = isinstance(x, torch.Tensor)
    xd = (x.to(device.device(), torch.float64) if on_device else device.to_device(np.asarray(x, np.float64)))
    n = xd.shape[0]
    out = device.empty(n)
    lib = _lib.load()
    wsb = ctypes.c_size_t()
    _lib.check(lib.pbh_rank_workspace_size(n, ctypes.byref(wsb)))
    ws = device.empty(int(wsb.value), "uint8")
    _lib.check(lib.pbh_rankdata_average(xd.data_ptr(), xd.stride(0), n, out.data_ptr(), ws.data_ptr(), wsb.value,
                                        device.stream()), "rankdata")
    return out if on_device else device.to_host(out)


# ------------------------------------------------------------------ permutation correlator
class SwapIndexGenerator:
    """Disjoint index sets (indices1, indices2) of length `size` from range(n)
    (correlation.py:428-470): each call takes the next 2 * size entries of a running
    permutation drawn from `rng`; when fewer remain they are dropped and a fresh permutation is
    drawn.  The stream is host state of the caller's numpy Generator, consumed exactly as the
    reference consumes it (the rng continues identically after the call)."""

    def __init__(self, rng, n: int):
        assert n >= 2
        self.rng = rng
        self.indices = np.arange(n)
        self.permutation = self.rng.permutation(self.indices)

    def __call__(self, size: int):
        assert size >= 1
        flat, offs = self._take_many(np.array([size]))
        s = (offs[1] - offs[0]) // 2
        return flat[:s], flat[s:2 * s]

    def _take_many(self, sizes):
        """The concatenated (i, j) lists of len(sizes) consecutive calls, step t occupying
        flat[offsets[t]:offsets[t + 1]] (i first, then j), without a Python call per step."""
        need = 2 * np.minimum(np.asarray(sizes, dtype=np.int64), len(self.indices) // 2)
        offs = np.zeros(len(need) + 1, dtype=np.int64)
        pieces, t = [], 0
        while t < len(need):
            window = need[t:t + len(self.permutation) // 2 + 1]  # every step takes >= 2 entries
            cum = np.cumsum(window)
            fit = int(np.searchsorted(cum, len(self.permutation), side="right"))
            if fit:
                used = int(cum[fit - 1])
                pieces.append(self.permutation[:used])
                self.permutation = self.permutation[used:]
                offs[t + 1:t + fit + 1] = offs[t] + cum[:fit]
                t += fit
            if t < len(need) and need[t] > len(self.permutation):
                self.permutation = self.rng.permutation(self.indices)  # the short rest is dropped
        flat = np.concatenate(pieces).astype(np.int64) if pieces else np.zeros(0, dtype=np.int64)
        return flat, offs


def _rank_block(block):
    """Column-wise rankdata('average') of a (K, N) device block (spearman space)."""
    out = device.empty(tuple(block.shape))
    for c in range(block.shape[0]):
        out[c] = rankdata(block[c])
    return out


def _private_block(X):
    """(N, K) input -> a (K, N) device block this module may modify, and whether X was a
    device tensor."""
    block, on_device = _as_block(X)
    if on_device and block.data_ptr() == X.data_ptr():
        block = block.clone()
    return block, on_device


class CorrelationMatrix:
    """Incrementally updated correlation matrix of X under row swaps within one column
    (correlation.py:757-921): swapping rows i and j of column k changes only row and column k
    of the matrix, by sum_s (X_[i_s] - X_[j_s]) (X_[j_s, k] - X_[i_s, k]) / (m std std_k).

    The data live on the device as a (K, N) block; the initial Gram matrix is computed there
    (pbh_centered_gram); a swap reads 2 s rows of K values back for the K-vector update, so the
    numerics of update_column / commit are the reference's numpy expressions on the same
    values.  The initial numerator comes from the device Gram (a different summation order
    than numpy's BLAS matmul), so it agrees with the reference to ~1e-15 relative."""

    def __init__(self, X, correlation_type="pearson", check=True):
        valid_corrs = ("pearson", "spearman")
        assert correlation_type in valid_corrs
        assert X.ndim == 2
        self.correlation_type = correlation_type
        self.check = check
        self._Xd, self._on_device = _private_block(X)
        self._Xsd = self._Xd if correlation_type == "pearson" else _rank_block(self._Xd)
        self.n, self.m = self._Xsd.shape
        _, G = _block_stats(self._Xsd)
        self.numerator = G / self.m
        self.denominator = np.sqrt(np.diag(G) / self.m)
        if np.any(np.isclose(self.denominator, 0)):
            raise ValueError("X has one or several constant columns")
        self.corr_mat = (self.numerator / self.denominator[None, :]) / self.denominator[:, None]

    @property
    def X(self):
        """The (permuted) data, (N, K): numpy, or a device tensor when X was one."""
        Y = self._Xd.t().contiguous()
        return Y if self._on_device else device.to_host(Y)

    @property
    def X_(self):
        Y = self._Xsd.t().contiguous()
        return Y if self._on_device else device.to_host(Y)

    def __repr__(self):
        return repr(self.corr_mat)

    def __getitem__(self, *args, **kwargs):
        return self.corr_mat.__getitem__(*args, **kwargs)

    def _rows(self, idx):
        import torch

        t = torch.as_tensor(np.asarray(idx, dtype=np.int64), device=self._Xsd.device)
        return device.to_host(self._Xsd.index_select(1, t).t())  # (len(idx), K)

    def _delta_numerator(self, col, i, j):
        if self.check:
            assert isinstance(col, int)
            assert 0 <= col < self.n
            if isinstance(i, int):
                i = [i]
            if isinstance(j, int):
                j = [j]
            assert len(i) == len(j)
            if set(i).intersection(set(j)):
                raise ValueError(f"Swaps must be two disjoint sets, got {i} and {j}")
        i, j = np.atleast_1d(i), np.atleast_1d(j)
        row_i, row_j = self._rows(i), self._rows(j)
        d = np.sum((row_i - row_j) * (row_j[:, col] - row_i[:, col])[:, None], axis=0)
        d[col] = 0.0
        return d

    def delta_column(self, col, i, j):
        return self._delta_numerator(col, i, j) / (self.m * self.denominator * self.denominator[col])

    def update_column(self, col, i, j):
        return self.corr_mat[:, col] + self.delta_column(col, i, j)

    def commit(self, col, i, j):
        import torch

        dnum = self._delta_numerator(col, i, j)
        dcol = dnum / (self.m * self.denominator * self.denominator[col])
        self.corr_mat[:, col] += dcol
        self.corr_mat[col, :] += dcol
        self.numerator[:, col] += dnum
        self.numerator[col, :] += dnum
        ii = torch.as_tensor(np.atleast_1d(i).astype(np.int64), device=self._Xd.device)
        jj = torch.as_tensor(np.atleast_1d(j).astype(np.int64), device=self._Xd.device)
        for blk in {id(self._Xsd): self._Xsd, id(self._Xd): self._Xd}.values():
            vi, vj = blk[col, ii].clone(), blk[col, jj].clone()
            blk[col, ii] = vj
            blk[col, jj] = vi
        return self


class PermutationCorrelator(Correlator):
    """Induces the target correlation by swapping rows within columns, keeping a swap when it
    lowers the weighted error of that variable's correlation column (randomized hill climbing,
    correlation.py:473-703).  Same constructor, validation, printed progress and rng stream as
    the reference; the loop runs on the device (pbh_permcorr_climb, one persistent workgroup)
    in chunks of whole cycles through the variables, with the swap lists of a chunk drawn up
    front from the correlator's numpy Generator (they do not depend on the accept decisions;
    after an early stop the rng is rewound and advanced by exactly the steps the reference
    takes).  Decisions are bit-exact given the initial correlation matrix, which is computed
    from the device Gram (~1e-15 relative to the reference's BLAS matmul)."""

    def __init__(self, *, weights=None, iterations=1000, tol=0.01, correlation_type="pearson", seed=None,
                 verbose=False):
        if not (weights is None or np.all(weights > 0)):
            raise ValueError("`weights` must have positive entries.")
        if not (isinstance(iterations, int) and iterations >= 0):
            raise ValueError("`iterations` must be non-negative integer.")
        if not isinstance(tol, float) and tol > 0:  # sic (correlation.py:561)
            raise ValueError("`tol` must be a positive float.")
        if not (seed is None or isinstance(seed, int)):
            raise TypeError("`seed` must be None or an integer")
        if not isinstance(verbose, bool):
            raise TypeError("`verbose` must be boolean")
        self.iters = iterations
        self.tol = tol
        self.rng = np.random.default_rng(seed)
        self.verbose = verbose
        self.correlation_type = correlation_type

    def set_target(self, correlation_matrix, *, weights=None):
        super().set_target(correlation_matrix)
        weights = np.ones_like(self.C) if weights is None else weights
        self.weights = weights / np.sum(weights)
        self.triu_indices = np.triu_indices(self.C.shape[0], k=1)
        return self

    def _error(self, observed, target):
        """Weighted RMSE over the strict upper triangle of corr(X) - target (:582-586)."""
        idx = self.triu_indices
        return float(np.sqrt(np.sum(self.weights[idx] * (observed[idx] - target[idx]) ** 2.0)))

    @staticmethod
    def subiters(n, i):
        """Swaps per step in iteration i of n: ceil((log2 n + 1) ** (1 - 2 i / n)) (:588-608)."""
        C = np.log2(n) + 1
        return int(np.ceil(C ** (1 - (2 * i / n))))

    def __call__(self, X):
        """A copy of X (N, K) with rows shuffled within columns (numpy in, numpy out; a device
        tensor in, a device tensor out)."""
        self._validate_X(X, check_rows_cols=False)
        block, on_device = _private_block(X)
        Y = self._transform_device(block, copy=False).t().contiguous()
        return Y if on_device else device.to_host(Y)

    def _transform_device(self, block, ev=None, copy=True):
        """(K, N) device block -> the permuted (K, N) block (a new one unless copy=False)."""
        K, N = block.shape
        if self.P.shape[0] != K:
            raise ValueError("Number of variables in `X` does not match `correlation_matrix`.")
        xo = block.clone() if copy else block
        if self.verbose:
            print(f"Running permutation correlator for {self.iters if self.iters else 'inf'} iterations.")
        gen = SwapIndexGenerator(rng=self.rng, n=N)
        assert self.correlation_type in ("pearson", "spearman")  # CorrelationMatrix.__init__ (:821)
        xs = xo if self.correlation_type == "pearson" else _rank_block(xo)
        _, G = _block_stats(xs)
        den = np.sqrt(np.diag(G) / N)
        if np.any(np.isclose(den, 0)):
            raise ValueError("X has one or several constant columns")
        corr = ((G / N) / den[None, :]) / den[:, None]
        if 0 < self.iters < 10:  # iteration % (iters // 10) at the first step (:660)
            raise ZeroDivisionError("integer modulo by zero")
        self._climb(xs, None if xs is xo else xo, corr, den, gen)
        return xo

    def _climb(self, xs, xo, corr, den, gen):
        import torch

        K, N = xs.shape
        lib = _lib.load()
        nb = ctypes.c_size_t()
        _lib.check(lib.pbh_permcorr_workspace_size(K, ctypes.byref(nb)), "pbh_permcorr_workspace_size")
        ws = device.empty(int(nb.value), "uint8")
        C = np.ascontiguousarray(self.C, dtype=np.float64)
        Wn = np.ascontiguousarray(self.weights, dtype=np.float64)
        den = np.ascontiguousarray(den, dtype=np.float64)
        corr_d = device.to_device(np.ascontiguousarray(corr, dtype=np.float64))
        chunk = max(1, 16384 // K)  # iterations per launch
        errlog = device.empty(chunk)
        state = device.zeros(2, "int64")
        n_sched = self.iters if self.iters else 10_000
        every = self.iters // 10 if self.iters else 0  # iterations == 0 never prints per iteration
        err = self._error(corr, C)
        it0 = 1
        while self.iters == 0 or it0 <= self.iters:
            n_it = chunk if self.iters == 0 else min(chunk, self.iters - it0 + 1)
            per_it = [self.subiters(n_sched, it) for it in range(it0, it0 + n_it)]
            sizes = np.repeat(np.array(per_it, dtype=np.int64), K)
            snap = (self.rng.bit_generator.state, gen.permutation)
            flat, offs = gen._take_many(sizes)
            sw = torch.as_tensor(flat, device=xs.device)
            of = torch.as_tensor(offs, device=xs.device)
            _lib.check(lib.pbh_permcorr_climb(xs.data_ptr(), device.ptr(xo), N, K, N, corr_d.data_ptr(),
                                              _lib.np_ptr(den), _lib.np_ptr(C), _lib.np_ptr(Wn), sw.data_ptr(),
                                              of.data_ptr(), n_it * K, float(self.tol), errlog.data_ptr(),
                                              state.data_ptr(), ws.data_ptr(), nb.value, device.stream()),
                       "pbh_permcorr_climb")
            steps, stopped = (int(v) for v in device.to_host(state))
            errs = device.to_host(errlog)
            reached = (steps + K - 1) // K  # iterations whose variable-0 step ran
            for q in range(reached):
                if self.verbose and every and (it0 + q) % every == 0:
                    print(f" Iter {it0 + q:>6}  Error: {err:.6f} Swaps: {per_it[q]:>2}")
                err = float(errs[q])
            if stopped:
                self.rng.bit_generator.state = snap[0]  # rewind: the reference stops drawing here
                gen.permutation = snap[1]
                gen._take_many(sizes[:steps])
                if self.verbose:
                    print(f""" Terminating at iteration {it0 + reached - 1} due to tolerance. Error: {err:.6f}""")
                return
            it0 += n_it
