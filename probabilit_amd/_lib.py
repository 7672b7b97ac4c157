"""ctypes binding of libprobabilit_hip.so (C-ABI declared in include/probabilit_hip.h).

The library is the only compute path of probabilit_amd: there is no CPU fallback.  Loading
fails loudly when the in-tree .so is missing (run `python -m probabilit_amd.build`).
"""

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libprobabilit_hip.so")
# (A/B measurements set LIB_PATH to a variant built by build.py --variant before the first load)

# pbh_status
OK, ERR_INVALID, ERR_HIP, ERR_NOT_PD, ERR_NONFINITE, ERR_WORKSPACE, ERR_UNSUPPORTED = range(7)

# pbh_dist
DIST_IDS = {"norm": 0, "uniform": 1, "expon": 2, "lognorm": 3, "triang": 4, "gamma": 5, "poisson": 6, "beta": 7,
            "truncnorm": 8, "binom": 9, "bernoulli": 10, "weibull_min": 11, "weibull_max": 12, "logistic": 13,
            "cauchy": 14, "laplace": 15, "gumbel_r": 16, "gumbel_l": 17, "pareto": 18, "loguniform": 19,
            "reciprocal": 19, "rayleigh": 20, "lomax": 21, "genextreme": 22, "gompertz": 23, "chi2": 24,
            "halfcauchy": 25, "halflogistic": 26, "halfnorm": 27, "arcsine": 28, "hypsecant": 29, "powerlaw": 30, "genpareto": 31, "fisk": 32, "burr": 33, "burr12": 34, "exponweib": 35, "exponpow": 36, "bradford": 37, "anglit": 38, "levy": 39, "levy_l": 40, "gibrat": 41, "invweibull": 42, "loglaplace": 43, "truncexpon": 44, "chi": 45, "maxwell": 46, "nakagami": 47, "dweibull": 48, "kappa3": 49, "genhalflogistic": 50, "alpha": 51, "fatiguelife": 52, "genlogistic": 53, "trapezoid": 54, "erlang": 5, "geom": 55, "randint": 56, "nbinom": 57, "invgamma": 58, "t": 59,
            "trapz": 54, "johnsonsu": 60, "johnsonsb": 61, "powernorm": 62, "laplace_asymmetric": 63, "mielke": 64,
            "truncpareto": 65, "tukeylambda": 66, "gengamma": 67, "loggamma": 68, "dgamma": 69, "f": 70, "rdist": 71,
            "semicircular": 72, "betaprime": 73, "dlaplace": 74, "planck": 75, "boltzmann": 76,
            "pearson3": 77, "gennorm": 78, "halfgennorm": 79, "wrapcauchy": 80, "skewcauchy": 81, "moyal": 82,
            "kappa4": 83, "crystalball": 84, "powerlognorm": 85, "jf_skew_t": 86, "foldcauchy": 87, "foldnorm": 88,
            "cosine": 89, "invgauss": 90, "wald": 91, "betabinom": 92, "hypergeom": 93, "skewnorm": 94,
            "recipinvgauss": 95, "exponnorm": 96, "argus": 97, "kstwobign": 98,
            "nhypergeom": 99, "yulesimon": 100, "zipfian": 101,
            "rel_breitwigner": 102}

# pbh_table_kind
TABLE_INTERP, TABLE_QUANTILE, TABLE_SEARCH = 0, 1, 2

# pbh_dtype
BOOL, INT64, FLOAT64 = 0, 1, 2

# pbh_op
OPS = {}
for _i, _name in enumerate(["add", "sub", "mul", "truediv", "floordiv", "mod", "pow", "max", "min", "and", "or",
                            "eq", "ne", "lt", "le", "gt", "ge", "isclose", "arctan2"]):
    OPS[_name] = _i
for _i, _name in enumerate(["neg", "abs", "log", "exp", "floor", "ceil", "sign", "sqrt", "square", "log10", "sin",
                            "cos", "tan", "arcsin", "arccos", "arctan", "sinh", "cosh", "tanh", "arcsinh",
                            "arccosh", "arctanh"]):
    OPS[_name] = 32 + _i
OPS["cast"] = 63

# exported symbols (tests check the .so exports every one of them)
SYMBOLS = ["pbh_version", "pbh_last_error", "pbh_init", "pbh_fill_lhs", "pbh_fill_uniform", "pbh_fill_sobol",
           "pbh_ppf", "pbh_lhs_ppf", "pbh_ic_workspace_size", "pbh_iman_conover", "pbh_rank_workspace_size",
           "pbh_rankdata_average", "pbh_elementwise", "pbh_average", "pbh_transpose", "pbh_timing_enable",
           "pbh_timing_reset", "pbh_kernel_name", "pbh_timing_read", "pbh_lhs_sorted_ppf", "pbh_sorted_check",
           "pbh_run_heads_workspace_size", "pbh_run_heads", "pbh_lhs_scores", "pbh_gram_workspace_size",
           "pbh_column_sums", "pbh_centered_gram", "pbh_ic_factor", "pbh_ic_apply", "pbh_ic_reorder_workspace_size",
           "pbh_ic_reorder", "pbh_mt19937_workspace_size", "pbh_mt19937_random", "pbh_mt19937_advance",
           "pbh_pcg64_workspace_size",
           "pbh_pcg64_random", "pbh_halton_workspace_size", "pbh_fill_halton",
           "pbh_affine_workspace_size", "pbh_affine_rows", "pbh_table_ppf", "pbh_permcorr_workspace_size",
           "pbh_permcorr_climb", "pbh_sobol_ppf", "pbh_lhs_reference_workspace_size",
           "pbh_lhs_reference", "pbh_lhs_reference_strata", "pbh_lhs_reference_perms", "pbh_lhs_reference_band", "pbh_lhs_reference_stats", "pbh_table_cache_stats", "pbh_table_cache_clear", "pbh_hbm_copy", "pbh_dag_eval",
           "pbh_lhs_sorted_counts", "pbh_sort_heads", "pbh_ic_owned_workspace_size", "pbh_ic_owned_create",
           "pbh_ic_owned_column", "pbh_ic_owned_finish", "pbh_lhs_values_at", "pbh_lhs_ppf_columns", "pbh_ic_owned_destroy", "pbh_event_create",
           "pbh_event_destroy", "pbh_event_record", "pbh_stream_wait_event", "pbh_event_synchronize",
           "pbh_set_serial", "pbh_ic_column_scores"]

# kernel ids of pbh_kernel_name / pbh_timing_read (csrc/pbh_timing.h)
KERNELS = ["k_lhs_ppf", "k_ppf", "k_scatter", "k_upsweep", "k_digit_hist", "k_rank_finish<scores>",
           "k_rank_finish<gather>", "k_load_keys", "k_gram", "k_apply", "k_elementwise", "k_head_bounds", "k_scan",
           "k_lhs_sorted_ppf", "k_perm_scores", "k_code_runs",
           "k_make_codes", "k_scatter<u32>", "k_upsweep<u32>", "k_digit_hist<u32>",
           "k_upsweep<place>", "k_scatter<place>", "k_place", "k_streams", "k_affine", "k_table_ppf",
           "k_permcorr", "k_hbm_copy", "k_hist16", "k_msd1", "k_msd2", "k_finish", "k_place_msd",
           "k_place_gen", "k_dag", "k_transpose"]


class Param(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("value", ctypes.c_double)]


class Operand(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("dtype", ctypes.c_int32), ("f", ctypes.c_double), ("i", ctypes.c_int64)]


class ICColumn(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("lhs_col", ctypes.c_int32), ("dist", ctypes.c_int32),
                ("params", ctypes.c_double * 4), ("nparams", ctypes.c_int32), ("nonfinite_flag", ctypes.c_void_p)]


class ICArgs(ctypes.Structure):
    _fields_ = [("columns", ctypes.POINTER(ICColumn)), ("X", ctypes.c_void_p), ("n", ctypes.c_int64), ("k", ctypes.c_int32), ("x_rs", ctypes.c_int64),
                ("x_cs", ctypes.c_int64), ("target_chol_host", ctypes.c_void_p), ("Y", ctypes.c_void_p),
                ("y_rs", ctypes.c_int64), ("y_cs", ctypes.c_int64), ("ws", ctypes.c_void_p),
                ("ws_bytes", ctypes.c_size_t), ("scores_out", ctypes.c_void_p), ("cscores_out", ctypes.c_void_p),
                ("idx_out", ctypes.c_void_p), ("corr_host_out", ctypes.c_void_p),
                ("strata", ctypes.c_void_p)]


class DagOp(ctypes.Structure):  # pbh_dag_op
    _fields_ = [("kind", ctypes.c_int32), ("op", ctypes.c_int32), ("dst", ctypes.c_int32), ("a", ctypes.c_int32),
                ("b", ctypes.c_int32), ("src", ctypes.c_int32), ("flag", ctypes.c_int32), ("store", ctypes.c_int32),
                ("value", ctypes.c_double), ("params", ctypes.c_double * 3)]


class DagSource(ctypes.Structure):  # pbh_dag_qsource
    _fields_ = [("kind", ctypes.c_int32), ("col", ctypes.c_int32), ("bits", ctypes.c_int32), ("shift", ctypes.c_uint32),
                ("sv", ctypes.c_uint32 * 32), ("seed", ctypes.c_uint64), ("n_total", ctypes.c_int64),
                ("q", ctypes.c_void_p), ("stride", ctypes.c_int64)]


DAG_GEN, DAG_LOAD, DAG_CONST, DAG_BINARY, DAG_UNARY, DAG_STORE = range(6)
QSRC_SOBOL, QSRC_LHS, QSRC_VECTOR = range(3)
DAG_MAX_REGS = 16


class NativeError(RuntimeError):
    """A HIP runtime failure inside libprobabilit_hip."""


_lib = None


def load():
    """Load (once) and return the native library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"probabilit_amd native library not built: {LIB_PATH} is missing "
                          "(run `python -m probabilit_amd.build`)")
    # torch loads its own libamdhip64.so.7 by path; importing it first makes this library's
    # NEEDED libamdhip64.so.7 resolve (by SONAME) to that same runtime instance instead of
    # loading a second HIP runtime into the process.
    import torch  # noqa: F401

    lib = ctypes.CDLL(LIB_PATH)
    vp, i64, i32, dbl, sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
    u64 = ctypes.c_uint64
    sig = {
        "pbh_version": ([], i32),
        "pbh_last_error": ([], ctypes.c_char_p),
        "pbh_init": ([i32], i32),
        "pbh_fill_lhs": ([u64, i64, i64, i64, i32, i32, vp, i64, vp], i32),
        "pbh_fill_uniform": ([u64, i64, i64, i32, i32, vp, i64, vp], i32),
        "pbh_fill_sobol": ([vp, vp, i32, i32, i64, i64, i32, i32, vp, i64, vp], i32),
        "pbh_ppf": ([i32, vp, i64, i64, ctypes.POINTER(Param), i32, vp, vp, vp], i32),
        "pbh_lhs_ppf": ([u64, i64, i64, i64, i32, i32, ctypes.POINTER(Param), i32, vp, vp, vp], i32),
        "pbh_ic_workspace_size": ([i64, ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_iman_conover": ([ctypes.POINTER(ICArgs), vp], i32),
        "pbh_rank_workspace_size": ([i64, ctypes.POINTER(sz)], i32),
        "pbh_rankdata_average": ([vp, i64, i64, vp, vp, sz, vp], i32),
        "pbh_elementwise": ([i32, i32, i32, ctypes.POINTER(Operand), ctypes.POINTER(Operand), vp, i64, vp, vp], i32),
        "pbh_average": ([ctypes.POINTER(vp), i32, i64, vp, vp, vp], i32),
        "pbh_transpose": ([vp, i64, i64, i64, vp, i64, vp], i32),
        "pbh_timing_enable": ([i32], i32),
        "pbh_timing_reset": ([], i32),
        "pbh_kernel_name": ([i32], ctypes.c_char_p),
        "pbh_timing_read": ([i32, ctypes.POINTER(dbl), ctypes.POINTER(i64)], i32),
        "pbh_lhs_sorted_ppf": ([u64, i64, i64, i64, i32, i32, vp, i32, vp, vp, vp], i32),
        "pbh_sorted_check": ([vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i64), vp, vp], i32),
        "pbh_run_heads_workspace_size": ([i64, ctypes.POINTER(sz)], i32),
        "pbh_run_heads": ([vp, i64, i64, i32, vp, ctypes.POINTER(i64), vp, sz, vp], i32),
        "pbh_lhs_scores": ([u64, i64, i32, i64, i64, vp, i64, vp, vp], i32),
        "pbh_gram_workspace_size": ([ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_column_sums": ([vp, i64, ctypes.c_int32, i64, vp, vp, sz, vp], i32),
        "pbh_centered_gram": ([vp, i64, ctypes.c_int32, i64, vp, vp, vp, sz, vp], i32),
        "pbh_ic_factor": ([vp, i64, ctypes.c_int32, vp, vp], i32),
        "pbh_ic_apply": ([vp, i64, ctypes.c_int32, i64, vp, vp, vp, sz, vp], i32),
        "pbh_ic_reorder_workspace_size": ([i64, ctypes.POINTER(sz)], i32),
        "pbh_ic_reorder": ([vp, i64, vp, vp, i64, vp, vp, sz, vp], i32),
        "pbh_mt19937_workspace_size": ([i64, ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_mt19937_random": ([vp, ctypes.c_int32, i64, i64, ctypes.c_int32, vp, i64, vp, sz, vp], i32),
        "pbh_mt19937_advance": ([vp, ctypes.c_int32, i64, vp, ctypes.POINTER(ctypes.c_int32), vp, sz, vp], i32),
        "pbh_pcg64_workspace_size": ([ctypes.POINTER(sz)], i32),
        "pbh_pcg64_random": ([vp, vp, i64, i64, ctypes.c_int32, vp, i64, vp, sz, vp], i32),
        "pbh_halton_workspace_size": ([vp, vp, i32, ctypes.POINTER(sz)], i32),
        "pbh_fill_halton": ([vp, vp, vp, i32, i64, i64, i32, i32, vp, i64, vp, sz, vp], i32),
        "pbh_affine_workspace_size": ([ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_table_ppf": ([i32, vp, i64, i64, vp, vp, i64, i32, i32, vp, vp, vp], i32),
        "pbh_affine_rows": ([vp, i64, ctypes.c_int32, i64, i64, vp, vp, vp, vp, vp, i64, i64, vp, sz, vp], i32),
        "pbh_sobol_ppf": ([vp, vp, i32, i32, i64, i64, i32, i32, ctypes.POINTER(Param), i32, vp, vp, vp], i32),
        "pbh_permcorr_workspace_size": ([ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_lhs_reference_workspace_size": ([i64, ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_lhs_reference": ([vp, vp, ctypes.c_int32, ctypes.c_uint32, i64, ctypes.c_int32, vp, i64, vp, sz, vp], i32),
        "pbh_lhs_reference_strata": ([vp, vp, ctypes.c_int32, ctypes.c_uint32, i64, ctypes.c_int32, vp, i64, vp, i64, vp,
                                      sz, vp], i32),
        "pbh_hbm_copy": ([vp, vp, sz, i32, vp], i32),
        "pbh_dag_eval": ([ctypes.POINTER(DagOp), i32, ctypes.POINTER(DagSource), i32, ctypes.POINTER(vp), i32, i64, i64,
                          vp, vp], i32),
        "pbh_lhs_reference_perms": ([vp, vp, ctypes.c_int32, ctypes.c_uint32, i64, ctypes.c_int32, vp, vp], i32),
        "pbh_lhs_reference_band": ([ctypes.c_double, ctypes.POINTER(ctypes.c_double)], i32),
        "pbh_lhs_reference_stats": ([ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i64)], i32),
        "pbh_table_cache_stats": ([ctypes.POINTER(i64), ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "pbh_table_cache_clear": ([ctypes.POINTER(i64), ctypes.POINTER(i64)], i32),
        "pbh_ic_column_scores": ([vp, i64, i64, vp, vp, vp, vp, sz, vp], i32),
        "pbh_permcorr_climb": ([vp, vp, i64, ctypes.c_int32, i64, vp, vp, vp, vp, vp, vp, i64, dbl, vp, vp, vp, sz, vp],
                               i32),
        "pbh_lhs_sorted_counts": ([u64, i64, i64, i64, i32, i32, vp, i32, vp, vp, vp, ctypes.c_uint32, vp, i32, vp],
                                  i32),
        "pbh_sort_heads": ([vp, i64, vp], i32),
        "pbh_ic_owned_workspace_size": ([i64, ctypes.c_int32, ctypes.POINTER(sz)], i32),
        "pbh_ic_owned_create": ([ctypes.POINTER(ICColumn), ctypes.c_int32, i64, vp, sz, ctypes.POINTER(vp), vp], i32),
        "pbh_ic_owned_column": ([vp, ctypes.c_int32, vp, vp, i64, vp, vp, vp, vp], i32),
        "pbh_lhs_values_at": ([ctypes.POINTER(ICColumn), i64, vp, i64, vp, i64, vp], i32),
        "pbh_lhs_ppf_columns": ([ctypes.POINTER(ICColumn), i32, i64, i64, i64, vp, i64, vp], i32),
        "pbh_ic_owned_finish": ([vp, vp, vp], i32),
        "pbh_ic_owned_destroy": ([vp, vp], i32),
        "pbh_event_create": ([ctypes.POINTER(vp)], i32),
        "pbh_event_destroy": ([vp], i32),
        "pbh_event_record": ([vp, vp], i32),
        "pbh_stream_wait_event": ([vp, vp], i32),
        "pbh_event_synchronize": ([vp], i32),
        "pbh_set_serial": ([i32], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def last_error():
    return load().pbh_last_error().decode(errors="replace")


def check(status, what=""):
    """Map a pbh_status to the exception type the reference raises for the same condition."""
    if status == OK:
        return
    msg = last_error()
    if what:
        msg = f"{what}: {msg}"
    if status in (ERR_INVALID, ERR_NOT_PD, ERR_NONFINITE):
        raise ValueError(msg)
    if status == ERR_UNSUPPORTED:
        raise NotImplementedError(msg)
    if status == ERR_WORKSPACE:
        raise MemoryError(msg)
    raise NativeError(msg)


def np_ptr(a):
    """Host pointer of a C-contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)

