/*
 * probabilit_hip.h -- C-ABI of libprobabilit_hip.so, the MI355X (gfx950) native library behind
 * the probabilit_amd drop-in for tommyod/probabilit's Monte Carlo sampling hot path.
 *
 * Every entry point is extern "C", takes plain pointers and sizes (device pointers unless
 * the name says _host), an opaque HIP stream (hipStream_t passed as void*; NULL = legacy
 * default stream), and returns a pbh_status.  No exception crosses the ABI: on failure the
 * call returns a non-zero status and pbh_last_error() returns a message (thread-local).
 *
 * Each function names the reference interface it replaces (file:line in tommyod/probabilit
 * @ 2025-09-19, src/probabilit/...; "scipy:" = scipy 1.15.3, the reference's L0 dependency).
 * The Python side (probabilit_amd/_lib.py) binds these with ctypes; INTEGRATION.md shows the
 * binding a maintainer of the reference would add.
 */
#ifndef PROBABILIT_HIP_H_
#define PROBABILIT_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum pbh_status {
  PBH_OK = 0,
  PBH_ERR_INVALID = 1,     /* bad argument (maps to ValueError / TypeError)                 */
  PBH_ERR_HIP = 2,         /* HIP runtime failure                                          */
  PBH_ERR_NOT_PD = 3,      /* IC rank-score correlation not positive definite (ValueError,
                              correlation.py:399-403)                                      */
  PBH_ERR_NONFINITE = 4,   /* non-finite input where the reference raises                   */
  PBH_ERR_WORKSPACE = 5,   /* workspace too small                                          */
  PBH_ERR_UNSUPPORTED = 6  /* distribution / op without a native kernel                    */
} pbh_status;

/* ---- distributions with a native inverse-CDF kernel (scipy.stats.<name>.ppf) ---- */
typedef enum pbh_dist {
  PBH_DIST_NORM = 0,    /* params: loc, scale                 scipy norm._ppf = ndtri        */
  PBH_DIST_UNIFORM = 1, /* params: loc, scale                                              */
  PBH_DIST_EXPON = 2,   /* params: loc, scale                 -log1p(-q)                     */
  PBH_DIST_LOGNORM = 3, /* params: s, loc, scale              exp(s * ndtri(q))              */
  PBH_DIST_TRIANG = 4,  /* params: c, loc, scale                                             */
  PBH_DIST_GAMMA = 5,   /* params: a, loc, scale              gammaincinv(a, q)              */
  PBH_DIST_POISSON = 6, /* params: mu, loc  (discrete)        smallest k: pdtr(k, mu) >= q   */
  PBH_DIST_BETA = 7,    /* params: a, b, loc, scale           I_x(a, b) = q (Boost ibeta_inv) */
  PBH_DIST_TRUNCNORM = 8, /* params: a, b, loc, scale         truncnorm._ppf (log space)     */
  PBH_DIST_BINOM = 9,   /* params: n, p, loc (discrete)       smallest k: bdtr(k, n, p) >= q */
  PBH_DIST_BERNOULLI = 10, /* params: p, loc (discrete)       binom with n = 1               */
  /* closed-form scipy _ppf bodies (scipy 1.15 stats/_continuous_distns.py), params: shapes,
   * loc, scale; any other scipy.stats name the reference's getattr(stats, distr) would take
   * (modeling.py:805-807) has no kernel */
  PBH_DIST_WEIBULL_MIN = 11, /* c                                pow(-log1p(-q), 1/c)           */
  PBH_DIST_WEIBULL_MAX = 12, /* c                                -pow(-log(q), 1/c)             */
  PBH_DIST_LOGISTIC = 13,    /*                                  logit(q)                       */
  PBH_DIST_CAUCHY = 14,      /*                                  Boost cauchy quantile          */
  PBH_DIST_LAPLACE = 15,     /*                                  +-log(2 min(q, 1 - q))         */
  PBH_DIST_GUMBEL_R = 16,    /*                                  -log(-log(q))                  */
  PBH_DIST_GUMBEL_L = 17,    /*                                  log(-log1p(-q))                */
  PBH_DIST_PARETO = 18,      /* b                                pow(1 - q, -1/b)               */
  PBH_DIST_LOGUNIFORM = 19,  /* a, b   (also scipy's reciprocal) exp(log a + q (log b - log a)) */
  PBH_DIST_RAYLEIGH = 20,    /*                                  sqrt(-2 log1p(-q))             */
  PBH_DIST_LOMAX = 21,       /* c                                expm1(-log1p(-q) / c)          */
  PBH_DIST_GENEXTREME = 22,  /* c                                -expm1(-c x) / c, x = gumbel_r */
  PBH_DIST_GOMPERTZ = 23,    /* c                                log1p(-log1p(-q) / c)          */
  PBH_DIST_CHI2 = 24,        /* df                               2 gammaincinv(df / 2, q)       */
  /* round 4: 30 more closed-form (or ndtri / gammaincinv based) scipy _ppf bodies; erlang is
   * gamma (the same _ppf) and reuses PBH_DIST_GAMMA */
  PBH_DIST_HALFCAUCHY = 25,   /*          tan(pi / 2 q) */
  PBH_DIST_HALFLOGISTIC = 26, /*          2 atanh(q) */
  PBH_DIST_HALFNORM = 27,     /*          ndtri((1 + q) / 2) */
  PBH_DIST_ARCSINE = 28,      /*          sin(pi / 2 q)^2 */
  PBH_DIST_HYPSECANT = 29,    /*          log(tan(pi q / 2)) */
  PBH_DIST_POWERLAW = 30,     /* a        pow(q, 1/a) */
  PBH_DIST_GENPARETO = 31,    /* c        -boxcox1p(-q, -c) */
  PBH_DIST_FISK = 32,         /* c        burr with d = 1 */
  PBH_DIST_BURR = 33,         /* c, d     (q^(-1/d) - 1)^(-1/c) */
  PBH_DIST_BURR12 = 34,       /* c, d     expm1(-log1p(-q) / d)^(1/c) */
  PBH_DIST_EXPONWEIB = 35,    /* a, c     (-log1p(-q^(1/a)))^(1/c) */
  PBH_DIST_EXPONPOW = 36,     /* b        log1p(-log1p(-q))^(1/b) */
  PBH_DIST_BRADFORD = 37,     /* c        expm1(q log1p(c)) / c */
  PBH_DIST_ANGLIT = 38,       /*          asin(sqrt(q)) - pi/4 */
  PBH_DIST_LEVY = 39,         /*          1 / ndtri(q/2)^2 */
  PBH_DIST_LEVY_L = 40,       /*          -1 / ndtri((q+1)/2)^2 */
  PBH_DIST_GIBRAT = 41,       /*          exp(ndtri(q)) */
  PBH_DIST_INVWEIBULL = 42,   /* c        (-log q)^(-1/c) */
  PBH_DIST_LOGLAPLACE = 43,   /* c        (2q)^(1/c) | (2(1-q))^(-1/c) */
  PBH_DIST_TRUNCEXPON = 44,   /* b        -log1p(q expm1(-b)) */
  PBH_DIST_CHI = 45,          /* df       sqrt(2 gammaincinv(df/2, q)) */
  PBH_DIST_MAXWELL = 46,      /*          sqrt(2 gammaincinv(1.5, q)) */
  PBH_DIST_NAKAGAMI = 47,     /* nu       sqrt(gammaincinv(nu, q) / nu) */
  PBH_DIST_DWEIBULL = 48,     /* c        +-(-log(2 min(q, 1-q)))^(1/c) */
  PBH_DIST_KAPPA3 = 49,       /* a        (a / (q^-a - 1))^(1/a) */
  PBH_DIST_GENHALFLOGISTIC = 50,/* c        (1 - ((1-q)/(1+q))^c) / c */
  PBH_DIST_ALPHA = 51,        /* a        1 / (a - ndtri(q ndtr(a))) */
  PBH_DIST_FATIGUELIFE = 52,  /* c        (c z + sqrt((c z)^2 + 4))^2 / 4 */
  PBH_DIST_GENLOGISTIC = 53,  /* c        -log(powm1(q, -1/c)) */
  PBH_DIST_TRAPEZOID = 54,    /* c, d     three pieces at cdf(c), cdf(d) */
  /* round 5: modeling.py:805-807 samples any scipy.stats name */
  PBH_DIST_GEOM = 55,         /* p, loc (discrete)   ceil(log1p(-q) / log1p(-p)), one step down */
  PBH_DIST_RANDINT = 56,      /* low, high, loc (discrete)  ceil(q (high - low) + low) - 1, one step down */
  PBH_DIST_NBINOM = 57,       /* n, p, loc (discrete)  smallest k: I_p(n, k + 1) >= q (Boost) */
  PBH_DIST_INVGAMMA = 58,     /* a        1 / gammainccinv(a, q) */
  PBH_DIST_T = 59,            /* df       stdtrit(df, q), through the incomplete beta */
  /* round 6: more scipy.stats names; trapz is trapezoid (PBH_DIST_TRAPEZOID) */
  PBH_DIST_JOHNSONSU = 60,    /* a, b     sinh((ndtri(q) - a) / b) */
  PBH_DIST_JOHNSONSB = 61,    /* a, b     expit(1 / b (ndtri(q) - a)) */
  PBH_DIST_POWERNORM = 62,    /* c        -ndtri(pow(1 - q, 1 / c)) */
  PBH_DIST_LAPLACE_ASYMMETRIC = 63, /* kappa  two log branches at kappa / (kappa + 1 / kappa) */
  PBH_DIST_MIELKE = 64,       /* k, s     pow(q^(s/k) / (1 - q^(s/k)), 1 / s) */
  PBH_DIST_TRUNCPARETO = 65,  /* b, c     pow(1 - (1 - c^-b) q, -1 / b) */
  PBH_DIST_TUKEYLAMBDA = 66,  /* lam      boxcox(q, lam) - boxcox1p(-q, lam) */
  PBH_DIST_GENGAMMA = 67,     /* a, c     (c > 0 ? gammaincinv : gammainccinv)(a, q)^(1 / c) */
  PBH_DIST_LOGGAMMA = 68,     /* c        log(gammaincinv(c, q)), the one-term tail below DBL_MIN */
  PBH_DIST_DGAMMA = 69,       /* a        +-gammaincinv / gammainccinv of 2 q - 1 / 2 q */
  PBH_DIST_F = 70,            /* dfn, dfd dfd w / (dfn (1 - w)), w = I^-1(q; dfn / 2, dfd / 2) */
  PBH_DIST_RDIST = 71,        /* c        2 I^-1(q; c / 2, c / 2) - 1 */
  PBH_DIST_SEMICIRCULAR = 72, /*          rdist with c = 3 */
  PBH_DIST_BETAPRIME = 73,    /* a, b     r / (1 - r), r = I^-1(q; a, b); 1 / isf - 1 near r = 1 */
  PBH_DIST_DLAPLACE = 74,     /* a, loc (discrete)   log branches, one step down by its cdf */
  PBH_DIST_PLANCK = 75,       /* lambda, loc (discrete)   ceil(-log1p(-q) / lambda - 1), one step down */
  PBH_DIST_BOLTZMANN = 76,    /* lambda, N, loc (discrete) the truncated planck */
  PBH_DIST_PEARSON3 = 77,     /* skew     gammaincinv(alpha, q or 1 - q) / beta + zeta; ndtri for |skew| < 1.6e-5 */
  PBH_DIST_GENNORM = 78,      /* beta     sign(q - 0.5) gammainccinv(1 / beta, (1 + c) - 2 c q)^(1 / beta) */
  PBH_DIST_HALFGENNORM = 79,  /* beta     gammaincinv(1 / beta, q)^(1 / beta) */
  PBH_DIST_WRAPCAUCHY = 80,   /* c        2 atan(val tan(pi q)), or 2 pi - 2 atan(val tan(pi (1 - q))) */
  PBH_DIST_SKEWCAUCHY = 81,   /* a        tan(pi / (1 -+ a) (q - (1 - a) / 2)) (1 -+ a) */
  PBH_DIST_MOYAL = 82,        /*          -log(2 erfcinv(q)^2), erfcinv(y) = -ndtri(y / 2) / sqrt(2) */
  PBH_DIST_KAPPA4 = 83,       /* h, k     the four closed forms of kappa4._ppf */
  PBH_DIST_CRYSTALBALL = 84,  /* beta, m  power-law tail below pbeta, ndtri of the gaussian core above */
  PBH_DIST_POWERLOGNORM = 85, /* c, s     exp(-ndtri((1 - q)^(1 / c)) s) */
  PBH_DIST_JF_SKEW_T = 86,    /* a, b     (2 d - 1) sqrt(a + b) / (2 sqrt(d (1 - d))), d = I^-1(q; a, b) */
  PBH_DIST_FOLDCAUCHY = 87,   /* c        the root of atan(x - c) + atan(x + c) = pi q in closed form */
  PBH_DIST_FOLDNORM = 88,     /* c        cdf / sf root by bracketed Newton (scipy: brentq on its cdf) */
  PBH_DIST_COSINE = 89,       /*          the root of x + sin x = pi (2 q - 1) by Newton */
  PBH_DIST_INVGAUSS = 90,     /* mu       log-cdf / log-sf root in log x by bracketed Newton */
  PBH_DIST_WALD = 91,         /*          invgauss with mu = 1 */
  PBH_DIST_BETABINOM = 92,    /* n, a, b, loc (discrete)  first k with sum of the pmf over [0, k] >= q */
  PBH_DIST_HYPERGEOM = 93,    /* M, n, N, loc (discrete)  the same over [max(0, N - M + n), min(n, N)] */
  PBH_DIST_SKEWNORM = 94,     /* a        cdf / sf root by bracketed Newton, Owen's T by Gauss-Legendre */
  PBH_DIST_RECIPINVGAUSS = 95, /* mu      1 / invgauss's (1 - q)-quantile */
  PBH_DIST_EXPONNORM = 96,    /* K        cdf / sf root by bracketed Newton */
  PBH_DIST_ARGUS = 97,        /* chi      cdf / sf root by bracketed Newton, sf from gammainc(1.5, .) */
  PBH_DIST_KSTWOBIGN = 98,    /*          kolmogci: theta-series cdf / alternating-series sf root */
  PBH_DIST_NHYPERGEOM = 99,   /* M, n, r, loc (discrete)  first k with sum of the pmf over [0, k] >= q */
  PBH_DIST_YULESIMON = 100,   /* alpha, loc (discrete)  first k >= 1 with 1 - k B(k, alpha + 1) >= q */
  PBH_DIST_ZIPFIAN = 101,     /* a, n, loc (discrete)  scipy's bisection on H(k, a) / H(n, a) */
  PBH_DIST_REL_BREITWIGNER = 102 /* rho   cdf root by bracketed Newton (scipy's complex-form cdf) */
} pbh_dist;

/* A distribution parameter: a scalar (ptr == NULL) or a length-n device vector of float64
 * (the composite-parameter broadcast of modeling.py:796-802, where a parent node's
 * samples_ array is passed as the argument). */
typedef struct pbh_param {
  const double* ptr;
  double value;
} pbh_param;

int pbh_version(void);
const char* pbh_last_error(void);
/* Fails (PBH_ERR_HIP) when no gfx950 device is visible; the product never runs without one. */
int pbh_init(int device);

/* ---------------------------------------------------------------- quantile generators
 * All generators write column-major quantiles: column c of the (N, d) quantile matrix of
 * modeling.py:478-489 at q[(c - col0) * ldq + (r - row0)], rows [row0, row0 + nrows).
 * Rows are counter-addressed, so any row range (a shard) is generated independently. */

/* Native Latin hypercube (replaces scipy.stats.qmc.LatinHypercube._random_lhs reached via
 * modeling.py:480,488): q = (pi_c(r) + 1 - u_c(pi_c(r))) / n where pi_c is a keyed bijection of
 * [0, n) (4-round Feistel network + cycle walking) and u_c(t) the jitter of stratum t (output t
 * of a SplitMix64 generator keyed by (seed, c)). */
int pbh_fill_lhs(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col0, int ncols, double* q,
                 int64_t ldq, void* stream);

/* Native pseudo-random uniforms in [0, 1) (Philox4x32-10), replaces modeling.py:484-486. */
int pbh_fill_uniform(uint64_t seed, int64_t row0, int64_t nrows, int col0, int ncols, double* q, int64_t ldq,
                     void* stream);

/* numpy's np.random.RandomState(...).random((N, d)) bit for bit (MT19937, legacy double
 * a >> 5, b >> 6): what check_random_state(int | None | RandomState).random((size, d)) gives at
 * modeling.py:484-486, rows [row0, row0 + nrows) of it.  key_host / pos: the generator's state
 * (RandomState.get_state()[1:3]).  Workspace: pbh_mt19937_workspace_size (8 B per draw + the
 * 107 KB jump table).  pbh_mt19937_advance returns numpy's state after nwords 32-bit draws (key
 * block + pos), so that a caller-owned or the global RandomState advances exactly as in numpy. */
int pbh_mt19937_workspace_size(int64_t nrows, int32_t d, size_t* bytes);
int pbh_mt19937_random(const uint32_t* key_host, int32_t pos, int64_t row0, int64_t nrows, int32_t d, double* q,
                       int64_t ldq, void* ws, size_t ws_bytes, void* stream);
int pbh_mt19937_advance(const uint32_t* key_host, int32_t pos, int64_t nwords, uint32_t* key_out_host,
                        int32_t* pos_out, void* ws, size_t ws_bytes, void* stream);

/* numpy's Generator(PCG64).random((nrows, d)) bit for bit, starting at draw index draw0 of the
 * stream whose 128-bit state / increment are state_host / inc_host ({low, high} words; numpy's
 * bit_generator.state["state"]): random_state=Generator at modeling.py:484-486, and the
 * rng.uniform(size=(n, d)) of scipy.stats.qmc.LatinHypercube._random_lhs. */
int pbh_pcg64_workspace_size(size_t* bytes);
int pbh_pcg64_random(const uint64_t* state_host, const uint64_t* inc_host, int64_t draw0, int64_t nrows, int32_t d,
                     double* q, int64_t ldq, void* ws, size_t ws_bytes, void* stream);

/* The reference's own Latin hypercube stream, opt-in parity mode (the default "lhs" path is the
 * native design of pbh_fill_lhs): scipy.stats.qmc.LatinHypercube(d, rng).random(n) bit for bit
 * (modeling.py:480,488 -> scipy:stats/_qmc.py LatinHypercube._random_lhs).  state_host / inc_host /
 * has32 / buf32: the engine Generator's PCG64 state before the call ({low, high} words and numpy's
 * buffered 32-bit half).  u = rng.uniform(size=(n, d)) is drawn on the device, the d Fisher-Yates
 * shuffles of arange(1, n + 1) (numpy Generator.shuffle: random_interval with masked rejection
 * on buffered 32-bit draws; one sequential stream) are decoded on the device: every draw is
 * classified against the band of states its column can be in, the few ambiguous ones are walked
 * in order on the host, and every decision is then re-checked against the rule at the state its
 * prefix implies; the permutation follows from the swap targets without replaying the swaps.  A
 * failed check retries with a wider band, then falls back to the host shuffles (parallel threads
 * after a counting pass).  q = (perm - u) / n is combined on the device into q (column-major,
 * column c at q + c * ldq).  n < 2^31.  Workspace: pbh_lhs_reference_workspace_size.
 * pbh_lhs_reference_perms is the host half alone: the d permutations (d x n int32, row c = the
 * shuffled column c) from the stream state at the first shuffle draw; state_out_host (optional,
 * 4 words) receives the state after the last one (state low, high, has32, buf32). */
int pbh_lhs_reference_workspace_size(int64_t n, int32_t d, size_t* bytes);
int pbh_lhs_reference(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32, uint32_t buf32, int64_t n,
                      int32_t d, double* q, int64_t ldq, void* ws, size_t ws_bytes, void* stream);
/* As pbh_lhs_reference, and strata (device int32, column c at strata + c * lds, lds >= n; may be
 * NULL) receives each row's stratum: strata[c][r] = perms[r, c] - 1, so q[c][r] lies in
 * (strata / n, (strata + 1) / n] -- the rank - 1 of q[c][r] in its column. */
int pbh_lhs_reference_strata(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32, uint32_t buf32,
                             int64_t n, int32_t d, double* q, int64_t ldq, int32_t* strata, int64_t lds, void* ws,
                             size_t ws_bytes, void* stream);
int pbh_lhs_reference_perms(const uint64_t* state_host, const uint64_t* inc_host, int32_t has32, uint32_t buf32,
                            int64_t n, int32_t d, int32_t* perms_host, uint64_t* state_out_host);
/* The device decode's band half-width in standard deviations of the steps done (default 6; each
 * retry doubles it); sigmas = 0 only reads it.  pbh_lhs_reference_stats: the last call's record
 * (device = 1: decoded on the device; attempts; ambiguous draws walked on the host). */
int pbh_lhs_reference_band(double sigmas, double* previous);
/* The process cache of inverse-CDF setup tables (gamma / beta guides, poisson / binom / nbinom CDF
 * tables, keyed by their scalar parameters; pbh_table_cache.hip): tables held, their bytes, and
 * the calls served from it.  The cache holds at most 1 GiB and 4 096 tables of <= 64 MiB each
 * (larger ones are built per call); when full, the least recently used table no call holds is
 * evicted.  pbh_table_cache_clear frees every table no call holds (after the kernels that read
 * them), reporting how many it freed and kept; safe between calls. */
int pbh_table_cache_stats(int64_t* entries, int64_t* bytes, int64_t* hits);
int pbh_table_cache_clear(int64_t* freed, int64_t* kept);
int pbh_lhs_reference_stats(int32_t* device, int32_t* attempts, int64_t* ambiguous);

/* Scrambled Halton points, bit-exact with scipy.stats.qmc.Halton(d, rng=...) (modeling.py:481,488):
 * column c is the van der Corput sequence in base bases_host[c] with counts_host[c] digit
 * permutations (perms_host: concatenated counts_host[c] x bases_host[c] tables, produced by the
 * host-side engine setup from the engine's Generator).  Rows [row0, row0 + nrows) = sequence
 * indices; columns [col0, col0 + ncols).  Workspace: pbh_halton_workspace_size. */
int pbh_halton_workspace_size(const int32_t* bases_host, const int32_t* counts_host, int d, size_t* bytes);
int pbh_fill_halton(const int32_t* bases_host, const int32_t* counts_host, const int32_t* perms_host, int d,
                    int64_t row0, int64_t nrows, int col0, int ncols, double* q, int64_t ldq, void* ws,
                    size_t ws_bytes, void* stream);

/* Scrambled Sobol' points, bit-exact with scipy.stats.qmc.Sobol (modeling.py:482,488):
 * x_r[c] = (shift[c] ^ XOR_{b in gray(r)} sv[c][b]) * 2^-bits.  sv_host is d x bits (row-major),
 * shift_host has d entries (both produced by the host-side engine setup). */
int pbh_fill_sobol(const uint32_t* sv_host, const uint32_t* shift_host, int d, int bits, int64_t row0,
                   int64_t nrows, int col0, int ncols, double* q, int64_t ldq, void* stream);

/* One scrambled Sobol' column (as pbh_fill_sobol: column `col` of d, `bits`, rows [row0, row0 +
 * nrows)) pushed through the inverse CDF of `dist` in one kernel, the quantile never stored:
 * out[r] = ppf(q(row0 + r)) (replaces the "sobol" branch of Node.sample, modeling.py:482,488,
 * followed by Distribution._sample, :795-807).  dist < PBH_DIST_BETA; others return
 * PBH_ERR_UNSUPPORTED (materialise with pbh_fill_sobol + pbh_ppf). */
int pbh_sobol_ppf(const uint32_t* sv_host, const uint32_t* shift_host, int d, int bits, int64_t row0, int64_t nrows,
                  int col, int dist, const pbh_param* params, int nparams, double* out, int32_t* nonfinite_flag,
                  void* stream);

/* ---------------------------------------------------------------- inverse CDF sweep
 * Distribution._sample (modeling.py:795-807) -> scipy rv_continuous.ppf / rv_discrete.ppf:
 * out[i] = ppf(q[i * q_stride]; params) with scipy's argument checks, support bounds at
 * q == 0 / 1, NaN for invalid input and `_ppf(q) * scale + loc` rounding (no FMA).
 * When nonfinite_flag != NULL it is set to 1 if any output is non-finite (the check of
 * modeling.py:600-606, fused into the producing kernel). */
int pbh_ppf(int dist, const double* q, int64_t q_stride, int64_t n, const pbh_param* params, int nparams,
            double* out, int32_t* nonfinite_flag, void* stream);

/* Fused generator + inverse CDF (q never touches HBM): column `col` of the native LHS
 * design of pbh_fill_lhs pushed through `dist`.  Bit-identical to pbh_fill_lhs + pbh_ppf. */
int pbh_lhs_ppf(uint64_t seed, int64_t n, int64_t row0, int64_t nrows, int col, int dist,
                const pbh_param* params, int nparams, double* out, int32_t* nonfinite_flag, void* stream);

/* ---------------------------------------------------------------- Iman-Conover
 * ImanConover.__call__ (correlation.py:368-425) on device:
 *   step 1  ranks = rankdata(X, axis=0, 'average') / (N + 1); S = ndtri(ranks)     (:394-395)
 *   step 2  E = corrcoef(S); E must be PD; L = cholesky(E)                        (:398-405)
 *   step 3  CS = S L^-T P^T  with P = cholesky(target) (target_chol_host, K x K
 *           row-major lower triangular, Correlator.set_target :177-178)         (:409-414)
 *   step 4  idx = rankdata(CS[:, k]).astype(int) - 1; Y[:, k] = sort(X[:, k])[idx]  (:418-423)
 * X element (r, c) is read at X[r * x_rs + c * x_cs]; Y is written at Y[r * y_rs + c * y_cs].
 * Returns PBH_ERR_NOT_PD when E is not positive definite, PBH_ERR_NONFINITE for NaN/inf in X.
 * The optional outputs (device pointers, column-major K x N, may be NULL) expose the
 * intermediates for parity tests: scores S, correlated scores CS, step-4 indices idx. */
/* An Iman-Conover input column that is GENERATED instead of read: column `lhs_col` of the
 * native LHS design of pbh_fill_lhs(seed, n) pushed through distribution `dist` (scalar
 * params).  This is how the DAG evaluator hands over initial sampling nodes that feed a
 * correlate() (modeling.py:529-538, 571-583): their pre-correlation samples are never
 * observable, so the device generates each column directly in sorted (stratum) order,
 * verifies it is non-decreasing, and derives the step-1 ranks from the LHS permutation --
 * no sort of X.  A column whose ppf is not monotone on the grid falls back to the sort path.
 * nonfinite_flag (optional, device) is set when a generated value is NaN / inf. */
typedef struct pbh_ic_column {
  uint64_t seed;
  int32_t lhs_col;
  int32_t dist;
  double params[4];
  int32_t nparams;
  int32_t* nonfinite_flag;
} pbh_ic_column;

typedef struct pbh_ic_args {
  const pbh_ic_column* columns; /* host array of k generated columns, or NULL: read X */
  const double* X;
  int64_t n;
  int32_t k;
  int64_t x_rs, x_cs;
  const double* target_chol_host;
  double* Y;
  int64_t y_rs, y_cs;
  void* ws;
  size_t ws_bytes;
  double* scores_out;
  double* cscores_out;
  int32_t* idx_out;
  double* corr_host_out; /* optional K x K host buffer: E = corrcoef(S) */
  /* optional (X only): host array of k device pointers, NULL entries allowed.  strata[c][r] =
   * rank - 1 of row r in column c when known (an LHS column's strata, e.g. the reference
   * stream's decoded shuffles, pbh_lhs_reference_strata): step 1 then puts X[:, c] in order by
   * one scatter instead of a sort, and keeps it only if the result is certified sorted (no
   * inversion, no stratum missed); otherwise the column is sorted as usual.  Results are the
   * same either way. */
  const int32_t* const* strata;
} pbh_ic_args;

int pbh_ic_workspace_size(int64_t n, int32_t k, size_t* bytes);
int pbh_iman_conover(const pbh_ic_args* args, void* stream);

/* ---------------------------------------------------------------- Iman-Conover phases
 * The four steps of pbh_iman_conover as separate calls, for row-sharded execution across
 * GPUs (probabilit_amd/distributed.py): every rank holds rows
 * [row0, row0 + nrows) of the N-row problem, sums its Gram partials with the other ranks
 * (one K x K all-reduce), and each column's step 4 runs on the rank that owns the column. */

/* Sorted values of a generated LHS column for the strata [t0, t0 + nt) (t = rank - 1 of the
 * point in its column): out[t - t0] = ppf((t + 1 - u) / n).  params_host: the scalar
 * parameters in pbh_dist order.  This is np.sort(X[:, k]) of correlation.py:423 for a
 * column the DAG generates (modeling.py:480, 488 + 807). */
int pbh_lhs_sorted_ppf(uint64_t seed, int64_t n, int64_t t0, int64_t nt, int col, int dist,
                       const double* params_host, int nparams, double* out, int32_t* nonfinite_flag,
                       void* stream);
/* The same segment [t0, t0 + nt) counted, not stored (asynchronous; the step-1 check of a
 * shard before its scores, correlation.py:394): counts_dev (2 device u64, zeroed first) +=
 * (#(x[t] == x[t+1]), #!(x[t] <= x[t+1])) over the pairs inside the segment.  heads (optional,
 * device u32, hcap entries): the run heads -- every t in (t0, t0 + nt) whose value differs from
 * stratum t - 1's, plus t0 itself when t0 == 0 -- unordered, at most hcap written; *hcur_dev
 * (device u32) counts them all.  A shard starting at row0 > 0 passes t0 = row0 - 1, so that the
 * pair across the shard boundary is counted exactly once.  certify != 0 (continuous columns,
 * no heads): the tie / inversion certificate instead of the counts -- the inverse CDF evaluated
 * only at the pairs whose quantile gap its error bound could close (see pbh_ppf.hip); counts
 * then read non-zero unless the segment is certified free of ties and inversions, and a caller
 * that sees non-zero recounts exactly. */
int pbh_lhs_sorted_counts(uint64_t seed, int64_t n, int64_t t0, int64_t nt, int col, int dist,
                          const double* params_host, int nparams, unsigned long long* counts_dev, uint32_t* heads,
                          uint32_t* hcur_dev, uint32_t hcap, int32_t* nonfinite_flag, int certify, void* stream);
/* heads[0 .. nh) in increasing order, nh <= 16384 (the run heads pbh_lhs_sorted_counts appends). */
int pbh_sort_heads(uint32_t* heads, int64_t nh, void* stream);
/* Adjacent-pair check of a column: *ties = #(x[t] == x[t+1]), *inversions = #!(x[t] <= x[t+1]).
 * ws: 256 bytes of device memory.  Synchronises the stream. */
int pbh_sorted_check(const double* x, int64_t n, int64_t* ties, int64_t* inversions, void* ws, void* stream);
/* Run heads of a sorted segment x[0..m) = strata [t0, t0 + m): the positions whose value
 * differs from the previous one (scipy _rankdata's `obs` flags, reached from
 * correlation.py:394).  With first_is_prev, x[0] is the value of stratum t0 - 1 and is not
 * itself reported.  heads (device, u32) receive t values in order; *count their number. */
int pbh_run_heads_workspace_size(int64_t m, size_t* bytes);
int pbh_run_heads(const double* x, int64_t m, int64_t t0, int first_is_prev, uint32_t* heads, int64_t* count,
                  void* ws, size_t ws_bytes, void* stream);
/* Step 1 for rows [row0, row0 + nrows) of a generated LHS column (correlation.py:394-395):
 * S[r - row0] = ndtri(rank / (N + 1)), rank = pi(r) + 1, or the 'average' rank of the run of
 * stratum pi(r) when heads (all run heads of the sorted column, heads[0] == 0) is given. */
int pbh_lhs_scores(uint64_t seed, int64_t n, int col, int64_t row0, int64_t nrows, const uint32_t* heads,
                   int64_t nheads, double* S, void* stream);
/* Step 2 pieces (correlation.py:398): column sums and the centered Gram matrix sum over rows
 * (S - means)^T (S - means) of a column-major block S (column stride ld); K x K row-major. */
int pbh_gram_workspace_size(int32_t k, size_t* bytes);
int pbh_column_sums(const double* S, int64_t n, int32_t k, int64_t ld, double* sums, void* ws, size_t ws_bytes,
                    void* stream);
int pbh_centered_gram(const double* S, int64_t n, int32_t k, int64_t ld, const double* means, double* gram,
                      void* ws, size_t ws_bytes, void* stream);
/* Host: E = corrcoef from the summed Gram matrix over n rows (np.cov / np.corrcoef order),
 * the positive-definiteness check and L = cholesky(E) (correlation.py:398-405).  Returns
 * PBH_ERR_NOT_PD with the reference's message. */
int pbh_ic_factor(const double* gram_host, int64_t n, int32_t k, double* corr_host_out, double* L_host_out);
/* Step 3 in place (correlation.py:409-414): S <- (S L^-T) P^T, P = cholesky(target).
 * ws >= (2 K^2 + K) doubles of device memory. */
int pbh_ic_apply(double* S, int64_t n, int32_t k, int64_t ld, const double* L_host, const double* target_chol_host,
                 void* ws, size_t ws_bytes, void* stream);
/* Step 4 for one column (correlation.py:418-423): y[r * y_rs] = sorted_src[rank(cs[r]) - 1],
 * idx_out[r] = rank - 1 (optional). */
int pbh_ic_reorder_workspace_size(int64_t n, size_t* bytes);
int pbh_ic_reorder(const double* cs, int64_t n, const double* sorted_src, double* y, int64_t y_rs, int32_t* idx_out,
                   void* ws, size_t ws_bytes, void* stream);
/* Step 1 for one materialised column on its owner (correlation.py:394-395): scores[r] =
 * ndtri(rankdata(x)[r] / (n + 1)) and, when sorted_x is not NULL, sorted_x = np.sort(x) (the
 * sort(X[:, k]) of :423, kept for the owner's pbh_ic_reorder).  Same kernels as a materialised
 * column of pbh_iman_conover; a NaN in x sets *nonfinite_flag (device, optional).
 * ws >= pbh_rank_workspace_size(n).  Synchronises the stream. */
int pbh_ic_column_scores(const double* x, int64_t stride, int64_t n, double* scores, double* sorted_x,
                         int32_t* nonfinite_flag, void* ws, size_t ws_bytes, void* stream);

/* Step 4 of the columns a rank owns in a row-sharded run (correlation.py:418-423 for the column
 * owner): m generated columns (as pbh_iman_conover's `columns`) of an
 * n-row design whose correlated scores arrive whole, one column at a time.
 *   pbh_ic_owned_create   gen tables + workspace carve (stream-ordered on `stream`)
 *   pbh_ic_owned_column   column i: y[r * y_rs] = sort(X[:, i])[rank(cs[r]) - 1] by the single-GPU
 *                         step-4 passes (codes, top-16 histogram with the adaptive code map, MSD
 *                         code passes, bucket finish, row placement, sort(X)[p] regenerated), on a
 *                         step-4 side stream that first waits for ready_event (a pbh event; NULL:
 *                         `stream`'s work so far); done_event (optional) is recorded when y is
 *                         complete.  With p_out (device u32, n) the sorted positions p[r] =
 *                         rank(cs[r]) - 1 are written instead of y (y may be NULL): 4 bytes a row
 *                         to send back, the row owners regenerate Y with pbh_lhs_values_at.  No
 *                         host synchronisation.  cs, y / p_out must stay valid until
 *                         pbh_ic_owned_finish returns.
 *   pbh_ic_owned_finish   the caller's stream joins the lanes; one readback of every column's
 *                         verdict; a column the fast passes rejected (spiky codes, runs of equal
 *                         codes beyond the finish) is redone by the general path, redone_host[i]
 *                         = 1 for it (its y changed after done_event).  Synchronises `stream`.
 *   pbh_ic_owned_destroy  frees the tables (after the lanes).
 * Calls on one device are not concurrent (one host thread per device). */
typedef struct pbh_ic_owned pbh_ic_owned;
int pbh_ic_owned_workspace_size(int64_t n, int32_t m, size_t* bytes);
int pbh_ic_owned_create(const pbh_ic_column* columns, int32_t m, int64_t n, void* ws, size_t ws_bytes,
                        pbh_ic_owned** out, void* stream);
int pbh_ic_owned_column(pbh_ic_owned* h, int32_t i, const double* cs, double* y, int64_t y_rs, uint32_t* p_out,
                        void* ready_event, void* done_event, void* stream);
int pbh_ic_owned_finish(pbh_ic_owned* h, int32_t* redone_host, void* stream);
int pbh_ic_owned_destroy(pbh_ic_owned* h, void* stream);
/* Every uncorrelated native-LHS leaf of a graph in one call (the per-node loop of
 * Node.sample_from_quantiles, modeling.py:529-538, for leaf Distributions with scalar parameters):
 * column c of out (ld apart) = pbh_lhs_ppf of cols[c] over rows [row0, row0 + nrows); the columns'
 * setups and kernels run side by side on internal streams, joined to `stream`.  nonfinite_flag and
 * the params follow pbh_ic_column. */
int pbh_lhs_ppf_columns(const pbh_ic_column* cols, int32_t k, int64_t n, int64_t row0, int64_t nrows, double* out,
                        int64_t ld, void* stream);
/* y[i * y_rs] = sort(X[:, column])[p[i]] for i < m: a generated column's value at sorted
 * positions p (the row owner's half of a row-sharded step 4: Y[r] = sort(X)[rank - 1],
 * correlation.py:423, p from the column's owner). */
int pbh_lhs_values_at(const pbh_ic_column* column, int64_t n, const uint32_t* p, int64_t m, double* y, int64_t y_rs,
                      void* stream);
/* HIP events for ordering the caller's streams (torch / RCCL) with the library's lanes. */
int pbh_event_create(void** event);
int pbh_event_destroy(void* event);
int pbh_event_record(void* event, void* stream);
int pbh_stream_wait_event(void* stream, void* event);
int pbh_event_synchronize(void* event);

/* rankdata(x, method='average') of one device column (scipy:stats/_stats_py.py _rankdata,
 * called at correlation.py:394 and :422).  ws >= pbh_rank_workspace_size(n). */
int pbh_rank_workspace_size(int64_t n, size_t* bytes);
int pbh_rankdata_average(const double* x, int64_t stride, int64_t n, double* ranks, void* ws, size_t ws_bytes,
                         void* stream);

/* ---------------------------------------------------------------- transforms
 * Elementwise Transform nodes (modeling.py:933-1169): Variadic/Binary/UnaryTransform._sample
 * with numpy dtype semantics.  Operands are device vectors or scalars (ptr == NULL; the
 * lazily-broadcast Constant._sample of :760-763). */
typedef enum pbh_dtype { PBH_BOOL = 0, PBH_INT64 = 1, PBH_FLOAT64 = 2 } pbh_dtype;

typedef struct pbh_operand {
  const void* ptr; /* device vector, or NULL for a scalar                     */
  int32_t dtype;   /* pbh_dtype of the vector / scalar                        */
  double f;        /* scalar value when dtype == PBH_FLOAT64 (or BOOL as 0/1)  */
  int64_t i;       /* scalar value when dtype == PBH_INT64 / PBH_BOOL          */
} pbh_operand;

typedef enum pbh_op {
  /* binary */
  PBH_OP_ADD = 0, PBH_OP_SUB, PBH_OP_MUL, PBH_OP_TRUEDIV, PBH_OP_FLOORDIV, PBH_OP_MOD, PBH_OP_POW,
  PBH_OP_MAX, PBH_OP_MIN, PBH_OP_AND, PBH_OP_OR, PBH_OP_EQ, PBH_OP_NE, PBH_OP_LT, PBH_OP_LE, PBH_OP_GT,
  PBH_OP_GE, PBH_OP_ISCLOSE, PBH_OP_ARCTAN2,
  /* unary */
  PBH_OP_NEG = 32, PBH_OP_ABS, PBH_OP_LOG, PBH_OP_EXP, PBH_OP_FLOOR, PBH_OP_CEIL, PBH_OP_SIGN, PBH_OP_SQRT,
  PBH_OP_SQUARE, PBH_OP_LOG10, PBH_OP_SIN, PBH_OP_COS, PBH_OP_TAN, PBH_OP_ARCSIN, PBH_OP_ARCCOS,
  PBH_OP_ARCTAN, PBH_OP_SINH, PBH_OP_COSH, PBH_OP_TANH, PBH_OP_ARCSINH, PBH_OP_ARCCOSH, PBH_OP_ARCTANH,
  PBH_OP_CAST = 63
} pbh_op;

/* out = op(a, b) (b ignored for unary ops) computed in `compute_dtype` and stored as
 * `out_dtype` (the numpy result dtype decided on the host). */
int pbh_elementwise(int op, int compute_dtype, int out_dtype, const pbh_operand* a, const pbh_operand* b,
                    void* out, int64_t n, int32_t* nonfinite_flag, void* stream);

/* Avg (modeling.py:986-990): out = np.average(vstack(parents), axis=0) over m float64 vectors. */
int pbh_average(const double* const* parents_host, int m, int64_t n, double* out, int32_t* nonfinite_flag,
                void* stream);

/* ---------------------------------------------------------------- fused DAG program
 * One pass over the rows for a whole graph of scalar-parameter leaf Distributions
 * (norm / uniform / expon / lognorm / triang), Constants and float64 Transform nodes: the
 * per-node loop of Node.sample (modeling.py:586-612, Distribution._sample :795-807, the
 * Transform._sample methods :943-1075) as one kernel that keeps every intermediate row value
 * in registers and writes only the nodes the garbage collector keeps
 * (garbage_collector.py:40-71).  A straight-line program over row-vector registers r[0..7]
 * (an operand index of -1 reads the op's immediate `value` instead):
 *   PBH_DAG_GEN     r[dst] = ppf_{op = pbh_dist}(q(row); params)   q from sources[src]
 *   PBH_DAG_LOAD    r[dst] = vectors[src][row]
 *   PBH_DAG_CONST   r[dst] = value
 *   PBH_DAG_BINARY  r[dst] = op(r[a], r[b])        (float64 pbh_op, numpy semantics)
 *   PBH_DAG_UNARY   r[dst] = op(r[a])
 *   PBH_DAG_STORE   (nothing but the store below) of r[a]
 * Every op with store >= 0 also writes its value to vectors[store][row]; dst = -1 keeps it
 * out of the registers.  Values are bit-identical to the per-node kernels (pbh_sobol_ppf /
 * pbh_lhs_ppf / pbh_ppf, pbh_elementwise): same inline functions, -ffp-contract=off.  GEN /
 * LOAD / BINARY / UNARY with flag >= 0 OR bit 0 into flags[flag] when a value is non-finite. */
typedef enum pbh_dag_kind {
  PBH_DAG_GEN = 0, PBH_DAG_LOAD = 1, PBH_DAG_CONST = 2, PBH_DAG_BINARY = 3, PBH_DAG_UNARY = 4, PBH_DAG_STORE = 5
} pbh_dag_kind;
#define PBH_DAG_MAX_REGS 16
#define PBH_DAG_MAX_OPS 65536

typedef struct pbh_dag_op {
  int32_t kind;      /* pbh_dag_kind                                                   */
  int32_t op;        /* BINARY / UNARY: pbh_op; GEN: pbh_dist (norm..triang)            */
  int32_t dst, a, b; /* registers (-1: none / the immediate `value`)                    */
  int32_t src;       /* GEN: source index; LOAD: vector index                           */
  int32_t flag;      /* flag word index, -1 for none                                    */
  int32_t store;     /* vector index the value is also written to, -1 for none          */
  double value;      /* CONST, and the immediate operand of BINARY / UNARY / STORE      */
  double params[3];  /* GEN: scalar parameters in scipy order (shape..., loc, scale)    */
} pbh_dag_op;

/* Quantile source of a GEN op: the same streams as the per-node kernels.
 *   PBH_QSRC_SOBOL   q = (shift ^ xor of sv[b] over set bits of gray(row0 + i)) 2^-bits
 *                    (pbh_sobol_ppf; sv = the column's `bits` direction numbers)
 *   PBH_QSRC_LHS     the native LHS column `col` of an n_total-row design, row row0 + i
 *                    (pbh_lhs_ppf)
 *   PBH_QSRC_VECTOR  q[i * stride] (pbh_ppf) */
typedef enum pbh_qsource_kind { PBH_QSRC_SOBOL = 0, PBH_QSRC_LHS = 1, PBH_QSRC_VECTOR = 2 } pbh_qsource_kind;
typedef struct pbh_dag_qsource {
  int32_t kind;
  int32_t col;          /* LHS column                         */
  int32_t bits;         /* Sobol' bits (1..32)                */
  uint32_t shift;       /* Sobol' digital shift               */
  uint32_t sv[32];      /* Sobol' direction numbers           */
  uint64_t seed;        /* LHS seed                           */
  int64_t n_total;      /* LHS design rows                    */
  const double* q;      /* VECTOR quantiles (device)          */
  int64_t stride;       /* VECTOR stride (elements)           */
} pbh_dag_qsource;

/* Evaluate rows [0, n) (global rows row0 + i of the Sobol' / LHS streams).  vectors_host:
 * nvectors float64 device vectors of n rows (LOAD inputs and STORE outputs). */
int pbh_dag_eval(const pbh_dag_op* ops_host, int nops, const pbh_dag_qsource* sources_host, int nsources,
                 double* const* vectors_host, int nvectors, int64_t row0, int64_t n, int32_t* flags, void* stream);

/* Column-major <-> row-major transpose of an (rows x cols) float64 matrix (LDS-tiled). */
int pbh_transpose(const double* in, int64_t rows, int64_t cols, int64_t ld_in, double* out, int64_t ld_out,
                  void* stream);

/* ---------------------------------------------------------------- table distributions
 * Inverse CDF of the table-driven nodes (modeling.py:825-927): out[i] = f(q[i * q_stride]).
 *   PBH_TABLE_INTERP   CumulativeDistribution: np.interp(q, xp = t0, fp = t1)     (float64 out)
 *   PBH_TABLE_QUANTILE EmpiricalDistribution: np.quantile(t0 = sorted data, q, method)
 *                      method 0 linear, 1 lower, 2 higher, 3 nearest, 4 midpoint (float64 out)
 *   PBH_TABLE_SEARCH   DiscreteDistribution: t1[searchsorted(t0 = cumsum(p), q, 'right')],
 *                      t1 = values (float64 / int64 per out_dtype) or NULL for the index itself
 *                      (int64 out); an index past the table sets flag bit 2 (the reference
 *                      raises IndexError there).
 * Tables are device arrays of m entries; flag bit 0 = a non-finite float output. */
typedef enum pbh_table_kind { PBH_TABLE_INTERP = 0, PBH_TABLE_QUANTILE = 1, PBH_TABLE_SEARCH = 2 } pbh_table_kind;
int pbh_table_ppf(int kind, const double* q, int64_t q_stride, int64_t n, const double* t0, const void* t1, int64_t m,
                  int method, int out_dtype, void* out, int32_t* flag, void* stream);

/* ---------------------------------------------------------------- affine row transform
 * Y[r, j] = offset[j] + sum_i ((X[r, i] - shift[i]) / scale[i]) * M[i, j], rows r < n, k <= 128
 * (X[r, i] at X[r * x_rs + i * x_cs], likewise Y; M row-major k x k; scale_host NULL = 1).
 * The N-sized step of the Cholesky correlator (replaces correlation.py:271-285:
 * mean + ((X - mean) / std) @ (solve_triangular(P_x^T, P^T) * std)) and of decorrelate
 * (correlation.py:745-754: mean + (X - mean) @ inv(L)^T); the K x K factors come from
 * pbh_column_sums / pbh_centered_gram.  Workspace: pbh_affine_workspace_size. */
int pbh_affine_workspace_size(int32_t k, size_t* bytes);
int pbh_affine_rows(const double* X, int64_t n, int32_t k, int64_t x_rs, int64_t x_cs, const double* shift_host,
                    const double* scale_host, const double* offset_host, const double* M_host, double* Y,
                    int64_t y_rs, int64_t y_cs, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- permutation correlator
 * The hill-climbing loop of PermutationCorrelator.__call__ (replaces correlation.py:650-700 with
 * CorrelationMatrix.update_column / commit, :875-921, and _error, :582-586) as one persistent
 * workgroup.  xs: the measured columns X_ (k columns of n rows, column c at xs + c * ldx), swapped
 * in place; xo: the original X when it differs from X_ (spearman), swapped alongside, else NULL.
 * corr: device k x k row-major correlation matrix, updated in place.  den_host (k), target_host
 * and weights_host (k x k row-major, weights already divided by their sum): host, copied into
 * the workspace.  Step t (0 <= t < nsteps, nsteps a multiple of k) treats variable t % k with
 * swap rows swaps[offsets[t] .. offsets[t] + s) against the next s entries, s = (offsets[t + 1] -
 * offsets[t]) / 2 (device int64 arrays, the SwapIndexGenerator stream).  After each variable-0
 * step errlog[t / k] = the weighted RMS error; the loop stops after the first one below tol.
 * state[0] = steps run, state[1] = 1 when stopped by tol (device int64[2]).  1 <= k <= 128. */
int pbh_permcorr_workspace_size(int32_t k, size_t* bytes);
int pbh_permcorr_climb(double* xs, double* xo, int64_t n, int32_t k, int64_t ldx, double* corr, const double* den_host,
                       const double* target_host, const double* weights_host, const int64_t* swaps,
                       const int64_t* offsets, int64_t nsteps, double tol, double* errlog, int64_t* state, void* ws,
                       size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------- measurement
 * When enabled, every launch of the library's main kernels is bracketed by two HIP events
 * recorded on the launching stream; pbh_timing_read returns the summed device time and the
 * launch count of kernel `id` (names via pbh_kernel_name).  Used by bench.py's roofline. */
int pbh_timing_enable(int on);
/* Measurement mode (bench.py's standalone pass, the rocprof 1-stream profiles): with on != 0,
 * pbh_iman_conover runs every kernel on the caller's stream in order -- one step-4 lane, the
 * deferred tie checks in line -- so that each launch's duration is its own, not stretched by
 * concurrent kernels.  Results are identical either way. */
int pbh_set_serial(int on);
int pbh_timing_reset(void);
const char* pbh_kernel_name(int id);
int pbh_timing_read(int id, double* total_ms, int64_t* launches);
/* The box's HBM copy ceiling for bench.py (the measured peak reported beside the 8 TB/s spec):
 * dst = src over `bytes` (16-byte aligned), timed as kernel "k_hbm_copy".  variant 0: grid-stride
 * non-temporal 16-byte vectors; 1 / 2: one block per tile of 4 / 8 vectors per lane; 3 / 4: the
 * same non-temporal.  bench.py reports the fastest. */
int pbh_hbm_copy(const void* src, void* dst, size_t bytes, int variant, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PROBABILIT_HIP_H_ */
