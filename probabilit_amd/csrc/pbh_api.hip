// C-ABI entry points that orchestrate several kernels: Iman-Conover and rankdata.
//
// Host-side control stays here (plain C++, no Python): the K x K correlation assembly,
// the positive-definiteness check and the Cholesky factor of correlation.py:398-405 are
// O(K^3) with K <= 128 and run on the host between two device phases (one 8 KB D2H).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "pbh_error.h"
#include "pbh_ic.h"
#include "pbh_lhs.h"
#include "pbh_sort.h"
#include "pbh_step4.h"

namespace pbh {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

namespace {

struct Carver {
  char* p;
  size_t used = 0;
  explicit Carver(void* base) : p((char*)base) {}
  void* take(size_t bytes) {
    void* r = p + used;
    used += (bytes + 255) & ~(size_t)255;
    return r;
  }
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

struct IcLayout {
  double* S;
  double* sorted_x;
  void* reorder_ws;             // step 4 (its sort / tie buffers also serve step 1's sorts)
  double* partials;
  double* means;
  double* gram;
  double* L;
  double* inv_diag;
  double* P;
  int32_t* flag;
  double* tmp;                  // n doubles: fallback X column, or the run heads (u32) of a tied column
  unsigned long long* counts;   // ties, inversions of a generated sorted column
  void* heads_ws;
  uint32_t* codes;              // K x n step-4 sort keys, written by the step-3 kernel
  double* colpart;              // K x perm_scores_blocks(n) per-block score sums (step-2 means)
  void* s4shared;               // step 4 of generated columns: per-column histograms, cursors
  void* s4column;               //   and one column's staging (pbh_step4.hip)
  uint32_t* heads_all;          // K x kHeadsCap run heads of the generated columns (unordered, then sorted)
  uint32_t* hcur;               // K head counts
};

size_t ic_bytes(int64_t n, int k, bool carve, void* base, IcLayout* L) {
  Carver c(base);
  void* S = c.take((size_t)n * k * 8);
  void* sx = c.take((size_t)n * k * 8);
  void* rws = c.take(reorder_ws_bytes(n));
  void* part = c.take(gram_partials_bytes(k));
  void* means = c.take((size_t)k * 8);
  void* gram = c.take((size_t)k * k * 8);
  void* Lm = c.take((size_t)k * k * 8);
  void* invd = c.take((size_t)k * 8);
  void* P = c.take((size_t)k * k * 8);
  void* flag = c.take(256);
  void* tmp = c.take((size_t)n * 8);
  void* counts = c.take(16 * 128);  // ties, inversions per generated column (k <= 128)
  void* hws = c.take(run_heads_ws_bytes(n));
  void* codes = c.take((size_t)n * k * 4);
  void* colpart = c.take((size_t)k * perm_scores_blocks(n) * 8);
  void* s4s = c.take(step4_gen_shared_bytes(k));
  void* s4c = c.take(step4_gen_column_bytes(n) * step4_streams());
  void* hall = c.take((size_t)k * kHeadsCap * 4);
  void* hcur = c.take((size_t)k * 4);
  if (carve) {
    L->heads_all = (uint32_t*)hall;
    L->hcur = (uint32_t*)hcur;
    L->s4shared = s4s;
    L->s4column = s4c;
    L->colpart = (double*)colpart;
    L->codes = (uint32_t*)codes;
    L->S = (double*)S;
    L->sorted_x = (double*)sx;
    L->reorder_ws = rws;
    L->partials = (double*)part;
    L->means = (double*)means;
    L->gram = (double*)gram;
    L->L = (double*)Lm;
    L->inv_diag = (double*)invd;
    L->P = (double*)P;
    L->flag = (int32_t*)flag;
    L->tmp = (double*)tmp;
    L->counts = (unsigned long long*)counts;
    L->heads_ws = hws;
  }
  return c.used;
}

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_version(void) { return 10000; }  // 1.0.0

extern "C" const char* pbh_last_error(void) { return pbh::g_last_error.c_str(); }

extern "C" int pbh_init(int device) {
  int count = 0;
  PBH_CHECK_HIP(hipGetDeviceCount(&count));
  PBH_REQUIRE(device >= 0 && device < count, "pbh_init: device %d not visible (%d devices)", device, count);
  hipDeviceProp_t prop;
  PBH_CHECK_HIP(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error("pbh_init: device %d is %s; this library is built for gfx950 (MI355X) only", device,
              prop.gcnArchName);
    return PBH_ERR_UNSUPPORTED;
  }
  PBH_CHECK_HIP(hipSetDevice(device));
  return PBH_OK;
}

extern "C" int pbh_ic_workspace_size(int64_t n, int32_t k, size_t* bytes) {
  PBH_REQUIRE(bytes != nullptr && n >= 1 && k >= 1, "pbh_ic_workspace_size: bad arguments");
  *bytes = ic_bytes(n, k, false, nullptr, nullptr);
  return PBH_OK;
}

extern "C" int pbh_rank_workspace_size(int64_t n, size_t* bytes) {
  PBH_REQUIRE(bytes != nullptr && n >= 1, "pbh_rank_workspace_size: bad arguments");
  *bytes = sort_workspace_bytes(n) + tie_workspace_bytes(n) + 512;
  return PBH_OK;
}

extern "C" int pbh_rankdata_average(const double* x, int64_t stride, int64_t n, double* ranks, void* ws,
                                    size_t ws_bytes, void* stream) {
  PBH_REQUIRE(x && ranks && ws, "pbh_rankdata_average: null pointer");
  PBH_REQUIRE(n >= 1 && n < ((int64_t)1 << 32), "pbh_rankdata_average: n out of range");
  size_t need = 0;
  pbh_rank_workspace_size(n, &need);
  if (ws_bytes < need) {
    set_error("pbh_rankdata_average: workspace %zu < %zu bytes", ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  Carver c(ws);
  SortBuffers sb;
  sort_carve(c.take(sort_workspace_bytes(n)), n, sb);
  TieBuffers tb;
  tie_carve(c.take(tie_workspace_bytes(n)), n, tb);
  uint32_t hist_host[8 * 256];
  sb.hist_host = hist_host;
  int st = load_keys(x, stride, n, sb.keys[0], nullptr, s);
  if (st) return st;
  int buf = 0;
  st = radix_sort_keys(sb, n, s, &buf);
  if (st) return st;
  RankOut out = {};
  out.ranks = ranks;
  return rank_finish(kModeRanks, sb.keys[buf], sb.vals[buf], n, tb, out, s);
}

namespace {
constexpr int kRedo = 1000;  // internal: a deferred tie / inversion check failed, run again undeferred

// defer: the tie / inversion counts of the generated continuous columns (which tie or invert with
// probability ~1e-8 per column at N = 1e8) run on a side stream next to steps 1-3 instead of
// before them, their scores computed as untied; the counts are checked before step 4 and, if any
// is non-zero, the whole call is redone with them first (kRedo).  The VALU-bound counting
// overlaps the bandwidth-bound Gram and step 3.
int ic_run(const pbh_ic_args* a, void* stream, int defer);
}  // namespace

extern "C" int pbh_iman_conover(const pbh_ic_args* a, void* stream) {
  PBH_REQUIRE(a != nullptr, "pbh_iman_conover: args must not be NULL");
  // PBH_DEFER_COUNTS: 0 = counts first; 1 = next to steps 1-3, checked before step 4;
  // 2 = next to step 4 (latency-bound passes: room for VALU work), checked at the end;
  // 3 = next to steps 1-3 (as 1), checked at the end: step 4 does not wait for them
  static const int defer = [] {
    const char* e = getenv("PBH_DEFER_COUNTS");
    return e ? atoi(e) : 3;
  }();
  int st = ic_run(a, stream, defer);
  if (st == kRedo) st = ic_run(a, stream, 0);
  return st;
}

namespace {
int ic_run(const pbh_ic_args* a, void* stream, int defer) {
  const int64_t n = a->n;
  const int k = a->k;
  PBH_REQUIRE((a->X || a->columns) && a->Y && a->ws && a->target_chol_host,
              "pbh_iman_conover: null pointer argument");
  PBH_REQUIRE(k >= 1 && k <= 128, "pbh_iman_conover: K = %d outside [1, 128]", k);
  PBH_REQUIRE(n > k && n < ((int64_t)1 << 32), "pbh_iman_conover: need K < N < 2^32 (N=%lld, K=%d)", (long long)n, k);
  IcLayout L;
  size_t need = ic_bytes(n, k, true, a->ws, &L);
  if (a->ws_bytes < need) {
    set_error("pbh_iman_conover: workspace %zu < %zu bytes", a->ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  // host buffers that asynchronous copies read or write: declared before the guard, whose
  // destructor synchronises the stream on every return (error returns included), so that no
  // copy outlives them
  std::vector<unsigned long long> cnt_host(2 * (size_t)k, 0);
  std::vector<double> G((size_t)k * k), Lc((size_t)k * k), invd(k), P((size_t)k * k);
  std::vector<int32_t> state(k), flags(k);
  std::vector<uint32_t> hists_host;
  int32_t flag_host = 0;
  struct SyncOnExit {
    hipStream_t s;
    bool side = false;
    ~SyncOnExit() {
      if (side) step4_sync_side_streams();  // step 4's side streams too (an error return mid-loop)
      (void)hipStreamSynchronize(s);
    }
  } sync_on_exit{s};
  ReorderWs rw;
  int st = reorder_carve(L.reorder_ws, n, rw, s);
  if (st) return st;
  SortBuffers& sb = rw.sb;
  TieBuffers& tb = rw.tb;

  // ---- step 1: van der Waerden scores of every column (+ the sorted column for step 4)
  PBH_CHECK_HIP(hipMemsetAsync(L.flag, 0, sizeof(int32_t), s));
  bool all_generated = true;  // every column's scores came from perm_scores (with partial sums)
  std::vector<char> regenerable(k, 0);  // step 4 may regenerate sort(X[:, c])[p] from p (gen_place)
  // Generated columns: every sorted column first, with its tie / inversion counts and run heads
  // but without storing it (step 4 regenerates sort(X)[p]; the fallbacks materialise it on
  // demand), then one readback for all of them (instead of a stream sync per column).
  std::vector<char> have_sx(k, 0);  // sorted_x column c holds sort(X[:, c])
  // the generated columns' inverse-CDF setups (tables built once, for step 1 and step 4)
  struct Gens {
    std::vector<GenColumn*> g;
    hipStream_t s;
    ~Gens() {
      for (GenColumn* x : g) gen_destroy(x, s);
    }
  } gens{std::vector<GenColumn*>(a->columns ? k : 0, nullptr), s};
  auto materialise = [&](int c) -> int {  // sort(X[:, c]) into the workspace, once
    if (have_sx[c] || !a->columns || !gens.g[c]) return PBH_OK;
    int r = gen_sorted(gens.g[c], 0, n, L.sorted_x + (int64_t)c * n, nullptr, nullptr, s);
    if (r == PBH_OK) have_sx[c] = 1;
    return r;
  };
  std::vector<char> deferred(k, 0);
  bool any_deferred = false;
  if (a->columns && defer)
    for (int c = 0; c < k; ++c) any_deferred |= (deferred[c] = a->columns[c].dist != PBH_DIST_POISSON) != 0;
  if (a->columns) {
    for (int c = 0; c < k; ++c) {
      const pbh_ic_column& g = a->columns[c];
      pbh_param prm[3];
      for (int j = 0; j < 3; ++j) prm[j] = pbh_param{nullptr, g.params[j]};
      st = gen_create(g.seed, n, g.lhs_col, g.dist, prm, g.nparams, &gens.g[c], s);
      if (st) return st;
      if (deferred[c]) continue;  // counted next to steps 1-3 (below)
      // run heads only for a discrete column (few runs); a continuous one ties rarely, if ever,
      // and would append every stratum
      const bool discrete = g.dist == PBH_DIST_POISSON;
      st = gen_sorted(gens.g[c], 0, n, nullptr, g.nonfinite_flag, L.counts + 2 * c, s,
                      discrete ? L.heads_all + (int64_t)c * kHeadsCap : nullptr, discrete ? L.hcur + c : nullptr,
                      discrete ? kHeadsCap : 0);
      if (st) return st;
    }
    PBH_CHECK_HIP(hipMemcpyAsync(cnt_host.data(), L.counts, 16 * (size_t)k, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    for (int c = 0; c < k; ++c)
      if (deferred[c]) cnt_host[2 * c] = cnt_host[2 * c + 1] = 0;  // assumed; checked before step 4
  }
  for (int c = 0; c < k; ++c) {
    double* S_c = L.S + (int64_t)c * n;
    double* sx_c = L.sorted_x + (int64_t)c * n;
    const double* x_c = a->X ? a->X + (int64_t)c * a->x_cs : nullptr;
    int64_t x_stride = a->x_rs;
    if (a->columns) {
      // generated LHS column: sorted order straight from the inverse permutation
      const pbh_ic_column& g = a->columns[c];
      pbh_param prm[3];
      for (int j = 0; j < 3; ++j) prm[j] = pbh_param{nullptr, g.params[j]};
      const unsigned long long* cnt = cnt_host.data() + 2 * c;
      if (cnt[1] == 0) {
        uint32_t* heads = nullptr;
        int64_t nheads = 0;
        if (cnt[0] != 0) {  // ties (discrete ppf): 'average' ranks from the runs of the sorted column
          nheads = n - (int64_t)cnt[0];  // no inversion: one head per distinct value
          const int64_t cap = [] {  // PBH_HEADS_CAP (tests): a smaller list, to reach the fallback
            const char* e = getenv("PBH_HEADS_CAP");
            const int64_t v = e ? atoll(e) : kHeadsCap;
            return v < 1 ? 1 : (v > kHeadsCap ? (int64_t)kHeadsCap : v);
          }();
          if (a->columns[c].dist == PBH_DIST_POISSON && nheads <= cap) {  // appended heads, put in order
            heads = L.heads_all + (int64_t)c * kHeadsCap;
            st = sort_heads(heads, nheads, s);
          } else {  // too many distinct values for the list: from the materialised column
            heads = (uint32_t*)L.tmp;
            st = materialise(c);
            if (!st) st = run_heads(sx_c, n, 0, false, heads, &nheads, L.heads_ws, s);
          }
          if (st) return st;
        }
        st = perm_scores(g.seed, n, g.lhs_col, 0, n, heads, nheads, S_c, s,
                         L.colpart + (int64_t)c * perm_scores_blocks(n));
        if (st) return st;
        regenerable[c] = 1;
        continue;
      }
      // not monotone on this grid: materialise the column in row order and sort it
      st = pbh_lhs_ppf(g.seed, n, 0, n, g.lhs_col, g.dist, prm, g.nparams, L.tmp, nullptr, stream);
      if (st) return st;
      x_c = L.tmp;
      x_stride = 1;
    }
    all_generated = false;
    st = load_keys(x_c, x_stride, n, sb.keys[0], L.flag, s);
    if (st) return st;
    int buf = 0;
    st = radix_sort_keys(sb, n, s, &buf);
    if (st) return st;
    RankOut out = {};
    out.scores = S_c;
    out.sorted_x = sx_c;
    st = rank_finish(kModeScores, sb.keys[buf], sb.vals[buf], n, tb, out, s);
    if (st) return st;
    have_sx[c] = 1;
  }
  struct Ev {
    hipEvent_t e = nullptr;
    hipStream_t wait_on = nullptr;  // ev_counts: the caller's stream waits for the side stream
    ~Ev() {                         // (destroyed before gens, whose tables are freed on s)
      if (e && wait_on) (void)hipStreamWaitEvent(wait_on, e, 0);
      if (e) (void)hipEventDestroy(e);
    }
  } ev_scores, ev_counts;
  ev_counts.wait_on = s;
  hipStream_t side = any_deferred ? step4_side_stream(defer == 2 ? kStep4MaxStreams - 1 : 0) : nullptr;
  auto launch_counts = [&]() -> int {  // the deferred columns' counts on `side`, after s's work so far
    sync_on_exit.side = true;
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_scores.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_counts.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventRecord(ev_scores.e, s));
    PBH_CHECK_HIP(hipStreamWaitEvent(side, ev_scores.e, 0));
    for (int c = 0; c < k; ++c) {
      if (!deferred[c]) continue;
      int r = gen_sorted(gens.g[c], 0, n, nullptr, a->columns[c].nonfinite_flag, L.counts + 2 * c, side);
      if (r) return r;
    }
    PBH_CHECK_HIP(hipEventRecord(ev_counts.e, side));
    return PBH_OK;
  };
  auto check_counts = [&]() -> int {  // PBH_OK, or kRedo when a deferred column ties / inverts
    if (ev_counts.e) PBH_CHECK_HIP(hipStreamWaitEvent(s, ev_counts.e, 0));
    std::vector<unsigned long long> dc(2 * (size_t)k, 0);
    PBH_CHECK_HIP(hipMemcpyAsync(dc.data(), L.counts, 16 * (size_t)k, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    for (int c = 0; c < k; ++c)
      if (deferred[c] && (dc[2 * c] | dc[2 * c + 1])) return kRedo;
    return PBH_OK;
  };
  if (any_deferred && side && defer == 2) {
    // launched after step 3 (below)
  } else if (any_deferred && side) {
    sync_on_exit.side = true;
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_scores.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_counts.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventRecord(ev_scores.e, s));  // the gens' tables are built; the scores are queued
    PBH_CHECK_HIP(hipStreamWaitEvent(side, ev_scores.e, 0));
    for (int c = 0; c < k; ++c) {
      if (!deferred[c]) continue;
      st = gen_sorted(gens.g[c], 0, n, nullptr, a->columns[c].nonfinite_flag, L.counts + 2 * c, side);
      if (st) return st;
    }
    PBH_CHECK_HIP(hipEventRecord(ev_counts.e, side));
  } else if (any_deferred) {  // no side stream: count in order
    for (int c = 0; c < k; ++c) {
      if (!deferred[c]) continue;
      st = gen_sorted(gens.g[c], 0, n, nullptr, a->columns[c].nonfinite_flag, L.counts + 2 * c, s);
      if (st) return st;
    }
  }
  PBH_CHECK_HIP(hipMemcpyAsync(&flag_host, L.flag, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  if (a->scores_out)
    PBH_CHECK_HIP(hipMemcpyAsync(a->scores_out, L.S, (size_t)n * k * 8, hipMemcpyDeviceToDevice, s));

  // ---- step 2: E = corrcoef(S) on the host from the device Gram matrix
  if (all_generated)  // the scores kernels left per-block sums behind
    st = means_from_partials(L.colpart, (int)perm_scores_blocks(n), k, (double)n, L.means, s);
  else
    st = column_means(L.S, n, k, n, L.partials, L.means, s);
  if (st) return st;
  st = centered_gram(L.S, n, k, n, L.means, L.partials, L.gram, s);
  if (st) return st;
  PBH_CHECK_HIP(hipMemcpyAsync(G.data(), L.gram, (size_t)k * k * 8, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  if (flag_host) {
    set_error("Iman-Conover input contains NaN");
    return PBH_ERR_NONFINITE;
  }
  st = ic_factor(G.data(), n, k, a->corr_host_out, Lc.data());
  if (st) return st;
  for (int j = 0; j < k; ++j) invd[j] = 1.0 / Lc[(size_t)j * k + j];
  for (int i = 0; i < k; ++i)
    for (int j = 0; j < k; ++j) P[(size_t)i * k + j] = j <= i ? a->target_chol_host[(size_t)i * k + j] : 0.0;
  PBH_CHECK_HIP(hipMemcpyAsync(L.L, Lc.data(), (size_t)k * k * 8, hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(L.inv_diag, invd.data(), (size_t)k * 8, hipMemcpyHostToDevice, s));
  PBH_CHECK_HIP(hipMemcpyAsync(L.P, P.data(), (size_t)k * k * 8, hipMemcpyHostToDevice, s));

  // ---- step 3: CS = (S L^-T) P^T, in place
  st = apply_decorrelate_correlate(L.S, n, k, n, L.L, L.inv_diag, L.P, s, L.codes, n, &rw.cm);
  if (st) return st;
  if (a->cscores_out)
    PBH_CHECK_HIP(hipMemcpyAsync(a->cscores_out, L.S, (size_t)n * k * 8, hipMemcpyDeviceToDevice, s));

  // the deferred counts: any tie or inversion means the scores assumed untied were wrong
  if (any_deferred && side && defer == 2) {
    st = launch_counts();  // next to step 4; checked at the end
    if (st) return st;
  } else if (any_deferred && !(side && defer == 3)) {
    st = check_counts();
    if (st) return st;
  }

  // ---- step 4: Y[:, c] = sort(X[:, c])[rankdata(CS[:, c]).astype(int) - 1]
  auto general = [&](int c) {  // the general path (sorted X read from the workspace)
    int r = materialise(c);
    if (r) return r;
    return reorder_column(L.S + (int64_t)c * n, n, L.sorted_x + (int64_t)c * n, a->Y + (int64_t)c * a->y_cs, a->y_rs,
                          a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, rw, s, L.codes + (int64_t)c * n);
  };
  bool any_regen = false;
  for (int c = 0; c < k; ++c) any_regen |= regenerable[c] != 0;
  if (a->columns && any_regen && step4_gen_enabled(n)) {
    // generated columns: MSD code passes + bucket finish + row placement, sort(X)[p]
    // regenerated (pbh_step4.hip); one readback for all columns' flatness before, one for
    // over-long runs after
    Step4Shared sh;
    step4_gen_carve_shared(L.s4shared, k, sh);
    const int ns = step4_streams();
    sync_on_exit.side = sync_on_exit.side || ns > 1;
    Step4Column cbs[kStep4MaxStreams];
    hipStream_t ss[kStep4MaxStreams];
    for (int i = 0; i < ns; ++i) {
      step4_gen_carve_column((char*)L.s4column + (size_t)i * step4_gen_column_bytes(n), n, cbs[i]);
      ss[i] = ns > 1 ? step4_side_stream(i) : s;
      if (!ss[i]) ss[i] = s;
    }
    st = step4_gen_hist(L.codes, n, n, sh, s);
    if (st) return st;
    PBH_CHECK_HIP(hipMemcpyAsync(state.data(), sh.state, (size_t)k * 4, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));  // everything before is complete: the side streams may start
    int next = 0;
    for (int c = 0; c < k; ++c) {
      if (state[c] != 0 || !regenerable[c]) continue;
      const int i = next++ % ns;
      hipStream_t cs_ = ss[i];
      st = step4_gen_column(c, L.codes + (int64_t)c * n, L.S + (int64_t)c * n, n, sh, cbs[i], cs_);
      if (st) return st;
      int buf = 0;
      st = step4_gen_place_passes(c, n, sh, cbs[i], cs_, &buf);
      if (st) return st;
      st = gen_place(gens.g[c], cbs[i].pairs[buf], n, a->Y + (int64_t)c * a->y_cs, a->y_rs,
                     a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, sh.flags + c, cs_);
      if (st) return st;
    }
    for (int i = 0; i < ns; ++i) {  // the caller's stream continues after every side stream
      if (ss[i] == s) continue;
      PBH_CHECK_HIP(hipStreamSynchronize(ss[i]));
    }
    PBH_CHECK_HIP(hipMemcpyAsync(flags.data(), sh.flags, (size_t)k * 4, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    for (int c = 0; c < k; ++c) {
      if (state[c] == 0 && regenerable[c] && flags[c] == 0) continue;
      st = general(c);  // not flat, not regenerable, or a run of equal codes beyond the finish
      if (st) return st;
    }
  } else {
    // The code histograms of all columns up front, one readback for the bucket-path decisions.
    struct AsyncBuf {  // freed on every return (stream-ordered, before the guard's final sync)
      uint32_t* p = nullptr;
      hipStream_t s;
      ~AsyncBuf() {
        if (p) (void)hipFreeAsync(p, s);
      }
    } hb{nullptr, s};
    uint32_t*& hists = hb.p;
    if (code_buckets_enabled(n)) {
      PBH_CHECK_HIP(hipMallocAsync((void**)&hists, (size_t)k * 1024 * 4, s));
      for (int c = 0; c < k; ++c) {
        st = code_hist(L.codes + (int64_t)c * n, n, hists + (size_t)c * 1024, s);
        if (st) return st;
      }
      hists_host.resize((size_t)k * 1024);
      PBH_CHECK_HIP(hipMemcpyAsync(hists_host.data(), hists, (size_t)k * 1024 * 4, hipMemcpyDeviceToHost, s));
      PBH_CHECK_HIP(hipStreamSynchronize(s));
    }
    for (int c = 0; c < k && st == PBH_OK; ++c) {
      st = materialise(c);
      if (st) break;
      const uint32_t* hc = hists ? hists + (size_t)c * 1024 : nullptr;
      const int flat = hists ? (code_hist_flat(hists_host.data() + (size_t)c * 1024, n) ? 1 : 0) : 1;
      st = reorder_column(L.S + (int64_t)c * n, n, L.sorted_x + (int64_t)c * n, a->Y + (int64_t)c * a->y_cs, a->y_rs,
                          a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, rw, s, L.codes + (int64_t)c * n, hc,
                          flat);
    }
    if (st) return st;
  }
  if (any_deferred && side && defer >= 2) {
    st = check_counts();
    if (st) return st;
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // host vectors above were sources of async copies
  return PBH_OK;
}
}  // namespace
