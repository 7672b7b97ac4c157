// C-ABI entry points that orchestrate several kernels: Iman-Conover and rankdata.
//
// Host-side control stays here (plain C++, no Python): the K x K correlation assembly,
// the positive-definiteness check and the Cholesky factor of correlation.py:398-405 are
// O(K^3) with K <= 128 and run on the host between two device phases (one 8 KB D2H).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
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
  void* s4c = c.take(step4_gen_column_bytes(n) * step4_lanes_configured());
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
int launch_wait(hipEvent_t e, hipStream_t s) {
  if (e) PBH_CHECK_HIP(hipStreamWaitEvent(s, e, 0));
  return PBH_OK;
}

// Step 4's lanes: the side streams, each with one column's staging (and, for the owned columns
// of a row-sharded run, one column of codes); columns are dealt round robin.  begin(): every
// lane continues after the caller's stream so far; join(to): `to` continues after every lane.
// Events only, no host synchronisation.
struct Step4Lanes {
  int ns = 1;
  int rr = 0;
  hipStream_t s;
  hipStream_t ss[kStep4MaxStreams];
  Step4Column cb[kStep4MaxStreams];
  uint32_t* codes[kStep4MaxStreams];
  std::vector<hipEvent_t> events;
  Step4Lanes(int64_t n, void* column_ws, void* codes_ws, hipStream_t s_, int max_lanes = kStep4MaxStreams) : s(s_) {
    ns = step4_streams() < max_lanes ? step4_streams() : max_lanes;
    for (int i = 0; i < ns; ++i) {
      step4_gen_carve_column((char*)column_ws + (size_t)i * step4_gen_column_bytes(n), n, cb[i]);
      codes[i] = codes_ws ? (uint32_t*)((char*)codes_ws + (size_t)i * align256((size_t)n * 4)) : nullptr;
      ss[i] = ns > 1 ? step4_side_stream(i) : s;
      if (!ss[i]) ss[i] = s;
    }
  }
  ~Step4Lanes() {
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
  }
  int order(hipStream_t from, hipStream_t to) {  // `to` continues after `from`'s work so far
    if (from == to) return PBH_OK;
    hipEvent_t e = nullptr;
    PBH_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    events.push_back(e);
    PBH_CHECK_HIP(hipEventRecord(e, from));
    PBH_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
    return PBH_OK;
  }
  int begin() {
    for (int i = 0; i < ns; ++i) {
      int st = order(s, ss[i]);
      if (st) return st;
    }
    return PBH_OK;
  }
  int next() { return rr++ % ns; }
  int join(hipStream_t to = nullptr) {
    for (int i = 0; i < ns; ++i) {
      int st = order(ss[i], to ? to : s);
      if (st) return st;
    }
    return PBH_OK;
  }
};

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

extern "C" int pbh_set_serial(int on) {
  g_serial = on != 0;
  return PBH_OK;
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
  // the generated columns' inverse-CDF setups (tables built once, for step 1 and step 4);
  // declared before the guard below, so that on every return the tables are freed (stream
  // ordered, on s) only after the guard has synchronised the side streams that read them
  struct Gens {
    std::vector<GenColumn*> g;
    hipStream_t s;
    ~Gens() {
      for (GenColumn* x : g) gen_destroy(x, s);
    }
  } gens{std::vector<GenColumn*>(a->columns ? k : 0, nullptr), s};
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
  auto materialise = [&](int c) -> int {  // sort(X[:, c]) into the workspace, once
    if (have_sx[c] || !a->columns || !gens.g[c]) return PBH_OK;
    int r = gen_sorted(gens.g[c], 0, n, L.sorted_x + (int64_t)c * n, nullptr, nullptr, s);
    if (r == PBH_OK) have_sx[c] = 1;
    return r;
  };
  std::vector<char> deferred(k, 0);
  bool any_deferred = false;
  // a deferred column's check: the certificate (PBH_CERT=0: the exact counts) -- it can only
  // confirm "no tie, no inversion"; anything else reads as a count and redoes the call exactly
  static const bool cert_on = [] {
    const char* e = getenv("PBH_CERT");
    return !(e && e[0] == '0');
  }();
  auto count_deferred = [&](int c, hipStream_t cs_) -> int {
    double T = 0.0;
    uint32_t cap = 0;
    if (!cert_on || !gen_cert_plan(gens.g[c], n, &T, &cap))  // no bound, or as costly as the count
      return gen_sorted(gens.g[c], 0, n, nullptr, a->columns[c].nonfinite_flag, L.counts + 2 * c, cs_);
    uint32_t* list = nullptr;
    PBH_CHECK_HIP(hipMallocAsync((void**)&list, ((size_t)cap + 64) * 4, cs_));
    int r = gen_certify(gens.g[c], 0, n, T, list, cap, list + cap, a->columns[c].nonfinite_flag, L.counts + 2 * c,
                        cs_);
    PBH_CHECK_HIP(hipFreeAsync(list, cs_));
    return r;
  };
  if (a->columns && defer)
    for (int c = 0; c < k; ++c) any_deferred |= (deferred[c] = !gen_discrete(a->columns[c].dist)) != 0;
  if (a->columns) {
    // the columns' inverse-CDF tables (gamma / beta guides, poisson CDFs) and the discrete columns'
    // counts and run heads (small latency-bound kernels, ~1.8 ms one after another at cfg3) run
    // side by side on the step-4 lanes' streams, idle this early in the call; the caller's stream
    // then waits for all of them
    {
      const int nts = step4_streams();  // 1 in measurement mode (pbh_set_serial)
      // an early return below (a column's table or counts failing) leaves work queued on the side
      // streams that reads the tables ~Gens frees: join them on every exit path
      if (nts > 1) sync_on_exit.side = true;
      hipStream_t ts[kStep4MaxStreams];
      std::vector<hipEvent_t> tev;
      struct Cleanup {
        std::vector<hipEvent_t>& v;
        ~Cleanup() {
          for (hipEvent_t e : v) (void)hipEventDestroy(e);
        }
      } cleanup{tev};
      auto order = [&](hipStream_t from, hipStream_t to) -> int {
        if (from == to) return PBH_OK;
        hipEvent_t e = nullptr;
        PBH_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        tev.push_back(e);
        PBH_CHECK_HIP(hipEventRecord(e, from));
        PBH_CHECK_HIP(hipStreamWaitEvent(to, e, 0));
        return PBH_OK;
      };
      for (int i = 0; i < nts; ++i) {
        ts[i] = nts > 1 ? step4_side_stream(i) : s;
        if (!ts[i]) ts[i] = s;
        if ((st = order(s, ts[i]))) return st;
      }
      for (int c = 0; c < k; ++c) {
        const pbh_ic_column& g = a->columns[c];
        pbh_param prm[4];
        for (int j = 0; j < 4; ++j) prm[j] = pbh_param{nullptr, g.params[j]};
        st = gen_create(g.seed, n, g.lhs_col, g.dist, prm, g.nparams, &gens.g[c], ts[c % nts]);
        if (st) return st;
        if (deferred[c]) continue;  // counted next to steps 1-3 (below)
        // run heads only for a discrete column (few runs); a continuous one ties rarely, if ever,
        // and would append every stratum (on the stream that built the column's table)
        const bool discrete = gen_discrete(g.dist);
        st = gen_sorted(gens.g[c], 0, n, nullptr, g.nonfinite_flag, L.counts + 2 * c, ts[c % nts],
                        discrete ? L.heads_all + (int64_t)c * kHeadsCap : nullptr, discrete ? L.hcur + c : nullptr,
                        discrete ? kHeadsCap : 0);
        if (st) return st;
      }
      for (int i = 0; i < nts; ++i)
        if ((st = order(ts[i], s))) return st;
    }
    PBH_CHECK_HIP(hipMemcpyAsync(cnt_host.data(), L.counts, 16 * (size_t)k, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    for (int c = 0; c < k; ++c)
      if (deferred[c]) cnt_host[2 * c] = cnt_host[2 * c + 1] = 0;  // assumed; checked before step 4
  }
  // The operator API's row-major X (n, k) (correlation.py:368, numpy C order): every phase reads
  // whole columns, a 64-byte line per 8-byte value when strided, so the block is transposed once into
  // S (k x n; step 1 reads column c there before it writes c's scores over it) and Y is assembled
  // column-major in S (step 4 writes column c's values last, over its dead CS) and transposed back
  // (PBH_IC_TRANSPOSE=0: strided, the comparator)
  static const bool transpose_on = [] {
    const char* e = getenv("PBH_IC_TRANSPOSE");
    return !(e && e[0] == '0');
  }();
  const bool x_rows = transpose_on && a->X && !a->columns && k > 1 && a->x_cs == 1 && a->x_rs >= k;
  const bool y_rows = transpose_on && !a->columns && k > 1 && a->y_cs == 1 && a->y_rs >= k;
  const double* Xb = a->X;
  int64_t xb_rs = a->x_rs, xb_cs = a->x_cs;
  if (x_rows) {
    if ((st = rows_to_columns(a->X, a->x_rs, n, k, L.S, s))) return st;
    Xb = L.S;
    xb_rs = 1;
    xb_cs = n;
  }
  double* const Yb = y_rows ? L.S : a->Y;
  const int64_t yb_rs = y_rows ? 1 : a->y_rs, yb_cs = y_rows ? n : a->y_cs;
  // Materialised columns with known strata (a->strata[c]: each row's rank - 1, e.g. the
  // reference LHS stream's decoded shuffles): sort(X[:, c]) by one scatter, certified by its
  // tie / inversion counts (one readback for all of them); an inversion (a ppf not monotone on
  // the grid, a NaN, strata that are not a permutation) leaves the column to the sort below.
  std::vector<char> by_strata(k, 0);
  std::vector<unsigned long long> scnt(2 * (size_t)k, 0);
  if (a->strata && a->X && !a->columns) {
    bool any = false;
    for (int c = 0; c < k; ++c) {
      if (!a->strata[c]) continue;
      st = strata_sorted(Xb + (int64_t)c * xb_cs, xb_rs, a->strata[c], n, L.sorted_x + (int64_t)c * n,
                         L.counts + 2 * c, s);
      if (st) return st;
      by_strata[c] = any = true;
    }
    if (any) {
      PBH_CHECK_HIP(hipMemcpyAsync(scnt.data(), L.counts, 16 * (size_t)k, hipMemcpyDeviceToHost, s));
      PBH_CHECK_HIP(hipStreamSynchronize(s));
    }
  }
  // step 1's scores of a sorted column through the row placement rather than a random scatter
  // (PBH_SCORES_PLACE=0: the scatter, the comparator), where the placement passes pay: n >= 2^22
  static const bool scores_place_on = [] {
    const char* e = getenv("PBH_SCORES_PLACE");
    return !(e && e[0] == '0');
  }();
  const bool scores_placed = scores_place_on && n >= ((int64_t)1 << 22);
  for (int c = 0; c < k; ++c) {
    double* S_c = L.S + (int64_t)c * n;
    double* sx_c = L.sorted_x + (int64_t)c * n;
    const double* x_c = Xb ? Xb + (int64_t)c * xb_cs : nullptr;
    int64_t x_stride = xb_rs;
    if (by_strata[c] && scnt[2 * c + 1] == 0) {
      uint32_t* heads = nullptr;
      int64_t nheads = 0;
      if (scnt[2 * c] != 0) {  // ties: 'average' ranks from the runs of the sorted column
        heads = (uint32_t*)L.tmp;
        st = run_heads(sx_c, n, 0, false, heads, &nheads, L.heads_ws, s);
        if (st) return st;
      }
      st = strata_scores(a->strata[c], n, heads, nheads, S_c, s);
      if (st) return st;
      all_generated = false;
      have_sx[c] = 1;
      continue;
    }
    if (a->columns) {
      // generated LHS column: sorted order straight from the inverse permutation
      const pbh_ic_column& g = a->columns[c];
      pbh_param prm[4];
      for (int j = 0; j < 4; ++j) prm[j] = pbh_param{nullptr, g.params[j]};
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
          if (gen_discrete(a->columns[c].dist) && nheads <= cap) {  // appended heads, put in order
            heads = L.heads_all + (int64_t)c * kHeadsCap;
            st = sort_heads(heads, nheads, s);
            if (!st) st = gen_set_runs(gens.g[c], heads, nheads, s);  // step 4 reads each run's value
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
    bool redo = false;
    st = scores_placed ? radix_sort_keys_top48(sb, n, s, &buf, &redo) : radix_sort_keys(sb, n, s, &buf);
    if (st) return st;
    if (redo) {  // a long run of keys equal in their top 48 bits: every byte after all
      if ((st = load_keys(x_c, x_stride, n, sb.keys[0], L.flag, s))) return st;
      if ((st = radix_sort_keys(sb, n, s, &buf))) return st;
    }
    RankOut out = {};
    out.sorted_x = sx_c;
    if (scores_placed) {
      // the scores in rank order (contiguous), then into row order by the row placement (LSD
      // passes on the row, 8192-row blocks assembled in LDS): a random 8-byte scatter cost the
      // rank finish ~4.8x its bytes in HBM writes at 1e8 rows (pmc_traffic_r6p.json)
      out.scores = L.tmp;
      st = rank_finish(kModeScoresRank, sb.keys[buf], sb.vals[buf], n, tb, out, s);
      if (st) return st;
      PlaceBuffers pb;  // input rows: sb.vals[buf]; pass 1 -> [0], pass 2 -> [1] (the keys are dead)
      pb.rows[0] = sb.vals[buf ^ 1];
      pb.vals[0] = (double*)sb.keys[buf ^ 1];
      pb.rows[1] = sb.vals[buf];
      pb.vals[1] = (double*)sb.keys[buf];
      pb.counts = sb.counts;
      pb.partials = sb.partials;
      pb.status = sb.status;
      pb.sweep = &sb.sweep;
      pb.bases = sb.bases;
      st = place_by_row(sb.vals[buf], L.tmp, n, S_c, 1, pb, s);
    } else {
      out.scores = S_c;
      st = rank_finish(kModeScores, sb.keys[buf], sb.vals[buf], n, tb, out, s);
    }
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
  // PBH_COUNTS_STREAM (A/B): the side stream of the deferred counts -- lane 0 (default: the counts
  // run ahead of lane 0's first column) or the last one (never a step-4 lane with the default 3
  // lanes, but a 5th stream next to the caller's and the lanes, beyond the runtime's 4 hardware
  // queues: two streams then share a queue and serialise, measured 4-5 ms per step slower)
  static const int counts_stream = [] {  // lane 0: 161-162 ms per step against 166 on its own queue (r3 ab1)
    const char* e = getenv("PBH_COUNTS_STREAM");
    const int v = e ? atoi(e) : 0;
    return v < 0 ? 0 : (v >= kStep4MaxStreams ? kStep4MaxStreams - 1 : v);
  }();
  // (measurement mode, pbh_set_serial: the caller's stream, in order)
  hipStream_t side = any_deferred ? (g_serial ? s : step4_side_stream(counts_stream)) : nullptr;
  auto launch_counts = [&]() -> int {  // the deferred columns' counts on `side`, after s's work so far
    sync_on_exit.side = true;
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_scores.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventCreateWithFlags(&ev_counts.e, hipEventDisableTiming));
    PBH_CHECK_HIP(hipEventRecord(ev_scores.e, s));
    PBH_CHECK_HIP(hipStreamWaitEvent(side, ev_scores.e, 0));
    for (int c = 0; c < k; ++c) {
      if (!deferred[c]) continue;
      int r = count_deferred(c, side);
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
      st = count_deferred(c, side);
      if (st) return st;
    }
    PBH_CHECK_HIP(hipEventRecord(ev_counts.e, side));
  } else if (any_deferred) {  // no side stream: count in order
    for (int c = 0; c < k; ++c) {
      if (!deferred[c]) continue;
      st = count_deferred(c, s);
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
    // regenerated (pbh_step4.hip), on the side-stream lanes without a host round trip; a column
    // whose codes stay spiky after the adaptive code map, or that meets a run of equal codes
    // beyond the finish, is skipped on the device and redone by the general path after one
    // readback of every column's verdict at the end
    Step4Shared sh;
    step4_gen_carve_shared(L.s4shared, k, sh);
    Step4Lanes lanes(n, L.s4column, nullptr, s);
    sync_on_exit.side = sync_on_exit.side || lanes.ns > 1;
    st = step4_gen_hist(L.codes, n, nullptr, n, n, sh, 0, k, s);
    if (st) return st;
    // one readback of the flatness verdicts: the adaptive re-code is launched only for the
    // columns that need it (the gated kernels would otherwise be dispatched for every column)
    PBH_CHECK_HIP(hipMemcpyAsync(state.data(), sh.state, (size_t)k * 4, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    st = lanes.begin();
    if (st) return st;
    for (int c = 0; c < k; ++c) {
      if (!regenerable[c]) continue;
      const int i = lanes.next();
      hipStream_t cs_ = lanes.ss[i];
      if (state[c]) {
        st = step4_gen_adapt(L.codes + (int64_t)c * n, n, L.S + (int64_t)c * n, n, n, sh, c, 1, cs_);
        if (st) return st;
      }
      st = step4_gen_column(c, L.codes + (int64_t)c * n, L.S + (int64_t)c * n, n, sh, lanes.cb[i], cs_);
      if (st) return st;
      int buf = 0;
      st = step4_gen_place_passes(c, n, sh, lanes.cb[i], cs_, &buf);
      if (st) return st;
      st = gen_place(gens.g[c], lanes.cb[i].pairs[buf], n, a->Y + (int64_t)c * a->y_cs, a->y_rs,
                     a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, sh.flags + c, cs_);
      if (st) return st;
    }
    st = lanes.join();  // the caller's stream continues after every lane
    if (st) return st;
    // one readback: every column's state and flags (contiguous), and the deferred counts
    std::vector<int32_t> verdict(2 * (size_t)k);
    std::vector<unsigned long long> dc(2 * (size_t)k, 0);
    const bool late_counts = any_deferred && side && defer >= 2;
    if (late_counts) {
      st = launch_wait(ev_counts.e, s);
      if (st) return st;
      PBH_CHECK_HIP(hipMemcpyAsync(dc.data(), L.counts, 16 * (size_t)k, hipMemcpyDeviceToHost, s));
    }
    PBH_CHECK_HIP(hipMemcpyAsync(verdict.data(), sh.state, 8 * (size_t)k, hipMemcpyDeviceToHost, s));
    PBH_CHECK_HIP(hipStreamSynchronize(s));
    if (late_counts)
      for (int c = 0; c < k; ++c)
        if (deferred[c] && (dc[2 * c] | dc[2 * c + 1])) return kRedo;
    for (int c = 0; c < k; ++c) {
      if (verdict[c] == 0 && regenerable[c] && verdict[k + c] == 0) continue;
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
    // Materialised columns (X given) on the step-4 lanes, each lane with its own reorder
    // workspace carved from the generated path's per-lane staging (unused here): a column's code
    // sort waits for its run flags on the host (its lane only), while the other lanes go on with
    // the placements queued before it; the placements' look-back checks land in one device word
    // read once at the end.  (About half of a column's step 4 at 1e7 rows is latency: the
    // one-sweep look-back chains and the per-column readback.)  Two lanes: 75.7-76.3 ms per
    // reference-stream call at 1e7 x 32 against 77.2-78.5 with three (profiles/r05/ab_step_lanes_r5zd_refstream.log).
    const int nts = step4_streams();
    const bool lanes_on = !a->columns && nts > 1 && reorder_ws_bytes(n) <= step4_gen_column_bytes(n);
    if (lanes_on) {
      Step4Lanes lanes(n, L.s4column, nullptr, s, 2);
      std::vector<ReorderWs> lrw(lanes.ns);
      for (int i = 0; i < lanes.ns && st == PBH_OK; ++i)
        st = reorder_carve((char*)L.s4column + (size_t)i * step4_gen_column_bytes(n), n, lrw[i], s);
      if (st) return st;
      int32_t* err = L.flag + 1;
      PBH_CHECK_HIP(hipMemsetAsync(err, 0, sizeof(int32_t), s));
      sync_on_exit.side = true;
      if ((st = lanes.begin())) return st;
      for (int c = 0; c < k && st == PBH_OK; ++c) {
        const int i = lanes.next();
        const uint32_t* hc = hists ? hists + (size_t)c * 1024 : nullptr;
        const int flat = hists ? (code_hist_flat(hists_host.data() + (size_t)c * 1024, n) ? 1 : 0) : 1;
        st = reorder_column(L.S + (int64_t)c * n, n, L.sorted_x + (int64_t)c * n, Yb + (int64_t)c * yb_cs, yb_rs,
                            a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, lrw[i], lanes.ss[i],
                            L.codes + (int64_t)c * n, hc, flat, err);
      }
      const int sj = lanes.join();  // s (and the histograms' free on it) after every lane
      if (st) return st;
      if (sj) return sj;
      int32_t e = 0;
      PBH_CHECK_HIP(hipMemcpyAsync(&e, err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      PBH_CHECK_HIP(hipStreamSynchronize(s));
      if (e) {
        set_error("row placement: one-sweep look-back did not complete");
        return PBH_ERR_HIP;
      }
    } else {
      for (int c = 0; c < k && st == PBH_OK; ++c) {
        st = materialise(c);
        if (st) break;
        const uint32_t* hc = hists ? hists + (size_t)c * 1024 : nullptr;
        const int flat = hists ? (code_hist_flat(hists_host.data() + (size_t)c * 1024, n) ? 1 : 0) : 1;
        st = reorder_column(L.S + (int64_t)c * n, n, L.sorted_x + (int64_t)c * n, Yb + (int64_t)c * yb_cs, yb_rs,
                            a->idx_out ? a->idx_out + (int64_t)c * n : nullptr, rw, s, L.codes + (int64_t)c * n,
                            hc, flat);
      }
    }
    if (st) return st;
    if (y_rows && (st = columns_to_rows(L.S, n, k, a->Y, a->y_rs, s))) return st;
  }
  if (any_deferred && side && defer >= 2 && !(a->columns && any_regen && step4_gen_enabled(n))) {
    st = check_counts();  // (checked with the step-4 verdicts above on the generated path)
    if (st) return st;
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));  // host vectors above were sources of async copies
  return PBH_OK;
}
}  // namespace

// ---------------------------------------------------------------- owned columns (row-sharded runs)
// Step 4 of the columns a rank owns in the row-sharded Iman-Conover (probabilit_amd/
// distributed.py): each column's correlated scores arrive whole (an all-to-all from the row
// shards) and are ranked by the same passes as the single-GPU call -- codes, top-16 histogram
// (+ the adaptive code map), MSD code passes, bucket finish, row placement, gen_place -- on the
// step-4 lanes, column i starting when its `ready` event fires and recording `done` when its Y
// column is complete, so that exchanges and ranking overlap.  finish() reads every column's
// verdict once and redoes the rare rejected column by the general path.
struct pbh_ic_owned {
  int m = 0;
  int64_t n = 0;
  std::vector<GenColumn*> gens;
  Step4Shared sh;
  Step4Lanes* lanes = nullptr;
  ReorderWs rw;
  double* tmp = nullptr;   // the general path's sort(X)
  double* tmp2 = nullptr;  // and its Y when the caller asked for positions
  std::vector<const double*> cs;
  std::vector<uint32_t*> p_out;
  std::vector<double*> y;
  std::vector<int64_t> y_rs;
  std::vector<char> launched;
};

namespace {
struct OwnedLayout {
  void* shared;
  void* lanes;
  void* codes;
  void* reorder;
  void* tmp;
  void* tmp2;
};
size_t owned_bytes(int64_t n, int m, void* base, OwnedLayout* o) {
  Carver c(base);
  OwnedLayout l;
  l.shared = c.take(step4_gen_shared_bytes(m));
  l.lanes = c.take(step4_gen_column_bytes(n) * step4_lanes_configured());
  l.codes = c.take(align256((size_t)n * 4) * step4_lanes_configured());
  l.reorder = c.take(reorder_ws_bytes(n));
  l.tmp = c.take((size_t)n * 8);
  l.tmp2 = c.take((size_t)n * 8);
  if (o) *o = l;
  return c.used;
}
}  // namespace

extern "C" int pbh_ic_owned_workspace_size(int64_t n, int32_t m, size_t* bytes) {
  PBH_REQUIRE(bytes && n >= 2 && n < ((int64_t)1 << 32) && m >= 1 && m <= 128,
              "pbh_ic_owned_workspace_size: bad arguments");
  *bytes = owned_bytes(n, m, nullptr, nullptr);
  return PBH_OK;
}

extern "C" int pbh_ic_owned_create(const pbh_ic_column* columns, int32_t m, int64_t n, void* ws, size_t ws_bytes,
                                   pbh_ic_owned** out, void* stream) {
  PBH_REQUIRE(columns && ws && out && m >= 1 && m <= 128, "pbh_ic_owned_create: bad arguments");
  PBH_REQUIRE(n >= 2 && n < ((int64_t)1 << 32), "pbh_ic_owned_create: need 2 <= N < 2^32 (N=%lld)", (long long)n);
  const size_t need = owned_bytes(n, m, nullptr, nullptr);
  if (ws_bytes < need) {
    set_error("pbh_ic_owned_create: workspace %zu < %zu bytes", ws_bytes, need);
    return PBH_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  pbh_ic_owned* h = new pbh_ic_owned();
  h->m = m;
  h->n = n;
  h->gens.assign(m, nullptr);
  h->cs.assign(m, nullptr);
  h->y.assign(m, nullptr);
  h->y_rs.assign(m, 1);
  h->p_out.assign(m, nullptr);
  h->launched.assign(m, 0);
  OwnedLayout lay;
  owned_bytes(n, m, ws, &lay);
  step4_gen_carve_shared(lay.shared, m, h->sh);
  h->tmp = (double*)lay.tmp;
  h->tmp2 = (double*)lay.tmp2;
  int st = reorder_carve(lay.reorder, n, h->rw, s);
  for (int i = 0; st == PBH_OK && i < m; ++i) {
    const pbh_ic_column& g = columns[i];
    pbh_param prm[4];
    for (int j = 0; j < 4; ++j) prm[j] = pbh_param{nullptr, g.params[j]};
    st = gen_create(g.seed, n, g.lhs_col, g.dist, prm, g.nparams, &h->gens[i], s);
  }
  if (st == PBH_OK) {
    h->lanes = new Step4Lanes(n, lay.lanes, lay.codes, s);
    st = h->lanes->begin();  // the lanes start after the tables and the code map
  }
  if (st != PBH_OK) {
    (void)hipStreamSynchronize(s);
    for (GenColumn* g : h->gens) gen_destroy(g, s);
    delete h->lanes;
    delete h;
    return st;
  }
  *out = h;
  return PBH_OK;
}

extern "C" int pbh_ic_owned_column(pbh_ic_owned* h, int32_t i, const double* cs, double* y, int64_t y_rs,
                                   uint32_t* p_out, void* ready_event, void* done_event, void* stream) {
  PBH_REQUIRE(h && cs && (y || p_out) && i >= 0 && i < h->m, "pbh_ic_owned_column: bad arguments");
  PBH_REQUIRE(!h->launched[i], "pbh_ic_owned_column: column %d already launched", i);
  Step4Lanes& L = *h->lanes;
  const int j = L.next();
  hipStream_t ls = L.ss[j];
  if (ready_event)
    PBH_CHECK_HIP(hipStreamWaitEvent(ls, (hipEvent_t)ready_event, 0));
  else {
    int st = L.order(as_stream(stream), ls);
    if (st) return st;
  }
  const int64_t n = h->n;
  int st = make_codes(cs, n, h->rw.cm, L.codes[j], ls);
  if (!st) st = step4_gen_hist(L.codes[j], n, cs, n, n, h->sh, i, 1, ls);
  if (!st) st = step4_gen_column(i, L.codes[j], cs, n, h->sh, L.cb[j], ls);
  int buf = 0;
  if (!st) st = step4_gen_place_passes(i, n, h->sh, L.cb[j], ls, &buf);
  if (!st)
    st = p_out ? place_positions(L.cb[j].pairs[buf], n, p_out, h->sh.flags + i, ls)
               : gen_place(h->gens[i], L.cb[j].pairs[buf], n, y, y_rs, nullptr, h->sh.flags + i, ls);
  if (st) return st;
  if (done_event) PBH_CHECK_HIP(hipEventRecord((hipEvent_t)done_event, ls));
  h->cs[i] = cs;
  h->p_out[i] = p_out;
  h->y[i] = y;
  h->y_rs[i] = y_rs;
  h->launched[i] = 1;
  return PBH_OK;
}

extern "C" int pbh_ic_owned_finish(pbh_ic_owned* h, int32_t* redone_host, void* stream) {
  PBH_REQUIRE(h, "pbh_ic_owned_finish: null handle");
  hipStream_t s = as_stream(stream);
  const int m = h->m;
  int st = h->lanes->join(s);
  if (st) return st;
  std::vector<int32_t> verdict(2 * (size_t)m);
  PBH_CHECK_HIP(hipMemcpyAsync(verdict.data(), h->sh.state, 8 * (size_t)m, hipMemcpyDeviceToHost, s));
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  for (int i = 0; i < m; ++i) {
    const bool redo = h->launched[i] && (verdict[i] != 0 || verdict[m + i] != 0);
    if (redone_host) redone_host[i] = redo ? 1 : 0;
    if (!redo) continue;
    // the general path: sort(X) materialised, the column ranked by the code sort
    st = gen_sorted(h->gens[i], 0, h->n, h->tmp, nullptr, nullptr, s);
    if (!st && h->p_out[i])  // the positions: rank - 1 of every row (its Y is not needed)
      st = reorder_column(h->cs[i], h->n, h->tmp, h->tmp2, 1, (int32_t*)h->p_out[i], h->rw, s);
    else if (!st)
      st = reorder_column(h->cs[i], h->n, h->tmp, h->y[i], h->y_rs[i], nullptr, h->rw, s);
    if (st) return st;
  }
  PBH_CHECK_HIP(hipStreamSynchronize(s));
  return PBH_OK;
}

extern "C" int pbh_ic_owned_destroy(pbh_ic_owned* h, void* stream) {
  if (!h) return PBH_OK;
  hipStream_t s = as_stream(stream);
  if (h->lanes) (void)h->lanes->join(s);  // no lane may still read the tables being freed
  for (GenColumn* g : h->gens) gen_destroy(g, s);
  (void)hipStreamSynchronize(s);
  delete h->lanes;
  delete h;
  return PBH_OK;
}

// ---------------------------------------------------------------- events (stream ordering for callers)
extern "C" int pbh_event_create(void** event) {
  PBH_REQUIRE(event, "pbh_event_create: null pointer");
  hipEvent_t e = nullptr;
  PBH_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *event = (void*)e;
  return PBH_OK;
}

extern "C" int pbh_event_destroy(void* event) {
  if (event) PBH_CHECK_HIP(hipEventDestroy((hipEvent_t)event));
  return PBH_OK;
}

extern "C" int pbh_event_record(void* event, void* stream) {
  PBH_REQUIRE(event, "pbh_event_record: null event");
  PBH_CHECK_HIP(hipEventRecord((hipEvent_t)event, as_stream(stream)));
  return PBH_OK;
}

extern "C" int pbh_stream_wait_event(void* stream, void* event) {
  PBH_REQUIRE(event, "pbh_stream_wait_event: null event");
  PBH_CHECK_HIP(hipStreamWaitEvent(as_stream(stream), (hipEvent_t)event, 0));
  return PBH_OK;
}

extern "C" int pbh_event_synchronize(void* event) {
  PBH_REQUIRE(event, "pbh_event_synchronize: null event");
  PBH_CHECK_HIP(hipEventSynchronize((hipEvent_t)event));
  return PBH_OK;
}
