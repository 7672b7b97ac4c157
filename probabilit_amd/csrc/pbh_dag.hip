// Fused DAG program: the per-node loop of Node.sample (modeling.py:586-612) for graphs of
// scalar-parameter leaf Distributions, Constants and float64 Transforms, as ONE pass over the
// rows.  The host (probabilit_amd.dag) turns the graph into a straight-line program over
// row-vector registers; this kernel runs it tile by tile, so an intermediate node that the
// garbage collector frees (garbage_collector.py:40-71) never touches HBM and a kept node costs
// exactly its 8-byte store.
//
// Roofline: 8 B per stored node per row + 8 B per LOAD (+ 8 B per vector quantile), nothing
// else; the inverse CDFs are FP64-VALU work (ndtri: 73 instructions in the centre, ~400 in
// the tail).  The README mutual fund with gc_strategy=[] stores 8 B per row for 20 norm draws,
// so it is VALU-bound; with gc_strategy=None it stores all 60 nodes, 480 B per row.
//
// Layout: block = 256 threads, tile = 1024 rows, item j of thread t is row base + 256 j + t
// (coalesced global and conflict-free LDS accesses).  The registers are rows of an LDS array,
// regs[R][1024] (dynamic shared memory, R = the registers the program uses): every operand
// index is block-uniform and an LDS row costs 2 B of LDS bandwidth per row byte, far below the
// ndtri arithmetic, whereas a VGPR register file indexed by a runtime index is either demoted to
// scratch or multiplies the VGPR budget by R.  norm / lognorm GENs queue their tail quantiles in
// LDS and drain them with the whole block (the tail compaction of pbh_ppf.hip), writing straight
// into the destination row.  Same inline functions as the per-node kernels and
// -ffp-contract=off, so every value is bit-identical to the unfused evaluation.
//
// Measured (cfg5, N=1e8, profiles/r02/dag_ab.jsonl): the kernel is bound by ndtri's FP64 work
// (~1.1 ms per draw column); uncapped it takes 229 VGPRs (2 waves per SIMD: the rational
// functions' float64 constants are hoisted out of the program loop), capped at 4 waves per
// SIMD it spills a little in the tail and the generic-operator calls and runs 15% faster; 8
// items per thread did not pay.
#include <math.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "pbh_error.h"
#include "pbh_ops.h"
#include "pbh_ppf_core.h"
#include "pbh_rng.h"
#include "pbh_timing.h"

namespace pbh {
namespace {

constexpr int kDBlock = 256;
#ifndef PBH_DAG_IPT
#define PBH_DAG_IPT 4
#endif
#ifndef PBH_DAG_WAVES
#define PBH_DAG_WAVES 4
#endif
#if PBH_DAG_WAVES > 0
#define PBH_DAG_OCC __attribute__((amdgpu_waves_per_eu(PBH_DAG_WAVES)))
#else
#define PBH_DAG_OCC
#endif
constexpr int kDIpt = PBH_DAG_IPT;
constexpr int kDTile = kDBlock * kDIpt;

struct DagQueue {  // TailQueue sized to one DAG tile
  double arg[kDTile];
  uint16_t pos[kDTile];
  int count;
};

struct DagSrc {
  int32_t kind;
  int32_t col;
  uint32_t shift;
  int32_t pad;
  double scale;
  const uint32_t* T;  // Sobol': the four 256-entry XOR tables of the column (global)
  uint64_t seed;
  int64_t n_total;
  const double* q;
  int64_t stride;
  double p[3];  // the GEN's scalar parameters (one source per GEN)
};

// The program as the kernel reads it: 32 bytes per op, one scalar load (and the next op's
// load in flight while this one runs).
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
struct DOp {
  uint32_t head;  // kind | op << 8 | (dst + 1) << 16 | (a + 1) << 24
  int32_t b, src, flag, store, pad;
  double value;
};
static_assert(sizeof(DOp) == 32, "DOp is one 32-byte scalar load");

PBH_DI int item(int j) { return j * kDBlock + threadIdx.x; }

// Quantiles of the tile's items from source s (rows beyond n get 0.5).
PBH_DI void gen_quantiles(const DagSrc& s, const uint32_t* T, int64_t row0, int64_t base, int64_t n,
                          double (&q)[kDIpt]) {
  if (s.kind == PBH_QSRC_SOBOL) {
#pragma unroll
    for (int j = 0; j < kDIpt; ++j) {
      const int64_t i = base + item(j);
      q[j] = i < n ? (double)sobol_point(T, s.shift, (uint64_t)(row0 + i)) * s.scale : 0.5;
    }
  } else if (s.kind == PBH_QSRC_LHS) {
    Philox ph(s.seed);
    FeistelPerm fp(ph, (uint64_t)s.n_total, (uint32_t)s.col);
#pragma unroll
    for (int j = 0; j < kDIpt; ++j) {
      const int64_t i = base + item(j);
      q[j] = i < n ? lhs_quantile(ph, fp, (uint64_t)(row0 + i), (uint32_t)s.col) : 0.5;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kDIpt; ++j) {
      const int64_t i = base + item(j);
      q[j] = i < n ? s.q[i * s.stride] : 0.5;
    }
  }
}

// out[item] = ppf_D(q) for the tile, ndtri's tail drained by the whole block (norm / lognorm).
// The caller has reset tq.count and synchronised.  Returns whether a valid row's value is
// non-finite (each thread for the values it computed).
template <int D>
PBH_DI bool gen_compacted(const double (&q)[kDIpt], const bool (&valid)[kDIpt], const double* p, double* out,
                          DagQueue& tq) {
  const PoissonTable pt{};
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kDIpt; ++j) {
    const bool tail = normal_takes_tail(q[j], normal_loc<D>(p[0], p[1]));  // never for rows past n (q = 0.5)
    if (!tail) {
      const double x = ppf_one<D, 1>(q[j], p[0], p[1], p[2], pt);
      out[item(j)] = x;
      bad |= valid[j] && !isfinite(x);
    }
    tail_push(tq, tail, q[j], item(j));
  }
  __syncthreads();
  const int T = tq.count;
#pragma unroll 1
  for (int t = threadIdx.x; t < T; t += kDBlock) {
    const double x = ppf_one<D, 2>(tq.arg[t], p[0], p[1], p[2], pt);
    out[tq.pos[t]] = x;
    bad |= !isfinite(x);
  }
  return bad;
}

template <int D>
PBH_DI bool gen_plain(const double (&q)[kDIpt], const bool (&valid)[kDIpt], const double* p, double* out) {
  const PoissonTable pt{};
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kDIpt; ++j) {
    const double x = ppf_one<D>(q[j], p[0], p[1], p[2], pt);
    out[item(j)] = x;
    bad |= valid[j] && !isfinite(x);
  }
  return bad;
}

// The operators beyond + - * / (pow, atan2, the transcendental unary ops), one element per
// call, so that unrolled inline copies do not size the registers of the whole program loop.
__device__ __noinline__ double binary_call(int op, double a, double b) { return f_binary(op, a, b); }
__device__ __noinline__ double unary_call(int op, double a) { return f_unary(op, a); }

PBH_DI void binary(int op, const double (&x)[kDIpt], const double (&y)[kDIpt], double (&z)[kDIpt]) {
  switch (op) {  // block-uniform; the arithmetic that dominates DAGs gets straight-line code
    case PBH_OP_ADD:
#pragma unroll
      for (int j = 0; j < kDIpt; ++j) z[j] = x[j] + y[j];
      break;
    case PBH_OP_SUB:
#pragma unroll
      for (int j = 0; j < kDIpt; ++j) z[j] = x[j] - y[j];
      break;
    case PBH_OP_MUL:
#pragma unroll
      for (int j = 0; j < kDIpt; ++j) z[j] = x[j] * y[j];
      break;
    case PBH_OP_TRUEDIV:
#pragma unroll
      for (int j = 0; j < kDIpt; ++j) z[j] = x[j] / y[j];
      break;
    default:
#pragma unroll
      for (int j = 0; j < kDIpt; ++j) z[j] = binary_call(op, x[j], y[j]);
      break;
  }
}

PBH_DI void operand(const double* regs, int r, double imm, double (&x)[kDIpt]) {
#pragma unroll
  for (int j = 0; j < kDIpt; ++j) x[j] = r >= 0 ? regs[r * kDTile + item(j)] : imm;
}

__global__ __launch_bounds__(kDBlock) PBH_DAG_OCC void k_dag(const DOp* __restrict__ prog, int nops,
                                                             const DagSrc* __restrict__ src,
                                                             double* const* __restrict__ vec, int64_t row0, int64_t n,
                                                             int32_t* __restrict__ flags) {
  __shared__ DagQueue tq;
  __shared__ uint32_t T[1024];
  extern __shared__ double regs[];  // [nregs][kDTile]
  const u32x8* code = reinterpret_cast<const u32x8*>(prog);
  for (int64_t base = (int64_t)blockIdx.x * kDTile; base < n; base += (int64_t)gridDim.x * kDTile) {
    bool valid[kDIpt];
#pragma unroll
    for (int j = 0; j < kDIpt; ++j) valid[j] = base + item(j) < n;
    u32x8 next = code[0];
    for (int k = 0; k < nops; ++k) {
      const u32x8 w = next;
      if (k + 1 < nops) next = code[k + 1];  // in flight while this op runs
      const int kind = (int)(w[0] & 0xffu), opc = (int)((w[0] >> 8) & 0xffu);
      const int dst = (int)((w[0] >> 16) & 0xffu) - 1, ra = (int)(w[0] >> 24) - 1;
      const int rb = (int)w[1], si = (int)w[2], flag = (int)w[3], store = (int)w[4];
      const double value = __builtin_bit_cast(double, ((uint64_t)w[7] << 32) | w[6]);
      double x[kDIpt];
      bool have = true;  // x holds this op's result
      bool bad = false;
      if (kind == PBH_DAG_GEN) {
        // Every GEN ends with a barrier (below), so here the previous GEN's readers of T and of
        // the tail queue are done: refill T, reset the queue, one barrier.
        const DagSrc& s = src[si];
        if (s.kind == PBH_QSRC_SOBOL)
          for (int t = threadIdx.x; t < 1024; t += kDBlock) T[t] = s.T[t];
        if (threadIdx.x == 0) tq.count = 0;
        __syncthreads();
        double q[kDIpt];
        gen_quantiles(s, T, row0, base, n, q);
        const double p[3] = {s.p[0], s.p[1], s.p[2]};
        double* out = regs + dst * kDTile;
        switch (opc) {
          case PBH_DIST_NORM: bad = gen_compacted<PBH_DIST_NORM>(q, valid, p, out, tq); break;
          case PBH_DIST_LOGNORM: bad = gen_compacted<PBH_DIST_LOGNORM>(q, valid, p, out, tq); break;
          case PBH_DIST_UNIFORM: bad = gen_plain<PBH_DIST_UNIFORM>(q, valid, p, out); break;
          case PBH_DIST_EXPON: bad = gen_plain<PBH_DIST_EXPON>(q, valid, p, out); break;
          default: bad = gen_plain<PBH_DIST_TRIANG>(q, valid, p, out); break;
        }
        __syncthreads();  // drained tail values are in the row
        have = store >= 0;
        if (have) operand(regs, dst, 0.0, x);
      } else {
        if (kind == PBH_DAG_LOAD) {
          const double* v = vec[si];
#pragma unroll
          for (int j = 0; j < kDIpt; ++j) x[j] = valid[j] ? v[base + item(j)] : 0.0;
        } else if (kind == PBH_DAG_CONST) {
#pragma unroll
          for (int j = 0; j < kDIpt; ++j) x[j] = value;
        } else if (kind == PBH_DAG_BINARY) {
          double a[kDIpt], b[kDIpt];
          operand(regs, ra, value, a);
          operand(regs, rb, value, b);
          binary(opc, a, b, x);
        } else if (kind == PBH_DAG_UNARY) {
          double a[kDIpt];
          operand(regs, ra, value, a);
#pragma unroll
          for (int j = 0; j < kDIpt; ++j) x[j] = unary_call(opc, a[j]);
        } else {  // STORE
          operand(regs, ra, value, x);
        }
        if (kind != PBH_DAG_STORE && dst >= 0) {
#pragma unroll
          for (int j = 0; j < kDIpt; ++j) regs[dst * kDTile + item(j)] = x[j];
        }
        if (flag >= 0) {
#pragma unroll
          for (int j = 0; j < kDIpt; ++j) bad |= valid[j] && !isfinite(x[j]);
        }
      }
      if (have && store >= 0) {
        double* v = vec[store];
#pragma unroll
        for (int j = 0; j < kDIpt; ++j)
          if (valid[j]) __builtin_nontemporal_store(x[j], v + base + item(j));
      }
      if (flag >= 0) flag_nonfinite(flags + flag, bad);
    }
  }
}

bool gen_dist_ok(int d) {
  return d == PBH_DIST_NORM || d == PBH_DIST_UNIFORM || d == PBH_DIST_EXPON || d == PBH_DIST_LOGNORM ||
         d == PBH_DIST_TRIANG;
}

bool float_op_ok(int kind, int op) {  // the float64 operators of pbh_elementwise
  if (kind == PBH_DAG_BINARY) return op >= PBH_OP_ADD && op <= PBH_OP_ARCTAN2;
  return (op >= PBH_OP_NEG && op <= PBH_OP_ARCTANH) || op == PBH_OP_CAST;
}

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace
}  // namespace pbh

using namespace pbh;

extern "C" int pbh_dag_eval(const pbh_dag_op* ops_host, int nops, const pbh_dag_qsource* sources_host, int nsources,
                            double* const* vectors_host, int nvectors, int64_t row0, int64_t n, int32_t* flags,
                            void* stream) {
  PBH_REQUIRE(nops >= 0 && nops <= PBH_DAG_MAX_OPS, "pbh_dag_eval: 0 <= nops <= %d", PBH_DAG_MAX_OPS);
  PBH_REQUIRE(nops == 0 || ops_host != nullptr, "pbh_dag_eval: ops must not be NULL");
  PBH_REQUIRE(nsources >= 0 && (nsources == 0 || sources_host), "pbh_dag_eval: bad sources");
  PBH_REQUIRE(nvectors >= 0 && (nvectors == 0 || vectors_host), "pbh_dag_eval: bad vectors");
  PBH_REQUIRE(row0 >= 0 && n >= 0, "pbh_dag_eval: bad row range");
  int nregs = 1;
  bool any_flag = false;
  auto vec_ok = [&](int v) { return v >= 0 && v < nvectors && vectors_host[v] != nullptr; };
  for (int k = 0; k < nops; ++k) {
    const pbh_dag_op& o = ops_host[k];
    auto reg_ok = [](int r) { return r >= 0 && r < PBH_DAG_MAX_REGS; };
    auto opnd_ok = [](int r) { return r >= -1 && r < PBH_DAG_MAX_REGS; };
    switch (o.kind) {
      case PBH_DAG_GEN:
        PBH_REQUIRE(o.src >= 0 && o.src < nsources, "pbh_dag_eval: op %d: bad source %d", k, o.src);
        PBH_REQUIRE(gen_dist_ok(o.op), "pbh_dag_eval: op %d: distribution %d has no fused form", k, o.op);
        PBH_REQUIRE(reg_ok(o.dst), "pbh_dag_eval: op %d: GEN needs a register", k);
        break;
      case PBH_DAG_LOAD:
        PBH_REQUIRE(vec_ok(o.src), "pbh_dag_eval: op %d: bad vector", k);
        PBH_REQUIRE(opnd_ok(o.dst), "pbh_dag_eval: op %d: bad register", k);
        break;
      case PBH_DAG_CONST:
        PBH_REQUIRE(opnd_ok(o.dst), "pbh_dag_eval: op %d: bad register", k);
        break;
      case PBH_DAG_BINARY:
      case PBH_DAG_UNARY:
        PBH_REQUIRE(float_op_ok(o.kind, o.op), "pbh_dag_eval: op %d: unknown operator %d", k, o.op);
        PBH_REQUIRE(opnd_ok(o.dst) && opnd_ok(o.a) && (o.kind == PBH_DAG_UNARY || opnd_ok(o.b)),
                    "pbh_dag_eval: op %d: bad register", k);
        break;
      case PBH_DAG_STORE:
        PBH_REQUIRE(opnd_ok(o.a) && o.dst == -1, "pbh_dag_eval: op %d: bad STORE", k);
        PBH_REQUIRE(o.store >= 0, "pbh_dag_eval: op %d: STORE without a vector", k);
        break;
      default:
        PBH_REQUIRE(false, "pbh_dag_eval: op %d: unknown kind %d", k, o.kind);
    }
    PBH_REQUIRE(o.store == -1 || vec_ok(o.store), "pbh_dag_eval: op %d: bad store vector", k);
    PBH_REQUIRE(o.flag >= -1, "pbh_dag_eval: op %d: bad flag index", k);
    any_flag |= o.flag >= 0;
    nregs = std::max(nregs, 1 + std::max(o.dst, std::max(o.a, o.kind == PBH_DAG_BINARY ? o.b : -1)));
  }
  PBH_REQUIRE(!any_flag || flags != nullptr, "pbh_dag_eval: flag indices given without a flags array");
  int nsobol = 0;
  for (int s = 0; s < nsources; ++s) {
    const pbh_dag_qsource& q = sources_host[s];
    if (q.kind == PBH_QSRC_SOBOL) {
      PBH_REQUIRE(q.bits >= 1 && q.bits <= 32, "pbh_dag_eval: source %d: bits must be in [1, 32]", s);
      PBH_REQUIRE(row0 + n <= ((int64_t)1 << q.bits), "pbh_dag_eval: source %d: rows exceed 2^bits", s);
      ++nsobol;
    } else if (q.kind == PBH_QSRC_LHS) {
      PBH_REQUIRE(q.n_total >= 1 && row0 + n <= q.n_total && q.col >= 0, "pbh_dag_eval: source %d: bad LHS rows", s);
    } else {
      PBH_REQUIRE(q.kind == PBH_QSRC_VECTOR && q.q != nullptr && q.stride >= 1,
                  "pbh_dag_eval: source %d: bad quantile vector", s);
    }
  }
  if (n == 0 || nops == 0) return PBH_OK;

  // one upload: program | sources | vector table | Sobol' XOR tables.  Every GEN gets a source
  // entry of its own (the quantile stream plus the GEN's parameters).
  int ngen = 0;
  for (int k = 0; k < nops; ++k) ngen += ops_host[k].kind == PBH_DAG_GEN;
  const int nsrc = ngen;
  const size_t b_ops = align256((size_t)nops * sizeof(DOp));
  const size_t b_src = align256((size_t)std::max(nsrc, 1) * sizeof(DagSrc));
  const size_t b_vec = align256((size_t)std::max(nvectors, 1) * sizeof(double*));
  const size_t b_tab = (size_t)nsobol * 1024 * 4;
  std::vector<uint8_t> host(b_ops + b_src + b_vec + b_tab, 0);
  hipStream_t st = as_stream(stream);
  uint8_t* dev = nullptr;
  PBH_CHECK_HIP(hipMallocAsync((void**)&dev, host.size(), st));
  DagSrc* hs = (DagSrc*)(host.data() + b_ops);
  uint32_t* ht = (uint32_t*)(host.data() + b_ops + b_src + b_vec);
  const uint32_t* dt = (const uint32_t*)(dev + b_ops + b_src + b_vec);
  std::vector<int> table_of(nsources, -1);  // Sobol' XOR tables, one per source
  int t = 0;
  for (int s = 0; s < nsources; ++s) {
    const pbh_dag_qsource& q = sources_host[s];
    if (q.kind != PBH_QSRC_SOBOL) continue;
    uint32_t* tb = ht + (size_t)t * 1024;
    for (int e = 0; e < 256; ++e)
      for (int g = 0; g < 4; ++g) {
        uint32_t v = 0;
        for (int b = 0; b < 8; ++b)
          if (((e >> b) & 1) && 8 * g + b < q.bits) v ^= q.sv[8 * g + b];
        tb[g * 256 + e] = v;
      }
    table_of[s] = t++;
  }
  DOp* hp = (DOp*)host.data();
  int gi = 0;
  for (int k = 0; k < nops; ++k) {
    const pbh_dag_op& o = ops_host[k];
    DOp d = {};
    d.head = (uint32_t)o.kind | ((uint32_t)o.op << 8) | ((uint32_t)(o.dst + 1) << 16) | ((uint32_t)(o.a + 1) << 24);
    d.b = o.b;
    d.src = o.src;
    d.flag = o.flag;
    d.store = o.store;
    d.value = o.value;
    if (o.kind == PBH_DAG_GEN) {
      const pbh_dag_qsource& q = sources_host[o.src];
      DagSrc g = {};
      g.kind = q.kind;
      g.col = q.col;
      g.shift = q.shift;
      g.seed = q.seed;
      g.n_total = q.n_total;
      g.q = q.q;
      g.stride = q.stride;
      if (q.kind == PBH_QSRC_SOBOL) {
        g.scale = 1.0 / (double)((uint64_t)1 << q.bits);
        g.T = dt + (size_t)table_of[o.src] * 1024;
      }
      for (int j = 0; j < 3; ++j) g.p[j] = o.params[j];
      hs[gi] = g;
      d.src = gi++;
    }
    hp[k] = d;
  }
  if (nvectors) memcpy(host.data() + b_ops + b_src, vectors_host, (size_t)nvectors * sizeof(double*));
  int rc = PBH_OK;
  if (hipMemcpyAsync(dev, host.data(), host.size(), hipMemcpyHostToDevice, st) != hipSuccess) {
    set_error("pbh_dag_eval: upload failed");
    rc = PBH_ERR_HIP;
  } else {
    const DOp* prog = (const DOp*)dev;
    const DagSrc* srcs = (const DagSrc*)(dev + b_ops);
    double* const* vecs = (double* const*)(dev + b_ops + b_src);
    dim3 g(grid_for(n, kDTile, 256 * 16)), b(kDBlock);
    const size_t lds = (size_t)nregs * kDTile * sizeof(double);
    PBH_TIMED(kKDag, st, hipLaunchKernelGGL(k_dag, g, b, lds, st, prog, nops, srcs, vecs, row0, n, flags));
    if (hipGetLastError() != hipSuccess) {
      set_error("pbh_dag_eval: launch failed");
      rc = PBH_ERR_HIP;
    }
  }
  PBH_CHECK_HIP(hipFreeAsync(dev, st));
  return rc;
}
