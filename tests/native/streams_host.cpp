// TEST HARNESS: the MT19937 jump-ahead and PCG64 advance of probabilit_amd/csrc/pbh_mt.h
// compiled for the HOST, so that tests/test_streams_host.py can check the algebra against
// numpy's own generators on the CPU.  Never ships in the product library; the device
// kernels (pbh_streams.hip) are checked by tests/test_gpu_streams.py.
#include <vector>

#include "pbh_mt.h"
#include "pbh_rng.h"

using namespace pbh;

extern "C" {

int sh_mt_charpoly(uint64_t* phi) {
  std::vector<uint64_t> p;
  if (!mt::host::charpoly(p)) return 1;
  for (int i = 0; i < mt::kPolyWords; ++i) phi[i] = p[i];
  return 0;
}

// tempered words start_word .. start_word + count - 1 of the sequence whose first key block is
// key0 (x_0 .. x_623): jump to start_word - 1, then step, as the device kernel does.
int sh_mt_words(const uint32_t* key0, int64_t start_word, int64_t count, uint32_t* out) {
  static std::vector<uint64_t> table;
  if (table.empty() && !mt::host::jump_table(table)) return 1;
  uint32_t w[mt::kN];
  for (int i = 0; i < mt::kN; ++i) w[i] = key0[i];
  int64_t base = 0, skip = 0;
  if (start_word > 0) {
    const int64_t D = start_word - 1;
    for (int i = 0; i < mt::kJumpBits; ++i)
      if ((D >> i) & 1) mt::host::apply_jump(w, &table[(size_t)i * mt::kPolyWords]);
    base = D;
    skip = 1;
  }
  int64_t k = 0;
  while (k < count) {
    for (int m = (int)skip; m < mt::kN && k < count; ++m) out[k++] = mt::temper(w[m]);
    mt::twist(w);
    skip = 0;
    base += mt::kN;
  }
  return 0;
}

void sh_pcg_advance(uint64_t s_lo, uint64_t s_hi, uint64_t inc_lo, uint64_t inc_hi, uint64_t k, uint64_t* out) {
  pcg::u128 table[128];
  const pcg::u128 inc = ((pcg::u128)inc_hi << 64) | inc_lo;
  pcg::jump_table(inc, table);
  pcg::u128 s = pcg::advance(((pcg::u128)s_hi << 64) | s_lo, k, table);
  out[0] = (uint64_t)s;
  out[1] = (uint64_t)(s >> 64);
}

void sh_pcg_doubles(uint64_t s_lo, uint64_t s_hi, uint64_t inc_lo, uint64_t inc_hi, uint64_t k0, int64_t n, double* out) {
  pcg::u128 table[128];
  const pcg::u128 inc = ((pcg::u128)inc_hi << 64) | inc_lo;
  pcg::jump_table(inc, table);
  pcg::u128 s = pcg::advance(((pcg::u128)s_hi << 64) | s_lo, k0, table);
  for (int64_t i = 0; i < n; ++i) {
    s = s * pcg::kMult + inc;
    out[i] = pcg::to_double(pcg::output(s));
  }
}

// The native LHS quantiles (pbh_rng.h lhs_quantile: keyed Feistel stratum + SplitMix64 jitter)
// of columns col0 .. col0 + ncols - 1 for rows 0 .. n - 1, q[c * n + r] -- the same inline
// functions the device kernels evaluate, compiled for the host.
void sh_native_lhs(uint64_t seed, int64_t n, int col0, int ncols, double* q) {
  Philox ph(seed);
  for (int c = 0; c < ncols; ++c) {
    FeistelPerm fp(ph, (uint64_t)n, (uint32_t)(col0 + c));
    for (int64_t r = 0; r < n; ++r) q[(int64_t)c * n + r] = lhs_quantile(ph, fp, (uint64_t)r, (uint32_t)(col0 + c));
  }
}
}
