// TEST HARNESS: the device special functions of probabilit_amd/csrc/pbh_special.h compiled
// for the HOST (they are __host__ __device__), so that tests/test_special_host.py can sweep
// them against scipy on the CPU.  This never ships in the product library; device results
// are checked separately by tests/test_gpu_ppf.py (libm vs device math may differ by ulps).
#include <vector>

#include "pbh_special.h"

using namespace pbh;

extern "C" {

void sfh_ndtri(const double* q, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::ndtri(q[i]);
}

void sfh_igami(double a, const double* p, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::igami(a, p[i]);
}

void sfh_pdtr(const double* k, double mu, long n, double* out) {
  for (long i = 0; i < n; ++i) out[i] = sf::pdtr(k[i], mu);
}

// gamma ppf through the scalar-shape guide table, exactly as the device kernels use it.
void sfh_igami_guided(double a, const double* p, long n, double* out) {
  const int m = sf::kGammaGuideM;
  std::vector<double> y(m), dy(m);
  for (int j = 0; j < m; ++j) sf::gamma_guide_entry(a, sf::kGammaGuideZ0 + j * sf::kGammaGuideH, &y[j], &dy[j]);
  sf::GammaGuide T{y.data(), dy.data(), m, sf::kGammaGuideZ0, sf::kGammaGuideH, 1.0 / sf::kGammaGuideH};
  sf::GammaAux aux = sf::gamma_aux(a);
  for (long i = 0; i < n; ++i) out[i] = sf::igami_guided(a, p[i], &aux, T);
}

}
