// Host check of crmath.h's division by a shared reciprocal (div_mk) and its range test (mk_exp),
// as the prox kernels use them: for c > 0 in [2^-100, 2^100] and x = +-0 or |x| in
// [2^-900, 2^900], div_mk(x, c, RN(1/c)) must equal x / c bit for bit (random, near-midpoint and
// signed-zero operands); mk_exp must accept exactly those x.  Prints "ok <n>" or the first failure.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../mm-admm_amd/csrc/kernels/crmath.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  s ^= s << 13;
  s ^= s >> 7;
  s ^= s << 17;
  return s;
}
static double rd(int emin, int emax) {
  const uint64_t m = rnd() & ((1ull << 52) - 1);
  const int e = emin + (int)(rnd() % (uint64_t)(emax - emin + 1));
  uint64_t b = ((uint64_t)(e + 1023) << 52) | m;
  if (rnd() & 1) b |= 1ull << 63;
  double d;
  std::memcpy(&d, &b, 8);
  return d;
}
static bool same(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 20000000;
  long checked = 0;
  for (long it = 0; it < n; ++it) {
    const double c = std::fabs(rd(-100, 99));
    double x;
    switch (it % 5) {
      case 0: {  // quotient near a rounding midpoint
        const double q = rd(-700, 700), qn = std::nextafter(q, INFINITY);
        x = (q + (qn - q) / 2) * c;
        if (rnd() & 1) x = std::nextafter(x, (rnd() & 1) ? INFINITY : -INFINITY);
        break;
      }
      case 1: x = (rnd() & 1) ? 0.0 : -0.0; break;
      default: x = rd(-899, 899);
    }
    if (!(x == 0 || (std::fabs(x) >= 0x1p-900 && std::fabs(x) <= 0x1p900))) continue;
    if (mmx::mk_exp(x, 900) > 1799u) {
      std::printf("mk_exp rejects in-range x=%a\n", x);
      return 1;
    }
    const double got = mmx::div_mk(x, c, 1.0 / c), want = x / c;
    if (!same(got, want)) {
      std::printf("div_mk(%a, %a) = %a, want %a\n", x, c, got, want);
      return 1;
    }
    ++checked;
  }
  // mk_exp rejects what div_mk does not cover
  const double out[] = {0x1p-901, -0x1p-950, 0x1p-1070, 0x1p901, -0x1p1000};
  for (double x : out)
    if (mmx::mk_exp(x, 900) <= 1799u) {
      std::printf("mk_exp accepts out-of-range x=%a\n", x);
      return 1;
    }
  std::printf("ok %ld\n", checked);
  return 0;
}
