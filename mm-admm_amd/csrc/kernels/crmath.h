// crmath.h -- correctly rounded fractional powers for the Huang functional.
//
// AdaptationFunctional<D>::blockGrad (reference src/AdaptationFunctional.cpp:219-236) calls
// std::pow with the exponents d*p/2, d*p/2-1, p, 1-p, p-1 (p = 1.5):
//   D = 2: 1.5, 0.5, 1.5, -0.5, 0.5        D = 3: 2.25, 1.25, 1.5, -0.5, 0.5
// The GPU evaluates each power as a double-double (relative error < 2^-100) built on the
// correctly rounded sqrt and explicit fma, and rounds it once.  When the double-double sits
// within 2^-95 of a rounding midpoint (arguments a few ulps from 1 do this systematically),
// an exact comparison decides the rounding: x^(p/q) > m  <=>  x^p > m^q, evaluated with
// Shewchuk expansion arithmetic.  The result is the correctly rounded power (round to nearest,
// ties to even); tests/test_crmath.py and tests/test_gpu_parity.py check it against
// __float128 powq.  This matters: the first prox builds a finite-difference Hessian with
// h = 2*sqrt(eps) (reference src/Mesh.cpp:780), which amplifies any last-bit difference in
// the gradient by 1/h ~ 3e7.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__) || defined(__HIP__)
#define MMX_HD __host__ __device__ __forceinline__
#define MMX_HD_COLD __host__ __device__ __attribute__((noinline))
#else
#define MMX_HD inline
#define MMX_HD_COLD inline
#endif

namespace mmx {

MMX_HD double cr_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
MMX_HD double cr_sqrt(double x) { return __builtin_sqrt(x); }

// RN(x / c) from rc = RN(1 / c) without a division, for the BFGS update's divisions by c2
// (Markstein: with rc correctly rounded and q = RN(x rc) within one ulp of x/c, the residual
// e = q c - x is exact (FMA) and RN(q - e rc) is the correctly rounded quotient).  Three
// instructions instead of the ~11 of an IEEE division (one of them a quarter-rate v_rcp_f64).
// Exact when c > 0 with c in [2^-100, 2^100] and x = +-0 or |x| in [2^-900, 2^900]: the residual
// cannot underflow and q is normal.  Signed zeros: x = +0 gives +0, x = -0 gives -0 (e = +0,
// -e * rc = -0).  The CALLER checks the ranges (mk_exp) and takes the exact path otherwise;
// non-finite x gives NaN (the caller's finiteness check catches it).  Checked against IEEE
// division on 4e8 random and near-midpoint operand pairs on the host and on the
// device by tests/test_gpu_parity.py::test_device_division_by_reciprocal_is_correctly_rounded.
MMX_HD double div_mk(double x, double c, double rc) {
  const double q = x * rc;
  const double e = cr_fma(q, c, -x);
  return cr_fma(-e, rc, q);
}
// frexp exponent of x biased so that (unsigned) <= 2*lim - 1 <=> x = 0 or |x| in [2^-lim, 2^lim]
// (frexp: |x| in [2^(e-1), 2^e); 0 for zero, inf and NaN).  Non-finite x therefore counts as IN
// range: callers must check finiteness themselves (bfgs_update_row folds every new entry into its
// `fin` check, which a NaN or infinite operand reaches).
MMX_HD unsigned mk_exp(double x, int lim) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (unsigned)(__builtin_amdgcn_frexp_exp(x) + (lim - 1));
#else
  int e;
  (void)std::frexp(x, &e);
  if (!std::isfinite(x)) e = 0;
  return (unsigned)(e + (lim - 1));
#endif
}
constexpr double kRecip3 = 1.0 / 3.0;  // RN(1/3), for the divisions by D + 1 = 3

// The same without range guards, for call sites whose operands are known to be normal with a
// quotient that is zero or normal (grid coordinates): three instructions, no branch.
MMX_HD double div_nr(double x, double c, double rc) {
  const double q = x * rc;
  const double r = cr_fma(-q, c, x);
  return cr_fma(r, rc, q);
}

// argument ranges in which the exact fallback (x^p and m^q as expansions) cannot over- or
// underflow; outside them (never met by the functional) the device libm pow is used.
MMX_HD bool cr_in(double x, double lo, double hi) { return x > lo && x < hi; }

// ---------------------------------------------------------------- exact expansions
namespace xp {
constexpr int kCap = 48;
struct Ex {
  double t[kCap];  // nonoverlapping, increasing magnitude
  int n;
};

MMX_HD void two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
MMX_HD void fast_two_sum(double a, double b, double& s, double& e) {  // |a| >= |b|
  s = a + b;
  e = b - (s - a);
}
MMX_HD void two_prod(double a, double b, double& p, double& e) {
  p = a * b;
  e = cr_fma(a, b, -p);
}

// h = e * b  (Shewchuk scale_expansion_zeroelim)
MMX_HD_COLD void scale(const Ex& e, double b, Ex& h) {
  h.n = 0;
  if (e.n == 0) return;
  double Q, hh, p1, p0, sum;
  two_prod(e.t[0], b, Q, hh);
  if (hh != 0) h.t[h.n++] = hh;
  for (int i = 1; i < e.n; ++i) {
    two_prod(e.t[i], b, p1, p0);
    two_sum(Q, p0, sum, hh);
    if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
    fast_two_sum(p1, sum, Q, hh);
    if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
  }
  if ((Q != 0 || h.n == 0) && h.n < kCap) h.t[h.n++] = Q;
}

// h = e + f  (Shewchuk fast_expansion_sum_zeroelim)
MMX_HD_COLD void sum(const Ex& e, const Ex& f, Ex& h) {
  h.n = 0;
  int ei = 0, fi = 0;
  double Q, Qn, hh;
  double enow = e.n ? e.t[0] : 0.0, fnow = f.n ? f.t[0] : 0.0;
  if (e.n == 0 && f.n == 0) return;
  if (fi >= f.n || (ei < e.n && ((fnow > enow) == (fnow > -enow)))) {
    Q = enow;
    ++ei;
    enow = (ei < e.n) ? e.t[ei] : 0.0;
  } else {
    Q = fnow;
    ++fi;
    fnow = (fi < f.n) ? f.t[fi] : 0.0;
  }
  if (ei < e.n && fi < f.n) {
    if ((fnow > enow) == (fnow > -enow)) {
      fast_two_sum(enow, Q, Qn, hh);
      ++ei;
      enow = (ei < e.n) ? e.t[ei] : 0.0;
    } else {
      fast_two_sum(fnow, Q, Qn, hh);
      ++fi;
      fnow = (fi < f.n) ? f.t[fi] : 0.0;
    }
    Q = Qn;
    if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
    while (ei < e.n && fi < f.n) {
      if ((fnow > enow) == (fnow > -enow)) {
        two_sum(Q, enow, Qn, hh);
        ++ei;
        enow = (ei < e.n) ? e.t[ei] : 0.0;
      } else {
        two_sum(Q, fnow, Qn, hh);
        ++fi;
        fnow = (fi < f.n) ? f.t[fi] : 0.0;
      }
      Q = Qn;
      if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
    }
  }
  while (ei < e.n) {
    two_sum(Q, enow, Qn, hh);
    ++ei;
    enow = (ei < e.n) ? e.t[ei] : 0.0;
    Q = Qn;
    if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
  }
  while (fi < f.n) {
    two_sum(Q, fnow, Qn, hh);
    ++fi;
    fnow = (fi < f.n) ? f.t[fi] : 0.0;
    Q = Qn;
    if (hh != 0 && h.n < kCap) h.t[h.n++] = hh;
  }
  if ((Q != 0 || h.n == 0) && h.n < kCap) h.t[h.n++] = Q;
}

// Shewchuk compress: shortens an expansion without changing its value
MMX_HD_COLD void compress(Ex& e) {
  if (e.n <= 1) return;
  double g[kCap];
  int bottom = e.n - 1;
  double Q = e.t[bottom], q, Qn;
  for (int i = e.n - 2; i >= 0; --i) {
    fast_two_sum(Q, e.t[i], Qn, q);
    if (q != 0) {
      g[bottom--] = Qn;
      Q = q;
    } else {
      Q = Qn;
    }
  }
  g[bottom] = Q;
  int top = 0;
  for (int i = bottom + 1; i < e.n; ++i) {
    fast_two_sum(g[i], Q, Qn, q);
    Q = Qn;
    if (q != 0) e.t[top++] = q;
  }
  e.t[top++] = Q;
  e.n = top;
}

// dst = src, its n live components only (a whole-struct copy moves kCap doubles: on the device the
// expansions live in scratch, and the copies were most of the exact path's traffic)
MMX_HD void assign(Ex& dst, const Ex& src) {
  for (int i = 0; i < src.n; ++i) dst.t[i] = src.t[i];
  dst.n = src.n;
}

MMX_HD_COLD void mul(const Ex& a, const Ex& b, Ex& out) {
  Ex acc, part, tmp;
  acc.n = 0;
  for (int j = 0; j < b.n; ++j) {
    scale(a, b.t[j], part);
    sum(acc, part, tmp);
    compress(tmp);
    assign(acc, tmp);
  }
  assign(out, acc);
}

MMX_HD void single(double v, Ex& e) {
  e.t[0] = v;
  e.n = 1;
}

MMX_HD_COLD void ipow(double x, int p, Ex& out) {  // x^p exactly, p >= 1
  Ex base, r, t;
  single(x, base);
  single(1.0, r);
  while (p) {
    if (p & 1) {
      mul(r, base, t);
      assign(r, t);
    }
    p >>= 1;
    if (p) {
      mul(base, base, t);
      assign(base, t);
    }
  }
  assign(out, r);
}

MMX_HD int sign(const Ex& e) {  // sign of the largest nonzero component
  for (int i = e.n - 1; i >= 0; --i) {
    if (e.t[i] > 0) return 1;
    if (e.t[i] < 0) return -1;
  }
  return 0;
}
}  // namespace xp

MMX_HD double next_toward(double h, int dir) {  // neighbouring double (h > 0)
  uint64_t b;
  std::memcpy(&b, &h, 8);
  b = (dir > 0) ? b + 1 : b - 1;
  double r;
  std::memcpy(&r, &b, 8);
  return r;
}

// Exact decision of round(x^(num/den)) between h and its neighbour in direction dir:
// compares x^num with m^den (num > 0) or x^(-num) * m^den with 1 (num < 0), m = midpoint.
MMX_HD_COLD double cr_resolve(double x, int num, int den, double h, int dir) {
  const double nb = next_toward(h, dir);
  const double mhi = h, mlo = (nb - h) * 0.5;  // m = h + (nb - h)/2 exactly (two terms)
  xp::Ex m, mp, lhs, diff, neg;
  if (std::fabs(mlo) < std::fabs(mhi)) {
    m.t[0] = mlo;
    m.t[1] = mhi;
    m.n = 2;
  } else {
    xp::single(mhi, m);
  }
  // m^den
  xp::assign(mp, m);
  for (int i = 1; i < den; ++i) {
    xp::Ex t;
    xp::mul(mp, m, t);
    xp::assign(mp, t);
  }
  int s;
  if (num > 0) {  // sign(x^num - m^den)
    xp::ipow(x, num, lhs);
    xp::assign(neg, mp);
    for (int i = 0; i < neg.n; ++i) neg.t[i] = -neg.t[i];
    xp::sum(lhs, neg, diff);
    s = xp::sign(diff);
  } else {  // v > m  <=>  1 > m^den * x^(-num)
    xp::Ex xn, prod, one;
    xp::ipow(x, -num, xn);
    xp::mul(mp, xn, prod);
    for (int i = 0; i < prod.n; ++i) prod.t[i] = -prod.t[i];
    xp::single(1.0, one);
    xp::sum(one, prod, diff);
    s = xp::sign(diff);
  }
  // s > 0: v above m; s < 0: below; s == 0: exact tie -> even mantissa
  const bool vAboveM = (s > 0);
  if (s == 0) {
    uint64_t b;
    std::memcpy(&b, &h, 8);
    return (b & 1) ? nb : h;
  }
  if (dir > 0) return vAboveM ? nb : h;
  return vAboveM ? h : nb;
}

// Round a normalised double-double (hi = RN(hi + lo)) that approximates x^(num/den) with
// relative error < 2^-100; near a midpoint the exact decision (cr_resolve) is needed.
// EXACT = false is the fast path of the prox kernels: instead of resolving it raises `tie` and
// returns a placeholder; the caller discards the lane's results and recomputes the simplex with
// EXACT = true (so cr_resolve, its calls and its stack stay out of the hot kernel body).
template <bool EXACT>
MMX_HD double cr_round_t(double x, int num, int den, double hi, double lo, bool& tie) {
  double h, l;
  xp::two_sum(hi, lo, h, l);
  if (l == 0.0) {
    // v within 2^-100 |h| of a double: decided unless h itself is near a midpoint (no)
    return h;
  }
  const int dir = (l > 0) ? 1 : -1;
  const double nb = next_toward(h, dir);
  const double half = std::fabs(nb - h) * 0.5;
  const double dist = half - std::fabs(l);  // distance of the dd value to the midpoint
  if (dist > std::fabs(h) * 0x1p-95) return h;
  if constexpr (EXACT) {
    return cr_resolve(x, num, den, h, dir);
  } else {
    tie = true;
    return h;
  }
}

MMX_HD double cr_round(double x, int num, int den, double hi, double lo) {
  bool t = false;
  return cr_round_t<true>(x, num, den, hi, lo, t);
}

// sqrt(x) = s + e, |error| < 2^-104 |s|
MMX_HD void cr_sqrt_dd(double x, double& s, double& e) {
  s = cr_sqrt(x);
  const double r = cr_fma(-s, s, x);
  e = r / (2.0 * s);
}

// x^0.5 -- correctly rounded sqrt
MMX_HD double cr_pow_p05(double x) { return cr_sqrt(x); }

// MMX_DD_FAST (device only): the double-double square roots of the powers below from the
// hardware reciprocal square root, refined by two coupled Newton (Goldschmidt) steps -- no IEEE
// sqrt and no division.  g -> sqrt(x) and hh -> 1/(2 sqrt(x)) converge quadratically from any
// start within 2^-10, so after two steps both are within a few ulps; the residual x - s^2 is then
// formed by FMA with relative error <= 2^-53, and e = (x - s^2) hh (= r / (2s) to ~2^-50) leaves
// s + e within ~2^-101 |s| of sqrt(x) (the neglected term e^2 / (2s) is ~2^-103 |s|).  Only the
// double-double changes: every power is still rounded by cr_round_t, whose 2^-95 margin covers
// it, so the results are the same correctly rounded values (tests/test_gpu_parity.py).
#ifndef MMX_DD_FAST
#define MMX_DD_FAST 0
#endif
// sqrt(x) = s + e and hh ~ 1 / (2 sqrt(x)) (to a few ulps)
MMX_HD void dd_sqrt_h(double x, double& s, double& e, double& hh) {
#if defined(__HIP_DEVICE_COMPILE__) && MMX_DD_FAST
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  double r = cr_fma(-g, h, 0.5);
  g = cr_fma(g, r, g);
  h = cr_fma(h, r, h);
  r = cr_fma(-g, h, 0.5);
  g = cr_fma(g, r, g);
  h = cr_fma(h, r, h);
  s = g;
  e = cr_fma(-g, g, x) * h;
  hh = h;
#else
  s = cr_sqrt(x);
  const double r = cr_fma(-s, s, x);
  e = r / (2.0 * s);
  hh = 0.5 / s;
#endif
}

// Outside the ranges below the powers defer to the library pow (EXACT) or raise `tie` (fast
// path: the exact recomputation takes the library call).
#define MMX_CR_RANGE(lo, hi, e)         \
  if (!cr_in(x, lo, hi)) {              \
    if constexpr (EXACT) {              \
      return ::pow(x, e);               \
    } else {                            \
      tie = true;                       \
      return 1.0;                       \
    }                                   \
  }

// x^1.5
template <bool EXACT>
MMX_HD double cr_pow_p15(double x, bool& tie) {
  MMX_CR_RANGE(1e-90, 1e90, 1.5)
  double s, e;
#if MMX_DD_FAST
  double hh;
  dd_sqrt_h(x, s, e, hh);
#else
  cr_sqrt_dd(x, s, e);
#endif
  const double p = x * s;
  const double lo = cr_fma(x, s, -p) + x * e;
  return cr_round_t<EXACT>(x, 3, 2, p, lo, tie);
}

// x^-0.5
template <bool EXACT>
MMX_HD double cr_pow_m05(double x, bool& tie) {
  MMX_CR_RANGE(1e-100, 1e100, -0.5)
  double s, e;
#if MMX_DD_FAST && defined(__HIP_DEVICE_COMPILE__)
  // q = 2 hh is within a few ulps of 1/s: 1/(s + e) = q / (1 - u) = q (1 + u + u^2 + ...)
  double hh;
  dd_sqrt_h(x, s, e, hh);
  const double q = 2.0 * hh;
  const double d = cr_fma(-q, s, 1.0);  // 1 - q*s (error <= 2^-53 of it)
  const double u = d - q * e;           // 1 - q*(s + e)
  return cr_round_t<EXACT>(x, -1, 2, q, q * cr_fma(u, u, u), tie);
#else
  cr_sqrt_dd(x, s, e);
  const double q = 1.0 / s;
  const double d = cr_fma(-q, s, 1.0);  // 1 - q*s, exact
  const double u = d - q * e;           // 1 - q*(s + e)
  return cr_round_t<EXACT>(x, -1, 2, q, q * u, tie);
#endif
}

// x^0.25 as hi + lo, |error| < 2^-103 |hi|
MMX_HD void cr_qrt_dd(double x, double& hi, double& lo) {
#if MMX_DD_FAST && defined(__HIP_DEVICE_COMPILE__)
  double s, e, hs;
  dd_sqrt_h(x, s, e, hs);  // sqrt(x) = s + e, hs ~ 1/(2s)
  double b, eb, hb;
  dd_sqrt_h(s, b, eb, hb);  // sqrt(s) = b + eb
  hi = b;
  lo = eb + b * (e * hs);  // sqrt(s + e) = sqrt(s) (1 + e/(2s) - ...)
#else
  double s, e;
  cr_sqrt_dd(x, s, e);  // sqrt(x) = s + e
  double b, eb;
  cr_sqrt_dd(s, b, eb);  // sqrt(s) = b + eb
  hi = b;
  lo = eb + b * (e / (2.0 * s));  // sqrt(s + e) = sqrt(s) (1 + e/(2s) - ...)
#endif
}

// x^2.25 = x^2 * x^0.25
template <bool EXACT>
MMX_HD double cr_pow_p225(double x, bool& tie) {
  MMX_CR_RANGE(1e-30, 1e30, 2.25)
  double b, lo4;
  cr_qrt_dd(x, b, lo4);
  const double X2 = x * x;
  const double X2e = cr_fma(x, x, -X2);
  const double hi = X2 * b;
  const double lo = cr_fma(X2, b, -hi) + (X2 * lo4 + X2e * b);
  return cr_round_t<EXACT>(x, 9, 4, hi, lo, tie);
}

// x^1.25 = x * x^0.25
template <bool EXACT>
MMX_HD double cr_pow_p125(double x, bool& tie) {
  MMX_CR_RANGE(1e-50, 1e50, 1.25)
  double b, lo4;
  cr_qrt_dd(x, b, lo4);
  const double hi = x * b;
  const double lo = cr_fma(x, b, -hi) + x * lo4;
  return cr_round_t<EXACT>(x, 5, 4, hi, lo, tie);
}
#undef MMX_CR_RANGE

// the correctly rounded powers as plain functions
MMX_HD double cr_pow_p15(double x) {
  bool t = false;
  return cr_pow_p15<true>(x, t);
}
MMX_HD double cr_pow_m05(double x) {
  bool t = false;
  return cr_pow_m05<true>(x, t);
}
MMX_HD double cr_pow_p225(double x) {
  bool t = false;
  return cr_pow_p225<true>(x, t);
}
MMX_HD double cr_pow_p125(double x) {
  bool t = false;
  return cr_pow_p125<true>(x, t);
}

// c2^2 (reference src/Mesh.cpp:847 pow(c2, 2.0)) is exactly the rounded square.
MMX_HD double cr_pow_2(double x) { return x * x; }

}  // namespace mmx
