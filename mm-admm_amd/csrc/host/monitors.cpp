// monitors.cpp -- built-in monitor plugins (host, evaluated once at set-up).
//
// Restates Experiments/TestMonitors/MEx{0,1,2,3,4,5,13D,23D,33D,53D}.h and the MonType registry
// of main.cpp:836-864.  User monitors plug in through mmadmm_monitor_fn or the C++
// MonitorFunction<D> adapter in include/mmadmm/MonitorFunction.h.
#include <cmath>
#include <limits>

#include "common.h"

namespace mmx {
namespace {

void identity(int D, double* M) {
  for (int i = 0; i < D * D; ++i) M[i] = (i / D == i % D) ? 1.0 : 0.0;
}
void scaledIdentity(int D, double* M, double s) {  // M = I; M *= s
  identity(D, M);
  for (int i = 0; i < D * D; ++i) M[i] *= s;
}

// MEx1.h / MEx13D.h: isotropic bump 1 + mu1 / (1 + mu2 |x - 0.5|^2)
void bump(int D, const double* x, double* M) {
  const double mu_1 = 20, mu_2 = 20;
  double sq = 0.0;
  for (int d = 0; d < D; ++d) {
    const double t = x[d] - 0.5;
    sq = (d == 0) ? t * t : sq + t * t;
  }
  scaledIdentity(D, M, 1 + mu_1 / (1 + mu_2 * sq));
}

// MEx2.h: anisotropic, eigenvectors (1,1)/sqrt2 and (1,-1)/sqrt2
void aniso(const double* x, double* M) {
  const double lam1 = 1 + (1.0 / cosh(50 * (x[0] + x[1] - 1.0) * (x[0] + x[1] - 1.0)));
  const double lam2 = 1.0 / lam1;
  const double a = (1.0 / sqrt(2.0)) * 1.0;
  const double v[2] = {a, a}, vo[2] = {a, -(1.0 / sqrt(2.0)) * 1.0};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) M[i * 2 + j] = ((lam1 * v[i]) * v[j]) + ((lam2 * vo[i]) * vo[j]);
}

// MEx3.h / MEx23D.h / MEx33D.h: radial oscillation
void ring(int D, const double* x, double* M) {
  const double PI = 3.141592653589793238462643383;
  double s;
  if (D == 2)
    s = sqrt(0.01 / (2.0 + cos(8.0 * PI * sqrt(pow(x[0] - 0.5, 2) + pow(x[1] - 0.5, 2)))));
  else
    s = pow(0.01 / (2.0 + cos(8.0 * PI * sqrt(pow(x[0] - 0.5, 2) + pow(x[1] - 0.5, 2) +
                                             pow(x[2] - 0.5, 2)))),
            1.0 / 2.0);
  scaledIdentity(D, M, s);
}

// MEx4.h: gradient of a smoothed step across x + y = 1
void step2(int D, const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  const double eps = 0.01;
  const double g0 = ((1.0 / (1.0 + exp((x[0] + h + x[1] - 1) / (2.0 * eps)))) -
                     (1.0 / (1.0 + exp((x[0] - h + x[1] - 1) / (2.0 * eps))))) /
                    (2.0 * h);
  const double g1 = ((1.0 / (1.0 + exp((x[0] + x[1] + h - 1) / (2.0 * eps)))) -
                     (1.0 / (1.0 + exp((x[0] + x[1] - h - 1) / (2.0 * eps))))) /
                    (2.0 * h);
  scaledIdentity(D, M, pow(1 + pow(sqrt(g0 * g0 + g1 * g1), 2.0), 1.0 / 4.0));
}

// MEx5.h: spiral u(x, y); M = (1 + |grad u|^2)^(1/4) I with centred differences
double spiral(double x, double y) {
  const double r = sqrt(pow(x - 0.7, 2.0) + pow(y - 0.5, 2.0));
  const double theta = atan((y - 0.5) / (x - 0.7));
  return 1.0 + 9.0 / (1.0 + 100.0 * r * r * pow(cos(theta - 20.0 * r * r), 2.0));
}
void spiralMon(int D, const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  const double g0 = (spiral(x[0] + h, x[1]) - spiral(x[0] - h, x[1])) / (2.0 * h);
  const double g1 = (spiral(x[0], x[1] + h) - spiral(x[0], x[1] - h)) / (2.0 * h);
  scaledIdentity(D, M, pow(1 + pow(sqrt(g0 * g0 + g1 * g1), 2.0), 1.0 / 4.0));
}

// MEx53D.h: 3D spiral; its Vector<double,2> gradient and the overwritten grad(1) are kept
double spiral3(double x, double y, double z) {
  const double r = sqrt(pow(x - 0.7, 2.0) + pow(y - 0.5, 2.0) + pow(z - 0.5, 2));
  const double theta = atan((y - 0.5) / (x - 0.7));
  const double psi = atan((z - 0.5) / (x - 0.7));
  return 1.0 + 9.0 / (1.0 + 100.0 * r * r * pow(cos(theta + psi - 20.0 * r * r), 2.0));
}
void spiral3Mon(const double* x, double* M) {
  const double h = 2.0 * sqrt(std::numeric_limits<double>::epsilon());
  const double g0 = (spiral3(x[0] + h, x[1], x[2]) - spiral3(x[0] - h, x[1], x[2])) / (2.0 * h);
  double g1 = (spiral3(x[0], x[1] + h, x[2]) - spiral3(x[0], x[1] - h, x[2])) / (2.0 * h);
  g1 = (spiral3(x[0], x[1], x[2] + h) - spiral3(x[0], x[1], x[2] - h)) / (2.0 * h);
  scaledIdentity(3, M, pow(1 + pow(sqrt(g0 * g0 + g1 * g1), 2.0), 1.0 / 4.0));
}

// MonType 6 (no reference counterpart; BASELINE config 4 "anisotropic monitor"):
// MEx2's construction (Experiments/TestMonitors/MEx2.h) around a spherical (2D: circular) shell
// of radius 0.3: eigenvalue lam1 = 1 + sech(50 phi^2) along the radial unit vector n, 1/lam1 across
// it, phi = |x - c| - 0.3: M = lam2 I + (lam1 - lam2) n n^T.  Restated term for term in
// oracle/oracle.cpp (anisoShell).
void anisoShell(int D, const double* x, double* M) {
  double d[3], r2 = 0.0;
  for (int i = 0; i < D; ++i) {
    d[i] = x[i] - 0.5;
    r2 = (i == 0) ? d[i] * d[i] : r2 + d[i] * d[i];
  }
  const double r = sqrt(r2);
  const double phi = r - 0.3;
  const double lam1 = 1 + (1.0 / cosh(50 * phi * phi));
  const double lam2 = 1.0 / lam1;
  double n[3];
  for (int i = 0; i < D; ++i) n[i] = (r > 1e-12) ? d[i] / r : (i == 0 ? 1.0 : 0.0);
  for (int i = 0; i < D; ++i)
    for (int j = 0; j < D; ++j) M[i * D + j] = ((i == j) ? lam2 : 0.0) + ((lam1 - lam2) * n[i]) * n[j];
}

}  // namespace

// MonType 7 (no reference counterpart; BASELINE config 5 "time-varying monitor"):
// a bump moving on a circle, M = (1 + 5 / (1 + 50 |x - c(t)|^2)) I with
// c(t) = (0.5 + 0.2 cos 2 pi t, 0.5 + 0.2 sin 2 pi t, 0.5).  Set-up evaluates it at t = 0; with
// mmadmm_set_regrid the engine re-evaluates it on the device at every step start
// (regrid_kernels.hip k_monitor_tv, from this centre).  Restated in oracle/oracle.cpp (movingBump).
void moving_bump_centre(double t, double c[3]) {
  const double PI = 3.141592653589793238462643383;
  c[0] = 0.5 + 0.2 * cos((2.0 * PI) * t);
  c[1] = 0.5 + 0.2 * sin((2.0 * PI) * t);
  c[2] = 0.5;
}
static void movingBump(int D, const double* x, double t, double* M) {
  double c[3];
  moving_bump_centre(t, c);
  double sq = 0.0;
  for (int d = 0; d < D; ++d) {
    const double u = x[d] - c[d];
    sq = (d == 0) ? u * u : sq + u * u;
  }
  const double sc = 1 + 5.0 / (1 + 50.0 * sq);
  for (int i = 0; i < D * D; ++i) M[i] = (i / D == i % D) ? sc : 0.0;
}

void builtin_monitor_eval(int dim, int monType, const double* x, double* M) {
  if (monType == 7) {
    movingBump(dim, x, 0.0, M);
    return;
  }
  if (dim == 2) {
    switch (monType) {
      case 0: identity(2, M); return;
      case 1: bump(2, x, M); return;
      case 2: aniso(x, M); return;
      case 3: ring(2, x, M); return;
      case 4: step2(2, x, M); return;
      case 6: anisoShell(2, x, M); return;
      default: spiralMon(2, x, M); return;
    }
  }
  switch (monType) {  // Mvals3D = {MEx0, MEx13D, MEx23D, MEx33D, MEx0, MEx53D}
    case 0:
    case 4: identity(3, M); return;
    case 1: bump(3, x, M); return;
    case 2:
    case 3: ring(3, x, M); return;
    case 6: anisoShell(3, x, M); return;
    default: spiral3Mon(x, M); return;
  }
}

}  // namespace mmx

namespace {
struct BuiltinTag {
  int dim, monType;
};
BuiltinTag g_tags[2][8] = {{{2, 0}, {2, 1}, {2, 2}, {2, 3}, {2, 4}, {2, 5}, {2, 6}, {2, 7}},
                           {{3, 0}, {3, 1}, {3, 2}, {3, 3}, {3, 4}, {3, 5}, {3, 6}, {3, 7}}};
void builtin_trampoline(int dim, const double* x, double* M, void* user) {
  const BuiltinTag* t = static_cast<const BuiltinTag*>(user);
  mmx::builtin_monitor_eval(dim, t->monType, x, M);
}
}  // namespace

extern "C" int mmadmm_builtin_monitor(int dim, int mon_type, mmadmm_monitor_fn* fn, void** user) {
  return mmx::guarded([&] {
    if ((dim != 2 && dim != 3) || mon_type < 0 || mon_type > 7 || !fn || !user)
      throw mmx::Error(MMADMM_ERR_INVALID, "mmadmm_builtin_monitor: dim must be 2|3, mon_type 0..7");
    *fn = &builtin_trampoline;
    *user = &g_tags[dim - 2][mon_type];
  });
}

namespace mmx {
// the built-in monitor behind (fn, user), or -1 for a user callback
int builtin_monitor_kind(mmadmm_monitor_fn fn, void* user) {
  if (fn != &builtin_trampoline) return -1;
  for (int d = 0; d < 2; ++d)
    for (int k = 0; k < 8; ++k)
      if (user == &g_tags[d][k]) return k;
  return -1;
}
}  // namespace mmx
