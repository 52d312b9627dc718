// lasolver_ref_capi.cpp -- C entry points over the reference LASolver, linked against the
// reference sources compiled in place (oracle/Makefile.ref).  TEST INFRASTRUCTURE ONLY: used by
// tests/ and tests/golden/make_lasolver_golden.py to pin oracle/lasolver.cpp; never shipped, never
// timed as the product.
//
// The call sequence is the one src/Mesh.cpp uses for backward Euler: MatrixStruc + set_entry +
// pack (Mesh.cpp:309-345), MatrixIter(MatrixStruc&) (354), ParamIter as in buildMatrix (264-304),
// aValue/bValue (1283-1310), sfac + set_toler + solve (1315-1323).
#include <cstring>
#include <exception>
#include <vector>

#include "def_compiler.h"
#include "Standard.h"
#include "SparseItUtil.h"
#include "ILU_class.h"
#include "accel_class.h"
#include "MatrixIter.h"

using namespace SparseItObj;

extern "C" {

// MatrixStruc(n, no_diag) + set_entry(rows[e], cols[e]) + pack().  Writes ia (n+1) and, if it
// fits, ja (cap entries).  Returns nnz, or -1 on a reference exception.
int lsr_struc_pack(int n, int nent, const int* rows, const int* cols, int no_diag, int* ia, int* ja, int cap) {
  try {
    MatrixStruc s(n, no_diag);
    for (int e = 0; e < nent; ++e) s.set_entry(rows[e], cols[e]);
    s.pack();
    int* ia_ = s.getia();
    int* ja_ = s.getja();
    const int nnz = ia_[n];
    std::memcpy(ia, ia_, sizeof(int) * (n + 1));
    if (nnz <= cap) std::memcpy(ja, ja_, sizeof(int) * nnz);
    delete[] ia_;
    delete[] ja_;
    return nnz;
  } catch (...) {
    return -1;
  }
}

// MatrixIter(n, ia, ja); a, b loaded; sfac(param); set_toler(toler or zeros); solve(param, x,
// nitr, initial_guess).  x holds the initial guess on entry when initial_guess != 0.  Returns 0,
// or -1 on a reference exception.
int lsr_solve(int n, const int* ia, const int* ja, const double* a, const double* b, const double* toler,
              int order, int level, int iscal, int iaccel, int nitmax, double resid_reduc, int new_rhat,
              int initial_guess, double* x, int* nitr) {
  try {
    MatrixIter m(n, ia, ja);
    for (int k = 0; k < ia[n]; ++k) m.aValue(k) = a[k];
    for (int i = 0; i < n; ++i) m.bValue(i) = b[i];
    ParamIter p;
    p.order = order;
    p.level = level;
    p.drop_ilu = 0;
    p.iscal = iscal;
    p.nitmax = nitmax;
    p.ipiv = 0;
    p.resid_reduc = resid_reduc;
    p.info = 0;
    p.drop_tol = 1.e-3;
    p.new_rhat = new_rhat;
    p.iaccel = iaccel;
    p.north = 10;
    m.sfac(p);
    if (toler) {
      m.set_toler(toler);
    }
    int it = 0;
    m.solve(p, x, it, initial_guess);
    *nitr = it;
    return 0;
  } catch (...) {
    return -1;
  }
}

}  // extern "C"

namespace {
// The ILU row structures are protected members of scaler_ILU (ILU_class.h:146); a derived class
// reads them back so the fixtures can pin the numeric factor itself.
class RefILU : public scaler_ILU {
 public:
  RefILU(int n, int* lord, int* pord) : scaler_ILU(n, lord, pord) {}
  int rowNz(int i) const { return rowsp[i].nz; }
  int rowDiag(int i) const { return rowsp[i].diag; }
  const int* rowJaf(int i) const { return rowsp[i].jaf; }
  const double* rowAf(int i) const { return rowsp[i].af; }
};
}  // namespace

extern "C" {

// scaler_ILU(n, natural order) + sfac2(level) + factor(a) (ILU_class.cpp:90-444).  Writes the
// factor in CSR form: iaf (n+1), jaf/af (cap), diag (n, row-relative).  Returns nnz(ILU) or -1.
int lsr_ilu(int n, const int* ia, const int* ja, const double* a, int level, int* iaf, int* jaf, double* af,
            int* diag, int cap) {
  try {
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    RefILU ilu(n, ord.data(), nullptr);
    int nzero = 0, ier = 0;
    ilu.sfac2(ia, ja, level, &nzero, &ier);
    if (ier != 0) return -1;
    ilu.factor(ia, ja, a);
    iaf[0] = 0;
    for (int i = 0; i < n; ++i) iaf[i + 1] = iaf[i] + ilu.rowNz(i);
    if (iaf[n] <= cap)
      for (int i = 0; i < n; ++i) {
        diag[i] = ilu.rowDiag(i);
        for (int k = 0; k < ilu.rowNz(i); ++k) {
          jaf[iaf[i] + k] = ilu.rowJaf(i)[k];
          af[iaf[i] + k] = ilu.rowAf(i)[k];
        }
      }
    return iaf[n];
  } catch (...) {
    return -1;
  }
}

// The same factor, then scaler_ILU::solve(x, b) (ILU_class.cpp:447-527).
int lsr_ilu_solve(int n, const int* ia, const int* ja, const double* a, const double* b, double* x) {
  try {
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    RefILU ilu(n, ord.data(), nullptr);
    int nzero = 0, ier = 0;
    ilu.sfac2(ia, ja, 0, &nzero, &ier);
    if (ier != 0) return -1;
    ilu.factor(ia, ja, a);
    ilu.solve(x, b);
    return 0;
  } catch (...) {
    return -1;
  }
}

// matmult (accel_class.cpp:521-549).
int lsr_matmult(int n, const int* ia, const int* ja, const double* a, const double* x, double* y) {
  matmult(const_cast<double*>(x), y, n, const_cast<double*>(a), const_cast<int*>(ia), const_cast<int*>(ja));
  return 0;
}

}  // extern "C"
