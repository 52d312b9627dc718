// MatrixIter.h -- the reference's LASolver classes (lib/LASolver/MatrixIter.h:66-383,
// SparseItUtil.h:7-11) over the C-ABI of libmmadmm.so (include/mmx_sparse.h): the ILU-preconditioned
// CG-STAB solve runs on the MI355X.  Same namespace, class names, signatures and argument meaning, so
// the reference's own caller -- Mesh<D>::buildMatrix and Mesh<D>::backwardsEulerStep (src/Mesh.cpp:
// 262-382, 1112-1341) -- compiles unchanged against this header.
//
//   General_Exception(const char*), member p      SparseItUtil.h:7-11
//   MatrixStruc(n, no_diag)                       MatrixIter.cpp:88-116   -> mmx_struc_create
//   MatrixStruc::set_entry(row, col)              MatrixIter.cpp:125-142  -> mmx_struc_set_entry
//   MatrixStruc::pack / getia / getja / getnja    MatrixIter.cpp:144-257  -> mmx_struc_pack / mmx_struc_get
//   ParamIter (public fields, the reference's     MatrixIter.h:113-175
//     defaults: order 1, level 1, iscal 1, ...)
//   MatrixIter(MatrixStruc&)                      MatrixIter.cpp:320-342  -> mmx_matrix_create_from_struc
//   MatrixIter(n, ia, ja) / init(n, ia, ja)       MatrixIter.cpp:344-427  -> mmx_matrix_create
//   aValue(k), aValue(row, col), bValue(i)        MatrixIter.h:308-320    host arrays, uploaded by solve
//   rowBegin / rowEndPlusOne / getColIndex        MatrixIter.h:367-371
//   get_n / get_ia / get_ja / getnonzero          MatrixIter.h:350, 377-381
//   check_entry, zeroa, zerob, mult_row,          MatrixIter.cpp (host-side accessors)
//     set_row, zero_row
//   sfac(ParamIter&)                              MatrixIter.cpp:455-489  -> mmx_matrix_sfac
//   set_toler(const double*)                      MatrixIter.cpp:443-453  -> mmx_matrix_set_toler
//   solve(ParamIter&, double* x, int& nitr, ig)   MatrixIter.cpp:635-819  -> mmx_matrix_set_values,
//                                                                            mmx_matrix_set_rhs, mmx_matrix_solve
//
// The matrix values and the right-hand side live in host arrays, as in the reference: aValue(k) and
// bValue(i) return references into them, and solve() hands both to the device (the values are
// factored again, as the reference re-factors in every solve, MatrixIter.cpp:684).  Non-convergence
// is nitr = -1, as in the reference.  Errors the reference throws as General_Exception (a bad entry,
// a packed structure) are thrown as General_Exception here too; so are the C-ABI's other failures
// (no GPU, an unsupported ParamIter setting: RCM ordering, drop-tolerance ILU, scaling, orthomin and
// CG are not implemented -- the reference's only caller uses none of them, src/Mesh.cpp:264-304).
// The device is mmx_device() (0 unless set).  Header-only; link with -lmmadmm.
#ifndef MATRIX_ITER_INC
#define MATRIX_ITER_INC

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../mmx_sparse.h"

namespace SparseItObj {

class General_Exception {
public:
    const char* p;
    General_Exception(const char* q) { p = q; }
};

// the device the matrices are created on
inline int& mmx_device() {
    static int dev = 0;
    return dev;
}

namespace detail {
inline void check(int rc) {
    if (rc == MMADMM_OK) return;
    static thread_local std::string msg;  // General_Exception keeps a pointer
    msg = mmadmm_last_error();
    throw General_Exception(msg.c_str());
}
}  // namespace detail

class MatrixStruc {
public:
    MatrixStruc(const int n_in, const int no_diag = 0) : n(n_in) {
        detail::check(mmx_struc_create(n_in, no_diag, &s_));
    }
    ~MatrixStruc(void) { mmx_struc_destroy(s_); }
    MatrixStruc(const MatrixStruc&) = delete;
    MatrixStruc& operator=(const MatrixStruc&) = delete;

    int get_sort_row(void) { return 1; }  // pack() sorts every row (the reference's sort_row = 1 after pack)

    void set_entry(int row, int col) { detail::check(mmx_struc_set_entry(s_, row, col)); }
    int* getia(void) {  // a new copy (delete[] by the caller); packs first, as the reference
        pack();
        int nn = 0;
        long long nnz = 0;
        detail::check(mmx_struc_get(s_, &nn, &nnz, nullptr, nullptr));
        int* ia = new int[nn + 1];
        detail::check(mmx_struc_get(s_, &nn, &nnz, ia, nullptr));
        return ia;
    }
    int* getja(void) {
        pack();
        int nn = 0;
        long long nnz = 0;
        detail::check(mmx_struc_get(s_, &nn, &nnz, nullptr, nullptr));
        int* ja = new int[nnz > 0 ? nnz : 1];
        detail::check(mmx_struc_get(s_, &nn, &nnz, nullptr, ja));
        return ja;
    }
    int getnja(void) {
        pack();
        int nn = 0;
        long long nnz = 0;
        detail::check(mmx_struc_get(s_, &nn, &nnz, nullptr, nullptr));
        return (int)nnz;
    }
    void pack(void) {
        if (!packed_) detail::check(mmx_struc_pack(s_));
        packed_ = true;
    }
    int getn(void) const { return n; }

    mmx_struc handle() { return s_; }

private:
    int n;
    bool packed_ = false;
    mmx_struc s_ = nullptr;
};

class ParamIter {
public:
    int order;
    int level;
    int drop_ilu;
    int ipiv;
    int iscal;
    int nitmax;
    double resid_reduc;
    int info;
    double drop_tol;
    int new_rhat;
    int iaccel;
    int north;

    ParamIter(void) {  // the reference's defaults (MatrixIter.h:154-167)
        order = 1;
        level = 1;
        drop_ilu = 0;
        iscal = 1;
        nitmax = 30;
        resid_reduc = 1.e-6;
        drop_tol = 1.e-3;
        info = 1;
        new_rhat = 0;
        iaccel = 0;
        north = 10;
        ipiv = 0;
    }
    ParamIter(const ParamIter&) = delete;
    ~ParamIter(void) {}

    mmx_param_iter abi() const {
        mmx_param_iter p{};
        p.order = order;
        p.level = level;
        p.drop_ilu = drop_ilu;
        p.ipiv = ipiv;
        p.iscal = iscal;
        p.nitmax = nitmax;
        p.resid_reduc = resid_reduc;
        p.info = info;
        p.drop_tol = drop_tol;
        p.new_rhat = new_rhat;
        p.iaccel = iaccel;
        p.north = north;
        return p;
    }
};

class MatrixIter {
public:
    MatrixIter(MatrixStruc& iaja_set) {
        iaja_set.pack();
        int* ia = iaja_set.getia();
        int* ja = iaja_set.getja();
        try {
            init(iaja_set.getn(), ia, ja);
        } catch (...) {
            delete[] ia;
            delete[] ja;
            throw;
        }
        delete[] ia;
        delete[] ja;
    }
    MatrixIter(const int n_in, const int* ia_in, const int* ja_in) { init(n_in, ia_in, ja_in); }
    MatrixIter(const MatrixIter&) = delete;
    MatrixIter& operator=(const MatrixIter&) = delete;
    ~MatrixIter(void) {
        if (m_) mmx_matrix_destroy(m_);
    }

    void init(const int n_in, const int* ia_in, const int* ja_in) {
        if (m_) mmx_matrix_destroy(m_);
        m_ = nullptr;
        n = n_in;
        ia.assign(ia_in, ia_in + n_in + 1);
        ja.assign(ja_in, ja_in + ia_in[n_in]);
        a.assign(ja.size(), 0.0);
        b.assign(n_in, 0.0);
        detail::check(mmx_matrix_create(mmx_device(), n_in, ia.data(), ja.data(), &m_));
    }

    // symbolic level-of-fill ILU (natural order)
    void sfac(ParamIter& param) {
        const mmx_param_iter p = param.abi();
        detail::check(mmx_matrix_sfac(m_, &p));
    }

    // x = A^-1 b (initial_guess = 0: x zeroed first) or x = x0 + A^-1 (b - A x0); nitr = -1 when
    // CG-STAB did not converge within param.nitmax
    void solve(ParamIter& param, double* x, int& nitr, const int initial_guess = 0) {
        const mmx_param_iter p = param.abi();
        detail::check(mmx_matrix_set_values(m_, a.data()));
        detail::check(mmx_matrix_set_rhs(m_, b.data()));
        int it = 0;
        detail::check(mmx_matrix_solve(m_, &p, x, &it, initial_guess));
        nitr = it;
    }

    void set_toler(const double* tol_in) { detail::check(mmx_matrix_set_toler(m_, tol_in)); }

    double& bValue(const int i) { return b[i]; }
    double& aValue(const int k) { return a[k]; }
    double& aValue(const int row, const int col) {
        for (int k = ia[row]; k < ia[row + 1]; ++k)
            if (ja[k] == col) return a[k];
        throw General_Exception("error: (row, col) not in the sparse matrix data structure\n");
    }
    double& aValue_bsearch(const int row, const int col) { return aValue(row, col); }
    int check_entry(int i, int j) {
        for (int k = ia[i]; k < ia[i + 1]; ++k)
            if (ja[k] == j) return 1;
        return 0;
    }
    void zeroa(void) { std::fill(a.begin(), a.end(), 0.0); }
    void zerob(void) { std::fill(b.begin(), b.end(), 0.0); }
    void set_row(const int i, double* row) {
        for (int k = ia[i]; k < ia[i + 1]; ++k) a[k] = row[ja[k]];
    }
    void zero_row(const int i, double* row) {
        for (int k = ia[i]; k < ia[i + 1]; ++k) row[ja[k]] = 0.0;
    }
    double mult_row(const int row, double* val) {  // sum over the row in storage order
        double s = 0.0;
        for (int k = ia[row]; k < ia[row + 1]; ++k) s += a[k] * val[ja[k]];
        return s;
    }
    int getnonzero(void) {  // nonzeros of the ILU factor (after sfac)
        long long nz = 0;
        detail::check(mmx_matrix_factor_nnz(m_, &nz));
        return (int)nz;
    }

    int rowBegin(const int row) const { return ia[row]; }
    int rowEndPlusOne(const int row) const { return ia[row + 1]; }
    int getColIndex(const int k) const { return ja[k]; }
    int get_n(void) { return n; }
    int* get_ia(void) { return ia.data(); }
    int* get_ja(void) { return ja.data(); }

    mmx_matrix handle() { return m_; }

private:
    int n = 0;
    std::vector<int> ia, ja;
    std::vector<double> a, b;
    mmx_matrix m_ = nullptr;
};

}  // namespace SparseItObj

#endif
