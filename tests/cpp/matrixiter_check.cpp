// matrixiter_check.cpp -- include/mmadmm/MatrixIter.h (the reference's SparseItObj::MatrixStruc /
// ParamIter / MatrixIter, lib/LASolver/MatrixIter.h:66-383) on the host: the structure calls, the
// reference's General_Exception cases and ParamIter's defaults.  Test infrastructure
// (tests/test_cpp_dropin.py::test_matrixiter_header); a MatrixIter needs a GPU, so without one its
// construction must throw General_Exception (the C-ABI's "no HIP device") rather than crash.
// Prints one "name ok|FAIL detail" line per check.
#include <cstdio>
#include <string>
#include <vector>

#include "SparseItObj.h"

using namespace SparseItObj;

static int fails = 0;
static void check(const char* name, bool ok, const std::string& why = "") {
    std::printf("%s %s %s\n", name, ok ? "ok" : "FAIL", why.c_str());
    if (!ok) fails++;
}

int main() {
    // MatrixStruc(n, 0): the diagonal is inserted (MatrixIter.cpp:99-104); set_entry, duplicates
    // merged by pack, rows sorted
    MatrixStruc s(4, 0);
    s.set_entry(0, 3);
    s.set_entry(2, 1);
    s.set_entry(2, 1);
    s.set_entry(3, 0);
    s.pack();
    int* ia = s.getia();
    int* ja = s.getja();
    const std::vector<int> eia = {0, 2, 3, 5, 7}, eja = {0, 3, 1, 1, 2, 0, 3};
    bool ok = s.getnja() == 7;
    for (int i = 0; i <= 4; ++i) ok = ok && ia[i] == eia[i];
    for (int k = 0; ok && k < 7; ++k) ok = ja[k] == eja[k];
    check("struc_pattern", ok);
    delete[] ia;
    delete[] ja;
    // MatrixStruc(n, 1): no diagonal
    MatrixStruc s1(3, 1);
    s1.set_entry(1, 2);
    check("struc_no_diag", s1.getnja() == 1);
    // General_Exception: an entry after pack, a row or column out of range (MatrixIter.cpp:125-142)
    auto throws = [](auto&& f) {
        try {
            f();
        } catch (const General_Exception& e) {
            return e.p != nullptr && e.p[0] != 0;
        }
        return false;
    };
    check("set_entry_after_pack", throws([&] { s.set_entry(0, 1); }));
    MatrixStruc s2(3, 0);
    check("row_out_of_range", throws([&] { s2.set_entry(3, 0); }));
    check("col_out_of_range", throws([&] { s2.set_entry(0, -1); }));
    // ParamIter's defaults (MatrixIter.h:154-167)
    ParamIter p;
    check("param_defaults", p.order == 1 && p.level == 1 && p.drop_ilu == 0 && p.iscal == 1 && p.nitmax == 30 &&
                                p.resid_reduc == 1.e-6 && p.drop_tol == 1.e-3 && p.info == 1 && p.new_rhat == 0 &&
                                p.iaccel == 0 && p.north == 10 && p.ipiv == 0);
    // MatrixIter on a GPU box: host accessors; without a GPU: General_Exception
    bool built = false, gpuless = false;
    try {
        MatrixIter m(s);
        built = true;
        ok = m.get_n() == 4 && m.rowBegin(2) == 3 && m.rowEndPlusOne(2) == 5 && m.getColIndex(4) == 2 &&
             m.check_entry(0, 3) && !m.check_entry(0, 1);
        m.aValue(2, 1) = 5.0;
        m.zerob();
        m.bValue(1) = 2.0;
        double v[4] = {1.0, 2.0, 3.0, 4.0};
        ok = ok && m.aValue(3) == 5.0 && m.mult_row(2, v) == 10.0;
        check("matrix_host_accessors", ok);
    } catch (const General_Exception& e) {
        gpuless = std::string(e.p).find("HIP") != std::string::npos || std::string(e.p).find("device") != std::string::npos;
    }
    check("matrix_built_or_gpuless", built || gpuless);
    return fails ? 1 : 0;
}
