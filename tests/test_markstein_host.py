"""The prox kernels' division by c2 through one reciprocal (crmath.h div_mk, Markstein's
correction) and its range test (mk_exp), checked on the host: bit-identical to IEEE division on
random, near-midpoint and signed-zero operands inside the ranges the kernels accept, and every
operand outside them rejected.  The device counterpart is
tests/test_gpu_parity.py::test_device_division_by_reciprocal_is_correctly_rounded."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG), reason="ROCm clang++ not installed")
def test_div_mk_matches_ieee_division(tmp_path):
    """Compiled by the device compiler's clang for the host (-mfma: the hardware FMA, as on the
    device).  GCC is not used: at -O2 it folds -fma(q, c, -x) into fnma(q, c, x), which turns the
    -0 quotient of x = -0 into +0 (LLVM keeps that fold behind no-signed-zeros)."""
    exe = tmp_path / "markstein_check"
    subprocess.run([CLANG, "-std=c++17", "-O2", "-mfma", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(ROOT, "tests", "cpp", "markstein_check.cpp")], check=True,
                   capture_output=True, text=True)
    r = subprocess.run([str(exe), "100000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok ")
