"""The element partition's failure handling: a rank that never joins, or stops,
must end the run with MMADMM_ERR_RCCL and a message, never a silent hang.

* CPU: the bounded polling loop behind every RCCL wait (mm-admm_amd/csrc/host/comm_poll.h) with a
  fake clock (tests/cpp/comm_poll_check.cpp).
* GPU: a two-rank RCCL communicator created by rank 0 alone (rank 1 never comes) returns
  MMADMM_ERR_RCCL after its deadline, aborted, instead of blocking in ncclCommInitRank forever.

The reference has no multi-process axis (its only parallelism is OpenMP over simplices,
/root/reference/src/Mesh.cpp:945-948); this covers the partition that replaces it."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")


def test_poll_bounded_host():
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "comm_poll_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-o", exe, os.path.join(ROOT, "tests", "cpp", "comm_poll_check.cpp")],
                   check=True, capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


def test_timeout_entry_exported():
    import ctypes
    import mmadmm_amd as mx
    L = mx.lib()
    assert isinstance(L.mmadmm_comm_create_rccl_timeout, ctypes._CFuncPtr)


_LONE_RANK = r"""
import sys, time
sys.path.insert(0, %r)
import mmadmm_amd as mx
uid = mx.Comm.unique_id()
t0 = time.time()
try:
    mx.Comm.rccl(2, 0, uid, 0, timeout_s=8.0)
    print("CREATED")
except mx.MMADMMError as e:
    print("CODE", e.code, "%%.1f" %% (time.time() - t0))
    print(str(e))
"""


@pytest.mark.gpu
def test_rccl_create_times_out_when_a_rank_never_joins():
    code = _LONE_RANK % os.path.join(ROOT, "mm-admm_amd", "python")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    out = r.stdout
    assert r.returncode == 0, (out + r.stderr)[-3000:]
    assert "CREATED" not in out
    line = [ln for ln in out.splitlines() if ln.startswith("CODE")][0]
    _, c, el = line.split()
    assert int(c) == 5, out  # MMADMM_ERR_RCCL
    assert 7.0 <= float(el) < 120.0, out
    assert "rank 0 of 2" in out and "ncclCommInitRankConfig" in out
