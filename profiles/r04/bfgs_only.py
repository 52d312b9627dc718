"""The BFGS-heavy section of bench.py alone (SquareGrid n = 707, MEx1, rho 1; bench.bfgs_bench),
for its own rocprofv3 counter pass: the prox launches here have the same grid size class as the
headline's, so they are profiled apart and summarised under "k_prox_lds<2, 128>@bfgs_heavy"."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
import bench  # noqa: E402
import mmadmm_amd as mx  # noqa: E402

print(json.dumps(bench.bfgs_bench(mx, False, 1, 10)), flush=True)
