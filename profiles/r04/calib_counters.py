"""Calibration of the rocprofv3 byte counters on this build's access widths (MI355X_MICROARCH.md
§HBM: FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads; other widths are
uncalibrated).  Runs each k_stream_copy calibration variant (include/mmx_sparse.h) once over
n = 2^27 doubles (1 GiB, four times the 256 MiB Infinity Cache) so that every byte comes from HBM.
Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`; the counters per
dispatch divided by the bytes below are the factors profiles/make_pmc_summary.py applies."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
import lasolver_amd as la  # noqa: E402

n = 1 << 27
dev = torch.device("cuda:0")
src = torch.rand(n, dtype=torch.float64, device=dev)
dst = torch.empty(n, dtype=torch.float64, device=dev)
flush = torch.empty(1 << 26, dtype=torch.float64, device=dev)  # 512 MiB written between variants
out = {}
for v, what, nbytes in ((3, "read 8 B/lane", 8 * n), (4, "read 24-B record/lane (3 x 8 B)", 8 * (n // 3) * 3),
                        (5, "read 16 B/lane", 8 * n), (6, "store 8 B/lane", 8 * n),
                        (7, "store 8 B/lane nontemporal", 8 * n), (8, "read random 24-B record/lane", 8 * (n // 3) * 3)):
    flush.fill_(float(v))
    torch.cuda.synchronize()
    ms = la.stream_copy_ms(src.data_ptr(), dst.data_ptr(), n, reps=1, device=0, variant=v)
    out[v] = {"what": what, "bytes": nbytes, "ms_1rep": round(ms, 4)}
print(json.dumps(out, indent=1), flush=True)
