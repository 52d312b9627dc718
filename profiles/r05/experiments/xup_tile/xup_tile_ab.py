"""C3 (hexdisc N=577, 1,000,519 nodes) x-update by node tiles staged in LDS (default) against the
gather form (MMX_XUP_TILE=0): x-update and prox kernel times and ADMM it/s from bench.py's C3 line,
alternating; run from the repository root."""
import json, os, subprocess, sys
B = [sys.executable, "-u", "bench.py", "--steps", "20", "--warmup", "3", "--no-spmv", "--no-be", "--no-bfgs",
     "--no-3d", "--no-cpu-baseline"]
for rep in range(2):
    for tile in ("1", "0"):
        env = dict(os.environ, MMX_XUP_TILE=tile)
        out = subprocess.run(B, env=env, capture_output=True, text=True, timeout=600)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        print(json.dumps({"tile": tile, "value": d["value"], "ms_per_step": d["ms_per_step"], "kernels": d["kernels"],
                          "c2": d["c2"]["value"]}), flush=True)
