"""Same-box comparison of build variants of libmmadmm (profiles/r04/variants.sh builds them with
extra -D flags into dev/lib_<name>/): for each library (MMADMM_LIB) in a fresh process, the
workload's prox / x-update times from HIP events and a hash of the node positions (variants must be
bit-identical).  Usage: python variant_bench.py <c3|c4|c2> <steps> <lib>[+VAR=VALUE...] [...]"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one(work, steps):
    import time
    sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))
    import mmadmm_amd as mx
    if work in ("c4", "c4mb"):  # c4mb: the isotropic moving-bump monitor (MonType 7) at t = 0
        m = mx.MeshData.rect(3, 63)
        M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(3, 6 if work == "c4" else 7), rho=2000.0, tau=0.5)
        dt = 0.025
    elif work == "c2":
        m = mx.MeshData.rect(2, 223)
        M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
        dt = 0.055
    else:
        m = mx.MeshData.hexdisc(577, 0.5, 0.5, 0.5)
        M = mx.Mesh(m.Xp, m.F, m.mask, mx.BuiltinMonitor(2, 1), rho=50.0, tau=0.5)
        dt = 0.055
    E = mx.Engine(M, dt)
    for _ in range(3):
        E.step(10, -1.0)
    E.set_timing(True)
    E.reset_stats()
    E.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        E.step(10, -1.0)
    E.sync()
    el = time.perf_counter() - t0
    st = E.stats()
    x = E.get("x")
    prox = st["t_prox_ms"] / st["n_prox"]
    return {"lib": os.environ.get("MMADMM_LIB", "default"), "work": work, "it_s": round(steps * 10 / el, 2),
            "prox_ms": round(prox, 4), "xup_ms": round(st["t_xupdate_ms"] / st["n_xupdate"], 4),
            "prox_GBs": round(st["prox_bytes"] / prox / 1e6, 1),
            "bfgs_per_prox": round(st["bfgs_iters"] / st["admm_iters"] / m.nF, 4),
            "xhash": hashlib.sha1(x.tobytes()).hexdigest()[:16]}


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        print(json.dumps(one(sys.argv[2], int(sys.argv[3]))), flush=True)
        sys.exit(0)
    work, steps, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
    for rep in range(2):  # two rounds, alternating, against box drift
        for spec in libs:
            # "<lib>[+VAR=VALUE...]": a library (or "default") and environment settings for it
            lib, *sets = spec.split("+")
            env = dict(os.environ)
            env.update(kv.split("=", 1) for kv in sets)
            if lib != "default":
                env["MMADMM_LIB"] = os.path.abspath(lib)
            r = subprocess.run([sys.executable, __file__, "--one", work, steps], env=env, capture_output=True,
                               text=True, timeout=600)
            if r.returncode != 0:
                print(json.dumps({"lib": lib, "error": r.stderr[-2000:]}), flush=True)
                sys.exit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            d["round"] = rep
            d["spec"] = spec
            print(json.dumps(d), flush=True)
