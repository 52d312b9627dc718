"""The element-partitioned engine across PROCESSES (one per rank, as bench.py's N > 1 run), each on
GPU 0 of the box, with the halo exchange and the block all-gathers carried by a host transport over
a torch.distributed gloo process group (mmadmm_comm_create_host + TorchDistTransport): every rank
makes its own calls in its own time, so the exchange ordering LoopbackComm's shared barrier hides is
exercised.  Node positions must equal the single-GPU run bit for bit.

* C4 (512,191 nodes, 3,000,564 tetrahedra, MonType 6), 2 ranks: 1 step x 10 ADMM iterations.
* a 2D disc with the moving-bump monitor rebuilt every step (partitioned regrid), 4 ranks: 3 steps.
* early exit (tol 1e-3) on 3 ranks: the same iteration counts as one GPU (summed residuals).
"""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))

pytestmark = pytest.mark.gpu

CASES = {
    # name: (mesh, dim, MonType, rho, tau, dt, steps, iters, tol, regrid, world)
    "c4_2ranks": (("rect", 3, 63), 3, 6, 2000.0, 0.5, 0.025, 1, 10, -1.0, False, 2),
    "disc_regrid_4ranks": (("disc", 2, 120), 2, 7, 200.0, 0.5, 0.05, 3, 5, -1.0, True, 4),
    "disc_early_exit_3ranks": (("disc", 2, 60), 2, 1, 50.0, 0.5, 0.055, 3, 10, 1e-3, False, 3),
}


def _mesh(mx, spec):
    kind, dim, n = spec
    return mx.MeshData.hexdisc(n, 0.5, 0.5, 0.5) if kind == "disc" else mx.MeshData.rect(dim, n)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, name, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mmadmm_amd as mx

        spec, dim, mon, rho, tau, dt, steps, iters, tol, regrid, _ = CASES[name]
        mesh = _mesh(mx, spec)
        M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=tau, device=0)
        tr = mx.TorchDistTransport()
        comm = mx.Comm.host(world, rank, tr)
        e = mx.Engine(M, dt, rank=rank, nranks=world, comm=comm)
        if regrid:
            e.set_regrid(True)
        ih, its = [], []
        for _ in range(steps):
            a, b = e.step(iters, tol)
            ih.append(a)
            its.append(b)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), x=e.get("x").reshape(-1, dim), ids=e.local_nodes(),
                 ih=np.array(ih), its=np.array(its), calls=tr.calls, sent=tr.bytes_sent)
        e.close()
        comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", list(CASES))
def test_multiprocess_partition_equals_single(name):
    import mmadmm_amd as mx

    spec, dim, mon, rho, tau, dt, steps, iters, tol, regrid, world = CASES[name]
    with tempfile.TemporaryDirectory() as outdir:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_rank_main, args=(r, world, port, name, outdir)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=600)
        codes = [p.exitcode for p in procs]
        assert codes == [0] * world, codes
        res = [dict(np.load(os.path.join(outdir, f"rank{r}.npz"))) for r in range(world)]
    mesh = _mesh(mx, spec)
    M = mx.Mesh(mesh.Xp, mesh.F, mesh.mask, mx.BuiltinMonitor(dim, mon), rho=rho, tau=tau, device=0)
    ref = mx.Engine(M, dt)
    if regrid:
        ref.set_regrid(True)
    ih_ref, its_ref = [], []
    for _ in range(steps):
        a, b = ref.step(iters, tol)
        ih_ref.append(a)
        its_ref.append(b)
    xr = ref.get("x").reshape(-1, dim)
    ref.close()
    covered = np.zeros(mesh.nP, bool)
    for r, d in enumerate(res):
        assert np.array_equal(d["x"], xr[d["ids"]]), f"rank {r}: node positions differ from one GPU"
        assert list(d["its"]) == its_ref, (r, list(d["its"]), its_ref)
        np.testing.assert_allclose(d["ih"], ih_ref, rtol=1e-12)
        assert int(d["calls"]) > 0 and int(d["sent"]) > 0  # the halo really went through the transport
        covered[d["ids"]] = True
    assert covered.all()

