"""Element partition of the ADMM consensus step on CPU ranks (torch.distributed, gloo): the
exchange plan of libmmadmm (host-only mmadmm_plan_*) plus an all-gather of interface-slot values
reproduces, bit for bit, the single-process per-node sums over incident slots in ascending
global simplex order -- the sums k_xupdate / k_predict form on each GPU."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))


def _expected_sums(F, nP, D, T):
    """Single process: node v sums T over its incident slots, ascending simplex id, from 0.0."""
    K = D * (D + 1)
    acc = [[0.0] * D for _ in range(nP)]
    for s in range(len(F)):
        for n in range(D + 1):
            v = int(F[s, n])
            for c in range(D):
                acc[v][c] = acc[v][c] + float(T[s * K + n * D + c])
    return np.array(acc)


def _rank_main(rank, world, port, dim, n, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mmadmm_amd as mx
        mesh = mx.MeshData.rect(dim, n)
        D, K = dim, dim * (dim + 1)
        F = mesh.F
        T = np.random.default_rng(5).standard_normal(len(F) * K) * np.exp(np.random.default_rng(6).uniform(-20, 20, len(F) * K))
        plan = mx.partition_plan(dim, mesh.nP, F, world, rank)
        s0 = plan["simplexBegin"]
        mxe = max(plan["maxExport"], 1)
        send = np.zeros((mxe, D))
        for e, off in enumerate(plan["exportOff"]):
            send[e] = T[s0 * K + off: s0 * K + off + D]
        gathered = [torch.zeros(mxe * D, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(send.reshape(-1)))
        remote = torch.cat(gathered).numpy().reshape(-1, D)
        nodes = plan["localNodes"]
        sums = np.zeros((len(nodes), D))
        for l in range(len(nodes)):
            acc = [0.0] * D
            for t in range(plan["incPtr"][l], plan["incPtr"][l + 1]):
                src = int(plan["incSrc"][t])
                vals = T[s0 * K + src: s0 * K + src + D] if src >= 0 else remote[-1 - src]
                for c in range(D):
                    acc[c] = acc[c] + float(vals[c])
            sums[l] = acc
        exp = _expected_sums(F, mesh.nP, D, T)[nodes]
        out[rank] = bool(np.array_equal(sums, exp)) and len(nodes) > 0
        # every simplex is owned by exactly one rank
        cnt = torch.tensor([plan["nLocalSimplices"]], dtype=torch.int64)
        dist.all_reduce(cnt)
        out[rank] = out[rank] and int(cnt.item()) == len(F)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,dim,n", [(2, 2, 8), (3, 2, 7), (2, 3, 3)])
def test_partition_exchange_gloo(world, dim, n):
    pytest.importorskip("mmadmm_amd")
    port = 29500 + world * 10 + dim * 100 + n
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, dim, n, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world))


def test_single_rank_plan_is_the_full_incidence():
    import mmadmm_amd as mx
    mesh = mx.MeshData.rect(2, 5)
    plan = mx.partition_plan(2, mesh.nP, mesh.F, 1, 0)
    assert np.array_equal(plan["localNodes"], np.arange(mesh.nP)) and plan["maxExport"] == 0
    assert (plan["incSrc"] >= 0).all() and plan["nLocalSimplices"] == len(mesh.F)
