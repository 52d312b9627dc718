"""Element partition of the ADMM consensus step on CPU ranks (torch.distributed, gloo): the
exchange plan of libmmadmm (host-only mmadmm_plan_*) plus a halo exchange with the neighbouring
ranks only (point-to-point send/recv of interface-slot values, as the engine does over RCCL)
reproduces, bit for bit, the single-process per-node sums over incident slots in ascending global
simplex order -- the sums k_xupdate / k_predict form on each GPU."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mm-admm_amd", "python"))


def _mesh(mx, kind, dim, n):
    if kind == "disc":
        return mx.MeshData.hexdisc(n, 0.5, 0.5, 0.5)
    return mx.MeshData.rect(dim, n)


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


def _rank_main(rank, world, port, kind, dim, n, method, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mmadmm_amd as mx
        mesh = _mesh(mx, kind, dim, n)
        D, K = dim, dim * (dim + 1)
        F = mesh.F
        T = np.random.default_rng(5).standard_normal(len(F) * K) * np.exp(np.random.default_rng(6).uniform(-20, 20, len(F) * K))
        plan = mx.partition_plan(dim, mesh.Xp, F, world, rank, method)
        ls = plan["localSimplices"]
        Tl = T.reshape(-1, K)[ls].reshape(-1)  # this rank's slot values, local simplex order
        send = np.zeros((max(len(plan["sendOff"]), 1), D))
        for e, off in enumerate(plan["sendOff"]):
            send[e] = Tl[off: off + D]
        recv = torch.zeros(max(plan["recvRows"], 1) * D, dtype=torch.float64)
        reqs, so, ro = [], 0, 0
        sendt = torch.from_numpy(send.reshape(-1))
        for q, ns, nr in plan["peers"]:
            reqs.append(dist.isend(sendt[so * D:(so + ns) * D].clone(), int(q)))
            reqs.append(dist.irecv(recv[ro * D:(ro + nr) * D], int(q)))
            so, ro = so + ns, ro + nr
        for r in reqs:
            r.wait()
        remote = recv.numpy().reshape(-1, D)
        nodes = plan["localNodes"]
        sums = np.zeros((len(nodes), D))
        for l in range(len(nodes)):
            acc = [0.0] * D
            for t in range(plan["incPtr"][l], plan["incPtr"][l + 1]):
                src = int(plan["incSrc"][t])
                vals = Tl[src: src + D] if src >= 0 else remote[-1 - src]
                for c in range(D):
                    acc[c] = acc[c] + float(vals[c])
            sums[l] = acc
        exp = _expected_sums(F, mesh.nP, D, T)[nodes]
        ok = bool(np.array_equal(sums, exp)) and len(nodes) > 0
        # every simplex is owned by exactly one rank; neighbours only (no rank talks to itself)
        cnt = torch.tensor([len(ls)], dtype=torch.int64)
        dist.all_reduce(cnt)
        ok = ok and int(cnt.item()) == len(F) and all(int(q) != rank for q in plan["peers"][:, 0])
        out[rank] = ok
    finally:
        dist.destroy_process_group()


CASES = [(2, "rect", 2, 8, "rcb"), (3, "rect", 2, 7, "rcb"), (2, "rect", 3, 3, "rcb"), (4, "disc", 2, 9, "rcb"),
         (4, "disc", 2, 9, "ranges"), (4, "rect", 3, 4, "rcb")]


@pytest.mark.parametrize("world,kind,dim,n,method", CASES)
def test_partition_exchange_gloo(world, kind, dim, n, method):
    pytest.importorskip("mmadmm_amd")
    port = 29500 + world * 10 + dim * 100 + n + (500 if method == "ranges" else 0) + (1000 if kind == "disc" else 0)
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, kind, dim, n, method, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world))


def test_single_rank_plan_is_the_full_incidence():
    import mmadmm_amd as mx
    mesh = mx.MeshData.rect(2, 5)
    plan = mx.partition_plan(2, mesh.Xp, mesh.F, 1, 0)
    assert np.array_equal(plan["localNodes"], np.arange(mesh.nP)) and len(plan["peers"]) == 0
    assert (plan["incSrc"] >= 0).all() and np.array_equal(plan["localSimplices"], np.arange(len(mesh.F)))


def _interface(mx, mesh, world, method):
    plans = [mx.partition_plan(mesh.dim, mesh.Xp, mesh.F, world, r, method) for r in range(world)]
    return plans, sum(p["interfaceNodes"] for p in plans)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rcb_disc_cuts_are_short(world):
    """The headline disc numbers its simplices ring by ring, so contiguous id ranges cut it into
    annuli (each cut a whole circle); RCB cuts it into sectors/strips with short interfaces, and
    balances the simplices to within 2% per cut (the plane snaps to the best nearby vertex
    coordinate)."""
    import mmadmm_amd as mx
    mesh = mx.MeshData.hexdisc(60, 0.5, 0.5, 0.5)
    plans, rcb = _interface(mx, mesh, world, "rcb")
    _, ranges = _interface(mx, mesh, world, "ranges")
    sizes = [len(p["localSimplices"]) for p in plans]
    assert max(sizes) <= 1.06 * len(mesh.F) / world and sum(sizes) == len(mesh.F)
    assert rcb < 0.5 * ranges, (rcb, ranges)
    assert max(len(p["peers"]) for p in plans) <= min(world - 1, 6)


def test_rcb_cuts_a_structured_cube_between_cell_layers():
    """An odd number of cell layers: the proportional cut falls inside the middle layer; the plane
    snaps to a layer boundary (one layer is within the 2% balance tolerance at n = 51), so the
    interface is one plane of (n+1)^2 nodes, not three."""
    import mmadmm_amd as mx
    n = 51
    mesh = mx.MeshData.rect(3, n)
    plans, total = _interface(mx, mesh, 2, "rcb")
    assert [p["interfaceNodes"] for p in plans] == [(n + 1) ** 2] * 2
    sizes = [len(p["localSimplices"]) for p in plans]
    assert abs(sizes[0] - sizes[1]) == len(mesh.F) // n  # one layer of cells off the half


def test_rcb_is_deterministic_and_rank_consistent():
    """Every rank derives the same owners: the simplex sets of all ranks tile the mesh, and what
    rank q sends to rank r is exactly what r expects from q (row counts agree pairwise)."""
    import mmadmm_amd as mx
    mesh = mx.MeshData.rect(3, 5)
    world = 5
    plans = [mx.partition_plan(3, mesh.Xp, mesh.F, world, r) for r in range(world)]
    own = np.concatenate([p["localSimplices"] for p in plans])
    assert np.array_equal(np.sort(own), np.arange(len(mesh.F)))
    cnt = {(r, int(q)): (int(s), int(v)) for r, p in enumerate(plans) for q, s, v in p["peers"]}
    for (r, q), (s, v) in cnt.items():
        assert cnt[(q, r)] == (v, s)
    again = mx.partition_plan(3, mesh.Xp, mesh.F, world, 2)
    assert np.array_equal(again["localSimplices"], plans[2]["localSimplices"])


@pytest.mark.parametrize("dim,n,world", [(2, 1, 4), (2, 2, 13), (2, 3, 32), (2, 4, 50), (2, 4, 64), (2, 5, 7),
                                         (3, 1, 6)])
def test_rcb_gives_every_rank_a_simplex(dim, n, world):
    """Small parts (nF = 4n^2 triangles in 2D): a snapped cut plane never leaves one side with
    fewer simplices than ranks, so no rank is left without simplices (each of the first five cases
    left ranks empty before the cut was restricted)."""
    import mmadmm_amd as mx
    mesh = mx.MeshData.rect(dim, n)
    assert len(mesh.F) >= world
    plans = [mx.partition_plan(dim, mesh.Xp, mesh.F, world, r) for r in range(world)]
    sizes = [len(p["localSimplices"]) for p in plans]
    assert min(sizes) >= 1 and sum(sizes) == len(mesh.F), sizes
    assert all(len(p["localNodes"]) >= dim + 1 for p in plans)


def _transport_main(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import mmadmm_amd as mx
        tr = mx.TorchDistTransport()
        ok = True
        # all-gather of a block per rank into one buffer (the engine's per-step scalar partials, and
        # the partitioned regrid's owned-vertex positions)
        send = np.arange(5, dtype=np.float64) + 10 * rank
        recv = np.zeros(5 * world)
        tr.allgather(send, recv)
        ok &= bool(np.array_equal(recv, np.concatenate([np.arange(5) + 10 * q for q in range(world)])))
        # halo exchange on a ring: rank r sends (r + 1) * 3 values to both neighbours, in views of one
        # host buffer at different offsets (as the engine's staging buffers), twice (tags by call order)
        for rep in range(2):
            peers = sorted({(rank + 1) % world, (rank - 1) % world} - {rank})
            buf = np.zeros(64)
            sends, recvs = [], []
            off = 0
            for q in peers:
                n = (rank + 1) * 3
                buf[off:off + n] = 1000 * rank + 100 * q + rep + np.arange(n)
                sends.append(buf[off:off + n])
                off += n
            rbuf = np.zeros(64)
            off = 0
            for q in peers:
                n = (q + 1) * 3
                recvs.append(rbuf[off:off + n])
                off += n
            tr.exchange(peers, sends, recvs)
            for q, r in zip(peers, recvs):
                ok &= bool(np.array_equal(r, 1000 * q + 100 * rank + rep + np.arange(len(r))))
            tr.exchange([], [], [])  # a rank with no peers still takes part in the call sequence
        ok &= tr.calls == 4
        out[rank] = ok
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_torch_dist_host_transport(world):
    """mmadmm_amd.TorchDistTransport, the host transport of mmadmm_comm_create_host, on gloo CPU ranks:
    the all-gather and the tagged neighbour exchange deliver every block where the engine's staging
    buffers expect it (the GPU-side staging is tests/test_gpu_multiprocess.py)."""
    pytest.importorskip("mmadmm_amd")
    port = 31800 + world
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    procs = [ctx.Process(target=_transport_main, args=(r, world, port, out)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    assert all(out[r] for r in range(world))


def test_host_comm_create_without_gpu():
    """mmadmm_comm_create_host validates its arguments and needs no device to be created."""
    import mmadmm_amd as mx

    class Null:
        def allgather(self, s, r):
            r[:] = 0

        def exchange(self, peers, sends, recvs):
            pass

    c = mx.Comm.host(2, 1, Null())
    c.close()
    with pytest.raises(mx.MMADMMError):
        mx.Comm.host(2, 2, Null())


def test_host_comm_failure_aborts_transport():
    """A transport call that raises: the callback reports status 1 to the engine (MMADMM_ERR_RCCL)
    and first calls the transport's abort(), so that the other ranks do not wait forever."""
    import ctypes
    import mmadmm_amd as mx

    class Failing:
        aborted = 0

        def allgather(self, s, r):
            raise RuntimeError("peer gone")

        def exchange(self, peers, sends, recvs):
            raise RuntimeError("peer gone")

        def abort(self):
            Failing.aborted += 1

    tr = Failing()
    c = mx.Comm.host(2, 0, tr)
    ag, ex = c._keep[0], c._keep[1]
    s = np.zeros(4)
    r = np.zeros(8)
    dp = ctypes.POINTER(ctypes.c_double)
    assert ag(None, s.ctypes.data_as(dp), r.ctypes.data_as(dp), 4) == 1
    assert Failing.aborted == 1
    ll = (ctypes.c_longlong * 1)
    assert ex(None, 1, (ctypes.c_int * 1)(1), s.ctypes.data_as(dp), ll(0), ll(4), r.ctypes.data_as(dp), ll(0),
              ll(4)) == 1
    assert Failing.aborted == 2
    c.close()


def _abort_main(rank, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    import time
    import mmadmm_amd as mx
    tr = mx.TorchDistTransport()
    if rank == 1:
        time.sleep(1.0)
        tr.abort()  # what Comm.host does when this rank's transfer failed
        out[rank] = True
        return
    try:
        tr.allgather(np.ones(3), np.zeros(6))
        out[rank] = False
    except Exception:  # noqa: BLE001 -- the peer's abort ends the collective with an error
        out[rank] = True
        dist.destroy_process_group()


def test_torch_dist_transport_abort_releases_peers():
    """TorchDistTransport.abort ends the gloo group: a rank blocked in the all-gather with it raises
    (within seconds) instead of hanging until gloo's 30-minute timeout."""
    pytest.importorskip("mmadmm_amd")
    ctx = mp.get_context("spawn")
    out = ctx.Manager().dict()
    procs = [ctx.Process(target=_abort_main, args=(r, 31811, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert out[0] and out[1]
