"""bench.py's --gpus N contract: N ranks or a non-zero exit, decided before
anything touches the GPU.  The reference's only parallelism knob is its thread count
(/root/reference/main.cpp:788-799 -> src/Mesh.cpp:436-438); here it is N ranks, one per GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def never():
    raise AssertionError("device count queried when it does not matter")


def test_single_gpu_default():
    assert bench.launch_plan(None, {}, never) == ("run", 1)
    assert bench.launch_plan(1, {}, never) == ("run", 1)


def test_spawn_when_no_launcher():
    assert bench.launch_plan(8, {}, lambda: 8) == ("spawn", 8)
    assert bench.launch_plan(2, {}, lambda: 8) == ("spawn", 2)


def test_too_few_gpus_is_an_error():
    plan, msg = bench.launch_plan(2, {}, lambda: 1)
    assert plan == "error" and "only 1 GPU" in msg and "device 1 is missing" in msg
    plan, msg = bench.launch_plan(8, {}, lambda: 0)
    assert plan == "error"


def test_under_launcher():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_plan(8, env, lambda: 8) == ("run", 8)
    assert bench.launch_plan(None, env, lambda: 8) == ("run", 8)
    assert bench.launch_plan(4, env, lambda: 8)[0] == "error"  # --gpus disagrees with the launcher
    assert bench.launch_plan(8, env, lambda: 4)[0] == "error"  # fewer devices than ranks
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, never) == ("run", 1)


def test_parallelism_label():
    assert bench.parallelism_label(1) == "single"
    assert bench.parallelism_label(8).startswith("element-partition x8")


def test_relaunch_command(monkeypatch):
    seen = {}

    def fake_run(cmd, **kw):
        seen["cmd"] = cmd
        return subprocess.CompletedProcess(cmd, 0)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "5"])
    assert bench.relaunch(8) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-3:] == ["--gpus", "8", "--steps", "5"][-3:]


def test_no_gpu_here_exits_nonzero():
    """here (no GPU) a 2-GPU bench must exit non-zero and print no result line"""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present (the -m gpu test covers the one-GPU box)")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "only 0 GPU" in r.stderr and r.stdout.strip() == ""


@pytest.mark.gpu
def test_one_gpu_box_refuses_two_ranks():
    import torch
    n = torch.cuda.device_count()
    if n >= 2:
        pytest.skip("%d GPUs visible" % n)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 2, r.stderr[-2000:]
    assert ("only %d GPU" % n) in r.stderr and ("device %d is missing" % n) in r.stderr
    assert r.stdout.strip() == ""


def test_host_comm_may_share_gpus():
    assert bench.launch_plan(2, {}, never, share=True) == ("spawn", 2)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, never, share=True) == ("run", 4)
    assert "gloo" in bench.parallelism_label(2, "host")


@pytest.mark.gpu
def test_bench_two_ranks_host_transport_rehearsal():
    """bench.py's N-rank path end to end on a one-GPU box: `--gpus 2 --comm host` re-launches itself
    under torch.distributed.run, builds the element-partitioned engine on both ranks (sharing the
    GPU; halo exchange over a gloo host transport), times the steps with the barrier and the max
    over ranks, and prints one line from rank 0 with both ranks' shares.  Only the transport differs
    from the RCCL measurement (covered at one rank in tests/test_gpu_partition.py)."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "host", "--steps", "3",
                        "--warmup", "1", "--disc-n", "120", "--no-cpu-baseline"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["ranks"] == 2 and d["n_gpus"] >= 1 and d["steps"] == 3
    cfg = d["config"]
    assert cfg["parallelism"].startswith("element-partition x2") and cfg["comm"] == "host"
    assert cfg["comm_nranks"] == 2 and cfg["rccl_nranks"] is None and len(cfg["nodes_per_rank"]) == 2
    assert sum(cfg["simplices_per_rank"]) == cfg["global_simplices"]
    # the halo exchange per rank (round 6): device time per ADMM iteration, bytes, overlap, balance
    assert len(cfg["exchange_us_per_iter"]) == 2 and all(v and v > 0 for v in cfg["exchange_us_per_iter"])
    assert all(h["send"] > 0 and h["recv"] > 0 for h in cfg["halo_bytes_per_iter"])
    assert cfg["halo_overlap"] is True and 1.0 <= cfg["imbalance"] < 1.01
    assert d["value"] > 0 and d["early_exit"]["admm_iters_per_step"] > 0


def _env_no_launcher(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MMX_BENCH_PROGRESS",
                                                            "MMX_BENCH_TEST_STALL_RANK")}
    env.update(extra)
    return env


def test_rendezvous_two_ranks():
    """--gpus 2 --rendezvous-only: the re-launch, both ranks' phase lines and the gloo rendezvous, no GPU"""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rendezvous-only",
                        "--budget-s", "120"], capture_output=True, text=True, timeout=400, env=_env_no_launcher())
    assert r.returncode == 0, r.stderr[-3000:]
    for rk in (0, 1):
        for ph in ("start", "rendezvous", "setup", "done"):
            assert "rank %d/2: phase %s" % (rk, ph) in r.stderr, r.stderr[-3000:]


def test_stalled_rank_fails_within_budget_and_is_named():
    """one of two ranks never joins the rendezvous.  The job must end non-zero
    within its budget (each rank's watchdog, and the parent's process-group kill behind it) and name
    the rank that never got there -- a driver time-out with no diagnosis is the failure this prevents."""
    import time
    budget = 20
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rendezvous-only",
                        "--budget-s", str(budget)], capture_output=True, text=True, timeout=budget + 240,
                       env=_env_no_launcher(MMX_BENCH_TEST_STALL_RANK="1"))
    el = time.time() - t0
    assert r.returncode != 0, r.stderr[-3000:]
    assert el < budget + 90, el  # the watchdogs fire at the budget; the parent's kill is at budget + 60
    assert "ranks that never reached the rendezvous: 1" in r.stderr, r.stderr[-3000:]
    assert "rank 1: last phase start" in r.stderr
    assert "exceeded in phase" in r.stderr  # a watchdog's message
    assert r.stdout.strip() == ""


def test_relaunch_kills_group_after_budget(monkeypatch, tmp_path):
    """the parent's own budget: a launcher that outlives budget + 60 s is killed as a process group
    and the call returns 124 (here with a fake launcher and the grace shortened)"""
    import time
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    real_popen = subprocess.Popen

    def fake_popen(cmd, **kw):  # a 'launcher' that sleeps, with a child of its own in the group
        return real_popen([sys.executable, "-c", "import subprocess,sys,time; "
                           "subprocess.Popen([sys.executable,'-c','import time; time.sleep(600)']); time.sleep(600)"],
                          **kw)

    monkeypatch.setattr(subprocess, "Popen", fake_popen)
    t0 = time.time()
    rc = bench.relaunch(2, budget_s=-58.0)  # kill after 2 s
    assert rc == 124
    assert time.time() - t0 < 60
