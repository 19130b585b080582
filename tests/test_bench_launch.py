"""bench.py's N-rank launcher (no GPU): `python bench.py --gpus N` outside torch.distributed.run starts
N rank processes itself, before anything touches HIP, and never falls back to fewer ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in
           ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
            "HAKAI_RCCL_SHARED_GPU")}
    env.update(kw)
    return env


def test_dry_run_prints_one_environment_per_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-dry-run"], capture_output=True,
                       text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr
    envs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.strip()]
    assert len(envs) == 8
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and int(ports.pop()) > 0
    for i, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(i)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "8"
        assert e["MASTER_ADDR"] == "127.0.0.1"


def test_launcher_process_never_imports_torch():
    code = ("import sys; sys.argv = ['bench.py', '--gpus', '4', '--launch-dry-run']; sys.path.insert(0, %r)\n"
            "import bench\n"
            "try:\n    bench.main()\nexcept SystemExit as e:\n    assert not e.code, e.code\n"
            "assert 'torch' not in sys.modules, 'the launcher imported torch'\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(), timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout


def test_world_size_mismatch_is_fatal():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], capture_output=True, text=True, timeout=300,
                       env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", LOCAL_WORLD_SIZE="2",
                                MASTER_ADDR="127.0.0.1", MASTER_PORT="29999"))
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_failing_rank_fails_the_launch():
    """On this GPU-less host every rank refuses to run (0 visible GPUs): the launch must fail, not print
    a line from fewer ranks."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=_env(), timeout=300)
    assert r.returncode != 0
    assert "visible GPU" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def _devices_check(idents, shared=None):
    """bench.check_distinct_devices on `len(idents)` ranks (threads) over one in-memory store, each
    rank's GPU identity given; returns the per-rank outcome (None or the SystemExit message)."""
    import threading
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    store = dist.HashStore()
    out = [None] * len(idents)
    orig = bench.device_identity
    bench.device_identity = lambda d: idents[d]
    old = os.environ.pop("HAKAI_RCCL_SHARED_GPU", None)
    if shared:
        os.environ["HAKAI_RCCL_SHARED_GPU"] = "1"
    try:
        def rank(r):
            try:
                bench.check_distinct_devices(store, r, len(idents), r)
            except SystemExit as e:
                out[r] = str(e)
        ts = [threading.Thread(target=rank, args=(r,)) for r in range(len(idents))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
    finally:
        bench.device_identity = orig
        os.environ.pop("HAKAI_RCCL_SHARED_GPU", None)
        if old is not None:
            os.environ["HAKAI_RCCL_SHARED_GPU"] = old
    return out


def test_ranks_on_one_gpu_stop_at_the_guard():
    """one global HIP_VISIBLE_DEVICES=0 with --gpus 2 maps both ranks to the same GPU; the
    guard compares the ranks' PCI identities after the rendezvous and stops both with a clear message
    (per-rank masks that give each rank its own GPU pass; HAKAI_RCCL_SHARED_GPU=1 declares sharing)."""
    assert _devices_check(["0000:05:00 a", "0000:15:00 b", "0000:25:00 c"]) == [None, None, None]
    out = _devices_check(["0000:05:00 a", "0000:05:00 a"])
    assert all(o and "same GPU" in o for o in out)
    assert _devices_check(["0000:05:00 a", "0000:05:00 a"], shared=True) == [None, None]
