"""bench.py --gpus N starts N ranks itself (no torchrun) and fails loudly on a rank mismatch.

--check-ranks runs the launcher, the rank bootstrap and the process group (gloo here) and
prints one line from rank 0; no GPU work, so it runs on the CPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


def test_gpus2_launches_two_ranks():
    r = _run(["--gpus", "2", "--check-ranks"])
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks_joined"] == 2 and line["backend"] == "gloo"


def test_gpus1_single_rank():
    r = _run(["--gpus", "1", "--check-ranks"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_rank_count_mismatch_fails_loudly():
    # a torchrun-style environment of 1 rank while --gpus asks for 2
    r = _run(["--gpus", "2", "--check-ranks"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2 but 1 rank(s)" in (r.stderr + r.stdout)


def test_node_shape_devices(monkeypatch):
    """The node-shape leg's devices (bench.node_devices): every GPU at N > 1; under the one-GPU
    rehearsal (BGV_BENCH_DEVICE) the rehearsal's device once per rank, so `BGV_BENCH_DEVICE=0
    bench.py --gpus 2` runs the leg on devices that exist."""
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.delenv("BGV_BENCH_DEVICE", raising=False)
    assert bench.node_devices(8, 3) == list(range(8))
    assert bench.node_devices(2, 1) == [0, 1]
    assert bench.node_devices(1, 0) == [0, 0]
    monkeypatch.setenv("BGV_BENCH_DEVICE", "0")
    assert bench.node_devices(2, 0) == [0, 0]
    assert bench.node_devices(4, 0) == [0, 0, 0, 0]
    assert bench.node_devices(1, 0) == [0, 0]
