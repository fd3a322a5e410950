"""bench.py launches its own ranks: ``--gpus N`` with no launcher around it
runs N processes (one per GPU; here gloo on CPU) and reports n_gpus = N; a
box with fewer visible GPUs fails fast instead of hanging in RCCL init."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args),
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def _json(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout  # rank 0 only
    return json.loads(lines[0])


def test_self_launch_two_ranks_cpu():
    r = _bench("--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1",
               "--batch", "1500")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2+kvshard2"
    assert d["config"]["global_batch"] == 3000
    assert d["rank_ms_per_step_max"] >= d["rank_ms_per_step_min"] > 0
    w = d["wire_bytes_per_gpu_step"]
    assert w["c1"] > 0 and w["c2"] > 0 and w["c3"] > 0  # keys, pull reply, push crossed


def test_self_launch_linear_two_ranks_cpu():
    r = _bench("--gpus", "2", "--device", "cpu", "--steps", "2", "--warmup", "1",
               "--batch", "1500", "--model", "linear")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json(r.stdout)
    assert d["n_gpus"] == 2 and d["vs_baseline"] is not None


def test_too_few_gpus_fails_fast():
    import torch
    n = torch.cuda.device_count()
    r = _bench("--gpus", str(max(n + 1, 2)), "--steps", "1", "--warmup", "0", timeout=120)
    assert r.returncode == 2
    assert "visible" in r.stderr and "only %d device" % n in r.stderr
