"""Stage tracing / metrics: stage times accumulate,
roctx ranges are optional, the worker's overhead line and the JSON-lines
metrics stream of a real job."""
import json
import os
import subprocess
import sys

from wormhole_amd.utils import trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stage_accumulates():
    trace.take()
    for _ in range(3):
        with trace.stage("a"):
            pass
    with trace.stage("b"):
        pass
    st = trace.take()
    assert st["a"][1] == 3 and st["b"][1] == 1 and st["a"][0] >= 0
    assert trace.take() == {}
    line = trace.overhead_line({"process": (0.5, 10), "parse": (0.3, 10)}, 1.0, 10)
    assert "done 10 minibatches" in line and "overhead 50.0%" in line


def test_job_metrics_stream(tmp_path):
    os.symlink(os.path.join(ROOT, "learn"), tmp_path / "learn")
    env = dict(os.environ, WH_DEVICE="cpu", WH_METRICS=str(tmp_path / "m{rank}.jsonl"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tracker", "dmlc_local.py"), "-n", "1",
                        "-s", "1", os.path.join(ROOT, "bin", "linear.dmlc"),
                        "learn/linear/guide/demo.conf"], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "minibatches" in r.stderr and "overhead" in r.stderr
    recs = [json.loads(l) for l in open(tmp_path / "m0.jsonl")]
    done = [x for x in recs if x["event"] == "pass_done"]
    assert done and all(x["examples"] > 0 and "process" in x["stages_sec"] for x in done)
