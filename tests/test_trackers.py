"""Launchers other than dmlc_local (ssh / mpi / sge / yarn): dry-run command
construction and the env-rank contract (no cluster here)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TR = os.path.join(ROOT, "tracker")


def _run(script, *args):
    r = subprocess.run([sys.executable, os.path.join(TR, script)] + list(args),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_ssh_plan(tmp_path):
    hf = tmp_path / "hosts"
    hf.write_text("nodeA\nnodeB  # second\n")
    out = _run("dmlc_ssh.py", "-n", "3", "-s", "1", "-H", str(hf), "--gpus-per-host", "2",
               "--host-ip", "10.0.0.1", "--dry-run", "bin/linear.dmlc", "demo.conf")
    lines = out.strip().splitlines()
    assert lines[0].startswith("local: ")
    assert [l.split(":")[0] for l in lines[1:]] == ["nodeA", "nodeA", "nodeB"]
    assert "RANK=2" in lines[3] and "LOCAL_RANK=0" in lines[3] and "MASTER_ADDR=10.0.0.1" in lines[3]


def test_mpi_sge_yarn_dry_run():
    out = _run("dmlc_mpi.py", "-n", "4", "--dry-run", "bin/kmeans.dmlc", "d", "3", "5", "o")
    assert "mpirun -n 4" in out and "-x WORLD_SIZE=4" in out
    out = _run("dmlc_sge.py", "-n", "4", "-q", "gpu.q", "--dry-run", "bin/lbfgs.dmlc", "d")
    assert "#$ -t 1-4" in out and "RANK=$((SGE_TASK_ID - 1))" in out and "#$ -q gpu.q" in out
    out = _run("dmlc_yarn.py", "-n", "2", "--vcores", "2", "--dry-run", "bin/xgboost.dmlc", "c")
    assert "-nworker 2" in out and "-vcores 2" in out


def test_env_rank_contract(monkeypatch):
    from wormhole_amd.parallel import comm
    for v in ("RANK", "DMLC_TASK_ID", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK",
              "SLURM_PROCID", "SGE_TASK_ID", "LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK"):
        monkeypatch.delenv(v, raising=False)
    assert comm.env_rank() == 0
    monkeypatch.setenv("SGE_TASK_ID", "3")
    assert comm.env_rank() == 2
    monkeypatch.setenv("OMPI_COMM_WORLD_RANK", "5")
    monkeypatch.setenv("OMPI_COMM_WORLD_LOCAL_RANK", "1")
    assert comm.env_rank() == 5 and comm.env_local_rank() == 1
