"""End-to-end apps on the GPU (single process, HIP kernels): the PS learners
(demo confs), L-BFGS linear/FM, k-means; results must match the CPU path."""
import os
import re

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRAIN = os.path.join(ROOT, "learn", "data", "agaricus.txt.train")


@pytest.fixture()
def work(tmp_path, monkeypatch):
    os.symlink(os.path.join(ROOT, "learn"), tmp_path / "learn")
    monkeypatch.chdir(tmp_path)
    for k in ("DMLC_ROLE", "RANK", "WORLD_SIZE", "WH_CKPT_DIR", "WH_FAULT"):
        monkeypatch.delenv(k, raising=False)
    return tmp_path


def _val_lines(out):
    return [l for l in out.splitlines() if re.match(r"^\s+\d+\s+1(\.61e\+03|611)\s", l)]


@pytest.mark.parametrize("app,conf", [("linear", "learn/linear/guide/demo.conf"),
                                      ("difacto", "learn/difacto/guide/demo.conf")])
def test_ps_demo_gpu_matches_cpu(work, capsys, monkeypatch, app, conf):
    from wormhole_amd.apps.ps_app import main
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main(app, [conf, "rand_shuffle=0"]) == 0
    gpu = capsys.readouterr().out
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main(app, [conf, "rand_shuffle=0"]) == 0
    cpu = capsys.readouterr().out
    g, c = _val_lines(gpu), _val_lines(cpu)
    assert len(g) == len(c) == 3
    for lg, lc in zip(g, c):
        # logloss / AUC columns agree to a few ulps of the printed precision
        vg = [float(x) for x in re.findall(r"\d+\.\d{5,}", lg)]
        vc = [float(x) for x in re.findall(r"\d+\.\d{5,}", lc)]
        assert vg and all(abs(a - b) < 2e-3 for a, b in zip(vg, vc)), (lg, lc)


def test_lbfgs_gpu(work, capsys, monkeypatch):
    from wormhole_amd.apps.lbfgs_app import main
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main("linear", [TRAIN, "reg_L1=1", "max_lbfgs_iter=10"]) == 0
    gpu = [float(x) for x in re.findall(r"new_objval=([-\d.e+]+)", capsys.readouterr().out)]
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main("linear", [TRAIN, "reg_L1=1", "max_lbfgs_iter=10"]) == 0
    cpu = [float(x) for x in re.findall(r"new_objval=([-\d.e+]+)", capsys.readouterr().out)]
    assert len(gpu) == len(cpu) > 5
    assert abs(gpu[-1] - cpu[-1]) < 1e-3 * cpu[-1]
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main("fm", [TRAIN, "nfactor=8", "max_lbfgs_iter=10", "reg_L2=1"]) == 0
    fm = [float(x) for x in re.findall(r"new_objval=([-\d.e+]+)", capsys.readouterr().out)]
    assert fm[-1] < 0.5 * fm[0]


def test_kmeans_gpu_matches_cpu(work, monkeypatch):
    from wormhole_amd.apps.kmeans_app import main
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main([TRAIN, "6", "5", "g.txt"]) == 0
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main([TRAIN, "6", "5", "c.txt"]) == 0
    g = [list(map(float, l.split())) for l in open("g.txt")]
    c = [list(map(float, l.split())) for l in open("c.txt")]
    assert len(g) == len(c) == 6
    for a, b in zip(g, c):
        assert max(abs(x - y) for x, y in zip(a, b)) < 1e-3
