"""BSP (rabit-style) apps on CPU through tracker/dmlc_local.py: L-BFGS linear
and FM, checkpoint-restart after an injected rank failure, and the solver's
numerics against a plain PyTorch reference of the reference objective."""
import os
import re
import struct
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACKER = os.path.join(ROOT, "tracker", "dmlc_local.py")
TRAIN = os.path.join(ROOT, "learn", "data", "agaricus.txt.train")
TEST = os.path.join(ROOT, "learn", "data", "agaricus.txt.test")


def run(args, cwd, env_extra=None, timeout=300):
    env = dict(os.environ, WH_DEVICE="cpu")
    env.update(env_extra or {})
    return subprocess.run([sys.executable, TRACKER] + args, cwd=cwd, env=env,
                          capture_output=True, text=True, timeout=timeout)


def objvals(out):
    return [float(x) for x in re.findall(r"new_objval=([-\d.e+]+)", out)]


def test_lbfgs_ranks_agree_and_predict(tmp_path):
    r1 = run(["-n", "1", os.path.join(ROOT, "bin", "lbfgs.dmlc"), TRAIN, "reg_L1=1",
              "max_lbfgs_iter=15", "model_out=m1"], tmp_path)
    r2 = run(["-n", "2", os.path.join(ROOT, "bin", "lbfgs.dmlc"), TRAIN, "reg_L1=1",
              "max_lbfgs_iter=15", "model_out=m2"], tmp_path)
    assert r1.returncode == 0 and r2.returncode == 0, r2.stderr[-2000:]
    o1, o2 = objvals(r1.stdout), objvals(r2.stdout)
    assert len(o1) == len(o2) >= 10
    for a, b in zip(o1, o2):
        assert abs(a - b) <= 1e-3 * abs(a) + 1e-3
    assert o1[-1] < o1[0]
    raw = open(tmp_path / "m2", "rb").read()
    assert raw[:4] == b"binf" and len(raw) == 4 + 88 + 4 * 127
    bs, nf, lt = struct.unpack_from("<f4xQi", raw, 4)
    assert nf == 126 and lt == 1 and abs(bs) < 1e-6  # logit(0.5) == 0
    r3 = run(["-n", "1", os.path.join(ROOT, "bin", "lbfgs.dmlc"), TEST, "task=pred",
              "model_in=m2", "name_pred=p.txt"], tmp_path)
    assert r3.returncode == 0, r3.stderr[-2000:]
    preds = [float(x) for x in open(tmp_path / "p.txt")]
    labels = [float(l.split()[0]) for l in open(TEST)]
    acc = sum((p > 0.5) == (y > 0.5) for p, y in zip(preds, labels)) / len(labels)
    assert len(preds) == 1611 and acc > 0.95


def test_lbfgs_restart_from_checkpoint_matches(tmp_path):
    base = [os.path.join(ROOT, "bin", "lbfgs.dmlc"), TRAIN, "reg_L1=1", "max_lbfgs_iter=8"]
    ref = run(["-n", "2"] + base, tmp_path, {"WH_CKPT_DIR": str(tmp_path / "ck0")})
    rr = run(["-n", "2", "--max-restart", "1"] + base, tmp_path,
             {"WH_CKPT_DIR": str(tmp_path / "ck1"), "WH_FAULT": "die:1:4"})
    assert ref.returncode == 0 and rr.returncode == 0, rr.stderr[-2000:]
    assert "restart from version=4" in rr.stdout
    assert "WH_FAULT" in rr.stderr
    a, b = objvals(ref.stdout), objvals(rr.stdout)
    assert abs(a[-1] - b[-1]) <= 1e-4 * abs(a[-1])


def test_fm_lbfgs_trains(tmp_path):
    r = run(["-n", "2", os.path.join(ROOT, "bin", "fm.dmlc"), TRAIN, "nfactor=4",
             "max_lbfgs_iter=12", "reg_L2=1", "model_out=fm.model"], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    o = objvals(r.stdout)
    assert o[-1] < 0.5 * o[0]
    size = os.path.getsize(tmp_path / "fm.model")
    assert size == 4 + 88 + 4 * (126 * 5 + 1)


def test_fm_objective_gradient_matches_autograd():
    """FM objective + gradient (fused FM kernels' CPU path) against autograd
    on the reference formula (learn/lbfgs-fm/fm.h:84-107)."""
    from wormhole_amd import _native
    from wormhole_amd.models.lbfgs_models import FMObjective, _SplitData, margin_to_loss
    from wormhole_amd.parallel.bsp import BSP
    keys, off, val, lab, _ = _native.host().load_split(TRAIN, 0, 8, "libsvm")
    bsp = BSP(torch.device("cpu"))
    obj = FMObjective(bsp, _SplitData(keys, off, val, lab, torch.device("cpu")), torch.device("cpu"))
    obj.set_param("nfactor", "3")
    obj.set_param("reg_L2", "0.5")
    obj.set_param("reg_L2_V", "0.25")
    n = obj.init_num_dim()
    w = obj.init_model(n) * 10
    F, k = obj.param.num_feature, 3
    wt = w.clone().double().requires_grad_(True)
    rows = torch.repeat_interleave(torch.arange(off.numel() - 1), off[1:] - off[:-1])
    X = torch.zeros(off.numel() - 1, F, dtype=torch.float64)
    X[rows, keys] = 1.0
    V = wt[F:F * (k + 1)].view(F, k)
    py = obj.param.base_score + wt[-1] + X @ wt[:F] + 0.5 * ((X @ V) ** 2 - (X * X) @ (V * V)).sum(1)
    loss = margin_to_loss(1, lab.double(), py).sum() + 0.25 * (wt[:F] ** 2).sum() + \
        0.125 * (wt[F:F * (k + 1)] ** 2).sum()
    loss.backward()
    assert abs(obj.eval(w) - float(loss)) < 1e-3 * float(loss)
    g = obj.calc_grad(w)
    assert torch.allclose(g.double(), wt.grad, atol=1e-3, rtol=1e-3)


def test_kmeans_app_and_restart(tmp_path):
    base = [os.path.join(ROOT, "bin", "kmeans.dmlc"), TRAIN, "4", "6"]
    r = run(["-n", "2"] + base + ["km.txt"], tmp_path, {"WH_CKPT_DIR": str(tmp_path / "c0")})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Finish 5-th iteration" in r.stdout
    rows = [list(map(float, l.split())) for l in open(tmp_path / "km.txt")]
    assert len(rows) == 4 and all(len(x) == 126 for x in rows)  # feature ids 0..125
    for x in rows:  # centroids are L2-normalised
        assert abs(sum(v * v for v in x) - 1.0) < 1e-4
    r2 = run(["-n", "2", "--max-restart", "1"] + base + ["km2.txt"], tmp_path,
             {"WH_CKPT_DIR": str(tmp_path / "c1"), "WH_FAULT": "die:0:3"})
    assert r2.returncode == 0, r2.stderr[-2000:]
    rows2 = [list(map(float, l.split())) for l in open(tmp_path / "km2.txt")]
    for a, b in zip(rows, rows2):
        assert max(abs(x - y) for x, y in zip(a, b)) < 1e-4


def test_kmeans_converges_on_separated_clusters():
    from wormhole_amd.models.kmeans import KMeans
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(0)
    centers = torch.nn.functional.normalize(torch.randn(5, 16, generator=g), dim=1) * 10
    lab = torch.randint(0, 5, (2000,), generator=g)
    X = centers[lab] + 0.1 * torch.randn(2000, 16, generator=g)
    km = KMeans(BSP(torch.device("cpu")), X, 5)
    km.init_centroids(3)
    objs = []
    for _ in range(10):
        km.step()
        objs.append(km.objective())
    # spherical k-means never decreases the mean cosine similarity
    assert all(b >= a - 1e-6 for a, b in zip(objs, objs[1:]))
    assert objs[-1] > 0.85
    # seeding one centroid per true cluster recovers them exactly
    km.C = torch.nn.functional.normalize(centers, dim=1) + 0.01
    for _ in range(3):
        km.step()
    assert km.objective() > 0.99


def _sparse_rows(n, F, k, nnz, seed):
    g = torch.Generator().manual_seed(seed)
    lab = torch.randint(0, k, (n, 1), generator=g)
    pick = torch.rand(n, 40, generator=g).argsort(1)[:, :nnz]  # distinct columns per row
    cols = (lab * (F // k) + pick) % F
    cols = torch.sort(cols, 1).values.reshape(-1)
    off = torch.arange(0, n * nnz + 1, nnz, dtype=torch.int64)
    val = torch.rand(n * nnz, generator=g) + 0.5
    return cols, off, val


def test_kmeans_csr_matches_dense_path():
    """Sparse rows (KMeansCSR: never densified) follow the dense path's
    iterations exactly on the CPU: same assignments, same centroids."""
    from wormhole_amd.models.kmeans import KMeans, KMeansCSR, densify
    from wormhole_amd.parallel.bsp import BSP
    bsp = BSP(torch.device("cpu"))
    cols, off, val = _sparse_rows(600, 500, 6, 7, 1)
    kd = KMeans(bsp, densify(cols, off, val, 600, 500, "cpu"), 6)
    ks = KMeansCSR(bsp, cols, off, val, 500, 6, "cpu")
    kd.init_centroids(2)
    ks.init_centroids(2)
    assert torch.equal(kd.C, ks.C)
    for _ in range(4):
        a, b = kd.step(), ks.step()
        assert torch.equal(a, b)
        assert torch.allclose(kd.C, ks.C, atol=1e-6)
    assert abs(kd.objective() - ks.objective()) < 1e-6


def test_kmeans_input_form_choice(monkeypatch):
    from wormhole_amd.models.kmeans import use_sparse
    assert not use_sparse(6513, 126, 6513 * 22)          # agaricus: dense
    assert use_sparse(1_000_000, 1_000_000, 32_000_000)  # wide and sparse
    assert use_sparse(10_000_000, 1000, 10_000_000_000 // 2)  # dense split > 4 GiB
    monkeypatch.setenv("WH_KMEANS_INPUT", "sparse")
    assert use_sparse(6513, 126, 6513 * 22)


def test_kmeans_app_sparse_input_matches_dense(tmp_path):
    """bin/kmeans.dmlc on 2 ranks with the CSR form forced gives the dense
    form's centroids."""
    base = [os.path.join(ROOT, "bin", "kmeans.dmlc"), TRAIN, "4", "4"]
    r1 = run(["-n", "2"] + base + ["d.txt"], tmp_path, {"WH_KMEANS_INPUT": "dense"})
    r2 = run(["-n", "2"] + base + ["s.txt"], tmp_path, {"WH_KMEANS_INPUT": "sparse"})
    assert r1.returncode == 0 and r2.returncode == 0, r2.stderr[-2000:]
    d = [list(map(float, l.split())) for l in open(tmp_path / "d.txt")]
    s = [list(map(float, l.split())) for l in open(tmp_path / "s.txt")]
    assert len(d) == len(s) == 4
    for a, b in zip(d, s):
        assert max(abs(x - y) for x, y in zip(a, b)) < 1e-5
