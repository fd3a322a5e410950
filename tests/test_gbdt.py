"""Histogram GBDT (bin/xgboost.dmlc): exact-greedy agreement on binned data,
CLI tasks (train/pred/dump/eval), distributed = single-rank trees,
checkpoint-restart."""
import os
import re
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACKER = os.path.join(ROOT, "tracker", "dmlc_local.py")
XGB = os.path.join(ROOT, "bin", "xgboost.dmlc")


def run(args, cwd, env_extra=None, timeout=300):
    env = dict(os.environ, WH_DEVICE="cpu")
    env.update(env_extra or {})
    return subprocess.run([sys.executable, TRACKER] + args, cwd=cwd, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.fixture()
def work(tmp_path):
    os.symlink(os.path.join(ROOT, "learn"), tmp_path / "learn")
    return tmp_path


def test_mushroom_train_pred_dump(work):
    r = run(["-n", "1", XGB, "learn/xgboost/mushroom.conf", "model_out=m.model"], work)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("[")]
    assert len(lines) == 2 and "test-error" in lines[0] and "train-error" in lines[0]
    errs = [float(x) for x in re.findall(r"test-error:([\d.]+)", r.stdout)]
    assert errs[-1] < 0.05
    r2 = run(["-n", "1", XGB, "learn/xgboost/mushroom.conf", "task=pred", "model_in=m.model",
              "test:data=learn/data/agaricus.txt.test"], work)
    assert r2.returncode == 0, r2.stderr[-2000:]
    preds = [float(x) for x in open(work / "pred.txt")]
    assert len(preds) == 1611 and all(0 <= p <= 1 for p in preds)
    r3 = run(["-n", "1", XGB, "learn/xgboost/mushroom.conf", "task=dump", "model_in=m.model",
              "fmap=learn/data/featmap.txt", "name_dump=dump.nice.txt"], work)
    assert r3.returncode == 0
    dump = open(work / "dump.nice.txt").read()
    assert dump.startswith("booster[0]:\n0:[") and "booster[1]:" in dump
    assert re.search(r"\t\d+:leaf=-?[\d.]+", dump)
    assert "odor=" in dump
    r4 = run(["-n", "1", XGB, "learn/xgboost/mushroom.conf", "task=dump", "model_in=m.model"],
             work)
    raw = open(work / "dump.txt").read()
    assert re.search(r"^0:\[f\d+<[\d.e+-]+\] yes=\d+,no=\d+,missing=\d+$", raw, re.M)


def test_distributed_trees_equal_single_rank(work):
    r1 = run(["-n", "1", XGB, "learn/xgboost/mushroom.conf", "num_round=4", "max_depth=4",
              "eta=0.5", "model_out=a.model"], work)
    r2 = run(["-n", "3", XGB, "learn/xgboost/mushroom.conf", "num_round=4", "max_depth=4",
              "eta=0.5", "model_out=b.model"], work)
    assert r1.returncode == 0 and r2.returncode == 0, r2.stderr[-2000:]
    from wormhole_amd.models.gbdt import Booster, GBDTParam
    a = Booster.load(str(work / "a.model"), GBDTParam())
    b = Booster.load(str(work / "b.model"), GBDTParam())
    # the sketch differs per split only for >max_bin distinct values: agaricus is exact
    assert a.dump() == b.dump()
    rounds = lambda out: [l for l in out.splitlines() if re.match(r"^\[\d+\]\t", l)]  # noqa
    assert rounds(r1.stdout) == rounds(r2.stdout) and len(rounds(r1.stdout)) == 4


def test_gbdt_restart_from_checkpoint(work):
    args = [XGB, "learn/xgboost/mushroom.conf", "num_round=6", "eta=0.3"]
    ref = run(["-n", "2"] + args + ["model_out=r.model"], work, {"WH_CKPT_DIR": str(work / "c0")})
    rr = run(["-n", "2", "--max-restart", "1"] + args + ["model_out=s.model"], work,
             {"WH_CKPT_DIR": str(work / "c1"), "WH_FAULT": "die:1:3"})
    assert ref.returncode == 0 and rr.returncode == 0, rr.stderr[-2000:]
    from wormhole_amd.models.gbdt import Booster, GBDTParam
    a = Booster.load(str(work / "r.model"), GBDTParam())
    b = Booster.load(str(work / "s.model"), GBDTParam())
    assert a.dump() == b.dump()


def test_split_search_matches_brute_force():
    """Greedy split of the histogram builder == exhaustive search on bins."""
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(0)
    n, f = 600, 5
    X = torch.randn(n, f, generator=g)
    X[torch.rand(n, f, generator=g) < 0.2] = float("nan")
    y = ((X.nan_to_num(0)[:, 0] + 0.5 * X.nan_to_num(0)[:, 1]) > 0).float()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.max_depth = 1
    p.max_bin = 16
    p.eta = 1.0
    dm = G.DMatrix.from_dense(X, y, torch.device("cpu"))
    cuts = G.Cuts.build(dm, p.max_bin, bsp)
    B = cuts.bin(dm)
    obj = G.Objective("binary:logistic")
    gp = obj.gpair(torch.zeros(n), y, None)
    tb = G.TreeBuilder(p, bsp, dm, cuts, B)
    tree = tb.build(gp, torch.zeros(n))
    Gs, Hs = gp[:, 0].double(), gp[:, 1].double()
    best = (-1e30, None)
    o = cuts.offsets.tolist()
    for j in range(f):
        for b in range(o[j + 1] - o[j]):
            for defl in (0, 1):
                bins = B[:, j].long()
                left = torch.where(bins == 255, torch.tensor(bool(defl)), bins <= b)
                GL, HL = Gs[left].sum(), Hs[left].sum()
                GR, HR = Gs[~left].sum(), Hs[~left].sum()
                if HL < 1 or HR < 1:
                    continue
                gain = GL ** 2 / (HL + 1) + GR ** 2 / (HR + 1) - Gs.sum() ** 2 / (Hs.sum() + 1)
                if gain > best[0] + 1e-9:
                    best = (float(gain), (j, b))
    assert tree.feat[0] == best[1][0]
    assert abs(tree.gain[0] - best[0]) < 1e-6 * max(1.0, abs(best[0]))


def test_external_memory_cache_suffix(work):
    """xgboost's "data#name.cache" syntax: the first run writes a binary CRB
    page per rank, the second run loads it and trains the same model."""
    args = ["-n", "2", XGB, "learn/xgboost/mushroom.conf",
            "data=learn/data/agaricus.txt.train#dtrain.cache"]
    r = run(args + ["model_out=a.model"], work)
    assert r.returncode == 0, r.stderr[-2000:]
    pages = sorted(p.name for p in work.iterdir() if p.name.startswith("dtrain.cache"))
    assert pages == ["dtrain.cache.r0of2.crb", "dtrain.cache.r1of2.crb"]
    r2 = run(args + ["model_out=b.model"], work)
    assert r2.returncode == 0, r2.stderr[-2000:]
    assert open(work / "a.model", "rb").read() == open(work / "b.model", "rb").read()


def _agaricus():
    from wormhole_amd import _native
    host = _native.host()
    keys, off, val, lab, wt = host.load_split(os.path.join(ROOT, "learn", "data",
                                                           "agaricus.txt.train"), 0, 1, "libsvm")
    return keys, off, val, lab


def _train(G, bsp, dm, p, rounds, hess_sketch=True):
    obj = G.Objective(p.objective)
    margin = torch.zeros(dm.n, device=dm.device)
    hess = obj.gpair(margin, dm.label, None)[:, 1] if hess_sketch else None
    cuts = G.Cuts.build(dm, p.max_bin, bsp, hess=hess)
    tb = G.make_builder(p, bsp, dm, cuts, cuts.bin(dm))
    trees = [tb.build(obj.gpair(margin, dm.label, None), margin) for _ in range(rounds)]
    return trees, margin


def test_csr_matrix_grows_the_dense_trees():
    """Agaricus kept CSR (dsparse) grows the trees of the dense matrix: absent
    features are missing in both, the sketch and split search agree."""
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    keys, off, val, lab = _agaricus()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.objective, p.max_depth, p.eta = "binary:logistic", 3, 0.5
    ncol = int(keys.max()) + 1
    res = []
    for sparse in (False, True):
        dm = G.make_dmatrix(keys, off, val, lab, None, ncol, torch.device("cpu"), sparse=sparse)
        assert getattr(dm, "sparse", False) == sparse
        res.append(_train(G, bsp, dm, p, 2))
    for a, b in zip(res[0][0], res[1][0]):
        assert a.feat == b.feat and a.cond == b.cond and a.defl == b.defl
        assert all(abs(x - z) < 1e-9 for x, z in zip(a.leaf, b.leaf))
    assert torch.allclose(res[0][1], res[1][1])


def test_weighted_sketch_follows_hessian_mass():
    """Cuts split each feature's HESSIAN weight evenly: rows with 9x the
    weight pull the cuts into their value range."""
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    n = 20000
    x = torch.rand(n, 1)
    dm = G.DMatrix.from_dense(x, torch.zeros(n), torch.device("cpu"))
    bsp = BSP(torch.device("cpu"))
    w = torch.where(x[:, 0] < 0.5, torch.full((n,), 9.0), torch.ones(n))
    cuts = G.Cuts.build(dm, 16, bsp, hess=w)
    c = cuts.values[:-1]
    below = float((c < 0.5).float().mean())
    assert 0.85 < below < 0.95, c  # 90 % of the weight sits below 0.5
    cu = G.Cuts.build(dm, 16, bsp).values[:-1]  # unweighted: even in value
    assert 0.4 < float((cu < 0.5).float().mean()) < 0.6
