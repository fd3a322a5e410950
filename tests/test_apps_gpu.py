"""End-to-end apps on the GPU (single process, HIP kernels): the PS learners
(demo confs), L-BFGS linear/FM, k-means; results must match the CPU path."""
import math
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
def test_ps_demo_gpu_matches_cpu(work, capfd, monkeypatch, app, conf):
    # (capfd: the native scheduler prints the table on the process's fd 1)
    from wormhole_amd.apps.ps_app import main
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main(app, [conf, "rand_shuffle=0"]) == 0
    gpu = capfd.readouterr().out
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main(app, [conf, "rand_shuffle=0"]) == 0
    cpu = capfd.readouterr().out
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


def test_gbdt_kernels_match_cpu():
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(1)
    n, f = 20000, 40
    X = torch.randn(n, f, generator=g)
    X[torch.rand(n, f, generator=g) < 0.1] = float("nan")
    X[:, 3] = torch.randint(0, 3, (n,), generator=g).float()  # few distinct values
    y = (torch.nan_to_num(X[:, 0]) + torch.nan_to_num(X[:, 5]) > 0).float()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.max_depth = 6
    p.objective = "binary:logistic"
    dmc = G.DMatrix.from_dense(X, y, torch.device("cpu"))
    dmg = G.DMatrix.from_dense(X, y, torch.device("cuda", 0))
    cuts = G.Cuts.build(dmc, 64, bsp)
    Bc, Bg = cuts.bin(dmc), cuts.bin(dmg)
    assert torch.equal(Bc, Bg.cpu())
    obj = G.Objective("binary:logistic")
    trees = []
    for dm, B in ((dmc, Bc), (dmg, Bg)):
        margin = torch.zeros(n, device=dm.device)
        tb = G.TreeBuilder(p, bsp, dm, cuts, B)
        out = []
        for _ in range(3):
            t = tb.build(obj.gpair(margin, dm.label, None), margin)
            out.append(t)
        trees.append((out, margin.cpu()))
    # fp32 LDS histograms vs the fp64 CPU oracle. Deep nodes hold a handful of
    # rows, where several candidate splits can have mathematically equal gain;
    # fp32 rounding may break such a tie differently. So: the first nodes must
    # agree exactly and the boosted margins must give the same training loss.
    top = 7  # the first nodes created (root and its first levels)
    for tc, tg in zip(trees[0][0], trees[1][0]):
        assert tc.feat[:top] == tg.feat[:top] and tc.cond[:top] == tg.cond[:top]

    def logloss(m):
        return float(torch.nn.functional.binary_cross_entropy_with_logits(m, y))
    lc, lg = logloss(trees[0][1]), logloss(trees[1][1])
    assert abs(lc - lg) < 1e-3 * lc, (lc, lg)


@pytest.mark.parametrize("w32", [False, True])
@pytest.mark.parametrize("f,nbin", [(40, 255), (40, 16), (13, 200)])
def test_gbdt_hist_kernel(f, nbin, w32):
    """Per-segment histograms (dword-row and byte-row paths, one and several
    feature groups, several row chunks per segment) vs an fp64 index_add;
    w32: int32 LDS passes of <= 4096 rows (three per chunk) over rows rounded
    to the given scale: exact sums of the rounded values."""
    from wormhole_amd import _native
    g = torch.Generator().manual_seed(f + nbin)
    n = 300000
    B = torch.randint(0, nbin, (n, f), generator=g, dtype=torch.uint8)
    B[torch.rand(n, f, generator=g) < 0.05] = 255
    gp = torch.randn(n, 2, generator=g)
    ridx = torch.randperm(n, generator=g).to(torch.int32)
    segs = [(0, 170000), (170000, 170000), (170000, 299000)]
    fg = min(64, (160 * 1024) // (nbin * 16))
    fg -= fg % 4
    groups = [(j, min(fg, f - j)) for j in range(0, f, fg)]
    chunk = 4096 * 3
    tasks, red = [], []
    for s, (b, e) in enumerate(segs):
        if e <= b:
            continue
        t0, nch = len(tasks), 0
        for r in range(b, e, chunk):
            nch += 1
            for fb, fc in groups:
                tasks.append((s, fb, fc, r, min(e, r + chunk)))
        for k, (fb, fc) in enumerate(groups):
            red.append((s, fb, fc, t0 + k, nch, len(groups)))
    dev = torch.device("cuda", 0)
    hist = torch.zeros(len(segs), f, nbin, 2, dtype=torch.float64, device=dev)
    qscale = torch.tensor([2.0 ** 30, 2.0 ** 31], device=dev)
    if w32:
        R = 4096
        sc = [2.0 ** math.floor(math.log2(2 ** 30 / (R * float(gp[:, c].abs().max()))))
              for c in range(2)]
        qscale = torch.tensor(sc + [float(R)], device=dev)
        gp = torch.stack([torch.round(gp[:, c] * sc[c]) / sc[c] for c in range(2)], 1)
    _native.hip().gbdt_hist(B.to(dev), nbin, ridx.to(dev), gp.to(dev), qscale,
                            torch.tensor(tasks, dtype=torch.int32, device=dev),
                            torch.tensor(red, dtype=torch.int32, device=dev),
                            max(c for _, c in groups), hist)
    for s, (b, e) in enumerate(segs):
        ref = torch.zeros(f * nbin, 2, dtype=torch.float64)
        rows = ridx[b:e].long()
        bins = B[rows].long()
        ok = bins != 255
        flat = (torch.arange(f)[None, :] * nbin + bins.clamp(max=nbin - 1))[ok]
        for c in range(2):
            ref[:, c].index_add_(0, flat, gp[rows, c].double()[:, None].expand(-1, f)[ok])
        # int64 fixed point: exact up to the 2^-30 rounding of each gradient
        # (w32: gp is pre-rounded to the scale, so the sums are exact)
        torch.testing.assert_close(hist[s].cpu().view(-1, 2), ref, rtol=1e-9, atol=1e-6)


def test_xgboost_app_gpu(work, capsys, monkeypatch):
    from wormhole_amd.apps.xgboost_app import main
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main(["learn/xgboost/mushroom.conf", "num_round=3", "model_out=g.model"]) == 0
    gpu = [l for l in capsys.readouterr().out.splitlines() if l.startswith("[")]
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main(["learn/xgboost/mushroom.conf", "num_round=3", "model_out=c.model"]) == 0
    cpu = [l for l in capsys.readouterr().out.splitlines() if l.startswith("[")]
    assert gpu == cpu and len(gpu) == 3


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


@pytest.mark.parametrize("gamma,colsample,hist", [(0.0, 1.0, "32"), (2.0, 0.6, "32"),
                                                  (0.0, 1.0, "64")])
def test_gbdt_native_grower_matches_python_loop(gamma, colsample, hist, monkeypatch):
    """The C++ level loop (one sync per level, device child segments, fused
    sibling subtraction) grows the same trees as the Python level loop on the
    same GPU kernels (fixed-point histograms: exact), including gamma pruning
    (leaf values looked up before the BFS renumbering) and colsample.  The
    two loops cut rows into different chunks; both histogram precisions must
    give bit-identical sums for any chunking."""
    from wormhole_amd.models import gbdt as G
    monkeypatch.setattr(G, "HIST32", hist == "32")
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(2)
    n, f = 60000, 24
    X = torch.randn(n, f, generator=g)
    X[torch.rand(n, f, generator=g) < 0.05] = float("nan")
    y = (torch.nan_to_num(X[:, 0]) * torch.nan_to_num(X[:, 1]) + X[:, 2].abs() > 0.7).float()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.max_depth, p.objective, p.gamma, p.colsample_bytree = 7, "binary:logistic", gamma, colsample
    dev = torch.device("cuda", 0)
    dm = G.DMatrix.from_dense(X, y, dev)
    cuts = G.Cuts.build(dm, 128, bsp)
    B = cuts.bin(dm)
    obj = G.Objective(p.objective)
    res = []
    for native in (True, False):
        margin = torch.zeros(n, device=dev)
        tb = G.TreeBuilder(p, bsp, dm, cuts, B)
        gen = torch.Generator().manual_seed(5)
        trees = []
        for _ in range(3):
            tb.sample_features(gen)
            gp = obj.gpair(margin, dm.label, None)
            trees.append(tb._build_native(gp, margin) if native else tb._build_py(gp, margin))
        res.append((trees, margin.cpu()))
    for a, b in zip(res[0][0], res[1][0]):
        assert a.feat == b.feat and a.cond == b.cond and a.defl == b.defl
        assert a.left == b.left and a.right == b.right
        assert all(abs(x - z) < 1e-6 for x, z in zip(a.leaf, b.leaf))
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6)


@pytest.mark.parametrize("gamma,colsample,depth", [(0.0, 1.0, 6), (2.0, 0.6, 8)])
def test_gbdt_device_level_loop_matches_host_grower(gamma, colsample, depth, monkeypatch):
    """The level loop on the device (heap-numbered nodes, device split
    bookkeeping, device-built histogram tasks, one host read per tree) grows
    the same trees and margins as the per-level host grower."""
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(3)
    n, f = 50000, 20
    X = torch.randn(n, f, generator=g)
    X[torch.rand(n, f, generator=g) < 0.05] = float("nan")
    y = (torch.nan_to_num(X[:, 0]) * torch.nan_to_num(X[:, 1]) + X[:, 2].abs() > 0.7).float()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.max_depth, p.objective, p.gamma, p.colsample_bytree = depth, "binary:logistic", gamma, colsample
    dev = torch.device("cuda", 0)
    dm = G.DMatrix.from_dense(X, y, dev)
    cuts = G.Cuts.build(dm, 64, bsp)
    B = cuts.bin(dm)
    obj = G.Objective(p.objective)
    res = []
    for grower in ("dev", "host"):  # (the builder calls the device loop by default)
        monkeypatch.setattr(G, "HOST_GROWER", grower == "host")
        margin = torch.zeros(n, device=dev)
        tb = G.TreeBuilder(p, bsp, dm, cuts, B)
        gen = torch.Generator().manual_seed(5)
        trees = []
        for _ in range(3):
            tb.sample_features(gen)
            trees.append(tb._build_native(obj.gpair(margin, dm.label, None), margin))
        res.append((trees, margin.cpu()))
    assert sum(len(t.feat) for t in res[0][0]) > 3 * 7  # real trees, not stumps
    for a, b in zip(res[0][0], res[1][0]):
        assert a.feat == b.feat and a.cond == b.cond and a.defl == b.defl
        assert a.left == b.left and a.right == b.right
        assert all(abs(x - z) < 1e-9 for x, z in zip(a.leaf, b.leaf))
        assert all(abs(x - z) < 1e-6 * max(1.0, abs(z)) for x, z in zip(a.gain, b.gain))
    assert torch.equal(res[0][1], res[1][1])


def test_gbdt_csr_gpu_matches_dense_and_trains_wide_data():
    """CSR kernels (global-bin histograms, compact split search, CSR
    partition and tree walk) grow the dense path's trees on agaricus, and a
    libsvm-shaped matrix with a 1M-feature space trains without densifying
    (a dense float matrix of it would be 80 GB)."""
    from wormhole_amd import _native
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    dev = torch.device("cuda", 0)
    host = _native.host()
    keys, off, val, lab, _ = host.load_split(os.path.join(ROOT, "learn", "data",
                                                          "agaricus.txt.train"), 0, 1, "libsvm")
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.objective, p.max_depth, p.eta = "binary:logistic", 4, 0.5
    ncol = int(keys.max()) + 1
    obj = G.Objective(p.objective)
    res = []
    for sparse in (False, True):
        dm = G.make_dmatrix(keys, off, val, lab, None, ncol, dev, sparse=sparse)
        margin = torch.zeros(dm.n, device=dev)
        cuts = G.Cuts.build(dm, 64, bsp, hess=obj.gpair(margin, dm.label, None)[:, 1])
        tb = G.make_builder(p, bsp, dm, cuts, cuts.bin(dm))
        res.append(([tb.build(obj.gpair(margin, dm.label, None), margin) for _ in range(3)],
                    margin.cpu()))
    for a, b in zip(res[0][0], res[1][0]):
        assert a.feat == b.feat and a.cond == b.cond and a.defl == b.defl
    assert torch.allclose(res[0][1], res[1][1], atol=1e-6)
    # wide: 20k rows x 1M-feature space, ~40 stored values per row
    g = torch.Generator().manual_seed(3)
    n, F, per = 20000, 1_000_000, 40
    k = torch.randint(0, F, (n, per), generator=g)
    k[:, 0] = torch.randint(0, 50, (n,), generator=g)  # a few dense-ish informative ids
    k = torch.sort(k, 1).values
    y = ((k[:, 0] % 2) == 0).float()
    offs = torch.arange(n + 1, dtype=torch.int64) * per
    dm = G.make_dmatrix(k.reshape(-1), offs, None, y, None, F, dev)
    assert getattr(dm, "sparse", False)
    margin = torch.zeros(n, device=dev)
    cuts = G.Cuts.build(dm, 64, bsp)
    tb = G.make_builder(p, bsp, dm, cuts, cuts.bin(dm))
    err0 = G.eval_metric("error", torch.sigmoid(margin), dm.label, None, bsp)
    for _ in range(3):
        tb.build(obj.gpair(margin, dm.label, None), margin)
    err = G.eval_metric("error", torch.sigmoid(margin), dm.label, None, bsp)
    assert err < 0.5 * err0, (err0, err)


@pytest.mark.parametrize("algo", [1, 2, 3])
def test_native_linear_step_matches_python_step(algo):
    """The single-shard linear step as ONE native call (LinearStep) trains
    the same model as the Python-driven sequence of the same kernels, with
    the next minibatch's localize begun early, a table that has to grow, and
    SGD's request-count step size."""
    import torch
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.data.synthetic import criteo_batch
    from wormhole_amd.models.linear import LinearLearner
    from wormhole_amd.parallel.comm import Comm
    dev = torch.device("cuda", 0)
    card = [50, 400, 3000, 20, 7, 900, 100000]
    batches = [criteo_batch(3000, 5, s, dev, card) for s in range(8)]

    def run(native):
        conf = LinearConfig(algo=algo, lambda_l1=0.1, lr_eta=0.1)
        lr = LinearLearner(conf, Comm(dev, init=False), dev, cap=1 << 12, seed=1)
        assert lr._native is not None
        if not native:
            lr._native = None
        for s, (keys, label, off) in enumerate(batches):
            nb = (batches[s + 1][0], batches[s + 1][2], None) if s + 1 < len(batches) else None
            lr.process(keys, off, None, label, 0, 0, next_batch=nb)
        lr.flush()
        prog = lr.take_progress()
        st = lr.store
        occ = st.occupied().long()
        m = dict(zip(st.keys[occ].cpu().tolist(), st.w[occ].cpu().tolist()))
        keys, label, off = criteo_batch(2000, 6, 0, dev, card)  # unseen ids too
        py = lr.process(keys, off, None, label, 2, 0)  # PRED: no insert, no push
        return m, prog, lr, py
    a, pa, la, ya = run(True)
    assert la._native.direct  # the localize-free step is the default
    b, pb, lb, yb = run(False)
    assert torch.allclose(ya, yb, atol=1e-4, rtol=1e-4)
    assert la.kv.guard.grows >= 1  # the 4096-slot table had to grow on both paths
    assert a.keys() == b.keys()
    bad = sum(1 for k, w in b.items() if abs(w - a[k]) > 1e-5 * max(1.0, abs(w)))
    assert bad <= len(b) // 1000, bad
    for x, y in zip(pa, pb):
        assert abs(x - y) <= 1e-4 * max(1.0, abs(y)), (pa, pb)


def test_native_linear_lookahead_made_on_the_compute_stream(monkeypatch):
    """The file worker hands the look-ahead minibatch over without a producer
    event (slices and offset rebasing queued on the compute stream just
    before the step): the next localize must wait for the compute stream.
    Each look-ahead here is produced behind a slow kernel chain, and the
    model must equal the one trained on batches made long before."""
    import torch
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.data.synthetic import criteo_batch
    from wormhole_amd.models.linear import LinearLearner
    from wormhole_amd.parallel.comm import Comm
    from wormhole_amd.models import linear as L
    monkeypatch.setattr(L, "DIRECT_STEP", False)
    dev = torch.device("cuda", 0)
    card = [50, 400, 3000, 20, 7, 900, 100000]
    batches = [criteo_batch(3000, 5, s, dev, card) for s in range(8)]
    torch.cuda.synchronize()
    slow = torch.randn(2048, 2048, device=dev)

    def late(b):  # a copy of b made on the current stream behind ~ms of work
        x = slow
        for _ in range(8):
            x = x @ slow
        keys, label, off = b
        return keys + (x[0, 0] * 0).long(), label, off + (x[0, 1] * 0).long()

    def run(fresh):
        conf = LinearConfig(algo=3, lr_eta=0.1)
        lr = LinearLearner(conf, Comm(dev, init=False), dev, cap=1 << 16, seed=1)
        assert lr._native is not None and not lr._native.direct
        cur = batches[0]
        for s in range(len(batches)):
            nb = None
            if s + 1 < len(batches):
                nxt = late(batches[s + 1]) if fresh else batches[s + 1]
                nb = (nxt[0], nxt[2], None)
            keys, label, off = cur
            lr.process(keys, off, None, label, 0, 0, next_batch=nb)
            if nb is not None:
                cur = (nb[0], nxt[1], nb[1])
        lr.flush()
        st = lr.store
        occ = st.occupied().long()
        return dict(zip(st.keys[occ].cpu().tolist(), st.w[occ].cpu().tolist())), lr.take_progress()
    a, pa = run(True)
    b, pb = run(False)
    assert a.keys() == b.keys()
    assert max(abs(w - a[k]) for k, w in b.items()) <= 1e-6
    assert pa == pytest.approx(pb, rel=1e-6)


@pytest.mark.parametrize("f,walk", [(16, None), (13, None), (16, "global")])
def test_gbdt_leaf_walk_matches_raw_value_predict(f, walk, monkeypatch):
    """The training margins after each tree come from a per-row walk of the
    pruned tree on the bins (k_leaf_walk); predicting the same (compacted)
    trees on the raw values must give the same margins (missing values,
    gamma pruning included). f = 13: the LDS walk's byte tail (rows not a
    multiple of 4 bytes); walk = "global": the global-memory walk kernel."""
    from wormhole_amd.models import gbdt as G
    from wormhole_amd.parallel.bsp import BSP
    if walk:
        monkeypatch.setattr(G, "LEAF_WALK_LDS", False)
    g = torch.Generator().manual_seed(4)
    n = 50000
    X = torch.randn(n, f, generator=g)
    X[torch.rand(n, f, generator=g) < 0.08] = float("nan")
    y = (torch.nan_to_num(X[:, 0]) + torch.nan_to_num(X[:, 3]) * X[:, 5].abs() > 0.2).float()
    bsp = BSP(torch.device("cpu"))
    p = G.GBDTParam()
    p.max_depth, p.objective, p.gamma = 6, "binary:logistic", 1.0
    dev = torch.device("cuda", 0)
    dm = G.DMatrix.from_dense(X, y, dev)
    cuts = G.Cuts.build(dm, 64, bsp)
    tb = G.TreeBuilder(p, bsp, dm, cuts, cuts.bin(dm))
    obj = G.Objective(p.objective)
    margin = torch.zeros(n, device=dev)
    ref = torch.zeros(n, device=dev)
    for _ in range(4):
        tree = tb.build(obj.gpair(margin, dm.label, None), margin)
        dm.predict_tree(tree, ref)
        assert torch.allclose(margin, ref, atol=1e-5), (margin - ref).abs().max()


@pytest.mark.parametrize("r32", [0, 8192])
def test_gbdt_qscale_kernel_matches_torch(r32):
    """k_qscale (one launch) == the torch formula of GBTree._qscale."""
    from wormhole_amd import _native
    for mg, mh, n in [(0.5, 0.25, 11_000_000), (1e-7, 3.0, 1), (0.0, 0.0, 6513), (123.4, 1e-30, 10 ** 9)]:
        m = torch.tensor([mg, mh], dtype=torch.float32, device="cuda")
        got = _native.hip().gbdt_qscale(m, float(n), r32).cpu()
        md = m.double().clamp_min(1e-30)  # (the torch path ran on the device too)
        e = torch.floor(torch.log2(2.0 ** 61 / (n * md)))
        if r32:
            e = torch.minimum(e, torch.floor(torch.log2(2.0 ** 30 / (r32 * md))))
        want = torch.pow(2.0, e.clamp(-60, 100)).float().cpu()
        if r32:
            want = torch.cat([want, torch.tensor([float(r32)])])
        assert torch.equal(got, want), (mg, mh, n, got, want)


def test_kmeans_csr_gpu_matches_cpu():
    """Sparse k-means on the HIP kernels (k_assign_csr over the transposed
    centroids, k_accum_csr) vs the host path: same assignments, centroids."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_bsp_apps import _sparse_rows
    from wormhole_amd.models.kmeans import KMeansCSR
    from wormhole_amd.parallel.bsp import BSP
    cols, off, val = _sparse_rows(5000, 3000, 300, 9, 4)  # K = 300: 2 float4 groups per lane
    kc = KMeansCSR(BSP(torch.device("cpu")), cols, off, val, 3000, 300, "cpu")
    kg = KMeansCSR(BSP(torch.device("cuda", 0)), cols, off, val, 3000, 300, torch.device("cuda", 0))
    kc.init_centroids(5)
    kg.init_centroids(5)
    for _ in range(3):
        a, b = kc.step(), kg.step()
        assert (a != b.cpu()).sum() <= 2  # (double sums in another order: near-ties only)
        kg.C = kc.C.to(kg.C.device)  # continue from the same centroids
    assert abs(kc.objective() - kg.objective()) < 1e-4


def test_kmeans_csr_app_gpu_matches_cpu(work, monkeypatch):
    from wormhole_amd.apps.kmeans_app import main
    monkeypatch.setenv("WH_KMEANS_INPUT", "sparse")
    monkeypatch.setenv("WH_DEVICE", "auto")
    assert main([TRAIN, "6", "5", "g.txt"]) == 0
    monkeypatch.setenv("WH_DEVICE", "cpu")
    assert main([TRAIN, "6", "5", "c.txt"]) == 0
    g = [list(map(float, l.split())) for l in open("g.txt")]
    c = [list(map(float, l.split())) for l in open("c.txt")]
    assert len(g) == len(c) == 6
    for a, b in zip(g, c):
        assert max(abs(x - y) for x, y in zip(a, b)) < 1e-4
