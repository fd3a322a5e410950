"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references
(wormhole_amd.ops.ref) and the host parameter store (kv.cpu_store)."""
import numpy as np
import pytest
import torch

from wormhole_amd.ops import ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


@pytest.fixture(scope="module")
def hip():
    from wormhole_amd import _native
    return _native.hip()


def _rand_batch(nrows, nnz_per_row, nkeys, seed, with_val=False, skew=True):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, 2 * nnz_per_row, (nrows,), generator=g)
    off = torch.zeros(nrows + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(lens, 0)
    nnz = int(off[-1])
    if skew:
        u = torch.rand(nnz, generator=g)
        ids = (torch.exp(u * np.log(nkeys)) - 1).long()
    else:
        ids = torch.randint(0, nkeys, (nnz,), generator=g)
    keys = ids * 0x9E3779B97F4A7C15 % (1 << 62) + 7
    val = torch.rand(nnz, generator=g) + 0.5 if with_val else None
    label = (torch.rand(nrows, generator=g) < 0.3).float()
    return keys, off, val, label


def test_scan(hip):
    for n in [0, 1, 5, 2047, 2048, 2049, 100000, 3_000_001]:
        x = torch.randint(0, 7, (n,), dtype=torch.int32, device=DEV)
        o = hip.scan_excl(x)
        exp = torch.zeros(n + 1, dtype=torch.int64, device=DEV)
        exp[1:] = torch.cumsum(x.long(), 0)
        assert torch.equal(o, exp), n


@pytest.mark.parametrize("nshard", [1, 3, 8])
@pytest.mark.parametrize("with_val", [False, True])
@pytest.mark.parametrize("hint", [0, 1, 2000])  # 1: table overflows -> safe-size retry
def test_localize(hip, nshard, with_val, hint):
    keys, off, val, _ = _rand_batch(3000, 20, 5000, 1, with_val)
    k, o = keys.to(DEV), off.to(DEV)
    v = val.to(DEV) if val is not None else None
    uniq, ucnt, owner_cnt, lid, csc_off, csc_row, csc_val = hip.localize(k, o, v, nshard, hint)[:7]
    ru = torch.unique(keys)
    assert uniq.numel() == ru.numel()
    assert torch.equal(torch.sort(uniq.cpu()).values, ru)
    # lid maps every non-zero back to its key
    assert torch.equal(uniq[lid.long()].cpu(), keys)
    # counts
    cnt_ref = torch.bincount(lid.long().cpu(), minlength=uniq.numel())
    assert torch.equal(ucnt.cpu().long(), cnt_ref)
    # grouping by owner
    own = ref.owner_of(uniq.cpu(), nshard)
    assert torch.equal(torch.bincount(own, minlength=nshard), owner_cnt)
    assert bool((own[1:] >= own[:-1]).all())
    # CSC: occurrence rows of each key
    rows = torch.repeat_interleave(torch.arange(3000), off[1:] - off[:-1])
    assert torch.equal(csc_off.cpu()[1:] - csc_off.cpu()[:-1], cnt_ref)
    cr = csc_row.cpu().long()
    keyof = torch.repeat_interleave(torch.arange(uniq.numel()), cnt_ref)
    pairs = torch.sort(keyof * 10_000 + cr).values
    pairs_ref = torch.sort(lid.cpu().long() * 10_000 + rows).values
    assert torch.equal(pairs, pairs_ref)
    if with_val:
        # values follow their non-zeros
        got = torch.sort(keyof.double() * 1e4 + cr.double() + csc_val.cpu().double() / 10).values
        exp = torch.sort(lid.cpu().double() * 1e4 + rows.double() + val.double() / 10).values
        assert torch.allclose(got, exp)


def _pulled(U, vstride, dim, seed, frac_v=0.6):
    """A random variable-length pull: hdr {w, vidx} + compact V rows in a
    shuffled (non-monotone) row order, with spare rows past m."""
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(U, generator=g) * 0.3
    flag = torch.rand(U, generator=g) < frac_v
    m = int(flag.sum())
    vidx = torch.full((U,), -1, dtype=torch.int64)
    vidx[flag] = torch.randperm(m, generator=g)
    vc = torch.randn(m + 7, vstride, generator=g) * 0.2
    vc[:, dim:] = 0
    return ref.make_hdr(w, vidx), vc


@pytest.mark.parametrize("dim", [5, 16, 64])
@pytest.mark.parametrize("with_val", [False, True])
def test_fm_forward_backward(hip, dim, with_val):
    vs = ref.vstride_for(dim)
    keys, off, val, label = _rand_batch(2000, 15, 3000, 2, with_val)
    uniq, ucnt, oc, lid, csc_off, csc_row, csc_val = hip.localize(
        keys.to(DEV), off.to(DEV), val.to(DEV) if val is not None else None, 1)[:7]
    U = uniq.numel()
    hdr, vc = _pulled(U, vs, dim, 3)
    met = torch.zeros(4, dtype=torch.float64, device=DEV)
    py, dual, xv = hip.fm_forward(off.to(DEV), lid, val.to(DEV) if val is not None else None,
                                  hdr.to(DEV), vc.to(DEV), vs, label.to(DEV), 2, met)
    met_r = torch.zeros(4, dtype=torch.float64)
    py_r, dual_r, xv_r = ref.fm_forward(off, lid.cpu(), val, hdr, vc, vs, label, 2, met_r)
    assert torch.allclose(py.cpu(), py_r, atol=1e-4, rtol=1e-4)
    assert torch.allclose(dual.cpu(), dual_r, atol=1e-5, rtol=1e-4)
    assert torch.allclose(xv.cpu(), xv_r, atol=1e-4, rtol=1e-4)
    assert torch.allclose(met.cpu(), met_r, rtol=1e-5)
    gw, gvc = hip.fm_backward(csc_off, csc_row, csc_val if with_val else None, dual, xv,
                              hdr.to(DEV), vc.to(DEV), vs)
    gw_r, gvc_r = ref.fm_backward(csc_off.cpu(), csc_row.cpu(),
                                  csc_val.cpu() if with_val else None, dual.cpu(), xv.cpu(),
                                  hdr, vc, vs)
    assert torch.allclose(gw.cpu(), gw_r, atol=1e-4, rtol=1e-3)
    live = ref.hdr_vidx(hdr).long()
    live = live[live >= 0]
    assert torch.allclose(gvc.cpu()[live], gvc_r[live], atol=1e-4, rtol=1e-3)
    # the two-phase backward (plan on a side stream, run after the forward)
    side = torch.cuda.Stream(device=DEV)
    side.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(side):
        plan = hip.fm_backward_plan(csc_off, csc_row, hdr.to(DEV), vc.shape[0],
                                    off.numel() - 1, vs)
    torch.cuda.current_stream(DEV).wait_stream(side)
    gw2, gvc2 = hip.fm_backward_run(plan, csc_off, csc_row, csc_val if with_val else None, dual,
                                    xv, hdr.to(DEV), vc.to(DEV), vs)
    assert torch.allclose(gw2.cpu(), gw_r, atol=1e-4, rtol=1e-3)
    assert torch.allclose(gvc2.cpu()[live], gvc_r[live], atol=1e-4, rtol=1e-3)


def test_grad_post_and_renumber(hip):
    g = torch.Generator().manual_seed(8)
    gvc = torch.randn(50, 16, generator=g) * 3
    m = torch.tensor([40], dtype=torch.int64)
    a = gvc.clone().to(DEV)
    hip.fm_grad_post(a, m.to(DEV), 12, 1.0, 0.0, 1, True)
    r = gvc.clone()
    r[:40, :12].clamp_(-1, 1)
    r[:40, :12] /= float((r[:40, :12].double() ** 2).sum()) ** 0.5
    assert torch.allclose(a.cpu()[:40, :12], r[:40, :12], atol=1e-6)
    assert torch.equal(a.cpu()[40:], gvc[40:]) and torch.equal(a.cpu()[:, 12:], gvc[:, 12:])
    vidx = torch.tensor([5, -1, 9, 2, -1, -1, 7], dtype=torch.int64)
    h = ref.make_hdr(torch.arange(7).float(), vidx)
    hg = h.to(DEV)
    mg = hip.vidx_renumber(hg)
    assert int(mg) == 4
    assert ref.hdr_vidx(hg.cpu()).tolist() == [0, -1, 1, 2, -1, -1, 3]
    assert torch.equal(hg.cpu()[:, 0], h[:, 0])


@pytest.mark.parametrize("loss", [1, 2, 4])
def test_linear_forward_backward(hip, loss):
    keys, off, val, label = _rand_batch(5000, 30, 20000, 4, True)
    uniq, ucnt, oc, lid, csc_off, csc_row, csc_val = hip.localize(
        keys.to(DEV), off.to(DEV), val.to(DEV), 1)[:7]
    w = torch.randn(uniq.numel()) * 0.1
    met = torch.zeros(4, dtype=torch.float64, device=DEV)
    py, dual, _ = hip.fm_forward(off.to(DEV), lid, val.to(DEV), w.to(DEV), None, 0,
                                 label.to(DEV), loss, met)
    met_r = torch.zeros(4, dtype=torch.float64)
    py_r, dual_r, _ = ref.fm_forward(off, lid.cpu(), val, w, None, 0, label, loss, met_r)
    assert torch.allclose(py.cpu(), py_r, atol=1e-4, rtol=1e-4)
    assert torch.allclose(dual.cpu(), dual_r, atol=1e-4, rtol=1e-4)
    assert torch.allclose(met.cpu(), met_r, rtol=1e-5)
    g, _ = hip.fm_backward(csc_off, csc_row, csc_val, dual, None, w.to(DEV), None, 0)
    g_r, _ = ref.fm_backward(csc_off.cpu(), csc_row.cpu(), csc_val.cpu(), dual.cpu(), None, w,
                             None, 0)
    assert torch.allclose(g.cpu(), g_r, atol=1e-3, rtol=1e-3)


def test_auc(hip):
    g = torch.Generator().manual_seed(5)
    for n in [10, 1000, 100000]:
        py = torch.randn(n, generator=g)
        lab = (torch.rand(n, generator=g) < torch.sigmoid(py)).float()
        a = hip.auc(py.to(DEV), lab.to(DEV)).cpu()
        r = ref.auc(py, lab)
        assert abs(float(a) - float(r)) < 1e-9
    one = hip.auc(torch.randn(50, device=DEV), torch.ones(50, device=DEV))
    assert float(one) == 1.0


def test_auc_ties_and_accumulate(hip):
    """Sort-free AUC (pair counting up to 24576 examples, bucketed above)
    vs the stable-sort reference and the rocPRIM sort path: heavy ties
    (quantised scores), all-equal scores (a zero model), +-0, and on-device
    accumulation over repeated calls."""
    g = torch.Generator().manual_seed(6)
    cases = []
    for n in [1, 2, 777, 10000, 24576, 24577, 65536, 300001]:
        py = torch.randn(n, generator=g)
        cases.append((py, (torch.rand(n, generator=g) < torch.sigmoid(2 * py)).float()))
        q = torch.round(py * 4) / 4  # few distinct values: long tie runs
        cases.append((q, (torch.rand(n, generator=g) < 0.3).float()))
    z = torch.zeros(4096)
    z[::3] = -0.0
    cases.append((z, (torch.rand(4096, generator=g) < 0.5).float()))
    acc = torch.zeros(1, dtype=torch.float64, device=DEV)
    tot = 0.0
    for py, lab in cases:
        r = float(ref.auc(py, lab))
        a = float(hip.auc(py.to(DEV), lab.to(DEV)))
        b = float(hip.auc_sorted(py.to(DEV), lab.to(DEV)))
        assert abs(a - r) < 1e-9, (py.numel(), a, r)
        assert abs(b - r) < 1e-9
        hip.auc_acc(py.to(DEV), lab.to(DEV), acc)
        tot += r
    assert abs(float(acc) - tot) < 1e-8


def test_lookback_fused_paths_large(hip):
    """Fused single-pass scans over many tiles (multi-window look-back):
    pull, vidx renumbering and backward chunk planning at U ~ 200k."""
    from wormhole_amd.kv.cpu_store import CpuKVStore
    n = 200_003
    gk = torch.Generator().manual_seed(11)
    keys = torch.unique(torch.randint(1, 1 << 40, (2 * n,), generator=gk))[:n]
    keys = keys[torch.randperm(n, generator=gk)] * 2 + 1
    gs = hip.KVStore(1 << 19, 1 << 18, 16, 0)
    cs = CpuKVStore(1 << 19, 1 << 18, 16)
    hp = [0.1, 1.0, 0.0, 0.0, 0.1, 1.0, 0.0, 0.01]
    cnt = (torch.rand(n) * 4).floor()
    sg = gs.find(keys.to(DEV), True)
    sc = cs.find(keys, True)
    gs.difacto_push_cnt(sg, cnt.int().to(DEV), hp, 1, False, 3)
    cs.difacto_push_cnt(sc, cnt, hp, 1, False, 3)
    for _ in range(2):  # second call: a fresh epoch over stale granules
        hg, vg, vpg = gs.difacto_pull(sg, False)
    hc, vcc, vpc = cs.difacto_pull(sc, False)
    assert torch.equal(ref.hdr_vidx(hg.cpu()), ref.hdr_vidx(hc))
    assert torch.equal(vpg.cpu(), vpc)
    m = int(vpc[-1])
    assert torch.allclose(vg.cpu()[:m], vcc[:m])
    # renumber a header whose vidx are scattered
    h = hg.clone()
    vi = ref.hdr_vidx(h.cpu()).long()
    exp = torch.where(vi >= 0, torch.cumsum((vi >= 0).long(), 0) - 1, -1)
    mm = hip.vidx_renumber(h)
    assert int(mm) == int((vi >= 0).sum())
    assert torch.equal(ref.hdr_vidx(h.cpu()).long(), exp)
    # backward with ~200k unique ids
    keys2, off, _, label = _rand_batch(40000, 12, 400000, 9, False, skew=False)
    uniq, ucnt, oc, lid, csc_off, csc_row, csc_val = hip.localize(keys2.to(DEV), off.to(DEV),
                                                                  None, 1)[:7]
    U = uniq.numel()
    assert U > 100000
    hdr, vc = _pulled(U, 16, 16, 4)
    dual = torch.randn(40000)
    xv = torch.randn(40000, 16)
    gw, gvc = hip.fm_backward(csc_off, csc_row, None, dual.to(DEV), xv.reshape(-1).to(DEV),
                              hdr.to(DEV), vc.to(DEV), 16)
    gw_r, gvc_r = ref.fm_backward(csc_off.cpu(), csc_row.cpu(), None, dual, xv.reshape(-1), hdr,
                                  vc, 16)
    assert torch.allclose(gw.cpu(), gw_r, atol=1e-4, rtol=1e-3)
    live = ref.hdr_vidx(hdr).long()
    live = live[live >= 0]
    assert torch.allclose(gvc.cpu()[live], gvc_r[live], atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("algo", [1, 2, 3])
def test_linear_store_updates(hip, algo):
    from wormhole_amd.kv.cpu_store import CpuKVStore
    gs = hip.KVStore(1 << 12, 0, 0, 0)
    cs = CpuKVStore(1 << 12, 0, 0)
    g = torch.Generator().manual_seed(algo)
    keys = torch.randint(0, 1 << 40, (1000,), generator=g)
    keys = torch.unique(keys)
    for it in range(5):
        sel = keys[torch.randperm(keys.numel(), generator=g)[:600]] if it else keys
        grad = torch.randn(sel.numel(), generator=g)
        s_g = gs.find(sel.to(DEV), True)
        s_c = cs.find(sel, True)
        eta = (1.0 + (it + 1) ** 0.5) / 0.1
        gs.linear_push(s_g, grad.to(DEV), algo, 0.1, 1.0, 0.3, 0.05, eta)
        cs.linear_push(s_c, grad, algo, 0.1, 1.0, 0.3, 0.05, eta)
    s_g = gs.find(keys.to(DEV), False)
    s_c = cs.find(keys, False)
    assert torch.allclose(gs.linear_pull(s_g).cpu(), cs.linear_pull(s_c), atol=1e-5, rtol=1e-4)
    assert int(gs.stats[0]) == int(cs.stats[0])
    assert int(gs.stats[4]) == keys.numel()


@pytest.mark.parametrize("dim", [5, 64])
def test_difacto_store_updates(hip, dim):
    from wormhole_amd.kv.cpu_store import CpuKVStore
    gs = hip.KVStore(1 << 12, 1 << 10, dim, 0)
    cs = CpuKVStore(1 << 12, 1 << 10, dim)
    vs = gs.vstride
    hp = [0.05, 1.0, 0.01, 0.1, 0.02, 1.0, 0.5, 0.01]
    g = torch.Generator().manual_seed(dim)
    keys = torch.unique(torch.randint(0, 1 << 40, (800,), generator=g))
    for it in range(6):
        sel = keys[torch.randperm(keys.numel(), generator=g)[:500]]
        cnt = torch.randint(1, 4, (sel.numel(),), generator=g).float()
        s_g = gs.find(sel.to(DEV), True)
        s_c = cs.find(sel, True)
        gs.difacto_push_cnt(s_g, cnt.to(DEV), hp, 3, True, 42)
        cs.difacto_push_cnt(s_c, cnt, hp, 3, True, 42)
        hg, vg, _ = gs.difacto_pull(s_g, True)
        hc, vcc, _ = cs.difacto_pull(s_c, True)
        _same_pull(hg, vg, hc, vcc)
        gw = torch.randn(sel.numel(), generator=g) * 0.5
        m = vcc.shape[0]
        gvc = torch.randn(m, vs, generator=g) * 0.5
        # the GPU store numbers its rows by the same exclusive scan
        gs.difacto_push(s_g, hg, gw.to(DEV), gvc.to(DEV), hp, 3, True, 42)
        cs.difacto_push(s_c, hc, gw, gvc, hp, 3, True, 42)
    s_g = gs.find(keys.to(DEV), False)
    s_c = cs.find(keys, False)
    hg, vg, _ = gs.difacto_pull(s_g, False)
    hc, vcc, _ = cs.difacto_pull(s_c, False)
    assert vcc.shape[0] > 0
    _same_pull(hg, vg, hc, vcc)
    assert int(gs.stats[0]) == int(cs.stats[0])
    assert int(gs.stats[1]) == int(cs.stats[1])


def _same_pull(hg, vg, hc, vcc):
    hg = hg.cpu()
    assert torch.allclose(hg[:, 0], hc[:, 0], atol=1e-5, rtol=1e-4)
    assert torch.equal(ref.hdr_vidx(hg), ref.hdr_vidx(hc))
    m = vcc.shape[0]
    assert torch.allclose(vg.cpu()[:m], vcc, atol=1e-5, rtol=1e-4)


def test_synth_criteo(hip):
    from wormhole_amd.data.synthetic import CRITEO_TB_CARD
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=DEV)
    keys, label, off = hip.synth_criteo(10000, 1, 0, card)
    assert keys.numel() == 390000 and off[-1].item() == 390000
    f = (keys.cpu() >> 54) & 1023
    assert torch.equal(f.view(10000, 39), torch.arange(39).expand(10000, 39))
    ctr = float(label.mean())
    assert 0.05 < ctr < 0.6
    keys2, _, _ = hip.synth_criteo(10000, 1, 0, card)
    assert torch.equal(keys, keys2)


def test_difacto_learner_matches_cpu(hip):
    """A few GPU training steps track the CPU reference path."""
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    emb = Embedding(dim=8, threshold=2)
    conf = DifactoConfig(embedding=[emb], lambda_l1=0.01)
    lg = DifactoLearner(conf, Comm(DEV, init=False), DEV, cap=1 << 14, vcap=1 << 12, seed=5)
    lc = DifactoLearner(conf, Comm(torch.device("cpu"), init=False), "cpu", cap=1 << 14,
                        vcap=1 << 12, seed=5)
    for step in range(4):
        keys, off, val, label = _rand_batch(400, 10, 800, 10 + step)
        lg.process(keys.to(DEV), off.to(DEV), None, label.to(DEV), 0, 0)
        lc.process(keys, off, None, label, 0, 0)
    pg, pc = lg.take_progress(), lc.take_progress()
    assert abs(pg[0] - pc[0]) / pc[0] < 1e-3
    assert abs(pg[1] - pc[1]) < 1e-3
    assert pg[6] == pc[6] and pg[7] == pc[7]


def test_hist_dots_and_dir_fix_dot(hip):
    """The solver's history kernels: every row against up to 4 probe rows
    (exact fp64) and the direction build + sign fix + dot (fp32 in list
    order, as the reference AddScale loop)."""
    g = torch.Generator().manual_seed(5)
    for R, n in [(21, 100_000), (3, 4096), (9, 40)]:
        H = torch.randn(R, n, generator=g)
        for probes in ([R - 1], [0, R - 1], [R - 1, 1, 2], [0, 1, 2, R - 1][: min(4, R)]):
            out = hip.hist_dots(H.to(DEV), probes).cpu()
            ref_ = H.double() @ H[probes].double().t()
            assert out.shape == (R, len(probes))
            assert torch.allclose(out, ref_, rtol=1e-10, atol=1e-9)
        rows = list(range(R // 2, R)) + list(range(R // 2))
        coef = [float(x) for x in torch.randn(R, generator=g)]
        for fix in (False, True):
            d, v = hip.dir_fix_dot(H.to(DEV), rows, coef, R - 1, fix)
            acc = torch.zeros(n)
            for r, c in zip(rows, coef):
                acc = acc + H[r] * torch.tensor(c, dtype=torch.float32)
            st = H[R - 1]
            if fix:
                acc = torch.where(acc * st <= 0, torch.zeros_like(acc), acc)
            assert torch.allclose(d.cpu(), acc, rtol=1e-5, atol=1e-5)
            rv = float((d.cpu() * st).double().sum())
            assert abs(float(v) - rv) <= 1e-9 * max(1.0, abs(rv))


def test_glm_xtg_plain_csc(hip):
    """glm.hip's segmented X^T g over a plain CSC (run = column, stores for
    columns inside a wave, atomics at wave cuts) against torch."""
    keys, off, val, _ = _rand_batch(20000, 30, 3000, 17, with_val=True)
    uniq, _c, _o, _lid, csc_off, csc_row, csc_val = [
        t.to(DEV) if t is not None else None for t in
        __import__("wormhole_amd.ops", fromlist=["localize"]).localize(
            keys.to(DEV), off.to(DEV), val.to(DEV), 1)]
    nnz = csc_row.numel()
    g = torch.randn(off.numel() - 1, device=DEV)
    hb = hip.glm_heads(csc_off, nnz)
    waves = (nnz + 1023) // 1024
    col0 = (torch.searchsorted(csc_off, torch.arange(waves, device=DEV) * 1024, right=True)
            - 1).int()
    U = csc_off.numel() - 1
    ucol = torch.arange(U, device=DEV, dtype=torch.int32)
    out = torch.zeros(U, device=DEV)
    hip.glm_xtg(csc_row.contiguous(), csc_val, hb, col0, ucol, g, out)
    key = torch.repeat_interleave(torch.arange(U, device=DEV), csc_off[1:] - csc_off[:-1])
    ref_ = torch.zeros(U, dtype=torch.float64, device=DEV).index_add_(
        0, key, (csc_val * g[csc_row.long()]).double())
    assert torch.allclose(out.double(), ref_, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("with_val,loss", [(False, 1), (True, 1), (False, 0)])
def test_glm_objective_matches_cpu(with_val, loss):
    """L-BFGS linear objective on the GPU (glm.hip: fused margin + loss, the
    segmented CSC X^T g with power-law columns spanning many 1024-entry
    waves) against the torch path on the CPU."""
    from wormhole_amd.models.lbfgs_models import LinearObjective, _SplitData
    from wormhole_amd.parallel.bsp import BSP
    g = torch.Generator().manual_seed(3 + loss)
    nrows, F = 60_000, 50_000
    lens = torch.randint(1, 40, (nrows,), generator=g)
    off = torch.zeros(nrows + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(lens, 0)
    nnz = int(off[-1])
    u = torch.rand(nnz, generator=g)
    keys = (torch.exp(u * np.log(F * 1.2)) - 1).long()  # some ids >= F (outside the model)
    keys[:: 7] = 3  # one very heavy column
    val = (torch.rand(nnz, generator=g) + 0.5) if with_val else None
    label = (torch.rand(nrows, generator=g) < 0.3).float()
    objs = []
    for dev in (torch.device("cpu"), DEV):
        d = _SplitData(keys, off, val, label, dev)
        o = LinearObjective(BSP(torch.device("cpu")), d, dev)
        o.set_param("objective", "logistic" if loss == 1 else "linear")
        o.set_param("num_feature", str(F))
        o.param.base_score = 0.1
        objs.append(o)
    w = torch.randn(F + 1, generator=g) * 0.05
    wd = w.to(DEV)
    lc = objs[0].eval(w)
    lg = objs[1].eval(wd)
    assert abs(lg - lc) <= 1e-5 * abs(lc)
    gc = objs[0].calc_grad(w)
    scale = float(gc.abs().max())
    # the gradient at the weights just evaluated reuses their margins; a
    # second call recomputes them
    for _ in range(2):
        gg = objs[1].calc_grad(wd).cpu()
        assert torch.allclose(gg, gc, rtol=1e-4, atol=1e-5 * scale)
    mc = objs[0].margin(w)
    mg = objs[1].margin(w.to(DEV)).cpu()
    assert torch.allclose(mg, mc, rtol=1e-5, atol=1e-5)


def test_owlqn_trajectory_matches_cpu():
    """Ten OWL-QN iterations (learn/solver/lbfgs.h:168-196: gradient, the
    two-loop direction with the L1 sign fixes, the backtracking line search)
    on Criteo-shaped data hashed into 2^18 columns: the GPU path (glm.hip
    objective / gradient, lbfgs.hip history dots and direction) follows the
    CPU path's objective iteration by iteration and ends at the same
    weights."""
    from wormhole_amd.data.synthetic import CRITEO_TB_CARD, criteo_batch_cpu
    from wormhole_amd.models.lbfgs_models import LinearObjective, _SplitData
    from wormhole_amd.parallel.bsp import BSP
    from wormhole_amd.solver.lbfgs import LBFGSSolver
    F = 1 << 18
    keys, label, off = criteo_batch_cpu(100_000, 4242, 0, CRITEO_TB_CARD)
    keys = torch.remainder(keys, F)
    runs = []
    for dev in (torch.device("cpu"), DEV):
        bsp = BSP(torch.device("cpu"))
        obj = LinearObjective(bsp, _SplitData(keys, off, None, label, dev), dev)
        obj.set_param("objective", "logistic")
        obj.set_param("num_feature", str(F))
        sol = LBFGSSolver(bsp, obj)
        sol.silent = True
        for k, v in (("reg_L1", 1.0), ("size_memory", 10), ("lbfgs_stop_tol", 0.0),
                     ("min_lbfgs_iter", 1 << 30), ("max_lbfgs_iter", 10)):
            sol.set_param(k, str(v))
        sol.init()
        traj = [float(sol.old_objval)]
        for _ in range(10):
            sol.update_one_iter()
            traj.append(float(sol.old_objval))
        runs.append((traj, sol.weight.detach().cpu()))
    (tc, wc), (tg, wg) = runs
    assert tc[-1] < 0.95 * tc[0]  # it trains
    for i, (a, b) in enumerate(zip(tc, tg)):
        assert abs(a - b) <= 1e-5 * abs(a), (i, tc, tg)
    assert (wc != 0).sum() > 100
    assert torch.allclose(wg, wc, rtol=1e-3, atol=1e-4 * float(wc.abs().max()))


@pytest.mark.parametrize("n,f,k", [(1000, 5, 7), (4096, 64, 33), (5000, 127, 100),
                                   (3000, 128, 1000), (777, 200, 40)])
def test_kmeans_assign_accum(hip, n, f, k):
    g = torch.Generator().manual_seed(n + f + k)
    X = torch.randn(n, f, generator=g)
    C = torch.nn.functional.normalize(torch.randn(k, f, generator=g), dim=1)
    Xd = X.to(DEV)
    Xp = hip.kmeans_pack_x(Xd)
    Cp = hip.kmeans_pack_c(C.to(DEV))
    a, score = hip.kmeans_assign(Xp, n, f, Cp, k)
    S = X.double() @ C.double().t()
    ref_a = S.argmax(1)
    a = a.cpu().long()
    # exact fp32 MFMA: any disagreement must be a numerical near-tie
    best = S.gather(1, ref_a[:, None])[:, 0]
    got = S.gather(1, a[:, None])[:, 0]
    assert bool(((best - got) <= 1e-4 * best.abs().clamp_min(1)).all())
    assert (a == ref_a).float().mean() > 0.999
    assert torch.allclose(score.cpu().double(), got, atol=1e-3, rtol=1e-4)
    sums = hip.kmeans_accum(Xd, a.to(torch.int32).to(DEV), k).cpu()
    ref_s = torch.zeros(k, f + 1)
    ref_s[:, :f].index_add_(0, a, X)
    ref_s[:, f].index_add_(0, a, torch.ones(n))
    assert torch.allclose(sums, ref_s, atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("n,f,k,skew", [(200_003, 128, 1000, False), (100_000, 64, 5, True),
                                        (50_000, 600, 10, False), (70_000, 33, 20000, False)])
def test_kmeans_accum_sorted(hip, n, f, k, skew):
    """Counting-sort accumulation (multi-block histograms, segments crossing
    waves, a dominant cluster) and its atomic fallback (f > 512, k > 16384)
    against index_add."""
    g = torch.Generator().manual_seed(n + k)
    X = torch.randn(n, f, generator=g)
    a = torch.randint(0, k, (n,), generator=g)
    if skew:
        a[torch.rand(n, generator=g) < 0.9] = 3
    sums = hip.kmeans_accum(X.to(DEV), a.to(torch.int32).to(DEV), k).cpu()
    ref_s = torch.zeros(k, f + 1, dtype=torch.float64)
    ref_s[:, :f].index_add_(0, a, X.double())
    ref_s[:, f].index_add_(0, a, torch.ones(n, dtype=torch.float64))
    assert torch.equal(sums[:, f], ref_s[:, f].float())
    assert torch.allclose(sums.double(), ref_s, atol=5e-3 * (n / k) ** 0.5, rtol=1e-4)


def test_spmv_kernels(hip):
    keys, off, val, label = _rand_batch(3000, 20, 5000, 9, True)
    uniq, ucnt, oc, lid, csc_off, csc_row, csc_val = hip.localize(
        keys.to(DEV), off.to(DEV), val.to(DEV), 1)[:7]
    x = torch.randn(uniq.numel())
    y = hip.spmv(off.to(DEV), lid, val.to(DEV), x.to(DEV)).cpu()
    rows = torch.repeat_interleave(torch.arange(3000), off[1:] - off[:-1])
    ref_y = torch.zeros(3000).index_add_(0, rows, val * x[lid.cpu().long()])
    assert torch.allclose(y, ref_y, atol=1e-4, rtol=1e-4)
    p = torch.randn(3000)
    yt = hip.spmv_t(csc_off, csc_row, csc_val, p.to(DEV)).cpu()
    ref_t = torch.zeros(uniq.numel()).index_add_(0, lid.cpu().long(), val * p[rows])
    assert torch.allclose(yt, ref_t, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("l1_shrk", [False, True])
def test_difacto_open_pull_fused(hip, l1_shrk):
    """The one-launch find + count push + pull against the host store doing
    the three steps: slots resolve to the same keys, counts cross the
    threshold at the same step, and the pulled headers / rows agree."""
    from wormhole_amd.kv.cpu_store import CpuKVStore
    gs = hip.KVStore(1 << 16, 1 << 14, 16, 0)
    cs = CpuKVStore(1 << 16, 1 << 14, 16)
    hp = [0.1, 1.0, 0.0, 0.0, 0.1, 1.0, 0.0, 0.01]
    g = torch.Generator().manual_seed(12)
    for step in range(4):
        keys = torch.unique(torch.randint(1, 5000, (3000,), generator=g)) * 7 + 3
        keys = keys[torch.randperm(keys.numel(), generator=g)]
        cnt = torch.randint(0, 3, (keys.numel(),), generator=g)
        sg, hg, vg, pg = gs.difacto_open_pull(keys.to(DEV), True, cnt.int().to(DEV), hp, 2,
                                              l1_shrk, 5)
        sc, hc, vcc, pc = cs.difacto_open_pull(keys, True, cnt.float(), hp, 2, l1_shrk, 5)
        assert bool((sg >= 0).all())
        assert torch.equal(gs.keys.cpu()[sg.long().cpu()], keys)
        assert torch.equal(ref.hdr_vidx(hg.cpu()), ref.hdr_vidx(hc))
        assert torch.equal(pg.cpu(), pc)
        m = int(pc[-1])
        assert torch.allclose(vg.cpu()[:m], vcc[:m])
        assert torch.allclose(hg.cpu()[:, 0], hc[:, 0], atol=1e-6, rtol=1e-5)
        # a push so that w moves (l1_shrk then filters on w != 0)
        gw = torch.randn(keys.numel(), generator=g)
        gv = torch.randn(max(m, 1), 16, generator=g) * 0.1
        gs.difacto_push(sg, hg, gw.to(DEV), gv[:m].contiguous().to(DEV), hp, 2, l1_shrk, 5)
        cs.difacto_push(sc, hc, gw, gv[:m].contiguous(), hp, 2, l1_shrk, 5)


def test_localize_job_pipelined(hip):
    """Two-phase localize (begin: insert + counts + async read; finish): two
    jobs in flight on the double-buffered tables, an under-sized table that
    retries inside finish(), and the same results as the one-shot call."""
    from wormhole_amd import ops
    batches = [_rand_batch(2000, 20, 8000, s, s % 2 == 1) for s in range(4)]
    dev = [(k.to(DEV), o.to(DEV), v.to(DEV) if v is not None else None) for k, o, v, _ in batches]
    ref_out = [ops.localize(k, o, v, 3, 0) for k, o, v in dev]
    j0 = ops.localize_begin(*dev[0], 3, 1)       # hint 1: overflows, retries at the safe size
    j1 = ops.localize_begin(*dev[1], 3, 5000)    # second job in flight (other table)
    outs = [ops.localize_finish(j0), ops.localize_finish(j1)]
    j2 = ops.localize_begin(*dev[2], 3, 0)
    outs.append(ops.localize_finish(j2))
    j3 = ops.localize_begin(*dev[3], 3, 0)
    del j3  # abandoned: its table must be cleaned before reuse
    outs.append(ops.localize(*dev[3], 3, 0))
    for (k, o, v), a, b in zip(dev, outs, ref_out):
        assert torch.equal(torch.sort(a[0]).values, torch.sort(b[0]).values)
        assert torch.equal(a[0][a[3].long()], k)
        assert torch.equal(a[2], b[2])
        cnt_a = torch.zeros(a[0].numel(), dtype=torch.int64, device=DEV)
        assert torch.equal(a[1].long().sum(), torch.tensor(k.numel(), device=DEV))
        assert torch.equal(a[4][1:] - a[4][:-1], a[1].long())


def test_learner_pipelined_matches_plain(hip):
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.data.synthetic import CRITEO_TB_CARD
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=DEV)
    res = []
    for pipelined in (False, True):
        emb = Embedding(dim=16, threshold=2)
        lr = DifactoLearner(DifactoConfig(minibatch=5000, embedding=[emb]),
                            Comm(DEV, init=False), DEV, cap=1 << 20, vcap=1 << 16, seed=3)
        data = [hip.synth_criteo(5000, 9, s, card) for s in range(6)]
        for s, (k, l, o) in enumerate(data):
            nb = None
            if pipelined and s + 1 < len(data):
                nb = (data[s + 1][0], data[s + 1][2], None)
            lr.process(k, o, None, l, 0, 0, next_batch=nb)
        res.append(lr.take_progress())
    a, b = res
    assert a[4] == b[4] and a[5] == b[5] and a[7] == b[7]
    assert abs(a[0] - b[0]) < 1e-4 * abs(b[0]) and abs(a[1] - b[1]) < 1e-6


@pytest.mark.parametrize("l1_shrk", [False, True])
def test_difacto_direct_pull_matches_copy(hip, l1_shrk):
    """One shard: the FM kernels reading V in place in the slab (direct pull,
    the default) train the same model as the pulled compact copy, through a
    V-slab growth, with the next localize begun early; prediction agrees."""
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.data.synthetic import CRITEO_TB_CARD
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=DEV)
    data = [hip.synth_criteo(4000, 21, s, card) for s in range(8)]
    out = []
    for direct in (True, False):
        emb = Embedding(dim=16, threshold=2)
        conf = DifactoConfig(minibatch=4000, embedding=[emb], l1_shrk=l1_shrk, lambda_l1=0.01)
        lr = DifactoLearner(conf, Comm(DEV, init=False), DEV, cap=1 << 20, vcap=1 << 10, seed=3)
        assert lr.direct_pull
        lr.direct_pull = direct
        for s, (k, l, o) in enumerate(data):
            nb = (data[s + 1][0], data[s + 1][2], None) if s + 1 < len(data) else None
            lr.process(k, o, None, l, 0, 0, next_batch=nb)
        lr.flush()
        k, l, o = hip.synth_criteo(3000, 22, 0, card)
        py = lr.process(k, o, None, l, 2, 0)
        st = lr.store
        occ = st.occupied().long()
        rows = st.vrow[occ].long()
        V = torch.where((rows >= 0)[:, None], st.V[rows.clamp_min(0)], torch.zeros_like(st.V[:1]))
        keys = st.keys[occ]
        order = torch.argsort(keys)  # (slot order depends on insert timing)
        out.append((lr.take_progress(), keys[order].cpu(), st.w[occ][order].cpu(),
                    V[order].cpu(), py.cpu(), lr.kv.guard.vgrows))
    (pa, ka, wa, va, ya, ga), (pb, kb, wb, vb, yb, gb) = out
    assert ga >= 1  # the 1024-row V slab had to grow
    assert torch.equal(ka, kb)
    assert torch.allclose(wa, wb, atol=1e-6) and torch.allclose(va, vb, atol=1e-6)
    assert torch.allclose(ya, yb, atol=1e-5)
    assert pa[4:] == pb[4:] and abs(pa[0] - pb[0]) < 1e-5 * abs(pb[0])


def test_async_saver_snapshot(hip, tmp_path):
    """The background save writes the state at the save call: updates
    issued right after it (before the file is written) must not leak in, and
    the file equals the synchronous dump byte for byte."""
    from wormhole_amd.kv import checkpoint
    gs = hip.KVStore(1 << 14, 1 << 12, 16, 0)
    hp = [0.05, 1.0, 0.01, 0.1, 0.02, 1.0, 0.5, 0.01]
    g = torch.Generator().manual_seed(5)
    keys = torch.unique(torch.randint(0, 1 << 40, (3000,), generator=g)).to(DEV)

    def step():
        s = gs.find(keys, True)
        gs.difacto_push_cnt(s, torch.randint(1, 4, (keys.numel(),), generator=g).float().to(DEV),
                            hp, 3, False, 7)
        hd, vc, _ = gs.difacto_pull(s, False)
        gs.difacto_push(s, hd, torch.randn(keys.numel(), generator=g).to(DEV),
                        torch.randn(vc.shape[0], vc.shape[1], generator=g).to(DEV), hp, 3, False, 7)

    for _ in range(3):
        step()
    checkpoint.save_difacto(gs, str(tmp_path / "sync"))
    saver = checkpoint.AsyncSaver()
    saver.save("difacto", gs, str(tmp_path / "async"))
    for _ in range(3):
        step()  # mutates the live table while the snapshot is written
    saver.join()
    a = (tmp_path / "sync").read_bytes()
    assert len(a) > 0 and a == (tmp_path / "async").read_bytes()


@pytest.mark.parametrize("S,F,nbin,alpha,mcw", [(5, 7, 33, 0.0, 1.0), (3, 28, 256, 0.5, 0.1),
                                                (2, 4, 1000, 0.0, 5.0)])
def test_gbdt_split_kernel(hip, S, F, nbin, alpha, mcw):
    """Fused split search vs the torch reference (_find_splits_ref): same
    feature / bin / direction, gains and left sums to fp64 rounding; a node
    with no valid candidate reports -inf."""
    from wormhole_amd.models import gbdt as G
    g = torch.Generator().manual_seed(S * F + nbin)
    hist = torch.zeros(S, F, nbin, 2, dtype=torch.float64)
    hist[..., 0] = torch.randn(S, F, nbin, generator=g, dtype=torch.float64)
    hist[..., 1] = torch.rand(S, F, nbin, generator=g, dtype=torch.float64) * 2
    present = hist.sum(2)  # [S, F, 2]
    totals = present.max(1).values + torch.rand(S, 2, generator=g, dtype=torch.float64)
    totals[:, 0] = present[:, :, 0].mean(1)  # rows missing a feature move the totals
    valid = torch.rand(F, nbin, generator=g) < 0.8
    valid[0] = False
    tb = G.TreeBuilder.__new__(G.TreeBuilder)
    tb.p = G.GBDTParam()
    tb.p.alpha, tb.p.min_child_weight = alpha, mcw
    tb.nbin, tb.valid_mask, tb._valid_dev = nbin, valid, None
    ref = tb._find_splits_ref(hist, totals)
    if S > 2:
        hist[2].zero_()  # no candidate passes min_child_weight on either side
        totals[2] = 0.0
        ref = tb._find_splits_ref(hist, totals)
    got = tb._find_splits(hist.to(DEV), totals.to(DEV))
    ok = torch.isfinite(ref[0])
    assert torch.equal(torch.isfinite(got[0]), ok)
    assert torch.allclose(got[0][ok], ref[0][ok], rtol=1e-9, atol=1e-9)
    for k in (1, 2, 3):
        assert torch.equal(got[k][ok], ref[k][ok])
    assert torch.allclose(got[4][ok], ref[4][ok], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("l1", [0.0, 0.3])
def test_owlqn_kernels(hip, l1):
    """OWL-QN direction / sign fix + dot / fused step + |w|_1 and the batched
    history dots against the solver's torch forms (fp32 data, fp64 sums)."""
    from wormhole_amd.solver.lbfgs import LBFGSSolver
    g = torch.Generator().manual_seed(11)
    n = 100_003
    grad = torch.randn(n, generator=g)
    w = torch.randn(n, generator=g)
    w[torch.rand(n, generator=g) < 0.3] = 0.0
    sv = LBFGSSolver.__new__(LBFGSSolver)
    sv.reg_L1 = l1
    ref_d = sv.set_l1_dir(grad, w)
    d = hip.owlqn_dir(grad.to(DEV), w.to(DEV), l1)
    assert torch.equal(d.cpu(), ref_d)
    steep = torch.randn(n, generator=g)
    ref_fixed = sv.fix_dir_l1_sign(ref_d.clone(), steep)
    ref_v = float((ref_fixed * steep).double().sum())  # float products, fp64 sum (lbfgs.h Dot)
    v = hip.owlqn_fix_dot(d, steep.to(DEV), l1 != 0.0)
    assert torch.equal(d.cpu(), ref_fixed)
    assert abs(float(v) - ref_v) <= 1e-9 * max(1.0, abs(ref_v))
    nw, s1 = hip.owlqn_step(w.to(DEV), d, 0.37, l1 != 0.0)
    ref_nw = sv.fix_weight_l1_sign(w + ref_fixed * 0.37, w)
    assert torch.allclose(nw.cpu(), ref_nw, rtol=1e-6, atol=1e-6)
    assert abs(float(s1) - float(nw.cpu().double().abs().sum())) <= 1e-6 * float(s1)
    H = torch.randn(21, 5000, generator=g)
    ia = torch.tensor([0, 3, 20, 5, 7], dtype=torch.int32)
    ib = torch.tensor([20, 3, 20, 9, 1], dtype=torch.int32)
    dots = hip.multi_dot(H.to(DEV), ia.to(DEV), ib.to(DEV)).cpu()
    ref = (H[ia.long()].double() * H[ib.long()].double()).sum(1)
    assert torch.allclose(dots, ref, rtol=1e-10, atol=1e-9)


@pytest.mark.parametrize("n,f,k", [(1000, 5, 7), (4096, 64, 33), (5000, 127, 100),
                                   (3000, 128, 1000), (2000, 17, 300)])
def test_kmeans_split_precision_matches_fp32(hip, n, f, k):
    """bf16 x 3 MFMA scores + exact fp32 re-score of near-ties: the argmax is
    the fp32 kernel's on random data, and planted near-ties (duplicated
    centroids perturbed below the split's error bound) are re-scored."""
    g = torch.Generator().manual_seed(7 * n + f + k)
    X = torch.randn(n, f, generator=g)
    C = torch.nn.functional.normalize(torch.randn(k, f, generator=g), dim=1)
    if k >= 7:  # near-duplicate centroids: rows near them tie within the bound
        C[1] = torch.nn.functional.normalize(C[0] + 1e-6 * torch.randn(f, generator=g), dim=0)
        X[: n // 10] = C[0] * 3 + 1e-3 * torch.randn(n // 10, f, generator=g)
    Xd, Cd = X.to(DEV), C.to(DEV)
    a32, _ = hip.kmeans_assign(hip.kmeans_pack_x(Xd), n, f, hip.kmeans_pack_c(Cd), k)
    Xp3, xn = hip.kmeans_pack_x3(Xd)
    a3, s3, namb = hip.kmeans_assign_x3(Xp3, xn, Xd, hip.kmeans_pack_c3(Cd), Cd)
    S = X.double() @ C.double().t()
    best = S.max(1).values
    got = S.gather(1, a3.cpu().long()[:, None])[:, 0]
    assert bool(((best - got) <= 1e-5 * best.abs().clamp_min(1)).all())
    differ = (a3 != a32).cpu()
    if k >= 7:
        assert int(namb.item()) >= n // 10  # the planted ties took the exact path
        # any disagreement with the fp32 kernel is a planted (fp32-level) tie
        assert bool((differ.nonzero()[:, 0] < n // 10).all())
    else:
        assert not bool(differ.any())
    assert torch.allclose(s3.cpu().double(), got, atol=1e-4, rtol=1e-4)


def test_ps_open_rejects_more_than_2_24_keys(hip):
    """The owner open numbers a minibatch's keys in 24 bits (the duplicate
    chain links, kv/psx.py): a shard receiving 2^24 keys in one minibatch
    is refused loudly, before anything is launched, and the store stays
    usable."""
    from wormhole_amd.kv import make_store
    st = make_store(1 << 10, 1 << 8, 16, DEV)
    seg = torch.tensor([0, 1 << 24], dtype=torch.int64, device=DEV)
    hseg = torch.zeros(2, dtype=torch.int64, device=DEV)  # (no header rows)
    big = torch.arange(1 << 24, dtype=torch.int64, device=DEV)
    hp = [0.1, 1.0, 0.0, 0.0, 0.1, 1.0, 0.0, 0.01]
    with pytest.raises(RuntimeError, match="2\\^24"):
        st.ps_open(big, False, seg, hseg, 1 << 24, True, False, hp, 0, False, 0)
    del big
    small = torch.arange(100, dtype=torch.int64, device=DEV) * 7 + 1
    seg = torch.tensor([0, 100], dtype=torch.int64, device=DEV)
    out = st.ps_open(small, False, seg, hseg, 100, True, False, hp, 0, False, 0)
    assert int((out[0] >= 0).sum()) == 100  # every key got a slot


def test_ps_open_headers_uneven_segments(hip):
    """The owner open writes each peer region's headers itself (segment
    V-row prefixes published between tiles): empty leading / middle /
    trailing segments and segments spanning several 1024-key tiles land at
    (HS_p + VS_p) * vstride + 2 (i - S_p) with the row index inside the
    peer's V block, and vcnt[p] counts each peer's rows."""
    from wormhole_amd.kv import make_store
    st = make_store(1 << 14, 1 << 13, 16, DEV)
    sizes = [0, 700, 0, 1500, 3, 0, 2100, 0]
    P, n = len(sizes), sum(sizes)
    g = torch.Generator().manual_seed(9)
    keys = torch.randperm(1 << 20, generator=g)[:n].long() * 2654435761 + 5
    cnt = (torch.arange(n) % 3 == 0).to(torch.int32) * 5
    rec = torch.cat([keys.view(torch.int32).view(n, 2), cnt[:, None]], 1).contiguous()  # {lo, hi, count}
    vs = 16
    S = [0]
    for z in sizes:
        S.append(S[-1] + z)
    H = [0]
    for z in sizes:
        H.append(H[-1] + (2 * z + vs - 1) // vs)
    segS = torch.tensor(S, dtype=torch.int64, device=DEV)
    segHS = torch.tensor(H, dtype=torch.int64, device=DEV)
    hp = [0.1, 1.0, 0.0, 0.0, 0.1, 1.0, 0.0, 0.01]
    slot, vpos, chain, head, rbuf, vcnt = st.ps_open(rec.to(DEV), True, segS, segHS, H[-1] + n,
                                                     True, True, hp, 2, False, 0)
    assert rbuf.shape[1] == vs
    vp = vpos.cpu().tolist()
    assert vp[n] == sum(1 for i in range(n) if i % 3 == 0)  # count 5 > threshold 2
    flat = rbuf.cpu().view(-1)
    bits = flat.view(torch.int32)
    for p in range(P):
        VS = vp[S[p]]
        assert int(vcnt[p]) == vp[S[p + 1]] - VS
        base = (H[p] + VS) * vs
        for i in range(S[p], S[p + 1]):
            j = vp[i] - VS if vp[i + 1] > vp[i] else -1
            assert float(flat[base + 2 * (i - S[p])]) == 0.0  # fresh keys: w = 0
            assert int(bits[base + 2 * (i - S[p]) + 1]) == j, (p, i)


def test_localize_hint_scales_with_minibatch_size(hip):
    """Uneven minibatches (CRB records cut parts into short and long blocks):
    a job begun with the previous, much smaller minibatch's unique count as
    its hint is sized by the non-zero ratio, so its partition plan fits and
    nothing falls back to the hash path; results stay exact."""
    card = torch.tensor([50, 400, 3000, 20, 7, 900, 100000, 2000000], dtype=torch.int64,
                        device=DEV)
    before = hip.loc_retries()
    hint = 0
    for s, n in enumerate([200000, 2000, 200000, 500, 150000, 3000, 200000]):
        keys, label, off = hip.synth_criteo(n, 11, s, card)
        job = hip.LocalizeJob(keys, off, None, 1, hint)
        uniq, ucnt, oc, lid = job.finish()[:4]
        assert torch.equal(uniq[lid.long()], keys)
        hint = uniq.numel()
    assert hip.loc_retries() == before


def test_kmeans_update_matches_torch(hip):
    """One-launch centroid update = mean of the summed rows (the previous
    centroid for an empty cluster), L2-normalised as models/kmeans.py does."""
    from wormhole_amd.models.kmeans import normalize_rows
    g = torch.Generator().manual_seed(4)
    k, f = 37, 100
    sums = torch.randn(k, f + 1, generator=g)
    sums[:, f] = torch.randint(0, 50, (k,), generator=g).float()
    sums[3, f] = 0
    sums[11, f] = 0
    sums[20, :f] = 0  # a zero-norm mean stays unscaled
    C = normalize_rows(torch.randn(k, f, generator=g))
    cnt = sums[:, f]
    empty = cnt == 0
    exp = torch.where(empty[:, None], C, sums[:, :f] / torch.where(empty, 1.0, cnt)[:, None])
    exp = normalize_rows(exp)
    got, ne = hip.kmeans_update(sums.to(DEV), C.to(DEV))
    assert int(ne) == int(empty.sum())
    assert torch.allclose(got.cpu(), exp, atol=1e-6, rtol=1e-6)


def test_auc_acc_reused_range_stays_exact(hip):
    """Accumulated AUCs over minibatches whose scores drift far apart
    (shifted, rescaled, all equal, then back) sum to the exact AUCs: the
    persistent bucket workspace carries nothing between calls but counts
    it re-arms."""
    g = torch.Generator().manual_seed(8)
    acc = torch.zeros(1, dtype=torch.float64, device=DEV)
    tot = 0.0
    base = torch.randn(100000, generator=g)
    for py in (base, base + 50.0, base * 1e-3, torch.full((60000,), 0.25), base, -base,
               torch.round(base * 8) / 8):
        lab = (torch.rand(py.numel(), generator=g) < 0.3).float()
        tot += float(ref.auc(py, lab))
        hip.auc_acc(py.to(DEV), lab.to(DEV), acc)
        assert abs(float(acc) - tot) < 1e-8, (float(acc), tot)


def test_auc_side_host_threads_match_exact(hip):
    """auc_acc_side on large minibatches (the host-thread AUC: pinned copy on
    the side stream, exact AUC on a worker) interleaved over two sums, one
    small minibatch (the on-stream device path) among them: auc_join adds
    each sum's own AUCs, and freeing the inputs before the copy ran does
    not change them (the side stream holds them in the caching allocator)."""
    hip.auc_host_threads(2)
    try:
        _auc_side_checks(hip)
    finally:
        hip.auc_host_threads(0)
    _auc_side_checks(hip)  # and the device chain on the side stream


def _auc_side_checks(hip):
    g = torch.Generator().manual_seed(9)
    a = torch.zeros(1, dtype=torch.float64, device=DEV)
    b = torch.zeros(1, dtype=torch.float64, device=DEV)
    ta = tb = 0.0
    base = torch.randn(100000, generator=g)
    for k, py in enumerate((base, torch.sigmoid(base * 3), base[:3000], torch.full((50000,), 0.5),
                            torch.round(base * 4) / 4, -base, base * 1e-4)):
        lab = (torch.rand(py.numel(), generator=g) < 0.35).float()
        r = float(ref.auc(py, lab))
        pyd, labd = py.to(DEV), lab.to(DEV)
        if k % 2:
            tb += r
            hip.auc_acc_side(pyd, labd, b)
        else:
            ta += r
            hip.auc_acc_side(pyd, labd, a)
        del pyd, labd  # freed while the copy may still be queued: the allocator
        torch.empty(100000, device=DEV).fill_(7.0)  # must not hand them out before it
    hip.auc_join(a)
    hip.auc_join(b)
    assert abs(float(a) - ta) < 1e-9, (float(a), ta)
    assert abs(float(b) - tb) < 1e-9, (float(b), tb)
    hip.auc_join(a)  # nothing pending: unchanged
    assert abs(float(a) - ta) < 1e-9


@pytest.mark.parametrize("nshard", [1, 8])
def test_localize_few_distinct_ids_many_partitions(hip, nshard):
    """~2M non-zeros over 2000 power-law ids (the shape of bench_e2e.py's
    Criteo text: few distinct ids, heavy duplication): the plan splits them
    into many partitions of few ids (<= ~16K non-zeros each) and single-id
    partitions for the hot ids elected by the previous call; every output
    still matches the reference."""
    keys, off, _, _ = _rand_batch(50000, 20, 2000, 11, False, skew=True)
    k, o = keys.to(DEV), off.to(DEV)
    hint = 0
    for _ in range(3):  # the second and third calls use the elected hot ids
        uniq, ucnt, owner_cnt, lid = hip.localize(k, o, None, nshard, hint)[:4]
        hint = uniq.numel()
        ru = torch.unique(keys)
        assert torch.equal(torch.sort(uniq.cpu()).values, ru)
        assert torch.equal(uniq[lid.long()].cpu(), keys)
        assert torch.equal(ucnt.cpu().long(), torch.bincount(lid.long().cpu(), minlength=hint))
        own = ref.owner_of(uniq.cpu(), nshard)
        assert torch.equal(torch.bincount(own, minlength=nshard), owner_cnt)
