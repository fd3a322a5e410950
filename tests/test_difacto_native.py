"""The single-shard DiFacto step in one native call (csrc/bind/
difacto_step.inl DifactoStep) against the op-by-op Python step it replaces
(models/difacto.py, WH_DIFACTO_NATIVE=0): the same model -- keys, feature
counts and embedding allocation exactly, w and V to float tolerance -- the
same progress, with and without the look-ahead localize, with the gradient
post-processing, over a validation pass, and with a table that has to grow
(learn/difacto/async_sgd.h:363-425 on one server shard)."""
import pytest
import torch

from test_psx import CARD, _conf, _model

pytestmark = pytest.mark.gpu


def _train(native, conf, steps=10, rows=2000, nxt=True, cap=1 << 16, val_steps=0,
           monkeypatch=None):
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner, VAL
    from wormhole_amd.parallel.comm import Comm
    monkeypatch.setenv("WH_DIFACTO_NATIVE", "1" if native else "0")
    dev = torch.device("cuda", 0)
    lr = DifactoLearner(conf, Comm(dev, init=False), dev, cap=cap, vcap=1 << 12, seed=5)
    assert (lr._nat is not None) == native
    b = [[t.to(dev) for t in criteo_batch_cpu(rows, 17, s, CARD)] for s in range(steps)]
    for s, (keys, label, off) in enumerate(b):
        nb = (b[s + 1][0], b[s + 1][2], None) if nxt and s + 1 < steps else None
        lr.process(keys, off, None, label, 0, 0, next_batch=nb)
    lr.flush()
    prog = lr.take_progress()
    vprog = None
    if val_steps:
        v = [[t.to(dev) for t in criteo_batch_cpu(rows, 99, s, CARD)] for s in range(val_steps)]
        for keys, label, off in v:
            lr.process(keys, off, None, label, VAL, 0)
        vprog = lr.take_progress()
    return lr, prog, vprog


def _same(a, b, vtol=1e-4):
    ma, mb = _model(a), _model(b)
    assert ma.keys() == mb.keys() and len(ma) > 500
    bad = 0
    for k, (w, c, v) in ma.items():
        wb, cb, vb = mb[k]
        assert c == cb and (v is None) == (vb is None), k
        if abs(w - wb) > 1e-4 * max(1.0, abs(w)) or (v is not None and
                                                     not torch.allclose(v, vb, atol=vtol)):
            bad += 1
    assert bad <= len(ma) // 1000, bad


@pytest.mark.parametrize("opts,nxt", [("", True), ("", False), ("clipdropnorm", True),
                                      ("clip", True)])
def test_native_difacto_step_matches_python_step(opts, nxt, monkeypatch):
    runs = [_train(n, _conf(max_conc=2, opts=opts), nxt=nxt, monkeypatch=monkeypatch)
            for n in (True, False)]
    (ln, pn, _), (lp, pp, _) = runs
    assert ln._nat.direct == (opts == "")
    _same(ln, lp)
    for i, (a, c) in enumerate(zip(pn, pp)):
        tol = 0.02 * pn[4] if i == 1 else 1e-3 * max(1.0, abs(a))  # (AUC of near-tied scores)
        assert abs(a - c) <= tol, (i, pn, pp)
    assert pn[4] == 10


def test_native_difacto_step_validation_and_growth(monkeypatch):
    """A table that starts at 4096 slots grows under the native guard; a
    validation pass after training forwards without inserting."""
    runs = [_train(n, _conf(max_conc=2), cap=1 << 12, val_steps=3, monkeypatch=monkeypatch)
            for n in (True, False)]
    (ln, pn, vn), (lp, pp, vp) = runs
    assert ln.kv.guard.grows >= 1 and lp.kv.guard.grows >= 1
    _same(ln, lp)
    assert vn[4] == vp[4] == 3
    assert abs(vn[0] - vp[0]) <= 1e-3 * abs(vp[0])
