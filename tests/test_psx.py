"""The lean multi-shard DiFacto step (kv/psx.py, csrc/hip/psx.hip).

* loopback P shards in one process with max_concurrency=1 (staleness 0)
  computes the same model as the single-shard fused path;
* the default pipelined step (staleness 1) trains and drains cleanly;
* 2 ranks over gloo: the owners' feature counts are exactly the total
  occurrences over both workers, every embedding row exists where the count
  crossed the threshold, and every worker pulls exactly the owner's values;
* the HIP kernels of the same path match the host oracle (GPU).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

CARD = [50, 400, 3000, 20, 7, 900]


def _conf(max_conc=2, l1_shrk=False, dim=8, thr=3, opts=""):
    """opts: "fb<n>" the fixed_bytes filter, "clip" / "drop" / "norm" the
    embedding-gradient post-processing (learn/difacto/loss.h:145-155)."""
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    emb = Embedding(dim=dim, threshold=thr)
    if "clip" in opts:
        emb.grad_clipping = 0.05
    if "drop" in opts:
        emb.dropout = 0.1
    if "norm" in opts:
        emb.grad_normalization = True
    fb = int(opts[opts.index("fb") + 2]) if "fb" in opts else 0
    return DifactoConfig(embedding=[emb], lambda_l1=0.01, l1_shrk=l1_shrk,
                         max_concurrency=max_conc, fixed_bytes=fb)


def _run(comm, conf, device, steps=6, rows=300, seed=17, nxt=True, nshard=None):
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner
    lr = DifactoLearner(conf, comm, device, cap=1 << 14, vcap=1 << 12, seed=5, nshard=nshard)
    batches = [[t.to(device) for t in criteo_batch_cpu(rows, seed, s, CARD)] for s in range(steps)]
    for s, (keys, label, off) in enumerate(batches):
        nb = None
        if nxt and s + 1 < steps:
            nb = (batches[s + 1][0], batches[s + 1][2], None)
        lr.process(keys, off, None, label, 0, 0, next_batch=nb)
    lr.flush()  # (collective on several ranks; take_progress itself stays local)
    prog = lr.take_progress()
    return lr, prog, batches


def _model(lr):
    st = lr.store
    occ = st.occupied().long()
    keys = st.keys[occ.to(st.keys.device)].cpu().tolist()
    w = st.w[occ.to(st.w.device)].cpu().tolist()
    cnt = st.cnt[occ.to(st.cnt.device)].cpu().tolist()
    vrow = st.vrow[occ.to(st.vrow.device)].cpu().tolist()
    V = st.V.cpu()
    out = {}
    for k, ww, c, r in zip(keys, w, cnt, vrow):
        out[int(np.int64(k))] = (float(ww), int(c), None if r < 0 else V[r][:lr.dim].clone())
    return out


def test_loopback_strict_matches_single_shard():
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    one, p1, _ = _run(Comm("cpu", init=False), _conf(max_conc=1), "cpu")
    lb, p4, _ = _run(LoopbackComm(4, "cpu"), _conf(max_conc=1), "cpu")
    assert lb.psx is not None and one.psx is None
    m1, m4 = _model(one), _model(lb)
    assert m1.keys() == m4.keys()
    for k, (w, c, v) in m1.items():
        w4, c4, v4 = m4[k]
        assert c == c4, k
        assert abs(w - w4) < 1e-5, (k, w, w4)
        assert (v is None) == (v4 is None), k
        if v is not None:
            assert torch.allclose(v, v4, atol=1e-5), k
    for a, b in zip(p1, p4):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (p1, p4)


def test_embedding_free_difacto_loopback_matches_single_shard():
    """A DiFacto model without an embedding takes the multi-shard step's
    linear wire format; the owner push applies DiFacto's FTRL on w (algo 4,
    learn/difacto/async_sgd.h:262-286): the same model as one shard."""
    from wormhole_amd.config.schema import DifactoConfig
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    conf = lambda: DifactoConfig(lambda_l1=0.01, lambda_l2=0.1, max_concurrency=1)  # noqa
    one, p1, _ = _run(Comm("cpu", init=False), conf(), "cpu")
    lb, p4, _ = _run(LoopbackComm(4, "cpu"), conf(), "cpu")
    assert lb.psx is not None and lb.psx.linear and lb.psx.lin_hp[0] == 4
    m1, m4 = _model(one), _model(lb)
    assert m1.keys() == m4.keys() and len(m1) > 100
    assert sum(1 for w, _, _ in m1.values() if w != 0.0) > 10
    for k, (w, c, v) in m1.items():
        assert abs(w - m4[k][0]) < 1e-6, (k, w, m4[k][0])
    for a, c in zip(p1, p4):
        assert abs(a - c) <= 1e-4 * max(1.0, abs(a)), (p1, p4)


def test_loopback_pipelined_trains_and_drains():
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    lb, prog, batches = _run(LoopbackComm(3, "cpu"), _conf(), "cpu", steps=8)
    assert lb.psx.tau == 1
    assert lb.psx.pull is None and lb.psx.push is None and lb.psx.job is None
    assert prog[4] == 8 and prog[5] == 8 * 300  # every minibatch forwarded once
    one, prog1, _ = _run(Comm("cpu", init=False), _conf(), "cpu", steps=8)
    # staleness 1 perturbs the trajectory only slightly on this problem
    assert abs(prog[0] / prog[5] - prog1[0] / prog1[5]) < 0.02
    m, m1 = _model(lb), _model(one)
    assert m.keys() == m1.keys()
    # counts are exact regardless of the pipelining
    assert all(m[k][1] == m1[k][1] for k in m1)
    assert all((m[k][2] is None) == (m1[k][2] is None) for k in m1)


def test_loopback_without_lookahead():
    """next_batch omitted: every call begins its own localize; same model
    as with the lookahead."""
    from wormhole_amd.parallel.comm import LoopbackComm
    a, pa, _ = _run(LoopbackComm(2, "cpu"), _conf(), "cpu", nxt=True)
    b, pb, _ = _run(LoopbackComm(2, "cpu"), _conf(), "cpu", nxt=False)
    ma, mb = _model(a), _model(b)
    assert ma.keys() == mb.keys()
    for k in ma:
        assert ma[k][0] == mb[k][0] and ma[k][1] == mb[k][1]
    assert pa == pb


def test_loopback_validation_pass():
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.parallel.comm import LoopbackComm
    lb, _, _ = _run(LoopbackComm(3, "cpu"), _conf(), "cpu", steps=4)
    nkeys = len(_model(lb))
    keys, label, off = criteo_batch_cpu(200, 99, 0, CARD)
    py = lb.process(keys, off, None, label, 2, 0)  # PRED: no insert, no push
    assert py.shape == (200,) and bool(torch.isfinite(py).all())
    assert len(_model(lb)) == nkeys


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _two_rank_main(rank, world, port, out_dir, device, max_conc, nshard=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from wormhole_amd import ops
    from wormhole_amd.parallel.comm import Comm
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(0)
        comm = Comm(dev, backend="gloo")
    else:
        comm = Comm(dev)
    lr, prog, batches = _run(comm, _conf(max_conc=max_conc), dev, steps=6, seed=17 + rank,
                             nshard=nshard)
    assert lr.psx is not None
    if nshard is not None and rank >= nshard:
        assert not _model(lr)  # a worker that owns no shard stores nothing
    # every key's count on its owner = its occurrences over all workers
    occ = {}
    for keys, _, _ in batches:
        u, c = torch.unique(keys.cpu(), return_counts=True)
        for k, n in zip(u.tolist(), c.tolist()):
            occ[k] = occ.get(k, 0) + n
    allocc = comm.allgather_object(occ)
    mine = _model(lr)
    allm = comm.allgather_object({k: (w, c, None if v is None else v.tolist())
                                  for k, (w, c, v) in mine.items()})
    tot, owner = {}, {}
    for o in allocc:
        for k, n in o.items():
            tot[k] = tot.get(k, 0) + n
    for m in allm:
        assert not (owner.keys() & m.keys())  # each key lives on one shard
        owner.update(m)
    assert owner.keys() == tot.keys()
    for k, n in tot.items():
        w, c, v = owner[k]
        assert c == n, (k, c, n)
        assert (v is not None) == (n > 3), (k, n)
    # a fresh read-only pull through the exchange sees the owners' values
    uniq, wp, rows = lr.psx.pull_values(batches[-1][0].to(dev))
    rows = rows.cpu()
    for i, k in enumerate(uniq.cpu().tolist()):
        w, c, v = owner[k]
        assert abs(float(wp[i]) - w) < 1e-7
        if v is None:
            assert float(rows[i].abs().sum()) == 0.0
        else:
            assert torch.equal(rows[i, :len(v)], torch.tensor(v, dtype=torch.float32))
    comm.barrier()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("%r\n" % (prog[0] / prog[5]))
    comm.finalize()


@pytest.mark.parametrize("max_conc,nshard", [(1, None), (2, None), (2, 1)])
def test_psx_two_ranks_gloo(tmp_path, max_conc, nshard):
    """(nshard = 1: the demo's `-n 2 -s 1`, one server shard, two workers)"""
    mp.spawn(_two_rank_main, args=(2, _free_port(), str(tmp_path), "cpu", max_conc, nshard),
             nprocs=2, join=True)
    for r in range(2):
        assert 0 < float(open(tmp_path / ("r%d" % r)).read()) < 1.0


@pytest.mark.gpu
def test_psx_two_ranks_gpu_staged(tmp_path):
    """The same multi-rank invariants with the HIP kernels (2 ranks sharing
    the GPU, transfers staged through gloo)."""
    mp.spawn(_two_rank_main, args=(2, _free_port(), str(tmp_path), "cuda", 2), nprocs=2,
             join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("max_conc", [1, 2])
def test_loopback_gpu_matches_cpu(max_conc):
    """Loopback P=4 through the HIP kernels vs the host oracle: no duplicates
    across segments, so the model must agree to float tolerance."""
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    g, pg, _ = _run(LoopbackComm(4, dev), _conf(max_conc=max_conc), dev, steps=6, rows=2000)
    c, pc, _ = _run(LoopbackComm(4, "cpu"), _conf(max_conc=max_conc), "cpu", steps=6, rows=2000)
    mg, mc = _model(g), _model(c)
    assert mg.keys() == mc.keys()
    bad = 0
    for k, (w, cn, v) in mc.items():
        wg, cg, vg = mg[k]
        assert cn == cg, k
        assert (v is None) == (vg is None), k
        if abs(w - wg) > 1e-4 or (v is not None and not torch.allclose(v, vg, atol=1e-4)):
            bad += 1
    assert bad == 0, bad
    assert abs(pg[0] / pg[5] - pc[0] / pc[5]) < 1e-4


def _rccl_loopback_main(rank, port, out_dir, model, max_conc):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    rc = LoopbackComm(4, dev, rccl=True)
    assert rc.backend == "loopback-rccl"
    if model == "difacto":
        a, pa, _ = _run(rc, _conf(max_conc=max_conc), dev, steps=6, rows=2000)
        b, pb, _ = _run(LoopbackComm(4, dev), _conf(max_conc=max_conc), dev, steps=6, rows=2000)
        assert a.psx._nat and b.psx._nat  # the native step, over RCCL and the identity
        ma, mb = _model(a), _model(b)
        assert ma.keys() == mb.keys()
        for k, (w, c, v) in mb.items():
            wa, ca, va = ma[k]
            assert c == ca and (v is None) == (va is None), k
            assert abs(w - wa) <= 1e-5 and (v is None or torch.allclose(v, va, atol=1e-5)), k
        assert abs(pa[0] / pa[5] - pb[0] / pb[5]) < 1e-5
    else:
        a, pa, bt = _lin_run(rc, dev, 3, steps=6, rows=2000, max_conc=max_conc)
        b, pb, _ = _lin_run(LoopbackComm(4, dev), dev, 3, max_conc=max_conc, batches=bt)
        assert a.psx._nat and b.psx._nat
        ma, mb = _lin_model(a), _lin_model(b)
        assert ma.keys() == mb.keys() and len(ma) > 1000
        for k, w in mb.items():
            assert abs(w - ma[k]) <= 1e-5 * max(1.0, abs(w)), k
        assert abs(pa[0] / pa[4] - pb[0] / pb[4]) < 1e-5
    # the wire tally counts what crosses to the (virtual) peers
    assert sum(a.psx._nat.wire()) > 0
    rc.finalize()
    with open(os.path.join(out_dir, "ok"), "w") as f:
        f.write("ok\n")


@pytest.mark.gpu
@pytest.mark.parametrize("model,max_conc", [("difacto", 1), ("difacto", 2), ("linear", 1),
                                            ("linear", 2)])
def test_loopback_rccl_transport(tmp_path, model, max_conc):
    """The native multi-shard step over its own RCCL communicator (1 rank,
    every virtual peer's segment a grouped ncclSend / ncclRecv to self) trains
    the same model as the identity loopback: the stream ordering of C0-C3
    against the compute and side streams holds under RCCL."""
    mp.spawn(_rccl_loopback_main, args=(_free_port(), str(tmp_path), model, max_conc),
             nprocs=1, join=True)
    assert (tmp_path / "ok").read_text() == "ok\n"


def _lockstep(lr, batches, cap=64):
    """Every rank steps in lockstep: a rank past its own minibatches passes
    empty ones (solver/ps.py run_pass), always with a look-ahead (the SAME
    tensor objects the next call gets), until a call reports that no rank
    had data."""
    dev = batches[0][0].device if batches else lr.device
    items = [(k, o, lab) for k, lab, o in batches]
    items += [(torch.zeros(0, dtype=torch.int64, device=dev),
               torch.zeros(1, dtype=torch.int64, device=dev),
               torch.zeros(0, dtype=torch.float32, device=dev)) for _ in range(cap + 1)]
    for i in range(cap):
        k, o, lab = items[i]
        nk, no, _ = items[i + 1]
        lr.process(k, o, None, lab, 0, 0, next_batch=(nk, no, None))
        if lr.last_empty:
            break
    else:
        raise AssertionError("no empty step within %d calls" % cap)
    lr.flush()
    return lr.take_progress()


def _staged_main(rank, world, port, out_dir, model, max_conc, opts=""):
    """One rank of a gloo-staged group on the shared GPU: the native step
    (kTxStaged) and the Python step train on the same uneven data (rank r
    has 6 - r minibatches of 300 + 100 r rows); this rank's shard must agree."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.models.linear import LinearLearner
    from wormhole_amd.parallel.comm import Comm
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = Comm(dev, backend="gloo")
    assert comm.stage
    mine = [[t.to(dev) for t in criteo_batch_cpu(300 + 100 * rank, 31 + rank, s, CARD)]
            for s in range(6 - rank)]
    res = {}
    for native in ("0", "1"):
        os.environ["WH_PSX_NATIVE"] = native
        if model == "difacto":
            lr = DifactoLearner(_conf(max_conc=max_conc, opts=opts), comm, dev, cap=1 << 14,
                                vcap=1 << 12, seed=5)
        else:
            fb = int(opts[opts.index("fb") + 2]) if "fb" in opts else 0
            lr = LinearLearner(LinearConfig(algo=3, lambda_l1=0.1, lr_eta=0.1,
                                            max_concurrency=max_conc, fixed_bytes=fb), comm, dev,
                               cap=1 << 14, seed=5)
        prog = _lockstep(lr, mine)
        assert bool(lr.psx._nat) == (native == "1")
        res[native] = (_model(lr) if model == "difacto" else _lin_model(lr), prog)
    (mp_, pp), (mn, pn) = res["0"], res["1"]
    assert mp_.keys() == mn.keys() and len(mp_) > 100
    if model == "difacto":
        # The embedding rows are compared at 1e-2: two runs of the SAME step
        # differ there by up to 3e-3 (measured; float-atomic order in the
        # backward, then AdaGrad's first steps ~eta * sign(g) on near-zero
        # gradients); keys, counts and allocation are exact, w to 1e-4.
        kinds = {"count": 0, "w": 0, "has_v": 0, "v": 0}
        ex = []
        for k, (w, c, v) in mp_.items():
            wn, cn, vn = mn[k]
            kind = ("count" if c != cn else "has_v" if (v is None) != (vn is None) else
                    "w" if abs(w - wn) > 1e-4 * max(1.0, abs(w)) else
                    "v" if v is not None and not torch.allclose(v, vn, atol=1e-2) else None)
            if kind:
                kinds[kind] += 1
                if len(ex) < 4:
                    ex.append((k, kind, c, cn, w, wn))
        bad = sum(kinds.values())
        assert kinds["count"] == 0 and kinds["has_v"] == 0, (kinds, ex)
        nmb = pn[4]
    else:
        bad = sum(1 for k, w in mp_.items() if abs(w - mn[k]) > 1e-4 * max(1.0, abs(w)))
        kinds, ex = {"w": bad}, []
        nmb = pn[3]
    assert bad <= max(2, len(mp_) // 1000), (bad, len(mp_), kinds, ex)
    assert nmb == 6 - rank  # every minibatch of this rank forwarded exactly once
    # (the per-minibatch AUC of an early model ranks near-tied predictions:
    # 1e-6 differences in them move it by up to ~1 %)
    i_auc = 1 if model == "difacto" else 2
    for i, (a, c) in enumerate(zip(pn, pp)):
        tol = 0.02 * nmb if i == i_auc else 1e-3 * max(1.0, abs(a))
        assert abs(a - c) <= tol, (i, pn, pp)
    comm.barrier()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("ok\n")
    comm.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("world,model,max_conc,opts", [
    (2, "difacto", 2, ""), (2, "difacto", 1, ""), (2, "linear", 2, ""), (3, "difacto", 2, ""),
    (3, "linear", 1, ""), (4, "difacto", 2, ""), (5, "linear", 2, ""),
    (2, "difacto", 2, "fb1clip"), (3, "difacto", 1, "fb2dropnorm"), (2, "linear", 2, "fb1")])
def test_native_step_multi_process_staged(tmp_path, world, model, max_conc, opts):
    """The native multi-shard step in 2 to 5 processes (ranks sharing the
    GPU, transfers staged through gloo), uneven data per rank: every rank's
    shard equals the one the Python step trains on the same data, and every
    minibatch is forwarded once (learn/difacto/async_sgd.h:363-425 with W
    workers and S = W servers)."""
    mp.spawn(_staged_main, args=(world, _free_port(), str(tmp_path), model, max_conc, opts),
             nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok\n"


@pytest.mark.gpu
@pytest.mark.parametrize("max_conc", [1, 2])
def test_loopback_gpu_long_run_crosses_tag_wrap(max_conc):
    """300 minibatches: the duplicate-chain tag epoch (8 bits, one per owner
    open) wraps and the table's tags are swept once; the multi-shard model
    still matches the single-shard fused path (counts and embedding
    allocation exactly, weights to float tolerance)."""
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    dev = torch.device("cuda", 0)
    steps = 300
    lb, plb, _ = _run(LoopbackComm(4, dev), _conf(max_conc=max_conc), dev, steps=steps, rows=1000)
    assert lb.store.ps_opens >= steps and lb.psx is not None  # the 255-epoch wrap crossed
    one, p1, _ = _run(Comm(dev, init=False), _conf(max_conc=max_conc), dev, steps=steps, rows=1000)
    m, m1 = _model(lb), _model(one)
    assert m.keys() == m1.keys()
    bad = 0
    for k, (w, c, v) in m1.items():
        w4, c4, v4 = m[k]
        assert c == c4, k
        assert (v is None) == (v4 is None), k
        if max_conc == 1 and (abs(w - w4) > 1e-3 or (v is not None and
                                                     not torch.allclose(v, v4, atol=1e-3))):
            bad += 1
    assert bad <= len(m1) // 1000, bad
    assert plb[4] == steps and plb[5] == steps * 1000
    assert abs(plb[0] / plb[5] - p1[0] / p1[5]) < (1e-3 if max_conc == 1 else 0.02)


# ---------------------------------------------------------------- linear
def _lin_run(comm, device, algo=3, steps=6, rows=300, seed=17, max_conc=1, nshard=None,
             batches=None, fixed_bytes=0):
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.linear import LinearLearner
    conf = LinearConfig(algo=algo, lambda_l1=0.1, lr_eta=0.1, max_concurrency=max_conc,
                        fixed_bytes=fixed_bytes)
    lr = LinearLearner(conf, comm, device, cap=1 << 14, seed=5, nshard=nshard)
    if batches is None:
        batches = [[t.to(device) for t in criteo_batch_cpu(rows, seed, s, CARD)]
                   for s in range(steps)]
    for s, (keys, label, off) in enumerate(batches):
        nb = (batches[s + 1][0], batches[s + 1][2], None) if s + 1 < len(batches) else None
        lr.process(keys, off, None, label, 0, 0, next_batch=nb)
    lr.flush()
    return lr, lr.take_progress(), batches


def _lin_model(lr):
    st = lr.store
    occ = st.occupied().long()
    keys = st.keys[occ.to(st.keys.device)].cpu().tolist()
    w = st.w[occ.to(st.w.device)].cpu().tolist()
    return {int(np.int64(k)): float(x) for k, x in zip(keys, w)}


@pytest.mark.parametrize("algo", [1, 2, 3])
def test_linear_loopback_strict_matches_single_shard(algo):
    """The linear model through the multi-shard step (P = 4 virtual shards,
    staleness 0) trains the same model as the single-shard path, for SGD,
    AdaGrad and FTRL (learn/linear/async_sgd.h:71-180)."""
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    one, p1, b = _lin_run(Comm("cpu", init=False), "cpu", algo)
    lb, p4, _ = _lin_run(LoopbackComm(4, "cpu"), "cpu", algo, batches=b)
    assert lb.psx is not None and lb.psx.linear and one.psx is None
    m1, m4 = _lin_model(one), _lin_model(lb)
    assert m1.keys() == m4.keys()
    if algo == 1:  # SGD's eta follows ps-lite's request count t: 4 per step here vs 1
        return
    for k, w in m1.items():
        assert abs(w - m4[k]) < 1e-5, (k, w, m4[k])
    for a, c in zip(p1, p4):
        assert abs(a - c) <= 1e-4 * max(1.0, abs(a)), (p1, p4)


def test_linear_loopback_pipelined():
    from wormhole_amd.parallel.comm import LoopbackComm
    lb, prog, _ = _lin_run(LoopbackComm(3, "cpu"), "cpu", max_conc=2, steps=8)
    assert lb.psx.tau == 1 and lb.psx.pull is None and lb.psx.push is None
    assert prog[3] == 8 and prog[4] == 8 * 300
    assert 0 < prog[0] / prog[4] < 1.0


def _lin_oracle(all_batches, algo, l1, alpha, beta, fixed_bytes=0, nshard=1):
    """Two workers in lockstep against one server, strict order: every step
    both pull the same model, then the owner applies worker 0's push, then
    worker 1's (ps-lite: one request at a time). fixed_bytes: each worker's
    pushed gradients pass through the payload filter's quantisation (the
    host reference of the wire format, same records, seeds and rounding)."""
    from wormhole_amd import _native
    from wormhole_amd.kv.cpu_store import CpuKVStore
    from wormhole_amd.kv.psx import _QFilter
    from wormhole_amd.ops import ref
    st = CpuKVStore(1 << 16, 0, 0)
    host = _native.host()
    qf = [_QFilter(fixed_bytes, 0, 5, r, True) for r in range(len(all_batches))] \
        if fixed_bytes else None
    t = 0
    for step in range(len(all_batches[0])):
        pend = []
        for r in range(len(all_batches)):
            keys, label, off = all_batches[r][step]
            uniq, ucnt, oc, lid, co, cr, cv = host.localize_cpu(keys, off, None, nshard)
            slot = st.find(uniq, True)
            w = st.linear_pull(slot)
            met = torch.zeros(5, dtype=torch.float64)
            py, dual, _ = ref.fm_forward(off, lid, None, w, None, 0, label, 2, met)
            g, _ = ref.fm_backward(co, cr, cv, dual, None, w, None, 0)
            if qf is not None:
                n = [int(x) for x in oc[:nshard].tolist()] + [0] * (len(all_batches) - nshard)
                d, rows, _ = qf[r].layout(n, None, None)
                q = ref.ps_qpack(g, d, sum(rows), qf[r].W, fixed_bytes, qf[r].next_seed())
                g = ref.ps_qunpack(q, d, qf[r].W, fixed_bytes, torch.zeros_like(g))
            pend.append((slot, g))
        for slot, g in pend:
            t += 1
            st.linear_push(slot, g, algo, alpha, beta, l1, 0.0, (beta + t ** 0.5) / alpha)
    return {int(k): float(x) for k, x in zip(st.keys.tolist(), st.w.tolist())}


def _lin_two_rank_main(rank, world, port, out_dir, nshard, algo, fixed_bytes=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.parallel.comm import Comm
    comm = Comm("cpu")
    mine = [[t for t in criteo_batch_cpu(300, 17 + rank, s, CARD)] for s in range(5)]
    lr, prog, _ = _lin_run(comm, "cpu", algo=algo, max_conc=1, nshard=nshard, batches=mine,
                           fixed_bytes=fixed_bytes)
    assert (lr.psx.qf is not None) == bool(fixed_bytes)
    assert lr.psx is not None and lr.psx.nshard == nshard
    model = _lin_model(lr)
    if rank >= nshard:
        assert not model  # a worker that owns no shard stores nothing
    allm = comm.allgather_object(model)
    allb = comm.allgather_object(mine)
    owner = {}
    for m in allm:
        assert not (owner.keys() & m.keys())
        owner.update(m)
    ref_m = _lin_oracle(allb, algo, 0.1, 0.1, 1.0, fixed_bytes, nshard)
    assert owner.keys() == ref_m.keys()
    for k, w in ref_m.items():
        assert abs(owner[k] - w) < 1e-5, (k, owner[k], w)
    comm.barrier()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("ok\n")
    comm.finalize()


@pytest.mark.parametrize("nshard,algo", [(2, 3), (1, 3), (2, 1), (1, 2)])
def test_linear_two_ranks_gloo_matches_oracle(tmp_path, nshard, algo):
    """2 workers over gloo, S = 2 or 1 server shards (`-n 2 -s 1`): the
    owners' weights equal a host oracle of two lockstep workers pushing to
    one server in worker order, for FTRL, SGD (ps-lite's request count t)
    and AdaGrad."""
    mp.spawn(_lin_two_rank_main, args=(2, _free_port(), str(tmp_path), nshard, algo), nprocs=2,
             join=True)
    for r in range(2):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok\n"


@pytest.mark.parametrize("nshard,nb", [(2, 2), (1, 1)])
def test_linear_fixed_bytes_two_ranks_matches_quantized_oracle(tmp_path, nshard, nb):
    """FIXING_FLOAT on the linear push (learn/linear/async_sgd.h:290-301):
    the owners' weights equal the lockstep oracle whose pushes pass through
    the same n-byte records (quantise -> dequantise, same seeds)."""
    mp.spawn(_lin_two_rank_main, args=(2, _free_port(), str(tmp_path), nshard, 3, nb),
             nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok\n"


@pytest.mark.gpu
@pytest.mark.parametrize("algo,max_conc", [(3, 1), (2, 2), (1, 1)])
def test_linear_loopback_gpu_matches_cpu(algo, max_conc):
    """The linear multi-shard step through the HIP kernels (ps_open on a
    linear store, the chain-ordered ps_push_linear) vs the host oracle."""
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    g, pg, b = _lin_run(LoopbackComm(4, dev), dev, algo, steps=6, rows=2000, max_conc=max_conc)
    c, pc, _ = _lin_run(LoopbackComm(4, "cpu"), "cpu", algo, max_conc=max_conc,
                        batches=[[t.cpu() for t in x] for x in b])
    mg, mc = _lin_model(g), _lin_model(c)
    assert mg.keys() == mc.keys()
    # (float contraction and gradient summation order differ between the
    # device and the host: a weight near the L1 threshold may land on the
    # other side of it)
    bad = sum(1 for k, w in mc.items() if abs(w - mg[k]) > 1e-4 * max(1.0, abs(w)))
    assert bad <= len(mc) // 1000, bad
    assert abs(pg[0] / pg[4] - pc[0] / pc[4]) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("model,max_conc,opts", [
    ("difacto", 2, ""), ("difacto", 1, ""), ("linear", 2, ""), ("linear", 1, ""),
    ("difacto", 2, "fb1"), ("difacto", 1, "fb3clipdrop"), ("difacto", 2, "clipnorm"),
    ("linear", 2, "fb2")])
def test_native_step_matches_python_step(model, max_conc, opts, monkeypatch):
    """The C++ driver of the multi-shard step (csrc/bind/psx_native.inl
    PsxStep) trains the same model as the Python step it ports (kv/psx.py
    Psx.train, WH_PSX_NATIVE=0), pipelined and strict, on 4 loopback shards;
    with the fixed_bytes filter (the same stochastic-rounding seeds in the
    same order) and the embedding-gradient post-processing too."""
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    runs = {}
    for native in ("1", "0"):
        monkeypatch.setenv("WH_PSX_NATIVE", native)
        if model == "difacto":
            lr, prog, b = _run(LoopbackComm(4, dev), _conf(max_conc=max_conc, opts=opts), dev,
                               steps=8, rows=3000)
            runs[native] = (_model(lr), prog, bool(lr.psx._nat))
        else:
            fb = int(opts[opts.index("fb") + 2]) if "fb" in opts else 0
            lr, prog, b = _lin_run(LoopbackComm(4, dev), dev, 3, steps=8, rows=3000,
                                   max_conc=max_conc, fixed_bytes=fb)
            runs[native] = (_lin_model(lr), prog, bool(lr.psx._nat))
    (mn, pn, isn), (mp_, pp, isp) = runs["1"], runs["0"]
    assert isn and not isp
    assert mn.keys() == mp_.keys() and len(mn) > 1000
    if model == "difacto":
        bad = sum(1 for k, (w, c, v) in mp_.items()
                  if c != mn[k][1] or abs(w - mn[k][0]) > 1e-4 * max(1.0, abs(w)) or
                  (v is None) != (mn[k][2] is None) or
                  (v is not None and not torch.allclose(v, mn[k][2], atol=1e-4)))
    else:
        bad = sum(1 for k, w in mp_.items() if abs(w - mn[k]) > 1e-4 * max(1.0, abs(w)))
    assert bad <= len(mp_) // 1000, bad
    for a, c in zip(pn, pp):
        assert abs(a - c) <= 1e-3 * max(1.0, abs(a)), (pn, pp)


def _c10d_main(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from wormhole_amd import _native
    send = [rank + 1 + q for q in range(world)]
    x = torch.cat([torch.full((send[q], 3), float(100 * rank + q)) for q in range(world)])
    recv = [p + 1 + rank for p in range(world)]
    out = _native.hip().c10d_a2a_rows(pg=dist.group.WORLD, x=x, send_rows=send, recv_rows=recv)
    o = 0
    for p in range(world):
        assert bool((out[o:o + recv[p]] == 100 * p + rank).all()), (rank, p)
        o += recv[p]
    dist.destroy_process_group()


def test_native_c10d_all_to_all_three_ranks():
    """The transport of the native step from C++: the Python process group
    object cast to c10d::ProcessGroup, a row-wise uneven alltoall_base and
    its work's wait (here over gloo between 3 CPU ranks; RCCL on GPUs)."""
    mp.spawn(_c10d_main, args=(3, _free_port()), nprocs=3, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("model,max_conc", [("difacto", 3), ("difacto", 4), ("linear", 3),
                                            ("linear", 4)])
def test_native_deep_pipeline_bounded_drift(model, max_conc):
    """max_concurrency = tau + 1 > 2 (learn/solver/minibatch_solver.h:284-322:
    an arbitrary in-flight bound): the native step keeps tau pushes in flight,
    so a minibatch's pull misses at most the tau previous pushes. Against the
    strict order (max_concurrency 1): the same keys, feature counts and
    embedding allocation (both are exact at the open), every minibatch
    forwarded once, and the training loss within a small drift."""
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    if model == "difacto":
        deep, pd, b = _run(LoopbackComm(4, dev), _conf(max_conc=max_conc), dev, steps=12,
                           rows=2000)
        strict, ps, _ = _run(LoopbackComm(4, dev), _conf(max_conc=1), dev, steps=12, rows=2000)
        md, ms = _model(deep), _model(strict)
        assert all(md[k][1] == c and (md[k][2] is None) == (v is None)
                   for k, (w, c, v) in ms.items())
        i_n, i_ex = 4, 5
    else:
        deep, pd, b = _lin_run(LoopbackComm(4, dev), dev, 3, steps=12, rows=2000,
                               max_conc=max_conc)
        strict, ps, _ = _lin_run(LoopbackComm(4, dev), dev, 3, max_conc=1, batches=b)
        md, ms = _lin_model(deep), _lin_model(strict)
        i_n, i_ex = 3, 4
    assert deep.psx._nat and deep.psx.tau_max == max_conc - 1
    assert md.keys() == ms.keys()
    assert pd[i_n] == ps[i_n] == 12 and pd[i_ex] == ps[i_ex]
    # (a drift that grows with the staleness: 12 minibatches, tau of them stale)
    assert abs(pd[0] / pd[i_ex] - ps[0] / ps[i_ex]) < 0.02 * (max_conc - 1)
    assert not deep.psx._nat.busy  # flushed: every push applied


def test_max_concurrency_out_of_range_is_an_error():
    from wormhole_amd.parallel.comm import LoopbackComm
    with pytest.raises(ValueError, match="max_concurrency"):
        _run(LoopbackComm(2, "cpu"), _conf(max_conc=10), "cpu", steps=1)
    # the Python step pipelines one deep under any larger bound
    lb, _, _ = _run(LoopbackComm(2, "cpu"), _conf(max_conc=4), "cpu", steps=3)
    assert lb.psx.tau == 1 and lb.psx.tau_max == 3


def _rccl_a2av_main(rank, out_dir):
    from wormhole_amd import _native
    hip = _native.hip()
    torch.cuda.set_device(0)
    c = hip.RcclComm(bytes(hip.RcclComm.unique_id()), 1, 0, 0)
    assert c.size == 1 and c.rank == 0
    g = torch.Generator().manual_seed(3)
    for rows, width, dt in (([5, 0, 7, 1], 3, torch.float32), ([2, 2, 2, 2, 2, 2, 2, 2], 1,
                                                               torch.int64),
                            ([0, 0, 9], 16, torch.float32)):
        n = sum(rows)
        x = torch.randint(-1 << 20, 1 << 20, (n, width), generator=g).to(dt).cuda()
        y = c.a2av(x, rows, rows)  # 1 rank, len(rows) virtual peers: the identity
        torch.cuda.synchronize()
        assert y.shape == x.shape and torch.equal(x, y), rows
    c.close()
    with open(os.path.join(out_dir, "ok"), "w") as f:
        f.write("ok\n")


@pytest.mark.gpu
def test_rccl_comm_virtual_peers_identity(tmp_path):
    """RcclComm.a2av on a 1-rank communicator with P virtual peers (segment 0
    the own copy, the rest send / recv pairs to self): every row arrives
    where it left, for uneven and empty segments and any row width."""
    mp.spawn(_rccl_a2av_main, args=(str(tmp_path),), nprocs=1, join=True)
    assert (tmp_path / "ok").read_text() == "ok\n"
