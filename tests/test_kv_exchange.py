"""Sharded KV over a 2-rank gloo group (the ps-lite server group re-expressed
as all-to-all-v): variable-length DiFacto pull/push exchange on CPU, and the
same multi-rank code path with the HIP kernels (2 ranks sharing the GPU,
tensors staged through gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_dir, defer=True, device="cpu", fixed_bytes=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from wormhole_amd import ops
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(0)
        comm = Comm(dev, backend="gloo")
    else:
        comm = Comm(dev)
    emb = Embedding(dim=8, threshold=3)
    conf = DifactoConfig(embedding=[emb], lambda_l1=0.01, l1_shrk=False, fixed_bytes=fixed_bytes,
                         max_concurrency=1)  # (staleness 0 on both exchange paths)
    card = [50, 400, 3000, 20, 7]
    lr = DifactoLearner(conf, comm, device, cap=1 << 14, vcap=1 << 12, seed=5)
    lr.defer_push = defer
    for step in range(4):
        keys, label, off = [t.to(dev) for t in criteo_batch_cpu(300, 17 + rank, step, card)]
        lr.process(keys, off, None, label, 0, 0)
    lr.flush()  # (the multi-shard step keeps its last minibatch in flight)
    # pull check: every worker sees the owner's stored values (through the
    # exchange's payload filter when fixed_bytes > 0)
    keys, label, off = [t.to(dev) for t in criteo_batch_cpu(300, 99 + rank, 0, card)]
    uniq, wp, rows = lr.psx.pull_values(keys)
    wp, rows, uniq = wp.cpu(), rows.cpu(), uniq.cpu()
    st = lr.store
    occ = st.occupied().long()
    sk = st.keys[occ.to(st.keys.device)].cpu().tolist()
    sw = st.w[occ.to(st.w.device)].cpu().tolist()
    sv = st.vrow[occ.to(st.vrow.device)].cpu().tolist()
    V = st.V.cpu()
    mine = {}
    for k, w, row in zip(sk, sw, sv):
        mine[int(np.int64(k))] = (float(w), None if row < 0 else V[row][:8].tolist())
    allmaps = comm.allgather_object(mine)
    owner = {}
    for mp_ in allmaps:
        owner.update(mp_)
    nv = 0
    for i, k in enumerate(uniq.tolist()):
        w_o, v_o = owner.get(k, (0.0, None))
        assert abs(float(wp[i]) - w_o) < 1e-7, (k, float(wp[i]), w_o)
        if v_o is None:
            assert float(rows[i].abs().sum()) == 0.0
        else:
            nv += 1
            # (fixed_bytes: rows arrive as n-byte fixed point, one scale per row)
            tol = 1e-8 if not fixed_bytes else 2.0 * max(abs(x) for x in v_o) / (
                (1 << (8 * fixed_bytes - 1)) - 1) + 1e-8
            assert torch.allclose(rows[i, :8], torch.tensor(v_o), atol=tol, rtol=0), k
    assert nv > 0
    prog = lr.take_progress()
    comm.barrier()
    comm.finalize()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("%r %d\n" % (prog[0] / prog[5], nv))
    torch.save({k: v for k, v in sorted(mine.items())}, os.path.join(out_dir, "m%d" % rank))


def test_difacto_sharded_pull_push_two_ranks(tmp_path):
    port = _free_port()
    mp.spawn(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        ll, nv = open(tmp_path / ("r%d" % r)).read().split()
        assert 0 < float(ll) < 1.0 and int(nv) > 0


@pytest.mark.gpu
def test_difacto_sharded_two_ranks_gpu(tmp_path):
    """The multi-rank path (owner-grouped localize, per-segment push, V-row
    renumbering) with the HIP kernels; same numbers as the CPU path."""
    g, c = tmp_path / "g", tmp_path / "c"
    g.mkdir(), c.mkdir()
    mp.spawn(_rank_main, args=(2, _free_port(), str(g), True, "cuda"), nprocs=2, join=True)
    mp.spawn(_rank_main, args=(2, _free_port(), str(c), True, "cpu"), nprocs=2, join=True)
    for r in range(2):
        lg, nvg = open(g / ("r%d" % r)).read().split()
        lc, nvc = open(c / ("r%d" % r)).read().split()
        assert int(nvg) == int(nvc) > 0
        assert abs(float(lg) - float(lc)) < 1e-4 * float(lc)
        mg, mc = torch.load(g / ("m%d" % r)), torch.load(c / ("m%d" % r))
        assert mg.keys() == mc.keys()
        for k in mc:
            assert abs(mg[k][0] - mc[k][0]) < 1e-4, k
            assert (mg[k][1] is None) == (mc[k][1] is None), k


def _localize_ex_main(rank, world, port, device):
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
    g = torch.Generator().manual_seed(rank)

    def count_exchange(owner_cnt):  # {keys for peer, own overflow flag} per peer
        P = comm.size
        send = torch.zeros(2 * P, dtype=torch.int64, device=owner_cnt.device)
        send[0:2 * P:2] = owner_cnt[:P]
        send[1::2] = owner_cnt[P]
        return comm.exchange_counts_dev(send)
    nnz = 20000
    keys = torch.randint(0, 1 << 40, (nnz,), generator=g).to(dev)
    off = torch.arange(0, nnz + 1, 4, dtype=torch.int64).to(dev)
    # rank 0 under-sizes its scratch table (hint 1): on the GPU it overflows
    # and BOTH ranks must retry the fused count exchange together
    hint = 1 if rank == 0 else 0
    a = ops.localize(keys, off, None, comm.size, hint, exchange=count_exchange)
    b = ops.localize(keys, off, None, comm.size, 0)
    # (the order of ids inside an owner group follows the GPU hash table,
    # which concurrent inserts may permute; the key of every nnz may not change)
    assert torch.equal(a[2].cpu(), b[2].cpu())
    assert torch.equal(torch.sort(a[0].cpu())[0], torch.sort(b[0].cpu())[0])
    assert torch.equal(a[0][a[3].long()].cpu(), keys.cpu())
    assert a[7] == comm.exchange_counts([int(x) for x in b[2].tolist()])
    comm.barrier()
    comm.finalize()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_localize_fused_count_exchange(device):
    mp.spawn(_localize_ex_main, args=(2, _free_port(), device), nprocs=2, join=True)


@pytest.mark.parametrize("nb", [1, 3])
def test_fixed_bytes_filter_two_ranks(tmp_path, nb):
    """ps-lite FIXING_FLOAT / TRUNCATE_FLOAT (conf fixed_bytes): embedding rows
    cross ranks as n-byte fixed point, counts as uint8; training still
    converges, and with 3 bytes it tracks the exact run closely."""
    q, e = tmp_path / "q", tmp_path / "e"
    q.mkdir(), e.mkdir()
    mp.spawn(_rank_main, args=(2, _free_port(), str(q), True, "cpu", nb), nprocs=2, join=True)
    mp.spawn(_rank_main, args=(2, _free_port(), str(e), True, "cpu", 0), nprocs=2, join=True)
    for r in range(2):
        lq, nvq = open(q / ("r%d" % r)).read().split()
        le, nve = open(e / ("r%d" % r)).read().split()
        assert 0 < float(lq) < 1.0 and int(nvq) > 0
        if nb == 3:
            assert abs(float(lq) - float(le)) < 1e-3 * float(le)


def test_quant_rows_roundtrip():
    from wormhole_amd.ops import ref
    g = torch.Generator().manual_seed(3)
    x = torch.randn(300, 64, generator=g) * torch.rand(300, 1, generator=g)
    x[5] = 0
    for nb in (1, 2, 3):
        q = ref.quant_rows(x, nb, 7)
        assert q.shape == (300, ref.quant_record_bytes(64, nb)) and q.dtype == torch.uint8
        y = ref.dequant_rows(q, 64, nb)
        lim = (1 << (8 * nb - 1)) - 1
        step = x.abs().max(1, keepdim=True).values / lim
        assert bool(((y - x).abs() <= step * 1.001 + 3e-7 * x.abs() + 1e-9).all())
        assert bool((y[5] == 0).all())
    # unbiased random rounding: the mean error over many seeds vanishes
    x1 = torch.full((1, 64), 0.3)
    x1[0, 0] = 1.0
    ys = torch.stack([ref.dequant_rows(ref.quant_rows(x1, 1, s), 64, 1)[0] for s in range(400)])
    assert abs(float(ys[:, 1:].mean()) - 0.3) < 2e-3
    c = torch.tensor([0, 5, 255, 256, 100000], dtype=torch.int32)
    assert ref.trunc_u8(c).tolist() == [0, 5, 255, 255, 255]


@pytest.mark.gpu
def test_quant_rows_gpu_matches_ref():
    from wormhole_amd import _native
    from wormhole_amd.ops import ref
    hip = _native.hip()
    g = torch.Generator().manual_seed(4)
    x = torch.randn(1000, 64, generator=g)
    for nb in (1, 2, 3):
        qg = hip.quant_rows(x.cuda(), nb, 11).cpu()
        qr = ref.quant_rows(x, nb, 11)
        # same hash, same rounding (a rare 1-ulp difference in x/scale may flip one code)
        diff = (qg.view(-1) != qr.view(-1)).float().mean()
        assert float(diff) < 1e-3
        yg = hip.dequant_rows(qg.cuda(), 64, nb).cpu()
        assert torch.allclose(yg, ref.dequant_rows(qg, 64, nb))
    c = torch.tensor([0, 5, 255, 256, 100000], dtype=torch.int32)
    assert hip.trunc_u8(c.cuda()).cpu().tolist() == [0, 5, 255, 255, 255]


def _regions(linear, nb, seed=0):
    from wormhole_amd.kv.psx import _QFilter
    g = torch.Generator().manual_seed(seed)
    P, vs = 5, 16
    n = [int(x) for x in torch.randint(0, 200, (P,), generator=g)]
    n[2] = 0  # an empty peer
    v = [int(torch.randint(0, k + 1, (1,), generator=g)) for k in n]
    H = [-(-2 * k // vs) for k in n]
    qf = _QFilter(nb, 0 if linear else vs, 3, 1, linear)
    d, rows, ext = qf.layout(n, v, H)
    x = torch.randn(ext if linear else ext // vs, *(() if linear else (vs,)), generator=g)
    return qf, d, rows, x


@pytest.mark.parametrize("linear", [False, True])
def test_qregion_roundtrip_ref(linear):
    """The exchange's region filter (kv/psx.py _QFilter, quant.hip qregion):
    exact parts bit-exact, quantised parts within one step of their scale."""
    from wormhole_amd.ops import ref
    for nb in (1, 2, 3):
        qf, d, rows, x = _regions(linear, nb, nb)
        q = ref.ps_qpack(x, d, sum(rows), qf.W, nb, 77)
        assert q.shape == (sum(rows), qf.R)
        y = ref.ps_qunpack(q, d, qf.W, nb, torch.zeros_like(x))
        xf, yf = x.reshape(-1), y.reshape(-1)
        lim = (1 << (8 * nb - 1)) - 1
        for sf, a, vf, nf, sq, ha in d.tolist():
            assert torch.equal(xf[sf:sf + a], yf[sf:sf + a])
            for r0 in range(0, nf, qf.W):
                seg = slice(sf + vf + r0, sf + vf + min(nf, r0 + qf.W))
                step = float(xf[seg].abs().max()) / lim
                err = (xf[seg] - yf[seg]).abs()
                assert bool((err <= step * 1.001 + 3e-7 * xf[seg].abs() + 1e-9).all())


@pytest.mark.gpu
@pytest.mark.parametrize("linear", [False, True])
def test_qregion_gpu_matches_ref(linear):
    from wormhole_amd import ops
    from wormhole_amd.ops import ref
    dev = torch.device("cuda", 0)
    for nb in (1, 2, 3):
        qf, d, rows, x = _regions(linear, nb, 10 + nb)
        dd = torch.from_numpy(d).to(dev)
        qg = ops.ps_qpack(x.to(dev), d, dd, sum(rows), qf.W, nb, 77)
        qc = ref.ps_qpack(x, d, sum(rows), qf.W, nb, 77)
        assert qg.shape == qc.shape
        yg = ops.ps_qunpack(qg, d, dd, qf.W, nb, torch.zeros_like(x).to(dev)).cpu()
        yc = ref.ps_qunpack(qc, d, qf.W, nb, torch.zeros_like(x))
        lim = (1 << (8 * nb - 1)) - 1
        # (the device may contract x * inv + u into an FMA: a rare last-step
        # rounding difference, never more than one quantisation step)
        tol = float(x.abs().max()) / lim * 1.001 + 1e-6
        assert float((yg - yc).abs().max()) <= tol
        xf, ygf = x.reshape(-1), yg.reshape(-1)
        for sf, a, vf, nf, sq, ha in d.tolist():
            assert torch.equal(xf[sf:sf + a], ygf[sf:sf + a])


@pytest.mark.gpu
def test_fixed_bytes_loopback_gpu_matches_cpu():
    """DiFacto with fixed_bytes = 3 through the multi-shard step's region
    filter on the HIP kernels vs the host path: same model within the
    quantisation noise."""
    import sys
    sys.path.insert(0, os.path.dirname(__file__))
    from test_psx import _conf, _model, _run
    from wormhole_amd.parallel.comm import LoopbackComm
    dev = torch.device("cuda", 0)
    conf = lambda: _conf(max_conc=1)  # noqa
    cg, cc = conf(), conf()
    cg.fixed_bytes = cc.fixed_bytes = 3
    g, pg, _ = _run(LoopbackComm(4, dev), cg, dev, steps=6, rows=2000)
    c, pc, _ = _run(LoopbackComm(4, "cpu"), cc, "cpu", steps=6, rows=2000)
    assert g.psx.qf is not None and g.psx.wire_report(1)["c2"] > 0  # (native or Python tally)
    mg, mc = _model(g), _model(c)
    assert mg.keys() == mc.keys()
    bad = sum(1 for k, (w, n, v) in mc.items() if abs(w - mg[k][0]) > 1e-3 * max(1.0, abs(w)))
    assert bad <= len(mc) // 200, bad
    assert abs(pg[0] / pg[5] - pc[0] / pc[5]) < 1e-3
