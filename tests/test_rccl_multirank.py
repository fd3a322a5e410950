"""The multi-rank exchange of the native parameter-server step (csrc/bind/
rccl_comm.h, csrc/bind/psx_native.inl) with more than one rank.

* ``a2a_plan`` -- the per-peer plan every transport executes -- composes to
  the exact all-to-all-v over P ranks for uneven, empty and one-sided
  segments and every record width the step sends (CPU);
* several RCCL ranks on ONE GPU (``WH_BENCH_SAME_GPU=1``: a host id of its
  own per rank, so RCCL connects them through its network transport over
  loopback sockets instead of refusing the shared device): the grouped
  per-peer ``ncclSend`` / ``ncclRecv`` of ``RcclComm.a2av`` delivers every
  row, and the native RCCL step (three communicators, or one with
  ``WH_PSX_RCCL_COMMS=1``) trains the same shards as the Python step over
  c10d's collectives (GPU);
* the watchdog: a rank that never posts its half of an exchange
  (``WH_FAULT=xstall:<rank>:<step>``) ends every rank of the job with exit
  status 3 and a diagnostic line naming the stalled exchange, within the
  ``WH_RCCL_TIMEOUT_S`` deadline -- over the gloo-staged transport and over
  RCCL (GPU).

Reference: W workers and S servers exchange every minibatch
(learn/difacto/async_sgd.h:363-425, learn/linear/async_sgd.h:240-301).
"""
import os
import random
import time

import pytest
import torch
import torch.multiprocessing as mp

from test_psx import CARD, _conf, _free_port, _lin_model, _lockstep, _model


# ------------------------------------------------------------------ plan
def _simulate(world, row_bytes, rows):
    """Run every rank's a2a_plan over byte buffers; rows[p][q] = rows rank p
    sends rank q. Returns each rank's receive buffer."""
    from wormhole_amd import _native
    hip = _native.hip()
    send = []
    for p in range(world):
        n = sum(rows[p]) * row_bytes
        send.append(bytes((p * 37 + i * 11) % 251 for i in range(n)))
    recv = [bytearray(sum(rows[q][p] for q in range(world)) * row_bytes) for p in range(world)]
    plans = [hip.a2a_plan(rank=p, world=world, row_bytes=row_bytes, send_rows=list(rows[p]),
                          recv_rows=[rows[q][p] for q in range(world)]) for p in range(world)]
    esz = {pl[0] for pl in plans}
    assert len(esz) == 1  # every rank picks the same element size
    for p, (_, (src, dst, nb), sends, recvs) in enumerate(plans):
        recv[p][dst:dst + nb] = send[p][src:src + nb]
        assert all(b > 0 for _, _, b in sends + recvs)  # zero-byte segments skipped
        assert [q for q, _, _ in sends] == sorted(q for q, _, _ in sends)
        assert p not in [q for q, _, _ in sends + recvs]
    # every posted send meets exactly one posted receive of the same size
    for p, (_, _, sends, _) in enumerate(plans):
        for q, off, nb in sends:
            m = [(o, b) for (s, o, b) in plans[q][3] if s == p]
            assert len(m) == 1 and m[0][1] == nb, (p, q)
            recv[q][m[0][0]:m[0][0] + nb] = send[p][off:off + nb]
    for q, (_, _, _, recvs) in enumerate(plans):
        for p, _, nb in recvs:
            assert any(s == q and b == nb for s, _, b in plans[p][2]), (p, q)
    return send, recv, esz.pop()


@pytest.mark.parametrize("world", [2, 3, 5, 8])
@pytest.mark.parametrize("row_bytes", [8, 12, 256, 3])
def test_a2a_plan_composes_to_all_to_all(world, row_bytes):
    rng = random.Random(world * 1000 + row_bytes)
    for trial in range(6):
        rows = [[rng.choice([0, 0, 1, 2, 7, 40]) for _ in range(world)] for _ in range(world)]
        if trial == 0:
            rows = [[0] * world for _ in range(world)]  # nobody sends anything
        if trial == 1:
            rows[0] = [0] * world  # a rank with no data sends nothing
        send, recv, esz = _simulate(world, row_bytes, rows)
        assert esz == (8 if row_bytes % 8 == 0 else 4 if row_bytes % 4 == 0 else 1)
        # rank p's buffer holds, in peer order, what each q sent it
        for p in range(world):
            exp = b""
            for q in range(world):
                off = sum(rows[q][:p]) * row_bytes
                exp += send[q][off:off + rows[q][p] * row_bytes]
            assert bytes(recv[p]) == exp, (p, rows)


def test_a2a_plan_loopback_and_errors():
    from wormhole_amd import _native
    hip = _native.hip()
    # 1-rank communicator, 4 virtual peers: own copy + one pair to self
    esz, own, s, r = hip.a2a_plan(rank=0, world=1, row_bytes=8, send_rows=[2, 3, 0, 1],
                                  recv_rows=[2, 3, 0, 1])
    assert esz == 8 and own == (0, 0, 16) and s == [(0, 16, 32)] and r == [(0, 16, 32)]
    with pytest.raises(RuntimeError, match="symmetric"):
        hip.a2a_plan(rank=0, world=1, row_bytes=8, send_rows=[1, 2], recv_rows=[1, 3])
    with pytest.raises(RuntimeError, match="own segment"):
        hip.a2a_plan(rank=1, world=2, row_bytes=8, send_rows=[1, 2], recv_rows=[1, 3])
    with pytest.raises(RuntimeError, match="segments for"):
        hip.a2a_plan(rank=0, world=3, row_bytes=8, send_rows=[1, 2], recv_rows=[1, 2])


# ------------------------------------------------------- RCCL, one GPU
def _rank_env(rank, world, port, extra=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", WH_BENCH_SAME_GPU="1")
    os.environ.update(extra or {})
    torch.set_num_threads(1)


def _a2av_main(rank, world, port, out_dir):
    _rank_env(rank, world, port)
    from wormhole_amd.parallel.comm import Comm
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = Comm(dev, backend="nccl")
    assert comm.size == world and not comm.stage
    c = comm.rccl("t")
    assert c.size == world and c.rank == rank
    rng = random.Random(11)
    for trial in range(8):
        width, dt = [(3, torch.int32), (1, torch.int64), (64, torch.float32),
                     (3, torch.uint8)][trial % 4]
        rows = [[rng.choice([0, 1, 5, 300]) for _ in range(world)] for _ in range(world)]
        if trial == 5:
            rows[1] = [0] * world  # (every rank agrees: rank 1 sends nothing)
        mine = rows[rank]
        x = torch.cat([torch.full((mine[q], width), 10 * rank + q, dtype=dt)
                       for q in range(world)]).to(dev)
        if trial == 6 and rank == 0:  # a view 4 bytes into its storage (peers aligned)
            pad = torch.zeros(sum(mine) * width + 1, dtype=dt, device=dev)
            pad[1:] = x.reshape(-1)
            x = pad[1:].view(-1, width)
        y = c.a2av(x.contiguous(), mine, [rows[q][rank] for q in range(world)])
        torch.cuda.synchronize()
        o = 0
        for q in range(world):
            n = rows[q][rank]
            assert bool((y[o:o + n].long() == 10 * q + rank).all()), (trial, rank, q)
            o += n
        assert o == y.shape[0]
    comm.barrier()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("ok\n")
    comm.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 4])
def test_rccl_comm_a2av_multi_rank_same_gpu(tmp_path, world):
    """RcclComm.a2av's per-peer branch with real peers: uneven, empty and
    one-sided segments, 1- to 256-byte rows, a misaligned view."""
    mp.spawn(_a2av_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok\n"


def _rccl_step_main(rank, world, port, out_dir, model, max_conc, comms):
    """Both steps over RCCL on the shared GPU: the native step's own
    communicators, and the Python step's c10d all-to-all-v; this rank's
    shard must agree (tolerances as tests/test_psx.py _staged_main)."""
    _rank_env(rank, world, port, {"WH_PSX_RCCL_COMMS": str(comms)})
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.models.linear import LinearLearner
    from wormhole_amd.parallel.comm import Comm
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = Comm(dev, backend="nccl")
    assert not comm.stage and comm.backend == "nccl"
    mine = [[t.to(dev) for t in criteo_batch_cpu(300 + 100 * rank, 31 + rank, s, CARD)]
            for s in range(6 - rank)]
    res = {}
    for native in ("0", "1"):
        os.environ["WH_PSX_NATIVE"] = native
        if model == "difacto":
            lr = DifactoLearner(_conf(max_conc=max_conc), comm, dev, cap=1 << 14, vcap=1 << 12,
                                seed=5)
        else:
            lr = LinearLearner(LinearConfig(algo=3, lambda_l1=0.1, lr_eta=0.1,
                                            max_concurrency=max_conc), comm, dev, cap=1 << 14,
                               seed=5)
        prog = _lockstep(lr, mine)
        assert bool(lr.psx._nat) == (native == "1")
        if native == "1":
            xt = lr.psx._nat.xtime()
            assert lr.psx._nat.watchdog_deadline > 0
        res[native] = (_model(lr) if model == "difacto" else _lin_model(lr), prog)
    (mp_, pp), (mn, pn) = res["0"], res["1"]
    assert mp_.keys() == mn.keys() and len(mp_) > 100
    if model == "difacto":
        bad = 0
        for k, (w, c, v) in mp_.items():
            wn, cn, vn = mn[k]
            assert c == cn and (v is None) == (vn is None), k
            if abs(w - wn) > 1e-4 * max(1.0, abs(w)) or (v is not None and
                                                         not torch.allclose(v, vn, atol=1e-2)):
                bad += 1
        nmb = pn[4]
    else:
        bad = sum(1 for k, w in mp_.items() if abs(w - mn[k]) > 1e-4 * max(1.0, abs(w)))
        nmb = pn[3]
    assert bad <= max(2, len(mp_) // 1000), (bad, len(mp_))
    assert nmb == 6 - rank
    assert xt[4] + xt[5] + xt[6] + xt[7] > 0  # exchange timing sampled
    comm.barrier()
    with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
        f.write("ok\n")
    comm.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("world,model,max_conc,comms", [(2, "difacto", 2, 3), (3, "difacto", 2, 3),
                                                        (2, "linear", 2, 3), (3, "difacto", 2, 1),
                                                        (2, "difacto", 1, 3), (4, "difacto", 2, 3),
                                                        (4, "linear", 2, 1)])
def test_native_step_multi_rank_rccl_same_gpu(tmp_path, world, model, max_conc, comms):
    mp.spawn(_rccl_step_main, args=(world, _free_port(), str(tmp_path), model, max_conc, comms),
             nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok\n"


# ------------------------------------------------------------- watchdog
def _fault_main(rank, world, port, out_dir, backend):
    fd = os.open(os.path.join(out_dir, "err%d" % rank), os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(fd, 2)
    _rank_env(rank, world, port, {"WH_FAULT": "xstall:1:3", "WH_RCCL_TIMEOUT_S": "4"})
    from wormhole_amd.data.synthetic import criteo_batch_cpu
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = Comm(dev, backend=backend)
    mine = [[t.to(dev) for t in criteo_batch_cpu(300, 31 + rank, s, CARD)] for s in range(8)]
    lr = DifactoLearner(_conf(max_conc=2), comm, dev, cap=1 << 14, vcap=1 << 12, seed=5)
    _lockstep(lr, mine)
    with open(os.path.join(out_dir, "returned%d" % rank), "w") as f:
        f.write("the stalled exchange returned\n")


def _run_fault(tmp_path, backend, world=2, limit=90):
    ctx = mp.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_fault_main, args=(r, world, port, str(tmp_path), backend))
          for r in range(world)]
    t0 = time.time()
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=max(1.0, limit - (time.time() - t0)))
    alive = [p for p in ps if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    errs = [(tmp_path / ("err%d" % r)).read_text() for r in range(world)]
    assert not alive, errs
    return [p.exitcode for p in ps], errs, time.time() - t0


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_watchdog_ends_a_stalled_exchange(tmp_path, backend):
    """Rank 1 never posts its exchange of step 3: both ranks exit with status
    3 inside the deadline, rank 0 naming the step and the exchange it is
    blocked on, the rank that stalled naming the fault."""
    codes, errs, dt = _run_fault(tmp_path, backend)
    assert codes == [3, 3], (codes, errs)
    assert "[psx watchdog] rank 0: no progress" in errs[0], errs[0]
    assert "of step 3" in errs[0] and "C" in errs[0]
    assert "WH_FAULT: rank 1 stalls" in errs[1] and "[psx watchdog] rank 1" in errs[1], errs[1]
    assert "exiting with status 3" in errs[0] and "exiting with status 3" in errs[1]
    assert not any((tmp_path / ("returned%d" % r)).exists() for r in range(2))
