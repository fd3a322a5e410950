"""Feature-sharded GBDT histogram exchange (models/gbdt.py HistExchange,
SURVEY §7.3 P9): 2- and 4-rank gloo growers build the same trees as one rank,
and move fewer histogram bytes per rank than the allreduce exchange."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

ROWS, FEAT, TREES, DEPTH = 1500, 8, 3, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(3)
    # few distinct values per feature: the quantile cuts are exact, hence the
    # same for any rank count
    X = torch.randint(0, 120, (ROWS, FEAT), generator=g).float()
    X[torch.rand(ROWS, FEAT, generator=g) < 0.1] = float("nan")
    logit = 0.2 * torch.nan_to_num(X[:, 0] - X[:, 3], 0.0) + 0.05 * torch.nan_to_num(X[:, 5], 7.0)
    y = (torch.rand(ROWS, generator=g) < torch.sigmoid(logit - 1.0)).float()
    return X, y


def _train(bsp, device):
    from wormhole_amd.models import gbdt as G
    X, y = _data()
    rows = torch.arange(ROWS)[bsp.rank::bsp.world]
    dm = G.DMatrix.from_dense(X[rows], y[rows], device)
    p = G.GBDTParam()
    p.objective, p.max_depth, p.eta = "binary:logistic", DEPTH, 0.4
    cuts = G.Cuts.build(dm, p.max_bin, bsp)
    tb = G.TreeBuilder(p, bsp, dm, cuts, cuts.bin(dm))
    obj = G.Objective(p.objective)
    margin = torch.zeros(dm.n, device=device)
    dumps = []
    for _ in range(TREES):
        tree = tb.build(obj.gpair(margin, dm.label, None), margin)
        dumps.append(tree.dump(with_stats=True))
    return dumps, tb.hist_bytes(), tb.xchg is not None


def _main(rank, world, port, out, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), WH_GBDT_XCHG=mode)
    torch.set_num_threads(1)
    from wormhole_amd.parallel.bsp import BSP
    bsp = BSP(torch.device("cpu"))
    dumps, sent, sharded = _train(bsp, torch.device("cpu"))
    sent = bsp.allreduce_scalar(sent, "max")
    if rank == 0:
        json.dump({"dumps": dumps, "sent": sent, "sharded": sharded}, open(out, "w"))
    bsp.finalize()


def _run(world, mode, tmp_path):
    out = str(tmp_path / ("%d_%s.json" % (world, mode)))
    mp.spawn(_main, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    return json.load(open(out))


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    from wormhole_amd.parallel.bsp import BSP
    os.environ.pop("RANK", None)
    dumps, _, _ = _train(BSP(torch.device("cpu")), torch.device("cpu"))
    return dumps


@pytest.mark.parametrize("world", [2, 4])
def test_feature_sharded_trees_equal_single_rank(single, world, tmp_path):
    r = _run(world, "rs", tmp_path)
    assert r["sharded"]
    assert r["dumps"] == single
    assert any("yes=" in d for d in single)  # trees actually split


def test_feature_sharded_exchange_halves_the_bytes(single, tmp_path):
    rs = _run(4, "rs", tmp_path)
    ar = _run(4, "allreduce", tmp_path)
    assert not ar["sharded"] and ar["dumps"] == single == rs["dumps"]
    # a ring allreduce sends 2 (P-1)/P of the histogram bytes per rank, the
    # feature all-to-all (P-1)/P: 2x, less the [S, 6] candidate table per level
    assert ar["sent"] >= 1.9 * rs["sent"] > 0, (ar["sent"], rs["sent"])


def _gpu_main(rank, world, port, out, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), WH_GBDT_XCHG=mode, WH_COMM_BACKEND="gloo")
    torch.set_num_threads(1)
    torch.cuda.set_device(0)
    from wormhole_amd.parallel.bsp import BSP
    dev = torch.device("cuda", 0)
    bsp = BSP(dev)  # ranks share the GPU: gloo-staged collectives
    dumps, sent, sharded = _train(bsp, dev)
    sent = bsp.allreduce_scalar(sent, "max")
    if rank == 0:
        json.dump({"dumps": dumps, "sent": sent, "sharded": sharded}, open(out, "w"))
    bsp.finalize()


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode", [(2, "rs"), (3, "rs"), (2, "allreduce")])
def test_native_device_grower_feature_sharded(world, mode, tmp_path):
    """The device level loop (gbdt_grow_dev) with the feature reduce-scatter
    and candidate pick callbacks: identical trees to one rank (the GPU
    histograms are exact fixed-point sums)."""
    from wormhole_amd.parallel.bsp import BSP
    os.environ.pop("RANK", None)
    dev = torch.device("cuda", 0)
    one, _, _ = _train(BSP(dev), dev)
    out = str(tmp_path / "g.json")
    mp.spawn(_gpu_main, args=(world, _free_port(), out, mode), nprocs=world, join=True)
    r = json.load(open(out))
    assert r["sharded"] == (mode == "rs")
    assert r["dumps"] == one
