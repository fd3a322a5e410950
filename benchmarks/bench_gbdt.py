#!/usr/bin/env python3
"""GBDT benchmark (BASELINE.json config: hist GBDT depth 8 on Higgs-shaped
11M x 28; default 500 trees).  Strong scaling: --rows is the total, split over
the ranks (row split, histogram allreduce per level over RCCL).

    python benchmarks/bench_gbdt.py [--rows 11000000] [--trees 500] [--depth 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wormhole_amd.models import gbdt as G  # noqa: E402
from wormhole_amd.parallel.bsp import BSP  # noqa: E402
from wormhole_amd.parallel.comm import env_local_rank  # noqa: E402
from wormhole_amd.parallel import launch  # noqa: E402


def higgs_like(n, f, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    X = torch.randn(n, f, device=dev, generator=g)
    X[:, :7] = X[:, :7].abs()  # kinematic-like positive features
    w = torch.randn(f, device=dev, generator=g)
    logit = (X * w).sum(1) * 0.3 + torch.sin(X[:, 0] * X[:, 1]) + 0.5 * (X[:, 2] > 1).float()
    y = (torch.rand(n, device=dev, generator=g) < torch.sigmoid(logit)).float()
    return X, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--trees", type=int, default=500)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--max-bin", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the framework's PyTorch CPU path (anchor numbers)")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); > 1 without a launcher: started here")
    a = ap.parse_args()
    if a.gpus > 1 and not launch.launched():  # before any GPU call in this process
        return launch.self_launch(os.path.abspath(__file__), sys.argv[1:], a.gpus, a.device)
    if a.device == "cuda":
        torch.cuda.set_device(env_local_rank())
        dev = torch.device("cuda", env_local_rank())
    else:
        dev = torch.device("cpu")

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    bsp = BSP(dev)
    launch.verify_world(bsp.comm, a.gpus if launch.launched() else 1)
    n = a.rows // bsp.world
    X, y = higgs_like(n, a.features, 7 + bsp.rank, dev)
    dm = G.DMatrix.from_dense(X, y, dev)
    p = G.GBDTParam()
    p.objective = "binary:logistic"
    p.max_depth = a.depth
    p.eta = 0.1
    p.max_bin = a.max_bin
    sync()
    t_prep = time.perf_counter()
    cuts = G.Cuts.build(dm, p.max_bin, bsp)
    B = cuts.bin(dm)
    sync()
    t_prep = time.perf_counter() - t_prep
    obj = G.Objective(p.objective)
    tb = G.TreeBuilder(p, bsp, dm, cuts, B)
    margin = torch.zeros(n, device=dev)
    for _ in range(a.warmup):
        t = tb.build(obj.gpair(margin, dm.label, None), margin)
        if hasattr(t, "materialize"):
            t.materialize()
    sync()
    bsp.barrier()
    b0 = tb.hist_bytes()
    t0 = time.perf_counter()
    tree = None
    for _ in range(a.trees):
        tree = tb.build(obj.gpair(margin, dm.label, None), margin)
    # a device-grown tree's host lists are built one tree later: the last
    # one's inside the timed region too
    if tree is not None and hasattr(tree, "materialize"):
        tree.materialize()
    sync()
    bsp.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    bsp.allreduce(t, "max")
    dt = float(t.item())
    hb = bsp.allreduce_scalar((tb.hist_bytes() - b0) / max(a.trees, 1), "max")
    err = G.eval_metric("error", torch.sigmoid(margin), dm.label, None, bsp)
    if bsp.rank == 0:
        print(json.dumps({"metric": "GBDT trees/s (hist, depth %d, %dx%d)" % (a.depth, a.rows, a.features),
                          "value": a.trees / dt, "unit": "trees/s", "n_gpus": bsp.world if dev.type == "cuda" else 0, "ranks": bsp.world, "device": dev.type,
                          "ms_per_tree": 1000 * dt / a.trees,
                          "trees": a.trees, "sketch_bin_s": t_prep,
                          "hist_exchange": ("feature-reduce-scatter" if tb.xchg is not None
                                            else "allreduce") if bsp.world > 1 else None,
                          "hist_bytes_per_rank_per_tree": hb,
                          "train_error": err, "scaling": "strong", "data": "synthetic Higgs-shaped"}),
              flush=True)
    bsp.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
