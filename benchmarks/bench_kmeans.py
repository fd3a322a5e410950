#!/usr/bin/env python3
"""k-means benchmark (BASELINE.json config: k=1000 on dense 10M x 128).

Strong scaling: --rows is the TOTAL row count, split over the ranks.  Every
timed iteration is a full reference iteration (assign + accumulate + RCCL
allreduce of K x (F+1) + normalise).  Data: synthetic Gaussian mixture on
the device.

    python benchmarks/bench_kmeans.py [--rows 10000000] [--dim 128] [--k 1000] [--iters 5]

``--sparse F`` clusters synthetic CSR rows over F features instead
(``--nnz`` non-zeros per row, topic-structured: each row draws most of its
features from its cluster's window), never densified (models/kmeans.py
KMeansCSR).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wormhole_amd.models.kmeans import KMeans, KMeansCSR  # noqa: E402
from wormhole_amd.parallel.bsp import BSP  # noqa: E402
from wormhole_amd.parallel.comm import env_local_rank  # noqa: E402
from wormhole_amd.parallel import launch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sparse", type=int, default=0,
                    help="F > 0: CSR rows over F features (e.g. 1000000) instead of dense --dim")
    ap.add_argument("--nnz", type=int, default=32, help="non-zeros per sparse row")
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
    g = torch.Generator(device=dev).manual_seed(1234 + bsp.rank)
    if a.sparse:
        F = a.sparse
        lab = torch.randint(0, a.k, (n, 1), device=dev, generator=g)
        win = max(64, F // (4 * a.k))  # each cluster's feature window
        base = (lab * (F // a.k)) % F
        topic = (base + torch.randint(0, win, (n, a.nnz), device=dev, generator=g)) % F
        noise = torch.randint(0, F, (n, a.nnz), device=dev, generator=g)
        keep = torch.rand(n, a.nnz, device=dev, generator=g) < 0.75
        cols = torch.where(keep, topic, noise).reshape(-1)
        off = torch.arange(0, n * a.nnz + 1, a.nnz, dtype=torch.int64, device=dev)
        del lab, base, topic, noise, keep
        km = KMeansCSR(bsp, cols, off, None, F, a.k, dev)
        a.dim = F
    else:
        centers = torch.randn(a.k, a.dim, device=dev, generator=g)
        lab = torch.randint(0, a.k, (n,), device=dev, generator=g)
        X = centers[lab] + 0.5 * torch.randn(n, a.dim, device=dev, generator=g)
        del lab
        km = KMeans(bsp, X, a.k)
    km.init_centroids(0)
    for _ in range(a.warmup):
        km.step()
    sync()
    bsp.barrier()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        km.step()
    sync()
    bsp.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    bsp.allreduce(t, "max")
    dt = float(t.item())
    flops = 2.0 * a.rows * a.k * (a.nnz if a.sparse else a.dim) * a.iters
    if bsp.rank == 0:
        form = "sparse CSR %dx%d, %d nnz/row" % (a.rows, a.dim, a.nnz) if a.sparse else \
            "dense %dx%d" % (a.rows, a.dim)
        print(json.dumps({"metric": "k-means iterations/s (k=%d, %s)" % (a.k, form),
                          "value": a.iters / dt, "unit": "iter/s", "n_gpus": bsp.world if dev.type == "cuda" else 0, "ranks": bsp.world, "device": dev.type,
                          "ms_per_iter": 1000 * dt / a.iters, "rows_per_s": a.rows * a.iters / dt,
                          "assign_tflops": flops / dt / 1e12, "scaling": "strong",
                          "dtype": ("fp64 accumulation of fp32 products (CSR)" if a.sparse else "exact fp32 argmax (bf16x3 split MFMA + fp32 re-score of near-ties)" if km.split else "fp32 (exact fp32 MFMA)") if dev.type == "cuda" else "fp64 (CPU reference path)",
                          "objective": km.objective() if a.sparse else None,
                          "rescored_rows_last_iter": int(km.rescored.item()) if km.rescored is not None else None, "data": "synthetic gaussian mixture"}),
              flush=True)
    bsp.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
