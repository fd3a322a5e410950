#!/usr/bin/env python3
"""RCCL-over-xGMI microbenchmark for the exchanges this framework issues
(measure the link, not assume it). Run with one process per
GPU:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        benchmarks/bench_comm.py

Per message size it reports, for the patterns used:
  * all_to_all_v as one grouped point-to-point launch (ShardedKV push/pull:
    keys 8 B, headers 8 B, embedding rows 256 B per key) -- per-GPU send GB/s;
  * all_reduce (k-means centroid sums, GBDT histograms, L-BFGS gradients) --
    bus GB/s = algbw * 2 (n-1) / n.
(--device cpu runs the same code on gloo for a functional rehearsal.)
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wormhole_amd.parallel.comm import Comm, env_local_rank  # noqa: E402


def timeit(fn, sync, iters):
    for _ in range(3):
        fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    if args.device == "cuda":
        torch.cuda.set_device(env_local_rank())
        dev = torch.device("cuda", env_local_rank())
    else:
        dev = torch.device("cpu")
    comm = Comm(dev)
    P = comm.size

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
    out = []
    # all-to-all-v: per-peer rows of a given width (bytes per row = 4 * width)
    for rows_per_peer, width, what in [(8192, 2, "keys/headers 8B"), (65536, 2, "keys/headers 8B"),
                                       (1024, 64, "emb rows 256B"), (8192, 64, "emb rows 256B"),
                                       (16384, 64, "emb rows 256B")]:
        if dev.type == "cpu":
            rows_per_peer = min(rows_per_peer, 2048)
        x = torch.randn(rows_per_peer * P, width, device=dev)
        split = [rows_per_peer] * P
        dt = timeit(lambda: comm.all_to_all_v_multi([(x, split, split)]), sync, args.iters)
        sent = 4 * width * rows_per_peer * (P - 1)
        out.append({"op": "all_to_all_v", "what": what, "bytes_per_peer": 4 * width * rows_per_peer,
                    "us": 1e6 * dt, "send_GBps_per_gpu": sent / dt / 1e9})
    for n in [1 << 16, 1 << 20, 1 << 22, 1 << 24]:
        if dev.type == "cpu":
            n = min(n, 1 << 18)
        t = torch.randn(n, device=dev)
        dt = timeit(lambda: comm.allreduce(t), sync, args.iters)
        alg = 4 * n / dt
        out.append({"op": "all_reduce", "bytes": 4 * n, "us": 1e6 * dt,
                    "bus_GBps": alg * 2 * (P - 1) / max(P, 1) / 1e9})
    if comm.rank == 0:
        for r in out:
            print(json.dumps(dict(r, n_gpus=P)), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
