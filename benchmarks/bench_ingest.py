#!/usr/bin/env python3
"""Input-pipeline throughput, stage by stage, without training: how fast the
file worker's minibatch source can go (the ceiling of bench_e2e.py).

Stages (rows/s each, one file part after another as the worker reads them):
  host_text   host reader alone: whole-line text batches into pinned memory
  device_text + copy + device parse (+ shuffle buffer) -> device minibatches
  host_crb    CRB records decoded by the host reader threads
  device_crb  + copy + device shuffle / slicing

    python benchmarks/bench_ingest.py [--rows 8000000] [--files 4] [--minibatch 100000]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def drain(make, files):
    n = 0
    t = time.time()
    for f in files:
        it = make(f)
        while True:
            b = it.next()
            if b is None:
                break
            n += b
    return n, time.time() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8_000_000)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--minibatch", type=int, default=100000)
    ap.add_argument("--rand-shuffle", type=int, default=10)
    ap.add_argument("--crb", action="store_true")
    ap.add_argument("--dir", default=None)
    args = ap.parse_args()
    from bench_e2e import criteo_text
    import torch
    from wormhole_amd import _native
    from wormhole_amd.data import device_text
    work = args.dir or tempfile.mkdtemp(prefix="wh_ingest_")
    os.makedirs(work, exist_ok=True)
    per = args.rows // args.files
    txt, crb = [], []
    for i in range(args.files):
        p = os.path.join(work, "part_%d.txt" % i)
        with open(p, "wb") as f:
            f.write(criteo_text(per, 100 + i))
        txt.append(p)
        if args.crb:
            q = p[:-4] + ".crb"
            subprocess.run([os.path.join(ROOT, "bin", "convert.dmlc"), "-data_in", p,
                            "-data_out", q, "-format_in", "criteo", "-format_out", "crb"],
                           check=True)
            crb.append(q)
    host = _native.host()
    dev = torch.device("cuda", 0)
    mb, shuf = args.minibatch, args.rand_shuffle
    out = {"rows": args.rows, "files": args.files, "minibatch": mb, "rand_shuffle": shuf}

    class Count:  # adapts an iterator's items to row counts
        def __init__(self, it, rows):
            self.it, self.rows = it, rows

        def next(self):
            b = self.it.next()
            return None if b is None else self.rows(b)

    def dev_rows(b):
        return int(b.args[3].numel())

    def sync_rate(make, files):
        torch.cuda.synchronize()
        n, s = drain(make, files)
        torch.cuda.synchronize()
        return n / s / 1e6

    # H2D copy rates: pinned (torch), pageable, and a host reader batch
    def h2d_rate(x, reps=10):
        x.to(dev, non_blocking=True)
        torch.cuda.synchronize()
        t = time.time()
        for _ in range(reps):
            x.to(dev, non_blocking=True)
        torch.cuda.synchronize()
        return round(reps * x.numel() / (time.time() - t) / 1e9, 2)
    nbytes = 30 << 20
    out["h2d_GBs_pinned"] = h2d_rate(torch.empty(nbytes, dtype=torch.uint8, pin_memory=True))
    out["h2d_GBs_pageable"] = h2d_rate(torch.empty(nbytes, dtype=torch.uint8))
    b0 = host.TextBatches(txt[0], 0, 1, mb, True).next()[0]
    out["reader_batch_pinned"] = bool(b0.is_pinned())
    out["h2d_GBs_reader_batch"] = h2d_rate(b0)
    del b0
    # synchronous stage split of one part: host batch wait, H2D copy, device parse
    tb = host.TextBatches(txt[0], 0, 1, mb, True)
    st = {"read": 0.0, "h2d": 0.0, "parse": 0.0}
    nb = 0
    while True:
        t0 = time.time()
        b = tb.next()
        if b is None:
            break
        t1 = time.time()
        text = b[0].to(dev, non_blocking=True)
        torch.cuda.synchronize()
        t2 = time.time()
        device_text.parse_block(text, b[1], "criteo")
        torch.cuda.synchronize()
        t3 = time.time()
        st["read"] += t1 - t0
        st["h2d"] += t2 - t1
        st["parse"] += t3 - t2
        nb += 1
    out["sync_stage_ms_per_batch"] = {k: round(1e3 * v / max(nb, 1), 3) for k, v in st.items()}
    out["batch_bytes"] = int(os.path.getsize(txt[0]) // max(nb, 1))
    drain(lambda f: Count(host.TextBatches(f, 0, 1, mb, True), lambda b: int(b[1])), txt[:1])
    out["host_text_Mrows_s"] = sync_rate(
        lambda f: Count(host.TextBatches(f, 0, 1, mb, True), lambda b: int(b[1])), txt)
    for sh in (0, shuf):
        mk = (lambda f, sh=sh: Count(device_text.DeviceTextIter(
            host, f, 0, 1, "criteo", mb, sh, 1.0, 7, dev), dev_rows))
        out["device_text_shuffle%d_Mrows_s" % sh] = sync_rate(mk, txt)
    if crb:
        out["host_crb_Mrows_s"] = sync_rate(
            lambda f: Count(host.MinibatchIter(f, 0, 1, "crb", mb * max(1, shuf), 0, 1.0, 7, True),
                            lambda b: int(b[3].numel())), crb)
        mk = (lambda f: Count(device_text.DeviceTextIter(
            host, f, 0, 1, "crb", mb, shuf, 1.0, 7, dev), dev_rows))
        out["device_crb_Mrows_s"] = sync_rate(mk, crb)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
