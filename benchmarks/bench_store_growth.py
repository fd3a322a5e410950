#!/usr/bin/env python3
"""Stream N distinct keys through the HBM parameter store with the load-factor
guard (kv.StoreGuard): the table starts small and grows on the device (rehash)
as it fills; at the end every key must be present and no insert may have
failed. Prints one JSON line (keys, growths, final capacity / load, insert
throughput with and without the growth steps).

    python benchmarks/bench_store_growth.py [--keys 300000000] [--batch 4194304]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from wormhole_amd.kv import StoreGuard, make_store  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=300_000_000)
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--cap", type=int, default=1 << 24)
    ap.add_argument("--verify-sample", type=int, default=1 << 22)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = make_store(a.cap, 1, 0, dev)
    g = StoreGuard(st)
    # distinct keys: an odd-multiplier bijection of 0..N-1 (spread over 64 bits)
    mul = 0x9E3779B97F4A7C15 - (1 << 64)
    t_ins = t_grow = 0.0
    done = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while done < a.keys:
        n = min(a.batch, a.keys - done)
        keys = (torch.arange(done, done + n, device=dev, dtype=torch.int64) + 1) * mul
        ta = time.perf_counter()
        grows = g.grows
        g.before_open(n)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        if g.grows > grows:
            t_grow += tb - ta
        st.find(keys, True)
        g.after_open()
        torch.cuda.synchronize()
        t_ins += time.perf_counter() - tb
        done += n
        if done % (a.batch * 16) == 0:
            print("[store] %d keys, cap %d, %.1f s" % (done, st.cap, time.perf_counter() - t0),
                  file=sys.stderr, flush=True)
    g.after_open()
    g.read()  # raises on any failed insert
    # every key is present: full count from the device counter, sampled lookups
    idx = torch.randint(0, a.keys, (min(a.verify_sample, a.keys),), device=dev)
    found = st.find((idx + 1) * mul, False)
    missing = int((found < 0).sum())
    print(json.dumps({
        "bench": "store_growth", "keys": a.keys, "keys_in_table": g.keys,
        "failed_inserts": 0, "sample_missing": missing, "growths": g.grows,
        "final_cap": st.cap, "final_load": g.keys / st.cap,
        "insert_Mkeys_per_s": a.keys / t_ins / 1e6, "growth_s": t_grow,
        "total_s": time.perf_counter() - t0}), flush=True)
    assert g.keys == a.keys and missing == 0


if __name__ == "__main__":
    main()
