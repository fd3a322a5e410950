#!/usr/bin/env python3
"""Host -> device copy bandwidth from pinned memory (the ingest path's
link): one stream vs two concurrent copies, 64 MB and 256 MB chunks."""
import json
import time

import torch


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for mb in (32, 64, 256):
        n = mb << 20
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.fill_(1)
        d = torch.empty(n, dtype=torch.uint8, device=dev)
        for _ in range(3):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        out["h2d_%dMB_GBps" % mb] = round(reps * n / (time.perf_counter() - t0) / 1e9, 1)
        s2 = torch.cuda.Stream(dev)
        h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        d2 = torch.empty(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            d.copy_(h, non_blocking=True)
            with torch.cuda.stream(s2):
                d2.copy_(h2, non_blocking=True)
        torch.cuda.synchronize()
        out["h2d_2streams_%dMB_GBps" % mb] = round(2 * reps * n / (time.perf_counter() - t0) / 1e9, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
