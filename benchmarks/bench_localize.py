#!/usr/bin/env python3
"""Localize microbenchmark: one 100k-row Criteo-shaped minibatch (device
synthetic) localized repeatedly with the previous unique count as the hint;
prints mean ms per call (events) for the partitioned path (the hash path with WH_DETERMINISTIC=1).
TEXT=<criteo text file>: four minibatches of its lines instead (parsed on
the device), e.g. the files benchmarks/bench_e2e.py writes."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wormhole_amd import _native  # noqa: E402
from wormhole_amd.utils import trace  # noqa: E402
from wormhole_amd.data.synthetic import CRITEO_TB_CARD  # noqa: E402


def main():
    n = int(os.environ.get("ROWS", "100000"))
    iters = int(os.environ.get("ITERS", "30"))
    nshard = int(os.environ.get("NSHARD", "1"))
    hip = _native.hip()
    dev = torch.device("cuda", 0)
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=dev)
    batches = [hip.synth_criteo(n, 11, s, card) for s in range(4)]
    if os.environ.get("TEXT"):  # Criteo text (e.g. bench_e2e.py's files), parsed on the device
        raw = open(os.environ["TEXT"], "rb").read()
        cut, pos = [0], 0
        for _ in range(4):
            for _ in range(n):
                pos = raw.index(b"\n", pos) + 1
            cut.append(pos)
        batches = []
        for a, b in zip(cut, cut[1:]):
            t = torch.frombuffer(bytearray(raw[a:b]), dtype=torch.uint8).to(dev)
            k, l, o = hip.parse_criteo(t, n, True)
            batches.append((k, l, o))
    if os.environ.get("SKEW") == "0":  # uniform ids, same count of distinct ids
        g = torch.Generator(device=dev).manual_seed(5)
        batches = [(torch.randint(0, 600000, (k.numel(),), device=dev, generator=g) *
                    0x9E3779B97F4A7C15 % (1 << 62), l, o) for k, l, o in batches]
    hint = 0
    for k, _, o in batches:
        out = hip.localize(k, o, None, nshard, hint)
        hint = out[0].numel()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        k, _, o = batches[i % 4]
        out = hip.localize(k, o, None, nshard, hint)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"bench": "localize",
                      "mode": "hash" if os.environ.get("WH_DETERMINISTIC") == "1" else "part",
                      "rows": n, "nshard": nshard,
                      "uniq": hint, "skew": os.environ.get("SKEW", "1"),
                      "ms_per_call": e0.elapsed_time(e1) / iters}))
    if trace.timing_on("loc"):
        t = hip.loc_timing_read().view(-1, 4).cpu()
        t = t[t[:, 0] > 0]
        t0 = int(t[:, 0].min())
        ph1, ph2, ph3 = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
        q = lambda x: [round(float(v) / 100, 2) for v in torch.quantile(x.double(), torch.tensor(
            [0.0, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64))]
        print(json.dumps({"parts": int(t.shape[0]), "span_us": (int(t[:, 3].max()) - t0) / 100,
                          "start_spread_us": (int(t[:, 0].max()) - t0) / 100,
                          "phase1_us_q": q(ph1), "lookback_us_q": q(ph2), "phase3_us_q": q(ph3),
                          "slowest_total_us": float((t[:, 3] - t[:, 0]).max()) / 100}))


if __name__ == "__main__":
    main()
