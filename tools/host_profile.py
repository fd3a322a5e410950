#!/usr/bin/env python3
"""Host-side cost of one DiFacto training step: wall time of every native
call made by the learner (no synchronisation inside the step), averaged over
steps, plus the synchronised step time. Shows whether the step is bound by
the GPU or by the host's launch path.

    python tools/host_profile.py [--steps 50] [--batch 100000]
"""
import argparse
import collections
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=100000)
    args = ap.parse_args()
    from wormhole_amd import _native, ops
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.data.synthetic import CRITEO_TB_CARD
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm
    dev = torch.device("cuda", 0)
    hip = _native.hip()
    acc = collections.defaultdict(float)

    def wrap(mod, name, label):
        f = getattr(mod, name)

        def g(*a, **k):
            t = time.perf_counter()
            r = f(*a, **k)
            acc[label] += time.perf_counter() - t
            return r
        setattr(mod, name, g)
    for n in ["localize", "localize_begin", "localize_finish", "fm_forward", "fm_backward",
              "fm_grad_post", "auc_acc"]:
        wrap(ops, n, "ops." + n)
    emb = Embedding(dim=64, threshold=100, lambda_l2=1.0, lr_eta=0.01)
    emb._set = {"dim", "threshold", "lambda_l2", "lr_eta"}
    conf = DifactoConfig(minibatch=args.batch, lr_eta=0.01, embedding=[emb])
    lr = DifactoLearner(conf, Comm(dev, init=False), dev, cap=1 << 27, vcap=1 << 24, seed=1)
    for n in ["open", "difacto_open_pull", "difacto_push_cnt", "difacto_pull", "difacto_push"]:
        wrap(lr.kv, n, "kv." + n)
    from wormhole_amd.models import difacto as dmod
    wrap(dmod, "begin_next", "begin_next")
    wrap(dmod, "localize_current", "localize_current")
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=dev)

    def synth(s):
        t = time.perf_counter()
        r = hip.synth_criteo(args.batch, 1, s, card)
        acc["synth"] += time.perf_counter() - t
        return r

    def run(first, n):  # pipelined like bench.py (next minibatch's localize begun early)
        nxt = synth(first)
        for s in range(first, first + n):
            k, l, o = nxt
            nxt = synth(s + 1) if s + 1 < first + n else None
            lr.process(k, o, None, l, 0, 0,
                       next_batch=(nxt[0], nxt[2], None) if nxt is not None else None)
    run(0, 10)
    lr.flush()
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    run(10, args.steps)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    for k_, v in sorted(acc.items(), key=lambda x: -x[1]):
        print("%-22s %8.1f us/step" % (k_, 1e6 * v / args.steps))
    print("host loop %.1f us/step, synchronised %.1f us/step" % (
        1e6 * t_host / args.steps, 1e6 * t_all / args.steps))


if __name__ == "__main__":
    main()
