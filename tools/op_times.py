#!/usr/bin/env python3
"""Synchronised wall time of every learner-level op of a DiFacto step
(torch.cuda.synchronize() around each call), averaged over steps: the
unprofiled counterpart of a rocprof kernel trace.

    python tools/op_times.py [--steps 30] [--batch 100000]
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
    ap.add_argument("--steps", type=int, default=30)
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
        f = getattr(mod, name, None)
        if f is None:
            return

        def g(*a, **k):
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            acc[label] += time.perf_counter() - t
            return r
        setattr(mod, name, g)
    for n in ["localize", "fm_forward", "fm_backward", "fm_grad_post", "auc_acc", "auc"]:
        wrap(ops, n, "ops." + n)
    emb = Embedding(dim=64, threshold=100, lambda_l2=1.0, lr_eta=0.01)
    emb._set = {"dim", "threshold", "lambda_l2", "lr_eta"}
    conf = DifactoConfig(minibatch=args.batch, lr_eta=0.01, embedding=[emb])
    lr = DifactoLearner(conf, Comm(dev, init=False), dev, cap=1 << 27, vcap=1 << 24, seed=1)
    for n in ["open", "difacto_push_cnt", "difacto_pull", "difacto_push"]:
        wrap(lr.kv, n, "kv." + n)
    card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=dev)
    wrap(hip, "synth_criteo", "synth")
    for s in range(5):
        k, l, o = hip.synth_criteo(args.batch, 1, s, card)
        lr.process(k, o, None, l, 0, 0)
    torch.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    for s in range(args.steps):
        k, l, o = hip.synth_criteo(args.batch, 1, 10 + s, card)
        lr.process(k, o, None, l, 0, 0)
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    tot = 0
    for k_, v in sorted(acc.items(), key=lambda x: -x[1]):
        tot += v
        print("%-22s %8.1f us/step" % (k_, 1e6 * v / args.steps))
    print("sum %.1f us/step, wall %.1f us/step" % (1e6 * tot / args.steps,
                                                   1e6 * t_all / args.steps))


if __name__ == "__main__":
    main()
