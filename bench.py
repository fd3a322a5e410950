#!/usr/bin/env python3
"""Headline benchmark: DiFacto FM (embedding dim 64) training throughput on
Criteo-1TB-shaped sparse data, examples/sec over all GPUs (BASELINE.json).

Config follows the reference's own Criteo DiFacto conf
(learn/difacto/guide/criteo.conf: minibatch 100000, threshold 100, V lambda_l2
1, lr_eta .01) with the embedding dim set to 64 as BASELINE.json names.  Data
is synthetic (13 integer + 26 categorical fields, Criteo-1TB field
cardinalities, power-law values) generated on the device every step; the
model is random-initialised.  Every timed step is a full training step:
generate -> localize -> key all-to-all -> count push (data pass 0) -> pull ->
FM forward + loss + AUC -> FM backward -> push -> fused FTRL/AdaGrad update.

Weak scaling: each GPU processes its own minibatch of --batch rows per step;
the keys are sharded over all GPUs (ps-lite server group -> xGMI all-to-all).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model difacto|linear]

``--gpus N`` with N > 1 and no launcher around it starts the N ranks itself
(``torch.distributed.run`` on 127.0.0.1, one process per GPU, the launch the
driver uses); every rank checks that the group has N members on N distinct
GPUs. The JSON line also reports the RCCL rank count, the per-rank step time
spread and the bytes each GPU sends to its peers per step in each collective.
"""
import argparse
import json
import os
import sys
import time

# (before torch: the HIP runtime reads it when it initialises; see
# wormhole_amd/__init__.py)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from wormhole_amd.config.schema import DifactoConfig, Embedding, LinearConfig  # noqa: E402
from wormhole_amd.data.synthetic import CRITEO_TB_CARD  # noqa: E402
from wormhole_amd.parallel.comm import Comm, env_local_rank  # noqa: E402
from wormhole_amd.parallel import launch  # noqa: E402

LINEAR_REF_EX_PER_S = 1.85e6  # linear.dmlc FTRL, Criteo, CPU host


def build(args, comm, device):
    if args.model == "difacto":
        from wormhole_amd.models.difacto import DifactoLearner
        emb = Embedding(dim=args.dim, threshold=100, lambda_l2=1.0, lr_eta=0.01)
        emb._set = {"dim", "threshold", "lambda_l2", "lr_eta"}
        conf = DifactoConfig(minibatch=args.batch, lr_eta=0.01, embedding=[emb],
                             fixed_bytes=args.fixed_bytes, max_concurrency=args.max_concurrency)
        return DifactoLearner(conf, comm, device, cap=args.cap, vcap=args.vcap, seed=1)
    from wormhole_amd.models.linear import LinearLearner
    conf = LinearConfig(minibatch=args.batch, lambda_l1=4.0, lr_eta=0.1)
    return LinearLearner(conf, comm, device, cap=args.cap, seed=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="difacto", choices=["difacto", "linear"])
    ap.add_argument("--batch", type=int, default=None,
                    help="rows per GPU per step (default: difacto 100000 as the reference's "
                         "criteo.conf; linear 10000 as the published criteo_kaggle.rst run)")
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--cap", type=int, default=1 << 27, help="KV slots per GPU shard")
    ap.add_argument("--vcap", type=int, default=1 << 24, help="embedding rows per shard")
    ap.add_argument("--fixed-bytes", type=int, default=0, choices=[0, 1, 2, 3],
                    help="ps-lite FIXING_FLOAT filter on the exchanged embedding rows "
                         "(lossy; the reference default 0 is used for the headline)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo rehearsal of the distributed path (tiny batches only)")
    ap.add_argument("--prewarm", type=int, default=None,
                    help="untimed training steps run before --warmup to bring the model "
                         "to a fixed warm state (embedding rows allocated by the count "
                         "threshold grow with the steps seen; default 1000 for difacto)")
    ap.add_argument("--loopback", type=int, default=0,
                    help="P > 1: run the multi-shard exchange path with P virtual shards "
                         "in this one process (identity transport; measures that path's "
                         "device + host overhead on one GPU)")
    ap.add_argument("--loopback-rccl", action="store_true",
                    help="with --loopback: issue every exchange as a real RCCL all-to-all on a "
                         "1-rank group (the RCCL stream/async semantics of the multi-GPU step)")
    ap.add_argument("--max-concurrency", type=int, default=2,
                    help="minibatches in flight per worker (reference default 2): with >= 2 "
                         "the multi-shard step is pipelined one minibatch deep")
    ap.add_argument("--host-profile", default=None,
                    help="write a cProfile of the timed steps' host (Python) side to PATH.<rank>")
    ap.add_argument("--launch-timeout", type=int, default=540,
                    help="self-launched multi-rank runs are killed after this many seconds "
                         "(below the driver's 600 s bench limit, so a stuck run still ends "
                         "with this launcher's message; the native step's own watchdog, "
                         "WH_RCCL_TIMEOUT_S, ends a stalled exchange sooner)")
    args = ap.parse_args()
    if args.gpus > 1 and args.loopback <= 1 and not launch.launched():
        # no launcher around us: start the N ranks ourselves (before any GPU
        # call in this process) and pass their exit code through
        return launch.self_launch(os.path.abspath(__file__), sys.argv[1:], args.gpus,
                                  args.device, args.launch_timeout)
    if args.batch is None:
        args.batch = 100000 if args.model == "difacto" else 10000
    if args.prewarm is None:  # (the CPU rehearsal of the distributed path skips it)
        args.prewarm = 1000 if (args.model == "difacto" and args.device == "cuda") else 0

    local = env_local_rank()
    if os.environ.get("WH_BENCH_SAME_GPU") == "1":
        local = 0  # rehearsal aid: every rank on GPU 0 (1-GPU box, multi-rank code path)
    if args.device == "cuda":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
        args.cap, args.vcap = min(args.cap, 1 << 16), min(args.vcap, 1 << 14)
    if args.loopback > 1:
        from wormhole_amd.parallel.comm import LoopbackComm
        comm = LoopbackComm(args.loopback, device, rccl=args.loopback_rccl)
    else:
        # (c10d's own collectives time out well inside the driver's limit)
        comm = Comm(device, timeout_s=int(os.environ.get("WH_RCCL_TIMEOUT_S", "120")) + 60)
        # the group is what --gpus says, on distinct devices
        launch.verify_world(comm, args.gpus if launch.launched() else 1,
                            same_gpu_ok=os.environ.get("WH_BENCH_SAME_GPU") == "1")
    n = 1 if args.loopback > 1 else comm.size  # GPUs doing work
    learner = build(args, comm, device)
    seed = 1000 + comm.rank
    if device.type == "cuda":
        from wormhole_amd import _native
        hip = _native.hip()
        card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=device)

        def batch(step):
            return hip.synth_criteo(args.batch, seed, step, card)
    else:
        from wormhole_amd.data.synthetic import criteo_batch_cpu

        def batch(step):
            return criteo_batch_cpu(args.batch, seed, step, CRITEO_TB_CARD)

    # Minibatch i+1 is generated and its localization begun before minibatch
    # i trains (learner.process(next_batch=...)): the one host read of the
    # unique-id counts then overlaps i's kernels. The pipeline does not cross
    # the warm-up / timed boundary, so every timed step's work is timed.
    # On the GPU the next minibatch is generated on its own stream (as the
    # file path's H2D copies run on theirs), concurrently with this
    # minibatch's localize; the learner waits on its event just before the
    # next localize begins.
    gen = torch.cuda.Stream(device) if device.type == "cuda" else None
    main = torch.cuda.current_stream(device) if device.type == "cuda" else None
    if gen is not None:
        from wormhole_amd.utils import streams
        evs = streams.EventRing(8)

    def batch_async(step):
        if gen is None:
            return batch(step), None
        with streams.on(gen):
            out = batch(step)
        out[1].record_stream(main)  # the label (keys / offsets: recorded by the learner)
        return out, evs.record(gen)

    def run(first, n):
        nxt, ev = batch(first), None
        for s in range(first, first + n):
            keys, label, offset = nxt
            nxt, ev = batch_async(s + 1) if s + 1 < first + n else (None, None)
            learner.process(keys, offset, None, label, 0, 0,
                            next_batch=(nxt[0], nxt[2], None, ev) if nxt is not None else None)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    # fixed warm state: the same number of untimed steps whatever --warmup is
    # (seeded apart from the timed steps' data)
    if args.prewarm > 0:
        seed0 = seed
        seed = 7000000 + comm.rank
        run(0, args.prewarm)
        seed = seed0
    run(0, args.warmup)
    learner.flush()
    sync()
    comm.barrier()
    sync()
    prof = None
    if args.host_profile:  # host-side (Python) profile of the timed steps
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    psx = getattr(learner, "psx", None)
    if psx is not None:
        psx.wire_reset()  # count the timed steps' exchange bytes only
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    learner.flush()  # the last step's (deferred) push is part of the timed work
    sync()
    comm.barrier()
    sync()
    dt = time.perf_counter() - t0
    if prof is not None:
        import pstats
        prof.disable()
        with open(args.host_profile + ".%d" % comm.rank, "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(40)
            pstats.Stats(prof, stream=f).sort_stats("cumulative").print_stats(60)
    per_rank = [float(x) for x in comm.allgather_object(dt)] if comm.size > 1 and \
        args.loopback <= 1 else [dt]
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    comm.allreduce(t, "max")
    dt = float(t.item())
    wire = psx.wire_report(args.steps) if psx is not None else None
    # sampled GPU time of each exchange class on the native RCCL step, per rank
    nat = getattr(psx, "_nat", None) if psx is not None else None
    xt = [round(v, 1) for v in nat.xtime()[:4]] if nat else None
    xts = comm.allgather_object(xt) if comm.size > 1 and args.loopback <= 1 else [xt]
    prog = learner.take_progress()
    guard = learner.kv.guard
    guard.after_open()
    guard.read()  # raises on any dropped key or embedding row
    sizes = getattr(learner, "last_sizes", None)
    if sizes is not None:  # last minibatch: unique keys and embedding rows per GPU
        sizes = [int(sizes[0]), int(sizes[1].reshape(-1)[0].item()) if torch.is_tensor(sizes[1]) else int(sizes[1])]
    ex = args.batch * args.steps * n
    value = ex / dt
    if args.model == "difacto":
        metric = "examples/sec, DiFacto FM on Criteo-1TB-shaped sparse at 1/2/4/8 MI355X"
        vs = None
        model = "difacto-fm-dim%d" % args.dim
    else:
        metric = "examples/sec, linear FTRL logistic regression on Criteo-shaped sparse"
        vs = value / LINEAR_REF_EX_PER_S
        model = "linear-ftrl"
    if comm.rank == 0:
        if args.model == "difacto":  # learn/difacto/progress.h layout
            logloss, auc = prog[0] / max(prog[5], 1.0), prog[1] / max(prog[4], 1.0)
        else:  # learn/linear/progress.h layout
            logloss, auc = prog[0] / max(prog[4], 1.0), prog[2] / max(prog[3], 1.0)
        print(json.dumps({
            "metric": metric, "value": value, "unit": "examples/s", "n_gpus": n,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1000.0 * dt / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": vs, "dtype": "fp32",
            "data": "synthetic (Criteo-1TB-shaped: 13 int + 26 cat fields, power-law, device-generated each step); random-init model",
            "config": {"model": model, "global_batch": args.batch * n, "seq_len": 39,
                       "parallelism": ("loopback%d%s(1 GPU)" % (args.loopback, "-rccl" if args.loopback_rccl else "")
                                       if args.loopback > 1
                                       else "dp%d+kvshard%d" % (n, n)),
                       "minibatch_per_gpu": args.batch, "threshold": 100, "nnz_per_example": 39},
            "train_logloss": logloss, "train_auc": auc,
            "uniq_keys_per_gpu_step": sizes[0] if sizes else None,
            "emb_rows_per_gpu_step": sizes[1] if sizes else None,
            "prewarm_steps": args.prewarm,
            "table_keys_per_gpu": guard.keys, "table_load": guard.keys / learner.store.cap,
            "table_grows": guard.grows, "vslab_rows_per_gpu": guard.vused,
            "dropped_keys": 0, "max_concurrency": args.max_concurrency,
            "loopback_shards": args.loopback if args.loopback > 1 else None,
            "rccl_ranks": comm.size if (comm.backend == "nccl" and args.loopback <= 1) else 0,
            "comm_backend": comm.backend,
            "rank_ms_per_step_min": 1000.0 * min(per_rank) / args.steps,
            "rank_ms_per_step_max": 1000.0 * max(per_rank) / args.steps,
            "wire_bytes_per_gpu_step": wire,
            "exchange_gpu_us_per_rank": ({"C0": [x[0] for x in xts], "C1": [x[1] for x in xts],
                                          "C2": [x[2] for x in xts], "C3": [x[3] for x in xts]}
                                         if xts and xts[0] is not None else None),
            "watchdog_deadline_s": nat.watchdog_deadline if nat else None,
            "localize_retries": (_native.hip().loc_retries() if device.type == "cuda" else 0),
        }), flush=True)
    comm.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
