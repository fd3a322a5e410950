"""Parameter-server solver runtime, worker side; the
scheduler is native (csrc/host/scheduler.cc, ``_host.run_scheduler``).

Reference layering (learn/solver/): DataParScheduler/Worker (dynamic
workload dispatch, data_parallel.h) < IterScheduler/Server/Worker (model
load/save, progress, prediction files, iter_solver.h) < MinibatchScheduler/
Worker (epoch loop, minibatch streaming, minibatch_solver.h).

MI355X design: one worker process per GPU; every worker also owns a shard of
the parameter store (the ps-lite server group is folded into the workers and
push/pull are all-to-all collectives over xGMI).  The scheduler is a separate
CPU process that keeps the reference's control semantics: it matches files,
splits them into ``num_parts_per_file`` virtual parts, hands them out one at
a time from the native WorkloadPool, sum-merges progress and prints the
reference progress table every ``print_sec``, and fans out load/save.

Because collectives are group-synchronous, workers step in lockstep: a worker
whose current part is exhausted asks for another; once the pool is empty it
keeps joining the collectives with empty minibatches until no rank has data,
which every rank learns from the has-data flags the per-step count exchange
already carries (SURVEY §7.5 hard part 1; no extra collective per
minibatch).  ``max_concurrency`` bounds the minibatches in flight per worker
(the multi-shard step pipelines one minibatch deep by default).
"""
import json
import collections
import os
import sys
import time

import torch

from .. import _native
from ..kv import checkpoint
from ..utils.fs import open_uri  # noqa: E402
from ..utils import trace  # noqa: E402
from ..data import device_text

TRAIN, VAL, PRED = 0, 1, 2
_TYPE_NAME = {TRAIN: "training", VAL: "validation", PRED: "prediction"}


def _msg(**kw):
    return json.dumps(kw).encode()


def _log(*a):
    print(*a, file=sys.stderr, flush=True)


def _parse_fault(spec, rank):
    """WH_FAULT=kill:<rank>:<after_n_minibatches> | sleep:<rank>:<sec_per_minibatch>
    | stall:<rank>:<sec>[:<after_n_minibatches>] (once) -- fault injection for
    the failure / straggler tests. A kill fires only in the
    first attempt of a job (the launcher's restart runs clean)."""
    if not spec:
        return None
    kind, r, arg, *after = spec.split(":")
    if int(r) != rank:
        return None
    if kind == "stall":
        return kind, float(arg), int(after[0]) if after else 0
    if kind == "kill" and int(os.environ.get("WH_RESTART_ATTEMPT", "0") or 0) > 0:
        return None  # the injected failure happens once; the restarted job runs clean
    return kind, float(arg)


# --------------------------------------------------------------------------
# worker
# --------------------------------------------------------------------------
class Worker:
    """MinibatchWorker + IterServer of its shard (minibatch_solver.h:200-330,
    iter_solver.h:77-167)."""

    def __init__(self, conf, app, learner, comm, van, nshard, kind):
        self.conf = conf
        self.app = app
        self.learner = learner
        self.comm = comm
        self.van = van
        self.nshard = nshard
        self.kind = kind  # "linear" | "difacto"
        self.device = learner.device
        self.host = _native.host()
        self.report_sec = max(0.1, float(conf.print_sec) / 2)
        self.n_done = 0
        self.metrics = trace.MetricsStream(comm.rank)
        self.fault = _parse_fault(os.environ.get("WH_FAULT", ""), comm.rank)
        if os.environ.get("WH_HANG_DUMP"):  # debug aid: all threads' stacks every N s
            import faulthandler
            faulthandler.dump_traceback_later(float(os.environ["WH_HANG_DUMP"]), repeat=True)
        self.saver = checkpoint.AsyncSaver()

    def send(self, **kw):
        self.van.send("scheduler", _msg(**kw))

    def recv(self):
        while True:
            m = self.van.recv(1.0)
            if m is None:
                continue
            _, raw = m
            if raw == b"__closed__":
                raise SystemExit("scheduler connection lost")
            return json.loads(raw)

    def serve(self):
        self.send(msg="ready", rank=self.comm.rank)
        while True:
            d = self.recv()
            cmd = d.get("cmd")
            if cmd == "exit":
                self.saver.join()
                return
            if cmd in ("save", "load"):
                self.learner.flush()
            if cmd == "save":
                if self.comm.rank < self.nshard:
                    name = checkpoint.model_name(d["file"], d["iter"], self.comm.rank)
                    # periodic saves (save_iter) write in the background while
                    # the next pass trains; the final save completes before
                    # its ack
                    self.saver.save(self.kind, self.learner.store, name)
                    if d["iter"] < 0:
                        self.saver.join()
                self.comm.barrier()
                self.send(msg="ack")
            elif cmd == "load":
                self.saver.join()
                if self.comm.rank < self.nshard:
                    name = checkpoint.model_name(d["file"], d["iter"], self.comm.rank)
                    fn = checkpoint.load_linear if self.kind == "linear" else checkpoint.load_difacto
                    fn(self.learner.store, name)
                    if d.get("resume"):
                        checkpoint.load_state(self.learner.store, name)
                self.comm.barrier()
                self.send(msg="ack")
            elif cmd == "match":
                self.send(msg="matched", files=self.host.match_file(d["data"]))
            elif cmd == "iterate":
                self.run_pass(d["type"], d["data_pass"], d.get("fmt", self.conf.data_format))

    def _inject_fault(self):
        kind, arg = self.fault[:2]
        if kind == "kill" and self.n_done >= arg:
            _log("[worker %d] WH_FAULT: killing myself after %d minibatches" % (
                self.comm.rank, self.n_done))
            os._exit(17)
        if kind == "sleep":
            time.sleep(arg)
        if kind == "stall" and self.n_done >= self.fault[2]:
            self.fault = None
            _log("[worker %d] WH_FAULT: stalling %.1f s" % (self.comm.rank, arg))
            time.sleep(arg)

    # -------------------------------------------------------- one pass
    def _empty_batch(self):
        dev = self.device
        return (torch.zeros(0, dtype=torch.int64, device=dev),
                torch.zeros(1, dtype=torch.int64, device=dev), None,
                torch.zeros(0, dtype=torch.float32, device=dev))

    def _to_dev(self, b):
        if isinstance(b, device_text.DeviceBatch):
            return b.to_main(self.device)
        keys, off, val, label, _w = b
        dev = self.device
        nb = dev.type == "cuda"
        keys = keys.to(dev, non_blocking=nb)
        off = off.to(dev, non_blocking=nb)
        label = label.to(dev, non_blocking=nb)
        if val is not None:
            val = val.to(dev, non_blocking=nb)
        return keys, off, val, label

    def run_pass(self, wtype, data_pass, fmt):
        c = self.conf
        train = wtype == TRAIN
        mb = c.minibatch if train else 10_000_000 if wtype == PRED else 100_000
        shuf = c.minibatch * c.rand_shuffle if (train and c.rand_shuffle > 0) else 0
        neg = c.neg_sampling if train else 1.0
        pred_f = None
        pred_name = None
        last = time.time()
        seed = 1000003 * (data_pass + 1) + self.comm.rank
        # Workloads are prefetched one ahead: as soon as one starts, the next
        # is requested and its MinibatchIter built, so its parser threads run
        # while this one trains (the reference's worker keeps max_concurrency
        # minibatches in flight for the same reason). A finished workload is
        # reported by name, so the prefetched one stays assigned.
        queue = collections.deque()
        # workloads in flight: the threaded host parser keeps 16 threads busy
        # on one; device-parsed text only reads on the host (one thread per
        # workload), so more workloads read ahead in parallel
        dev_text = device_text.applies(fmt, "", self.device)
        prefetch = int(os.environ.get("WH_PREFETCH_PARTS", "4" if dev_text else "2"))
        exhausted = False
        done_prev = None
        n_pass = n_ex = ex_last = 0
        pass_stages = {}
        trace.take()  # stage times of this pass only
        t_pass = time.time()

        def fetch():
            nonlocal exhausted, done_prev
            if exhausted:
                if done_prev is not None:  # nothing left to request: report it alone
                    self.send(msg="finished", finished=done_prev)
                    done_prev = None
                return
            self.send(msg="request", finished=done_prev)
            done_prev = None
            d = self.recv()
            if d.get("file") is None:
                exhausted = True
                return
            if device_text.applies(fmt, d["file"], self.device):
                it = device_text.DeviceTextIter(self.host, d["file"], d["k"], d["n"], fmt, int(mb),
                                                int(shuf), float(neg), seed + d["k"], self.device)
            else:
                it = self.host.MinibatchIter(d["file"], d["k"], d["n"], fmt, int(mb), int(shuf),
                                             float(neg), seed + d["k"],
                                             self.device.type == "cuda")  # pinned: async H2D
            queue.append((d, it))

        def next_parsed():
            """The next minibatch of this worker (None once its parts are
            exhausted); prediction output files follow the workload."""
            nonlocal pred_f, pred_name, done_prev
            batch = None
            while queue and batch is None:
                d, it = queue[0]
                if wtype == PRED:
                    base = os.path.basename(d["file"])
                    name = "%s%s_part-%d" % (c.predict_out, base, d["k"])
                    if name != pred_name:
                        if pred_f:
                            pred_f.close()
                        pred_f = open_uri(name, "w")
                        pred_name = name
                if len(queue) < prefetch:
                    fetch()  # the next workload starts reading / parsing now
                with trace.stage("parse"):
                    batch = it.next()
                if batch is None:
                    queue.popleft()
                    done_prev = {"file": d["file"], "k": d["k"]}
                    if not queue:
                        fetch()
            return batch

        # Training parses one minibatch ahead and hands it to the learner
        # (next_batch), which begins its localization -- and, on several
        # ranks, the count exchange -- before training the current one, as
        # bench.py does.
        #
        # Several ranks (the multi-shard step, kv/psx.py): every rank calls
        # process() once per step, with an empty minibatch once its parts are
        # exhausted, and always hands a look-ahead (empty if it has none), so
        # the count collectives stay in lockstep. Each count exchange carries
        # a has-data flag per rank: the first call in which NO rank had data
        # reports learner.last_empty on every rank at once, and the pass ends
        # there -- no per-minibatch collective or host read of its own
        # (learn/solver/minibatch_solver.h:284-322). The embedding-free /
        # quantised-payload learners without that step fall back to one
        # "have data" allreduce per minibatch.
        multi = self.comm.size > 1
        flags = multi and getattr(self.learner, "psx", None) is not None
        # (the allreduce fallback gives no lockstep look-ahead decision, so it
        # runs without one)
        ahead = train and (flags or not multi)

        def dev_or_empty(b):
            return self._to_dev(b) if b is not None else self._empty_batch()

        fetch()
        batch = next_parsed()
        args = dev_or_empty(batch) if (batch is not None or multi) else None
        nxt = next_parsed() if (ahead and batch is not None) else None
        nargs = None
        if ahead and (nxt is not None or flags):
            nargs = dev_or_empty(nxt)
        while True:
            if not multi and batch is None:
                break
            if multi and not flags:
                flag = torch.tensor([1 if batch is not None else 0], dtype=torch.int32,
                                    device=self.comm.device)
                self.comm.allreduce(flag)
                if int(flag.item()) == 0:
                    break
            if self.fault and batch is not None:
                self._inject_fault()
            with trace.stage("process"):
                nb = (nargs[0], nargs[1], nargs[2]) if nargs is not None else None
                py = self.learner.process(*args, wtype=wtype, data_pass=data_pass,
                                          next_batch=nb)
            if flags and self.learner.last_empty:
                break  # no rank had data in this step: every rank stops here
            self.n_done += 1
            n_pass += 1
            n_ex += int(args[3].numel())
            if wtype == PRED and batch is not None:
                p = py.float().cpu()
                if c.prob_predict:
                    p = torch.sigmoid(p)
                pred_f.write("".join("%g\n" % v for v in p.tolist()))
            if time.time() - last > self.report_sec:
                now = time.time()
                if self.metrics.f is not None:
                    st = trace.take()
                    for k, v in st.items():
                        a = pass_stages.setdefault(k, [0.0, 0])
                        a[0] += v[0]
                        a[1] += v[1]
                    self.metrics.write(event="progress", wtype=int(wtype), data_pass=data_pass,
                                       examples=n_ex - ex_last,
                                       examples_per_sec=(n_ex - ex_last) / max(now - last, 1e-9),
                                       stages_sec={k: v[0] for k, v in st.items()})
                    ex_last = n_ex
                last = now
                self.send(msg="progress", data=self.learner.take_progress())
            with trace.stage("h2d"):
                if ahead:
                    # the look-ahead batch (already on the device, its
                    # localize begun) is the next step's: the SAME objects
                    batch, args = nxt, nargs
                    nxt = next_parsed() if batch is not None else None
                    nargs = dev_or_empty(nxt) if (nxt is not None or flags) else None
                    if args is None and multi:
                        args = self._empty_batch()
                else:
                    batch = next_parsed()
                    args = dev_or_empty(batch) if (batch is not None or multi) else None
        if pred_f:
            pred_f.close()
        # the reference worker's summary line (minibatch_solver.h:244-248)
        for k, v in trace.take().items():
            a = pass_stages.setdefault(k, [0.0, 0])
            a[0] += v[0]
            a[1] += v[1]
        wall = time.time() - t_pass
        if n_pass:
            _log("[worker %d] %s" % (self.comm.rank, trace.overhead_line(
                {k: tuple(v) for k, v in pass_stages.items()}, wall, n_pass)))
        self.metrics.write(event="pass_done", wtype=int(wtype), data_pass=data_pass,
                           minibatches=n_pass, examples=n_ex, wall_sec=wall,
                           examples_per_sec=n_ex / max(wall, 1e-9),
                           stages_sec={k: v[0] for k, v in pass_stages.items()})
        if done_prev is not None:
            self.send(msg="finished", finished=done_prev)
        self.learner.flush()  # collective: every rank leaves the loop together
        self.send(msg="pass_done", progress=self.learner.take_progress())
