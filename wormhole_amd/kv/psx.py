"""Lean multi-shard parameter-server step of DiFacto and the linear model:
P > 1 ranks over RCCL/xGMI, or P virtual shards on one GPU
(:class:`wormhole_amd.parallel.comm.LoopbackComm`); keys owned by the first
S <= P ranks (``-s S``).

Reference per-minibatch flow (learn/difacto/async_sgd.h:372-424): push the
feature counts (kPushFeaCnt) -> ZVPull(w, V) -> compute -> ZVPush(gw, gV),
with ``max_concurrency`` (default 2, learn/difacto/config.proto:154)
minibatches in flight per worker, so minibatch i+1 may pull before
minibatch i's push has landed.

Here a minibatch costs four collectives and no extra host synchronisation
(see csrc/hip/psx.hip for the row-aligned wire layout):

  C0  {key count, overflow flag, V rows of the previous pull, has data} per
      peer: the localize count exchange, read by the host together with the
      counts (the ONE host read of the step). The has-data flags end a pass
      without any other collective: once no rank has a minibatch left, every
      rank sees it in the same read (learn/solver/minibatch_solver.h:284-322
      streams minibatches without a per-minibatch barrier either).
  C1  keys (+ counts in data pass 0), 12-byte records
  C2  pull reply: per peer one region [header rows | V rows]
  C3  push: the same regions back, [gw | gV rows]

The owner's open (find/insert, count, lazy V, variable-length pull) and its
push are one kernel each over all P segments. With ``max_concurrency >= 2``
the step is software-pipelined one minibatch deep (staleness 1, as the
reference allows by default); a call of :meth:`Psx.train` enqueues,
on the compute stream S,

    unpack(i-1) fwd(i-1) | owner push(i-2) | owner open(i) pack(i) |
    bwd(i-1) pack_gw(i-1) [+ AUC(i-1) on its side stream]

while the localize of minibatch i+1 runs on its own stream, begun as soon as
minibatch i's localize is finished (its count collective deferred until
after open(i), whose V row counts it carries). The collectives go out in the
order C2(i-1), C3(i-2), C1(i), C0(i+1): RCCL runs them in issue order on the
process group's stream, so the push of the previous backward (C3(i-2)) is
issued behind this call's pull reply rather than at the end of that
backward -- C2 then overlaps the backward's tail and C3 the forward, instead
of the two big transfers running back to back between them. C1-C3 are
waited on (a stream dependency, not a host wait) right before the kernel
that consumes them; C0 and its pinned host read run from a side stream the
compute stream never waits on. The host's wait for the read of C0(i+1)
happens in the NEXT call while S still holds bwd(i-1), so S never drains.
``max_concurrency = 1`` gives the strict (staleness 0) order at the cost of
one pipeline drain per step.

The linear model (learn/linear/async_sgd.h:240-301: ZPull w -> gradient ->
ZPush) runs the same pipeline with C1 = 8-byte keys, C2 = one w per key, C3 =
one gradient per key; its owner push applies SGD / AdaGrad / FTRL over all
segments in one launch, each worker's gradients as one request in peer order.
An embedding-free DiFacto model takes the same wire format, its owner push
applying DiFacto's FTRL on w (push algo 4).

Payload filter (``fixed_bytes`` 1-3: ps-lite FIXING_FLOAT,
learn/difacto/async_sgd.h:428-445, learn/linear/async_sgd.h:290-301): the
embedding rows of C2 / C3 (DiFacto) and the gradients of C3 (linear: the
reference filters its pushes only) travel as n-byte fixed point with one
scale per 64-float record and unbiased random rounding, the {w, vidx}
headers exact (csrc/hip/quant.hip qregion kernels: packed on the producer's
stream right before the collective, unpacked by its consumer); the feature
counts of C1 saturate at 255 (TRUNCATE_FLOAT(1) of the count push).
"""
import contextlib
import os

import numpy as np
import torch

from .. import _native, ops
from ..utils import streams, trace

TRAIN, VAL, PRED = 0, 1, 2
# (Stream placements measured and dropped -- docs/performance.md "Measured
# dead ends": the owner push on its own stream beside the forward, the next
# localize on a side stream at the open instead of right after this one's
# localize, C3 issued at the end of the backward instead of behind the next
# call's C2, a training step's AUC right after its forward.)
_COMM_TIMING = trace.timing_on("comm")
# CUs the persistent FM kernels leave free for RCCL's channel workgroups when
# the exchange runs over RCCL (csrc/hip/fm.hip fm_set_cu_reserve): C2 / C3
# are issued while a forward / backward holds the machine, and must start
# then rather than after it drains. (The forward's persistent grid fills all
# 32 wave slots of every CU.) 16 CUs leave ~500 wave slots for RCCL's channel
# workgroups; on one GPU (RCCL loopback, one channel) the reserve costs 1 %
# at 16 CUs, 3 % at 32, 7 % at 64 (99.4 / 98.5 / 96.3 / 92.9 M ex/s).
_CU_RESERVE = int(os.environ.get("WH_RCCL_CU_RESERVE", "16"))


def _cdiv(a, b):
    return -(-a // b)


class _Step:
    """One minibatch in flight through the exchange."""

    __slots__ = ("train", "use_cnt", "U", "uniq", "ucnt", "lid", "offset", "val", "csc",
                 "label", "send", "recv", "Hw", "Ho", "tabs", "segS_w", "segHS_w", "segS_o",
                 "segHS_o", "keys_o", "slot", "vpos", "chain", "head", "rbuf", "vcnt",
                 "ev_open", "ev_grad",
                 "vown", "vrecv", "vrecv_d", "rrecv", "hdr", "rows", "py", "dual", "xv",
                 "gpush", "gvc", "seed_step", "w_c1", "w_c2", "w_c3", "q2", "q3")

    def __init__(self):
        for s in self.__slots__:
            setattr(self, s, None)


class _PinRing:
    """Host -> device uploads of small int64 tables through a ring of
    pre-pinned buffers (no pinned allocation per step); a slot is reused only
    after its previous copy's event completed (long before, in practice)."""

    def __init__(self, dev, n=8, width=4096):
        self.dev = dev
        self.buf = [torch.empty(width, dtype=torch.int64, pin_memory=True) for _ in range(n)]
        self.ev = [None] * n
        self.i = 0

    def put(self, arr):
        k = self.i
        self.i = (k + 1) % len(self.buf)
        if arr.shape[0] > self.buf[k].numel():
            self.buf[k] = torch.empty(2 * arr.shape[0], dtype=torch.int64, pin_memory=True)
        if self.ev[k] is not None:
            self.ev[k].synchronize()
        h = self.buf[k][:arr.shape[0]]
        h.numpy()[:] = arr
        d = h.to(self.dev, non_blocking=True)
        if self.ev[k] is None:
            self.ev[k] = torch.cuda.Event()
        self.ev[k].record()
        return d


class _CollTimer:
    """GPU time of each collective from the moment its inputs are ready on
    the issuing stream to the moment it has landed (a timing stream waits
    on the work, then records): RCCL's own queueing behind earlier
    collectives is included, which is what the step waits for."""

    def __init__(self, dev):
        self.ts = torch.cuda.Stream(device=dev)
        self.pairs = []
        self.pend = {}

    def ready(self, c):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.pend[c] = ev

    def done(self, c, work):
        w = getattr(work, "work", None)
        end = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.ts):
            if w is not None:
                w.wait()
            else:
                self.ts.wait_stream(torch.cuda.current_stream())
            end.record(self.ts)
        self.pairs.append((c, self.pend.pop(c), end))

    def reset(self):
        self.pairs = []

    def report(self):
        out = {}
        for c, a, b in self.pairs:
            b.synchronize()
            out[c] = out.get(c, 0.0) + a.elapsed_time(b)
        return out


class _QFilter:
    """The fixed_bytes payload filter's region tables (see the module doc):
    per peer {sf, a, vf, nf, sq, ha} -- float offset of the region, exact
    floats, offset and count of the quantised floats, first wire row, raw
    wire rows -- from the host-known key / row counts of a step."""

    def __init__(self, nb, vs, seed, rank, linear):
        from ..ops import ref
        self.nb = int(nb)
        self.vs = max(int(vs), 1)
        self.linear = linear
        self.W = 64 if linear else self.vs  # floats per record
        self.R = ref.quant_record_bytes(self.W, self.nb)
        self.seed = (int(seed) * 0x9E3779B1 + 17 * int(rank) + 1) & 0x7FFFFFFFFFFF
        self.calls = 0

    def layout(self, n, v, H):
        """n keys, v embedding rows, H header rows per peer -> (desc [P, 6],
        wire rows per peer, floats of the float layout)."""
        P = len(n)
        d = np.zeros((P, 6), dtype=np.int64)
        rows = []
        sf = sq = 0
        for p in range(P):
            if self.linear:
                a, vf, nf, ha = 0, 0, int(n[p]), 0
                nr, ext = _cdiv(int(n[p]), self.W), int(n[p])
            else:
                a, vf, nf = 2 * int(n[p]), int(H[p]) * self.vs, int(v[p]) * self.vs
                ha, nr = _cdiv(4 * a, self.R), int(v[p])
                ext = (int(H[p]) + int(v[p])) * self.vs
            d[p] = (sf, a, vf, nf, sq, ha)
            rows.append(ha + nr)
            sf += ext
            sq += ha + nr
        return d, rows, sf

    def next_seed(self):
        self.calls += 1
        return self.seed + (self.calls << 20)


class Psx:
    """The pipelined multi-shard step of both PS learners (DiFacto:
    vstride > 0; linear: vstride == 0, where C1 moves 8-byte keys, C2 one
    float w per key and C3 one float gradient per key). Keys are owned by
    the first S = ``lrn.kv.nshard`` ranks (the conf's ``-s S`` servers);
    every rank is a worker."""

    def __init__(self, lrn):
        self.lrn = lrn
        self.comm = lrn.comm
        self.store = lrn.store
        self.P = self.comm.size
        self.nshard = max(1, min(int(lrn.kv.nshard), self.P))
        self.vs = self.store.vstride
        self.linear = self.vs == 0
        self.dev = lrn.device
        self.cuda = self.dev.type == "cuda"
        self.cs = torch.cuda.Stream(device=self.dev) if self.cuda else None
        # the next minibatch's localize runs on its own stream, begun as soon
        # as this minibatch's localize is finished (as on one shard,
        # models/_pipeline.py), concurrently with the forward / push / open
        self.ls = torch.cuda.Stream(device=self.dev) if self.cuda else None
        # C2 / C3 are issued from xs, each behind its producer's event only
        # (see _a2a)
        self.xs = torch.cuda.Stream(device=self.dev) if self.cuda else None
        self._ring = streams.EventRing(32) if self.cuda else None
        self.S = torch.cuda.current_stream(self.dev) if self.cuda else None
        if self.cuda and getattr(self.comm, "backend", "") in ("nccl", "loopback-rccl"):
            _native.hip().set_cu_reserve(_CU_RESERVE)
        self.pins = _PinRing(self.dev) if self.cuda else None
        # staleness: max_concurrency - 1 minibatches may pull before a push
        # of theirs lands (the reference's in-flight bound,
        # learn/solver/minibatch_solver.h:284-322). The native step honours
        # any depth up to 8; this Python step (the oracle, and the payload-
        # filter configurations) pipelines at most one deep, which stays
        # within the bound.
        mc = int(getattr(lrn.conf, "max_concurrency", 2) or 2)
        if mc < 1 or mc > 9:
            raise ValueError("max_concurrency must be 1..9 (got %d)" % mc)
        self.tau_max = mc - 1
        self.tau = min(self.tau_max, 1)
        self.job = None     # (keys, LocalizeJob | finished tuple, carried step)
        self.pull = None    # opened, reply not yet exchanged
        self.push = None    # push in flight to the owners
        self.uhint = 0
        # set by train / evaluate: no rank had data for that call's minibatch
        # (read from the has-data flags every C0 carries), so the call did
        # nothing but its count exchange and the pass is over
        self.last_empty = False
        # linear SGD: push requests this owner has applied (ps-lite's t)
        self.requests = 0
        # bytes this rank sends to OTHER ranks per collective (C0..C3): what
        # crosses xGMI (own-segment rows stay in HBM)
        self.wire = [0, 0, 0, 0]
        # WH_TIMING=comm: per-collective (issue-ready -> landed) GPU times
        self.timer = _CollTimer(self.dev) if (self.cuda and _COMM_TIMING) else None
        fb = int(getattr(lrn.conf, "fixed_bytes", 0) or 0)
        if fb not in (0, 1, 2, 3):
            raise ValueError("fixed_bytes must be 0, 1, 2 or 3")
        self.qf = _QFilter(fb, self.vs, lrn.seed, getattr(self.comm, "rank", 0),
                           self.linear) if fb else None
        # the owner-side update of the linear wire format: (algo, alpha,
        # beta, l1, l2) -- the linear model's, or DiFacto's FTRL on w (algo 4)
        self.lin_hp = lrn.psx_linear_hp() if self.linear else None
        # the native driver of train() (csrc/bind/psx_native.inl PsxStep):
        # decided at the first training call; False = this Python step
        self._nat = None
        self._kmod_cache = None  # (keys, keys % max_key) of the last reduced tensor

    # ------------------------------------------------------------ wire stats
    def _tally(self, c, x, send_rows):
        row = x.element_size()
        for d in x.shape[1:]:
            row *= int(d)
        r = getattr(self.comm, "rank", 0)
        self.wire[c] += row * (sum(int(v) for v in send_rows) - int(send_rows[r]))

    def _qpack(self, x, send, recv, vsend, vrecv, Hs, Hr):
        """fixed_bytes: quantise the float regions x (this side: n = send,
        v = vsend, H = Hs per peer) into wire rows, on S behind x's producer.
        Returns (wire tensor, wire rows per peer out / in, the unpack plan of
        the receiving side)."""
        qf = self.qf
        ds, srows, ext = qf.layout(send, vsend, Hs)
        dr, rrows, rext = qf.layout(recv, vrecv, Hr)
        if ext != x.numel():
            raise RuntimeError("psx filter: region layout %d floats vs buffer %d" % (
                ext, x.numel()))
        P = len(send)
        a = np.concatenate([ds.reshape(-1), dr.reshape(-1)])
        t = self.pins.put(a) if self.cuda else torch.from_numpy(a)
        q = ops.ps_qpack(x, ds, t[:6 * P].view(P, 6), sum(srows), qf.W, qf.nb, qf.next_seed())
        return q, srows, rrows, (dr, t[6 * P:].view(P, 6), rext)

    def _qunpack(self, q, plan):
        """The receiving side: wire rows -> the float layout the consumer
        kernel expects (after the collective has landed)."""
        dr, dd, rext = plan
        vs = 1 if self.linear else self.vs
        out = torch.empty((rext // vs, vs) if not self.linear else (rext,),
                          dtype=torch.float32, device=q.device)
        return ops.ps_qunpack(q, dr, dd, self.qf.W, self.qf.nb, out)

    def _a2a(self, c, x, send_rows, recv_rows, ready=None):
        """Issue collective Cc (async) and account for its bytes.

        ready: an event recorded on the compute stream right after the
        kernel that produced ``x``. The collective is then issued from the
        exchange stream xs, which waits for that event only: RCCL's stream
        waits for the ISSUING stream's queued work, so issued from S it
        would also wait for every kernel enqueued on S after x's producer
        (C2 of minibatch i-1 behind the backward of i-2) and the transfer
        could not overlap that compute. The consumer still orders itself
        after the transfer with ``work.wait()`` on S. (RCCL loopback P = 8:
        104.5 / 105.3 vs 97.5 / 98.2 M ex/s issued from S.)"""
        self._tally(c, x, send_rows)
        if self.timer is not None:
            self.timer.ready(c)
        if ready is not None and self.cuda:
            xs = self.xs
            xs.wait_event(ready)
            x.record_stream(xs)
            with streams.on(xs):
                out, work = self.comm.all_to_all_v_async(x, send_rows, recv_rows)
            if out.is_cuda:
                out.record_stream(self.S)  # allocated on xs, read on S
        else:
            out, work = self.comm.all_to_all_v_async(x, send_rows, recv_rows)
        if self.timer is not None:
            self.timer.done(c, work)
        return out, work

    def _event(self):
        """An event recorded on S now (a ring: an event is re-recorded only
        long after the stream wait that consumed it was enqueued)."""
        if not self.cuda:
            return None
        return self._ring.record(self.S)

    def wire_reset(self):
        self.wire = [0, 0, 0, 0]
        if self._nat:
            self._nat.wire_reset()
        if self.timer is not None:
            self.timer.reset()

    def wire_report(self, steps):
        """Per-step averages since :meth:`wire_reset`: bytes each collective
        sent to peers (and, with WH_TIMING=comm, its GPU time in ms)."""
        steps = max(int(steps), 1)
        wire = list(self.wire)
        if self._nat:
            wire = [a + b for a, b in zip(wire, self._nat.wire())]
        out = {"c%d" % c: wire[c] / steps for c in range(4)}
        out["c0"] = 32 * (self.P - 1)  # {keys, overflow, V rows, has data} per peer
        if self.timer is not None:
            for c, ms in self.timer.report().items():
                out["c%d_ms" % c] = ms / steps
        elif self._nat and _COMM_TIMING:  # (the native step's per-exchange GPU time)
            xt = self._nat.xtime()
            for c in range(4):
                if xt[4 + c]:
                    out["c%d_ms" % c] = xt[c] / 1000.0 * xt[4 + c] / steps
        return out

    # ------------------------------------------------------------ streams
    @contextlib.contextmanager
    def _on_cs(self, *inputs):
        """Run work on the side stream (the C0 count exchange and its host
        read) after the compute stream's queued work, without making the
        compute stream wait for it."""
        if not self.cuda:
            yield
            return
        S = self.S
        ring = self._ring
        ring.wait(self.cs, S)
        if streams.current_id(self.dev.index) != S.stream_id:
            # called from a localize job on its own stream (ls)
            ring.wait(self.cs, self.ls)
        for t in inputs:
            if t is not None and t.is_cuda:
                t.record_stream(self.cs)
        with streams.on(self.cs):
            yield

    # ------------------------------------------------------------ localize
    def _exchange(self, carried, flag):
        """The C0 closure handed to localize: owner counts + overflow flag +
        the carried step's per-peer V row counts + this rank's has-data flag,
        all-to-all on the comm stream, then (payload, stream, 4, P) for the
        native job's read."""
        P, S = self.P, self.nshard

        def ex(owner_cnt):
            vc = carried.vcnt if carried is not None else None
            with self._on_cs(owner_cnt, vc):
                send, payload = ops.ps_c0(owner_cnt, vc, P, flag)
                payload[S + 1:S + 1 + 4 * P] = self.comm.exchange_counts_dev(send)
            if self.cuda:
                return payload, self.cs.cuda_stream, 4, P
            return payload
        return ex

    def _begin(self, keys, offset, val, carried, ready=None, defer=False):
        lrn = self.lrn
        flag = 1 if offset.numel() > 1 else 0  # (a host-side shape: no sync)
        S = self.nshard
        if self.cuda:
            # Outputs are allocated on ls and read on S; ls first waits for
            # everything queued on S, so a block the allocator hands back to
            # ls is rewritten only after the S kernels that read it have run.
            # S itself reads the job's outputs only after the host has waited
            # for the job's count read (which follows `ready` on ls).
            cs, ls = self.S, self.ls
            self._ring.wait(ls, cs)
            if ready is not None:
                ls.wait_event(ready)
            for t in (keys, offset, val):
                if t is not None:
                    t.record_stream(ls)
                    t.record_stream(cs)
            with streams.on(ls):
                k = ops.key_mod(keys, lrn.max_key) if lrn.max_key else keys
                job = _native.hip().LocalizeJob(k, offset, val, S, int(self.uhint),
                                                self._exchange(carried, flag), defer)
            self.job = (keys, job, carried)
            return
        k = ops.key_mod(keys, lrn.max_key) if lrn.max_key else keys
        out = list(_native.host().localize_cpu(k, offset, val, S))
        oc = torch.cat([out[2].to(torch.int64), torch.zeros(1, dtype=torch.int64)])
        payload = self._exchange(carried, flag)(oc)
        out[2] = oc[:S].clone()
        out.append(payload[S + 1:].clone())
        self.job = (keys, tuple(out), carried)

    def _exchange_deferred(self):
        """Issue C0 of an early-begun localize (after the open it carries)."""
        if self.job is not None and self.cuda and not isinstance(self.job[1], tuple):
            with streams.on(self.ls):
                self.job[1].exchange()  # (no-op unless the job deferred it)

    def _counts(self):
        """The one host read of the step (count exchange C0 of the begun
        localize): returns (send, recv, all_empty); fills the carried step's
        V counts. Idempotent (the job keeps its read)."""
        self._exchange_deferred()
        keys, job, carried = self.job
        if isinstance(job, tuple):
            oc, tail = job[2], job[7]
        else:
            oc, tail = job.counts()
        P = self.P
        tail = tail.tolist()
        if carried is not None and carried.vown is None:
            carried.vrecv = tail[2:4 * P:4]
            carried.vown = tail[4 * P:5 * P]
        send = [int(x) for x in oc.tolist()] + [0] * (P - self.nshard)
        empty = not any(tail[3:4 * P:4])
        return send, [int(x) for x in tail[0:4 * P:4]], empty

    def _finish(self):
        """Enqueue the rest of the begun localize (after :meth:`_counts`)."""
        keys, job, carried = self.job
        self.job = None
        return tuple(job) if isinstance(job, tuple) else tuple(job.finish())

    def _ensure_job(self, keys, offset, val):
        """This minibatch's localize: begun by the previous call, or now."""
        if self.job is None or self.job[0] is not keys:
            if self.job is not None:  # a stale job (never expected): finish it in order
                self._counts()
                self._finish()
            self._begin(keys, offset, val, self.pull if (self.pull is not None and
                                                         self.pull.vown is None) else None)

    def _vcount_exchange(self, st):
        """Standalone C0 for a step whose V row counts rode on no localize
        (pipeline drain, validation): one extra host read. (Linear models
        move no V rows: nothing to exchange.)"""
        P, S = self.P, self.nshard
        if self.linear:
            st.vrecv, st.vown = [0] * P, [0] * P
            return
        zero = torch.zeros(S + 1, dtype=torch.int64, device=self.dev)
        with self._on_cs(st.vcnt, zero):
            send, payload = ops.ps_c0(zero, st.vcnt, P, 1)
            payload[S + 1:S + 1 + 4 * P] = self.comm.exchange_counts_dev(send)
            v = payload.cpu().tolist()
        st.vrecv = v[S + 3:S + 1 + 4 * P:4]
        st.vown = v[S + 1 + 4 * P:S + 1 + 5 * P]

    # ---------------------------------------------------------------- tables
    def _upload(self, st, prev):
        """Device copies of the host-known segment tables of `st` (and the V
        row counts of `prev`): one pinned host -> device copy."""
        P = self.P
        vs = max(self.vs, 1)
        st.Hw = [_cdiv(2 * n, vs) for n in st.send] if not self.linear else [0] * P
        st.Ho = [_cdiv(2 * n, vs) for n in st.recv] if not self.linear else [0] * P
        a = np.zeros(4 * (P + 1) + P, dtype=np.int64)
        a[1:P + 1] = np.cumsum(st.send)
        a[P + 2:2 * P + 2] = np.cumsum(st.Hw)
        a[2 * P + 3:3 * P + 3] = np.cumsum(st.recv)
        a[3 * P + 4:4 * P + 4] = np.cumsum(st.Ho)
        if prev is not None:
            a[4 * P + 4:] = prev.vrecv
        t = self.pins.put(a) if self.cuda else torch.from_numpy(a)
        st.tabs = t
        st.segS_w, st.segHS_w = t[0:P + 1], t[P + 1:2 * P + 2]
        st.segS_o, st.segHS_o = t[2 * P + 2:3 * P + 3], t[3 * P + 3:4 * P + 4]
        if prev is not None:
            prev.vrecv_d = t[4 * P + 4:]

    # -------------------------------------------------------------- phases
    def _c1(self, st):
        """Issue C1: this minibatch's keys (+ counts) to their owners."""
        if self.linear:
            rec = st.uniq  # 8-byte keys
        else:
            cnt = st.ucnt if st.use_cnt else None
            if cnt is not None and self.qf is not None:
                cnt = cnt.clamp(max=255)  # TRUNCATE_FLOAT(1) of the count push
            rec = ops.ps_records(st.uniq, cnt)
        st.keys_o, st.w_c1 = self._a2a(1, rec, st.send, st.recv)

    def _open(self, st, insert):
        """Owner side: wait for C1, then one fused open (+ header pack)."""
        lrn = self.lrn
        st.w_c1.wait()
        n = sum(st.recv)
        if insert:
            lrn.kv.guard.before_open(n, self._remap)
        rows = sum(st.Ho) + n if not self.linear else 0
        st.slot, st.vpos, st.chain, st.head, st.rbuf, st.vcnt = self.store.ps_open(
            keys=st.keys_o, use_cnt=st.use_cnt, segS=st.segS_o, segHS=st.segHS_o, rows_cap=rows,
            insert=insert, chains=st.train, h=lrn.hp, threshold=lrn.threshold,
            l1_shrk=lrn.l1_shrk, seed=lrn.seed)
        st.keys_o = st.w_c1 = None
        st.ev_open = self._event()  # C2 of this step waits for this only
        if insert:
            lrn.kv.guard.after_open()

    def _c2(self, st):
        """Issue C2: the owner's pull reply regions back to the workers."""
        P = self.P
        send_rows = [st.Ho[p] + st.vown[p] for p in range(P)]
        recv_rows = [st.Hw[q] + st.vrecv[q] for q in range(P)]
        if self.linear:  # one w per key
            send_rows, recv_rows = st.recv, st.send
        x, ready = st.rbuf[:sum(send_rows)], st.ev_open
        st.q2 = None
        if self.qf is not None and not self.linear:  # (linear pulls travel exact)
            with streams.on(self.S) if self.cuda else contextlib.nullcontext():
                x, send_rows, recv_rows, st.q2 = self._qpack(x, st.recv, st.send, st.vown,
                                                             st.vrecv, st.Ho, st.Hw)
                ready = self._event()
        st.rrecv, st.w_c2 = self._a2a(2, x, send_rows, recv_rows, ready)
        st.ev_open = None
        st.rbuf = None

    def _reply(self, st):
        """Worker side: wait for C2, unpack, forward (+ AUC)."""
        lrn = self.lrn
        st.w_c2.wait()
        st.w_c2 = None
        if st.q2 is not None:
            st.rrecv, st.q2 = self._qunpack(st.rrecv, st.q2), None
        if self.linear:
            st.hdr = st.rrecv
            st.py, st.dual, st.xv = ops.fm_forward(st.offset, st.lid, st.val, st.rrecv, None, 0,
                                                   st.label, lrn.loss, lrn.met)
        else:
            st.hdr, st.rows = ops.ps_unpack(st.rrecv, st.U, st.segS_w, st.segHS_w, st.vrecv_d)
            st.py, st.dual, st.xv = ops.fm_forward(st.offset, st.lid, st.val, st.hdr, st.rrecv,
                                                   self.vs, st.label, lrn.loss, lrn.met)
        if not st.train:  # (a training step's AUC follows its backward)
            ops.auc_acc(st.py, st.label, lrn.auc_sum)
        if st.label.numel():
            lrn.n_mb += 1
        lrn.last_sizes = (st.U, sum(st.vrecv))

    def _c3(self, st):
        """Issue C3: the packed push regions back to their owners."""
        P = self.P
        send_rows = [st.Hw[q] + st.vrecv[q] for q in range(P)]
        recv_rows = [st.Ho[p] + st.vown[p] for p in range(P)]
        if self.linear:  # one gradient per key
            send_rows, recv_rows = st.send, st.recv
        x, ready = st.gvc, st.ev_grad
        st.q3 = None
        if self.qf is not None:
            with streams.on(self.S) if self.cuda else contextlib.nullcontext():
                x, send_rows, recv_rows, st.q3 = self._qpack(x, st.send, st.recv, st.vrecv,
                                                             st.vown, st.Hw, st.Ho)
                ready = self._event()
        st.gpush, st.w_c3 = self._a2a(3, x, send_rows, recv_rows, ready)
        st.ev_grad = None
        st.gvc = None

    def _grad(self, st, issue=True):
        """Backward + gradient post-processing, then issue C3 (the push), or
        leave it for :meth:`_c3` (issue=False)."""
        lrn = self.lrn
        emb = lrn.emb
        csc_off, csc_row, csc_val = st.csc
        if self.linear:
            gw, _ = ops.fm_backward(csc_off, csc_row, csc_val, st.dual, None, st.hdr, None, 0)
            st.gvc = gw.reshape(-1)
        else:
            gw, gvc = ops.fm_backward(csc_off, csc_row, csc_val, st.dual, st.xv, st.hdr,
                                      st.rrecv, self.vs)
            if emb is not None and (emb.grad_clipping > 0 or emb.dropout > 0 or
                                    emb.grad_normalization):
                if emb.grad_normalization:  # header rows must not enter the norm
                    self._zero_header_rows(st, gvc)
                ops.fm_grad_post(gvc, st.rows, lrn.dim, emb.grad_clipping, emb.dropout,
                                 lrn.seed + 7919 * st.seed_step + 1, bool(emb.grad_normalization))
            ops.ps_pack_gw(gw, gvc, st.segS_w, st.segHS_w, st.vrecv_d)
            st.gvc = gvc
        st.ev_grad = self._event()  # C3 of this step waits for this only
        if issue:
            self._c3(st)
        ops.auc_acc(st.py, st.label, lrn.auc_sum)
        # the worker-side tensors of this step are done
        st.rrecv = st.hdr = st.dual = st.xv = st.lid = st.csc = None

    def _zero_header_rows(self, st, gvc):
        idx, base = [], 0
        for q in range(self.P):
            idx.extend(range(base, base + st.Hw[q]))
            base += st.Hw[q] + st.vrecv[q]
        if idx:
            gvc[torch.tensor(idx, dtype=torch.int64, device=gvc.device)] = 0

    def _owner_push(self, st):
        """Apply a landed push on the owner (one launch over all segments)."""
        lrn = self.lrn
        st.w_c3.wait()
        if st.q3 is not None:
            st.gpush, st.q3 = self._qunpack(st.gpush, st.q3), None
        if self.linear:
            algo, alpha, beta, l1, l2 = self.lin_hp
            self.store.ps_push_linear(
                slot=st.slot, chain=st.chain, head=st.head, segS=st.segS_o, g=st.gpush,
                algo=algo, alpha=alpha, beta=beta, l1=l1, l2=l2, t0=float(self.requests))
            self.requests += self.P  # one request per worker (ps-lite SGD's t)
        else:
            self.store.ps_push(slot=st.slot, vpos=st.vpos, chain=st.chain, head=st.head,
                               segS=st.segS_o, segHS=st.segHS_o, gbuf=st.gpush, h=lrn.hp,
                               threshold=lrn.threshold, l1_shrk=lrn.l1_shrk, seed=lrn.seed)
        st.w_c3 = None
        st.gpush = st.slot = st.vpos = st.chain = st.head = st.keys_o = None

    def _remap(self, remap):
        """The table grew: translate the slot ids of in-flight steps."""
        for st in (self.pull, self.push):
            if st is not None and st.slot is not None and st.slot.numel():
                # (a -1 slot -- a failed insert or a miss -- stays -1)
                s_ = st.slot.long()
                st.slot = torch.where(s_ >= 0, remap[s_.clamp_min(0)], st.slot)

    # ----------------------------------------------------------------- API
    def _new_step(self, send, recv, label, train, data_pass, prev):
        st = _Step()
        st.send, st.recv = send, recv
        st.label = label
        st.train = train
        st.use_cnt = train and data_pass == 0 and not self.linear
        st.seed_step = self.lrn.step
        self._upload(st, prev)
        return st

    def _set_loc(self, st, loc, offset, val):
        st.uniq, st.ucnt, _, st.lid, csc_off, csc_row, csc_val = loc[:7]
        st.csc = (csc_off, csc_row, csc_val)
        st.U = st.uniq.numel()
        st.offset, st.val = offset, val
        self.uhint = st.U

    def _drop_empty(self):
        """Every rank's minibatch of this call is empty (C0's flags): the
        pass is over. Drop the job; the pipeline keeps what is in flight for
        :meth:`flush`."""
        self._finish()
        self.last_empty = True

    # ------------------------------------------------------------ native
    def _native(self):
        """The C++ driver of :meth:`train` (csrc/bind/psx_native.inl
        PsxStep) -- the default for every GPU configuration: RCCL ranks (its
        own communicator, grouped send / recv per peer), gloo-staged ranks
        sharing one GPU, the loopback identity and the 1-rank RCCL loopback.
        It covers the payload filter (fixed_bytes), the embedding-gradient
        post-processing and the exchange timing too; this Python step is the
        test oracle (``WH_PSX_NATIVE=0`` selects it) and the CPU path."""
        if self._nat is None:
            lrn, emb = self.lrn, self.lrn.emb
            post = emb is not None and (emb.grad_clipping > 0 or emb.dropout > 0 or
                                        bool(emb.grad_normalization))
            backend = getattr(self.comm, "backend", "")
            staged = bool(getattr(self.comm, "stage", False))
            hip = _native.hip()
            tx = {"loopback": hip.PSX_TX_IDENTITY, "loopback-rccl": hip.PSX_TX_RCCL,
                  "nccl": hip.PSX_TX_RCCL}.get(backend)
            if staged and backend == "gloo":
                tx = hip.PSX_TX_STAGED
            ok = self.cuda and os.environ.get("WH_PSX_NATIVE", "1") != "0" and tx is not None
            self._nat = False
            rccl = None
            if ok and tx == hip.PSX_TX_RCCL:
                ok = self._own_rccl()
                if ok:
                    rccl = ok
            if not ok and self.cuda and self.tau_max > 1:
                print("[psx] max_concurrency %d: the Python step keeps at most 2 minibatches in "
                      "flight (staleness 1)" % (self.tau_max + 1), flush=True)
            if ok:
                self._nat = hip.PsxStep(
                    store=self.store, P=self.P, S=self.nshard,
                    rank=int(getattr(self.comm, "rank", 0)), tx=tx,
                    pg=self.comm.pg if tx == hip.PSX_TX_STAGED else None,
                    rccl=rccl,
                    linear=self.linear,
                    lin_hp=list(self.lin_hp) if self.linear else [0.0] * 5,
                    hp=list(lrn.hp), threshold=int(lrn.threshold), l1_shrk=bool(lrn.l1_shrk),
                    seed=int(lrn.seed), loss=int(lrn.loss), met=lrn.met, auc_sum=lrn.auc_sum,
                    tau=int(self.tau_max), max_load=float(lrn.kv.guard.max_load),
                    cu_reserve=_CU_RESERVE if tx == hip.PSX_TX_RCCL else 0,
                    filt=[self.qf.nb, self.qf.seed] if self.qf is not None else [0, 0],
                    post=[float(emb.grad_clipping), float(emb.dropout),
                          1.0 if emb.grad_normalization else 0.0, float(lrn.dim)]
                    if post else [0.0, 0.0, 0.0, 0.0])
                self._nat.requests = self.requests
                self._nat.step = self.lrn.step
                self.timer = None  # (the native step times its own exchanges)
        return self._nat or None

    def _own_rccl(self):
        """The native step's own communicators: (c0, c1, c23) -- C0 and C1 on
        the path to the next open get their own, RCCL running one
        communicator's operations in issue order -- or one shared by all
        four exchanges with ``WH_PSX_RCCL_COMMS=1``. Creating them is
        collective; the ranks then agree on the outcome (a failure on one
        rank alone would leave it on the Python step's c10d collectives and
        its peers on the native ones, a deadlock), and the communicators
        made are closed again if any rank failed. Returns the communicators,
        or False (every rank then takes the Python step)."""
        one = os.environ.get("WH_PSX_RCCL_COMMS", "3") == "1"
        made, err = [], None
        try:
            for tag in (("c23",) if one else ("c0", "c1", "c23")):
                made.append(self.comm.rccl(tag))
        except RuntimeError as e:
            err = str(e).splitlines()[0]
        good = err is None
        if getattr(self.comm, "size", 1) > 1 and getattr(self.comm, "pg", None) is not None:
            flag = torch.tensor([1 if good else 0], dtype=torch.int64, device=self.dev)
            self.comm.allreduce(flag, "min")
            good = bool(int(flag.item()))
        if not good:
            self.comm._close_rccl()
            print("[psx] own RCCL communicators unavailable (%s): the Python step exchanges "
                  "over the c10d group" % (err or "failed on another rank"), flush=True)
            return False
        return made[0] if one else tuple(made)

    def _kmod(self, keys):
        """max_key (ps-lite's flag, learn/base/localizer.h:108-115): the
        native step localizes the keys modulo max_key; the same input tensor
        maps to the same reduced tensor (the begun localize of the next
        minibatch is matched by identity)."""
        if keys is None or not self.lrn.max_key:
            return keys
        c = self._kmod_cache
        if c is not None and c[0] is keys:
            return c[1]
        k = ops.key_mod(keys, self.lrn.max_key)
        self._kmod_cache = (keys, k)
        return k

    def _native_drain(self):
        """Hand the pipeline back to the Python step (an evaluation or a
        read-only pull): every minibatch in flight completed, the begun
        localize dropped (all ranks reach this at the same point)."""
        nat = self._nat
        if nat:
            self.lrn.n_mb += nat.flush()
            nat.drop_job()
            self.requests = nat.requests
            g = self.lrn.kv.guard
            g.grows, g.vgrows = max(g.grows, nat.grows), max(g.vgrows, nat.vgrows)

    def train(self, keys, offset, val, label, data_pass, next_batch):
        nat = self._native() if self.cuda else None
        if nat is not None:
            nk = no = nv = None
            ready = 0
            if next_batch is not None:
                nk, no, nv = next_batch[:3]
                if len(next_batch) > 3 and next_batch[3] is not None:
                    ready = next_batch[3].cuda_event
            keys = self._kmod(keys)
            if nat.step != self.lrn.step:  # (an evaluation pass counted steps in between)
                nat.step = self.lrn.step
            if nk is not None and self.lrn.max_key:
                if ready:  # the reduction reads the next keys on this stream
                    torch.cuda.current_stream(self.dev).wait_event(next_batch[3])
                nk = self._kmod(nk)
            has, nmb, u, v = nat.train(keys=keys, offset=offset, val=val, label=label,
                                       data_pass=int(data_pass), next_keys=nk, next_offset=no,
                                       next_val=nv, ready=ready)
            self.lrn.n_mb += nmb
            if nmb:
                self.lrn.last_sizes = (u, v)
            self.last_empty = not has
            if has:
                self.lrn.step += 1
            return
        if self.cuda and streams.current_id(self.dev.index) != self.S.stream_id:
            self.S = torch.cuda.current_stream(self.dev)
        self.last_empty = False
        self._ensure_job(keys, offset, val)
        send, recv, empty = self._counts()  # the step's one host read
        if empty:
            self._drop_empty()
            return
        prev = self.pull
        if prev is not None and prev.vown is None:
            self._vcount_exchange(prev)
        st = self._new_step(send, recv, label, True, data_pass, prev)
        if prev is not None:
            self._c2(prev)  # transfers while this minibatch's localize finishes
        if self.push is not None and self.push.gvc is not None:
            # the previous backward's push, issued only now: behind this
            # step's pull reply on the (in-order) RCCL stream, so the reply
            # overlaps the end of that backward and the push overlaps the
            # forward below, instead of both transfers running back to back
            # between the backward and the forward
            self._c3(self.push)
        self._set_loc(st, self._finish(), offset, val)
        early = self.cuda and next_batch is not None
        if early:  # next minibatch's localize kernels now; its C0 after the open
            nk, no, nv = next_batch[:3]
            self._begin(nk, no, nv, st, next_batch[3] if len(next_batch) > 3 else None,
                        defer=True)
        self._c1(st)        # transfers while the previous minibatch computes
        if prev is not None:
            self._reply(prev)
            if self.tau == 0 and prev.train:
                self._grad(prev)
                self._owner_push(prev)
        if self.push is not None:
            self._owner_push(self.push)
            self.push = None
        self._open(st, True)
        self.pull = st
        if early:
            self._exchange_deferred()
        elif next_batch is not None:
            nk, no, nv = next_batch[:3]
            self._begin(nk, no, nv, st, next_batch[3] if len(next_batch) > 3 else None)
        if self.tau == 1 and prev is not None and prev.train:
            self._grad(prev, issue=False)  # C3 goes out behind the next call's C2
            self.push = prev
        self.lrn.step += 1

    def evaluate(self, keys, offset, val, label):
        """A validation / prediction minibatch: drain the training pipeline,
        then open (no insert), reply and forward synchronously. Returns the
        predictions, or None when no rank had data (``last_empty``)."""
        self.flush()
        self._native_drain()
        self.last_empty = False
        self._ensure_job(keys, offset, val)
        send, recv, empty = self._counts()
        if empty:
            self._drop_empty()
            return None
        st = self._new_step(send, recv, label, False, 1, None)
        self._set_loc(st, self._finish(), offset, val)
        self._c1(st)
        self._open(st, False)
        self._vcount_exchange(st)
        self._upload_vrecv(st)
        self._c2(st)
        self._reply(st)
        self.lrn.step += 1
        return st.py

    def pull_values(self, keys):
        """Read-only pull of ``keys``' current values from their owners
        through the same exchange (no insert, no metrics) -- a collective,
        every rank calls it with its own keys. Returns (uniq, w [U], rows)
        with rows [U, vstride] (zero for keys without an embedding) or None
        for the linear wire format; None if no rank has keys."""
        self.flush()
        self._native_drain()
        n = int(keys.numel())
        dev = keys.device
        offset = torch.arange(n + 1, dtype=torch.int64, device=dev)
        self._ensure_job(keys, offset, None)
        send, recv, empty = self._counts()
        if empty:
            self._drop_empty()
            return None
        st = self._new_step(send, recv, None, False, 1, None)
        self._set_loc(st, self._finish(), offset, None)
        self._c1(st)
        self._open(st, False)
        self._vcount_exchange(st)
        self._upload_vrecv(st)
        self._c2(st)
        st.w_c2.wait()
        if st.q2 is not None:
            st.rrecv, st.q2 = self._qunpack(st.rrecv, st.q2), None
        if self.linear:
            return st.uniq, st.rrecv.reshape(-1), None
        hdr, _ = ops.ps_unpack(st.rrecv, st.U, st.segS_w, st.segHS_w, st.vrecv_d)
        vid = ops.hdr_vidx(hdr).long()
        rows = torch.zeros(st.U, self.vs, dtype=torch.float32, device=dev)
        has = vid >= 0
        rows[has] = st.rrecv[vid[has]]
        return st.uniq, hdr[:, 0].contiguous(), rows

    def _upload_vrecv(self, st):
        a = np.array(st.vrecv, dtype=np.int64)
        st.vrecv_d = self.pins.put(a) if self.cuda else torch.from_numpy(a)

    def flush(self):
        """Complete every minibatch in flight (end of a pass, before reading
        or saving the model, end of a timed run)."""
        if self._nat:
            self.lrn.n_mb += self._nat.flush()
            g = self.lrn.kv.guard
            g.grows = max(g.grows, self._nat.grows)
            g.vgrows = max(g.vgrows, self._nat.vgrows)
        if self.push is not None and self.push.gvc is not None:
            self._c3(self.push)
        if self.job is not None and self.job[2] is not None:
            # the next minibatch's localize already carries the last pull's
            # V counts: read them now (the job itself stays begun)
            self._counts()
        st = self.pull
        if st is not None:
            if st.vown is None:
                self._vcount_exchange(st)
            self._upload_vrecv(st)
            self._c2(st)
            self._reply(st)
            if st.train:
                self._grad(st)
        if self.push is not None:
            self._owner_push(self.push)
            self.push = None
        if st is not None and st.train:
            self._owner_push(st)
        self.pull = None


PsxDifacto = Psx  # (round-2 name)
