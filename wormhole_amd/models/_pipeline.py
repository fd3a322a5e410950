"""Minibatch localize pipeline shared by the PS learners (difacto, linear).

Localize minibatch i (finishing the job begun during minibatch i-1 when it
was told about i), then begin i+1, so the one host read of the unique-id
counts overlaps i's kernels (the reference overlaps the same stages with
threads: learn/solver/minibatch_solver.h:284-315 keeps max_concurrency
minibatches in flight).

``next_batch`` is ``(keys, offset, val)`` of the NEXT call, optionally with a
fourth item: a ``torch.cuda.Event`` recorded on the stream that produced the
tensors (a data generator or H2D copy stream). The compute stream waits on it
only right before the next minibatch's localize begins, so the producer runs
concurrently with minibatch i's localize finish. Every rank must pass
``next_batch`` in lockstep (the count exchange is a collective).
"""
import torch

from .. import ops
from ..utils import streams


def localize_pipelined(lrn, keys, offset, val, next_batch):
    loc = localize_current(lrn, keys, offset, val)
    if next_batch is not None:
        begin_next(lrn, next_batch, loc[0].numel())
    return loc


def localize_current(lrn, keys, offset, val):
    """This minibatch's localize: finish the job begun for it, or run it."""
    job, lrn._job = lrn._job, None
    if job is not None and job[0] is keys:
        return ops.localize_finish(job[1])
    k = ops.key_mod(keys, lrn.max_key) if lrn.max_key else keys
    return ops.localize(k, offset, val, lrn.kv.nshard, lrn.uhint)


# DiFacto begins the next minibatch's localize right AFTER enqueueing this
# minibatch's pull (localize_current + begin_next): the host reaches the pull
# launch sooner after its count read (127.0 -> 131.7 M ex/s). The linear
# model, whose step is short enough that the job's count read comes late, is
# 5 % slower that way and begins it before (localize_pipelined).


def begin_next(lrn, next_batch, uhint):
    """Begin the localize of ``next_batch`` (see the module docstring);
    ``uhint``: this minibatch's unique-id count (sizes the job's table)."""
    nk, no, nv = next_batch[:3]
    ready = next_batch[3] if len(next_batch) > 3 else None
    if nk.is_cuda:
        # The next minibatch's partitioned localize runs on its own stream,
        # concurrently with this minibatch's forward / backward / push on the
        # compute stream. The side stream first waits for everything queued
        # on the compute stream so far (memory safety, below); the job's
        # finish host-syncs its event before any compute-stream kernel reads
        # its buffers.
        cur = _cur_stream(nk.device)
        side = _loc_stream(nk.device)
        _ring(nk.device).wait(side, cur)
        if ready is not None:
            side.wait_event(ready)
        for t in (nk, no, nv):
            if t is not None:
                t.record_stream(side)
                t.record_stream(cur)
        with streams.on(side):
            k = ops.key_mod(nk, lrn.max_key) if lrn.max_key else nk
            job = ops.localize_begin(k, no, nv, lrn.kv.nshard, uhint)
        lrn._job = (nk, job)
        return
    if ready is not None and nk.is_cuda:
        cur = _cur_stream(nk.device)
        cur.wait_event(ready)
        for t in (nk, no, nv):  # produced on another stream, consumed here
            if t is not None:
                t.record_stream(cur)
    k = ops.key_mod(nk, lrn.max_key) if lrn.max_key else nk
    lrn._job = (nk, ops.localize_begin(k, no, nv, lrn.kv.nshard, uhint))


# Since the partitioned localize (LDS dedup, no global atomics) the side
# stream pays: DiFacto 117.5 -> 127 M ex/s on one MI355X. (With the round-1
# hash localize it was slower: its concurrent atomic inserts cost the
# gather-bound FM kernels more than they hid.) Memory safety of the side-stream outputs: they are allocated on the side
# stream and read on the compute stream; the side stream's next job first
# waits for the compute stream (side.wait_stream(cur) below), so a block the
# allocator hands back to the side stream is never rewritten before the
# compute-stream kernels that read it have run.
_streams = {}
_rings = {}
_cur = {}


def _ring(dev):
    r = _rings.get(dev)
    if r is None:
        r = _rings[dev] = streams.EventRing(8)
    return r


def _cur_stream(dev):
    """The current stream of dev (a cached Stream while it stays current)."""
    s = _cur.get(dev)
    if s is None or streams.current_id(dev.index) != s.stream_id:
        s = _cur[dev] = torch.cuda.current_stream(dev)
    return s


def _loc_stream(dev):
    s = _streams.get(dev)
    if s is None:
        s = _streams[dev] = torch.cuda.Stream(device=dev)
    return s
