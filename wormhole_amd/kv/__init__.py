"""Sharded key-value parameter store (the ps-lite server group, re-designed).

Every GPU process owns one shard: keys with ``mix64b(key) % P == rank`` live
in its HBM table (:class:`wormhole_amd._hip.KVStore`).  A minibatch's unique
keys are already grouped by owner by ``localize``, so a pull is

    all_to_all_v(keys) -> owner find/insert -> owner gather -> all_to_all_v(values)

and a push sends only the values back along the same splits (the keys and
owner-side slots are cached for the minibatch: ps-lite's KEY_CACHING filter).
Owner-side updates are applied per source rank in rank order, so each
worker's push is one atomic update like a ps-lite server request.

DiFacto values are variable length (ps-lite ZVPull/ZVPush with sizes 1 or
1+k, learn/difacto/async_sgd.h:234-244): every key moves an 8-byte header
{w, vidx} and only keys that own an embedding move their vstride floats, in
a second all-to-all whose per-peer row counts come from the owner's pull.
The gradient push mirrors it (4-byte gw per key + the embedding rows).
"""

import torch

from .. import _native, ops
from ..utils import streams
from .cpu_store import CpuKVStore


class StoreError(RuntimeError):
    """The parameter store lost data (a failed insert or a full V slab)."""


class StoreGuard:
    """Load-factor control and loud failure for one parameter store shard.

    The reference server allocates an entry per key without bound and grows
    V per key on demand (learn/difacto/async_sgd.h:139-160, 247-259). The
    HBM store is an open-addressing table plus a V-row slab, so this guard
    keeps it there: after every open it enqueues a 32-byte summary read
    (keys, failed inserts, V-slab overflows, V rows used), and before the
    next open it checks that read -- raising :class:`StoreError` on any lost
    key or row -- and grows the table (device rehash, at most ``max_load``
    occupancy) or the V slab so that the coming minibatch cannot overflow
    either, whatever it inserts. The read is one minibatch behind, so it
    never stalls the stream."""

    def __init__(self, store, max_load=0.7):
        self.store = store
        self.max_load = float(max_load)
        self.pend = None      # (pinned host tensor, event) of the last summary
        self.keys = 0
        self.vused = 0
        self.since = 0        # keys opened since the last completed summary
        self.grows = 0
        self.vgrows = 0
        # key counts of the last two opens: their pushes may still be in
        # flight (the deferred push; push(i-2) under the pipelined multi-shard
        # step) and each may allocate one V row per key after the summary
        self.recent = [0, 0]
        self._ring = None
        self._main = None  # the stream opens run on (cached)
        self.cuda = not isinstance(store, CpuKVStore)

    def after_open(self):
        if self.cuda:
            if getattr(self, "_ev", None) is None:  # two alternating host slots
                self._ev = [torch.cuda.Event() for _ in range(2)]
                self._k = 0
                self._side = torch.cuda.Stream()
            k = self._k = self._k ^ 1
            ev = self._ev[k]
            # the summary (a one-wave read of the table's counters, written
            # straight into host memory) runs on a side stream behind the
            # open, off the compute stream's critical path; read() waits for
            # it one open later
            side = self._side
            if self._ring is None:
                self._ring = streams.EventRing(4)
            main = torch.cuda.current_stream() if self._main is None else self._main
            if streams.current_id(main.device_index) != main.stream_id:
                main = torch.cuda.current_stream()
            self._main = main
            self._ring.wait(side, main)
            with streams.on(side):
                self.store.summary_async(k)
                ev.record(side)
            self.pend = (k, ev)
        else:
            self.pend = (self.store.summary(), None)
        self.since = 0

    def read(self):
        """Apply the last summary; raises StoreError on lost data."""
        if self.pend is None:
            return
        h, ev = self.pend
        self.pend = None
        if ev is not None:
            ev.synchronize()
            keys, fail, vover, vused = self.store.summary_read(h)
        else:
            keys, fail, vover, vused = [int(x) for x in h.tolist()]
        self.keys, self.vused = keys, vused
        if fail or vover:
            raise StoreError(
                "parameter store shard lost data: %d failed inserts, %d embedding rows "
                "dropped (table %d/%d keys, V slab %d/%d rows)" % (
                    fail, vover, keys, self.store.cap, vused, self.store.vcap))

    def before_open(self, n, remap_cb=None):
        """Make room for a minibatch of n incoming keys (before its open)."""
        self.read()
        st = self.store
        need = self.keys + self.since + n
        if need > self.max_load * st.cap:
            cap = st.cap
            while need > 0.5 * cap:  # leave room to grow into
                cap *= 2
            remap = st.grow(cap)
            self.grows += 1
            if remap_cb is not None:
                remap_cb(remap)
        if getattr(st, "vstride", 0) > 0:
            # V rows: this open, and the pushes of the previous opens not yet
            # in the summary, may each allocate one row per key at most
            vneed = self.vused + self.since + n + sum(self.recent)
            if vneed > st.vcap:
                vcap = max(st.vcap, 1)
                while vneed > vcap:
                    vcap *= 2
                st.grow_v(vcap)
                self.vgrows += 1
        self.since += n
        self.recent = [self.recent[1], n]


def make_store(cap, vcap, dim, device):
    device = torch.device(device)
    if device.type == "cuda":
        return _native.hip().KVStore(int(cap), int(vcap), int(dim), device.index or 0)
    return CpuKVStore(cap, vcap, dim)


class Session:
    """Per-minibatch exchange state (keys sent once, splits reused)."""

    __slots__ = ("send", "recv", "keys", "slots", "hdr_own", "vsend", "vrecv", "m", "cnt")

    def __init__(self, send, recv, keys):
        self.send = send
        self.recv = recv
        self.keys = keys
        self.slots = None
        self.hdr_own = None  # owner-side pull header (owner vidx numbering)
        self.vsend = None    # embedding rows this rank sent per peer in the pull
        self.vrecv = None    # ... and received per peer
        self.m = None        # device int64 [1]: embedding rows in the local model
        self.cnt = None      # owner-side feature counts (DiFacto pass 0)

    def segments(self):
        b = 0
        for n in self.recv:
            yield b, b + n
            b += n


class ShardedKV:
    def __init__(self, store, comm, nshard=None, fixed_bytes=0, seed=0):
        self.store = store
        self.comm = comm
        # ps-lite FIXING_FLOAT / TRUNCATE_FLOAT filters (conf fixed_bytes,
        # learn/difacto/async_sgd.h:429-446): embedding rows cross the wire as
        # n-byte fixed point with random rounding, feature counts as uint8.
        # Scalars (w, gw, the header) travel exact. Only applied to data that
        # actually moves between ranks.
        self.fixed_bytes = int(fixed_bytes or 0)
        if self.fixed_bytes not in (0, 1, 2, 3):
            raise ValueError("fixed_bytes must be 0, 1, 2 or 3")
        self.qseed = (int(seed) * 0x9E3779B1 + 17 * comm.rank + 1) & 0x7FFFFFFFFFFF
        self.qcalls = 0
        # keys are owned by the first `nshard` ranks (the conf's -s S servers)
        self.nshard = comm.size if nshard is None else max(1, min(int(nshard), comm.size))
        self.push_count = 0  # number of push requests applied (SGD's t)
        self.pending = None  # a deferred push: (handle, apply)
        self.guard = StoreGuard(store)

    # ------------------------------------------------------ payload filter
    def _rows_out(self, x):
        """rows about to be sent: quantised records when fixed_bytes > 0"""
        if not self.fixed_bytes or x.numel() == 0:
            return x
        self.qcalls += 1
        return ops.quant_rows(x, self.fixed_bytes, self.qseed + (self.qcalls << 20))

    def _rows_in(self, q, width):
        if not self.fixed_bytes:
            return q
        if q.numel() == 0:
            return torch.zeros((q.shape[0], width), dtype=torch.float32, device=q.device)
        return ops.dequant_rows(q, width, self.fixed_bytes)

    def flush(self):
        """Complete a deferred push (wait for its transfers, apply it)."""
        if self.pending is not None:
            handle, apply = self.pending
            self.pending = None
            handle.wait()
            apply()

    def count_exchange(self):
        """The per-minibatch key-count all-to-all, for ops.localize to run
        before its host read (None on one rank).  Each rank sends every peer
        {keys for that peer, own table-overflow flag}."""
        if self.comm.size == 1:
            return None
        P, ns = self.comm.size, self.nshard

        def ex(owner_cnt):
            send = torch.zeros(2 * P, dtype=torch.int64, device=owner_cnt.device)
            send[0:2 * ns:2] = owner_cnt[:ns]
            send[1::2] = owner_cnt[ns]
            return self.comm.exchange_counts_dev(send)
        return ex

    def open(self, uniq, owner_cnt, insert, cnt=None, recv=None):
        """Send this minibatch's unique keys to their owners (plus, for the
        DiFacto count push, their counts in the same exchange) and resolve
        them to owner-side slots.  recv: the per-rank receive counts when the
        count exchange already ran inside localize."""
        send = [int(x) for x in (owner_cnt.tolist() if hasattr(owner_cnt, "tolist") else owner_cnt)]
        send += [0] * (self.comm.size - len(send))
        if self.comm.size == 1:
            sess = Session(send, send, uniq)
            sess.cnt = cnt
        else:
            recv = self.comm.exchange_counts(send) if recv is None else [int(r) for r in recv]
            if cnt is None:
                keys = self.comm.all_to_all_v(uniq, send, recv)
                sess = Session(send, recv, keys)
            else:
                cw = ops.trunc_u8(cnt) if self.fixed_bytes else cnt
                keys, c = self.comm.all_to_all_v_multi([(uniq, send, recv), (cw, send, recv)])
                sess = Session(send, recv, keys)
                sess.cnt = c.int() if self.fixed_bytes else c
        self.flush()  # a deferred push lands before this minibatch's lookups
        if insert:
            self.guard.before_open(sess.keys.shape[0])
        sess.slots = self.store.find(sess.keys, insert)
        if insert:
            self.guard.after_open()
        return sess

    def _to_owner(self, sess, x):
        return x if self.comm.size == 1 else self.comm.all_to_all_v(x, sess.send, sess.recv)

    def _to_worker(self, sess, x):
        return x if self.comm.size == 1 else self.comm.all_to_all_v(x, sess.recv, sess.send)

    # ---------------------------------------------------------------- linear
    def linear_pull(self, sess):
        return self._to_worker(sess, self.store.linear_pull(sess.slots))

    def linear_push(self, sess, grad, algo, alpha, beta, l1, l2, defer=False):
        self.flush()

        def apply(g):
            for a, b in sess.segments():
                self.push_count += 1
                eta = (beta + float(self.push_count) ** 0.5) / alpha
                if b > a:
                    self.store.linear_push(sess.slots[a:b], g[a:b], algo, alpha, beta, l1, l2,
                                           eta)
        if self.comm.size == 1:
            apply(grad.reshape(-1))
            return
        (g,), handle = self.comm.all_to_all_v_multi(
            [(grad.reshape(-1).contiguous(), sess.send, sess.recv)], async_op=True)
        self.pending = (handle, lambda: apply(g))
        if not defer:
            self.flush()

    # --------------------------------------------------------------- difacto
    def difacto_push_cnt(self, sess, hp, threshold, l1_shrk, seed):
        """Feature-count push (kPushFeaCnt); the counts travelled with the
        keys in :meth:`open`."""
        c = sess.cnt
        if not (c.is_cuda and c.dtype == torch.int32) and c.dtype != torch.float32:
            c = c.float()  # (the GPU kernel takes int32 counts directly)
        for a, b in sess.segments():
            if b > a:
                self.store.difacto_push_cnt(sess.slots[a:b], c[a:b], hp, threshold, l1_shrk, seed)

    def difacto_open_pull(self, uniq, owner_cnt, insert, cnt, hp, threshold, l1_shrk, seed,
                          recv=None, direct=False):
        """open() + (pass 0) difacto_push_cnt() + difacto_pull() as one call.
        On one shard this is ONE fused device pass over the keys (find,
        count, lazy V allocation, variable-length pull); with peers it is the
        exchange sequence of the three calls. Returns (sess, hdr, vc).

        direct (one shard, device store): no pulled copy of the V rows --
        hdr's vidx column holds table rows and vc IS the store's V slab, so
        the FM kernels read the rows in place (the gradient rows then follow
        the slab numbering too; the push takes them that way)."""
        if self.comm.size > 1:
            sess = self.open(uniq, owner_cnt, insert, cnt=cnt, recv=recv)
            if cnt is not None:
                self.difacto_push_cnt(sess, hp, threshold, l1_shrk, seed)
            hdr, vc = self.difacto_pull(sess, l1_shrk)
            return sess, hdr, vc
        send = [int(x) for x in (owner_cnt.tolist() if hasattr(owner_cnt, "tolist") else owner_cnt)]
        sess = Session(send, send, uniq)
        self.flush()
        if cnt is not None and not (cnt.is_cuda and cnt.dtype == torch.int32):
            cnt = cnt.int() if cnt.is_cuda else cnt.float()
        if insert:
            self.guard.before_open(uniq.shape[0])
        slots, hdr, vc, vpos = self.store.difacto_open_pull(uniq, insert, cnt, hp, threshold,
                                                            l1_shrk, seed, direct)
        if insert:
            self.guard.after_open()
        sess.slots = slots
        sess.hdr_own = hdr
        sess.m = vpos[-1:]
        return sess, hdr, vc

    def difacto_pull(self, sess, l1_shrk):
        """Returns (hdr [U, 2], vc [mcap, vstride]) in the worker's key order;
        sess.m holds the live embedding-row count on the device."""
        hdr, vc, vpos = self.store.difacto_pull(sess.slots, l1_shrk)
        sess.hdr_own = hdr
        if self.comm.size == 1:
            sess.m = vpos[-1:]
            return hdr, vc
        # embedding rows per peer = vpos at the receive-segment boundaries;
        # exchanged on the device, then ONE host read for both directions
        bounds = [0]
        for n in sess.recv:
            bounds.append(bounds[-1] + n)
        vb = vpos[torch.tensor(bounds, dtype=torch.int64, device=vpos.device)]
        vrecv_d = (vb[1:] - vb[:-1]).contiguous()       # owner -> worker rows
        vsend_d = self.comm.exchange_counts_dev(vrecv_d)  # worker <- owner rows
        both = torch.cat([vrecv_d, vsend_d]).tolist()
        P = self.comm.size
        sess.vrecv, sess.vsend = both[:P], both[P:]
        hdr_w, vc_w = self.comm.all_to_all_v_multi([
            (hdr, sess.recv, sess.send),
            (self._rows_out(vc[:sum(sess.vrecv)]), sess.vrecv, sess.vsend)])
        vc_w = self._rows_in(vc_w, vc.shape[1])
        sess.m = ops.vidx_renumber(hdr_w)
        return hdr_w, vc_w

    def difacto_push(self, sess, gw, gvc, hp, threshold, l1_shrk, seed, defer=False):
        """Send the gradients to their owners and apply them there.  With
        defer=True (and more than one GPU) the transfer is only started: the
        caller overlaps it with independent work (the next minibatch's
        localize) and completes it with :meth:`flush` before the next pull,
        so every pull still sees every earlier push."""
        self.flush()

        def apply(g, gv):
            for a, b in sess.segments():
                if b > a:
                    self.store.difacto_push(sess.slots[a:b], sess.hdr_own[a:b], g[a:b], gv, hp,
                                            threshold, l1_shrk, seed)
        if self.comm.size == 1:
            apply(gw, gvc)
            return
        width = gvc.shape[1] if gvc.dim() == 2 else 0
        (g, gv), handle = self.comm.all_to_all_v_multi([
            (gw, sess.send, sess.recv),
            (self._rows_out(gvc[:sum(sess.vsend)]), sess.vsend, sess.vrecv)], async_op=True)
        self.pending = (handle, lambda: apply(g, self._rows_in(gv, width).contiguous()))
        if not defer:
            self.flush()
