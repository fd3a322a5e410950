"""Sharded key-value parameter store (the ps-lite server group, re-designed).

Every GPU process owns one shard: keys with ``mix64b(key) % S == rank`` live
in its HBM table (:class:`wormhole_amd._hip.KVStore`, or the host
:class:`CpuKVStore` of the CPU path), kept within its load factor by
:class:`StoreGuard`. One shard pulls and pushes through :class:`ShardedKV`;
with P > 1 ranks the minibatch exchange is the pipelined multi-shard step of
kv/psx.py (keys, variable-length DiFacto values -- ps-lite ZVPull/ZVPush with
sizes 1 or 1+k, learn/difacto/async_sgd.h:234-244 -- and the pushes as four
all-to-all collectives per minibatch, payload filters included).
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
    """Per-minibatch state of a one-shard open (the slots the push reuses:
    ps-lite's KEY_CACHING by construction)."""

    __slots__ = ("keys", "slots", "hdr_own", "m")

    def __init__(self, keys):
        self.keys = keys
        self.slots = None
        self.hdr_own = None  # pull header (this shard's vidx numbering)
        self.m = None        # device int64 [1]: embedding rows in the local model


class ShardedKV:
    """The parameter store front end of one process: its shard of the keys
    (``mix64b(key) % nshard``, the first ``nshard`` ranks owning them) and
    the one-shard pull / push. With more than one rank every exchange is the
    pipelined multi-shard step (kv/psx.py) -- also for the fixed_bytes
    payload filter and embedding-free models -- which reads ``nshard`` and
    ``guard`` from here."""

    def __init__(self, store, comm, nshard=None, fixed_bytes=0, seed=0):
        self.store = store
        self.comm = comm
        self.fixed_bytes = int(fixed_bytes or 0)
        if self.fixed_bytes not in (0, 1, 2, 3):
            raise ValueError("fixed_bytes must be 0, 1, 2 or 3")
        # keys are owned by the first `nshard` ranks (the conf's -s S servers)
        self.nshard = comm.size if nshard is None else max(1, min(int(nshard), comm.size))
        self.push_count = 0  # number of push requests applied (SGD's t)
        self.guard = StoreGuard(store)

    def _one(self):
        if self.comm.size != 1:
            raise RuntimeError("ShardedKV serves one shard; P > 1 runs through kv/psx.py")

    def flush(self):
        """(one shard: every push is applied when it is issued)"""

    def open(self, uniq, owner_cnt, insert, cnt=None, recv=None):
        """Resolve this minibatch's unique keys to slots (insert on train)."""
        self._one()
        sess = Session(uniq)
        if insert:
            self.guard.before_open(uniq.shape[0])
        sess.slots = self.store.find(uniq, insert)
        if insert:
            self.guard.after_open()
        return sess

    # ---------------------------------------------------------------- linear
    def linear_pull(self, sess):
        return self.store.linear_pull(sess.slots)

    def linear_push(self, sess, grad, algo, alpha, beta, l1, l2, defer=False):
        self.push_count += 1
        eta = (beta + float(self.push_count) ** 0.5) / alpha
        if sess.slots.shape[0]:
            self.store.linear_push(sess.slots, grad.reshape(-1), algo, alpha, beta, l1, l2, eta)

    # --------------------------------------------------------------- difacto
    def difacto_open_pull(self, uniq, owner_cnt, insert, cnt, hp, threshold, l1_shrk, seed,
                          recv=None, direct=False):
        """Find (insert), (data pass 0) count, lazy V allocation and the
        variable-length pull as ONE fused device pass over the keys. Returns
        (sess, hdr, vc).

        direct (device store): no pulled copy of the V rows -- hdr's vidx
        column holds table rows and vc IS the store's V slab, so the FM
        kernels read the rows in place (the gradient rows then follow the
        slab numbering too; the push takes them that way)."""
        self._one()
        sess = Session(uniq)
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

    def difacto_push(self, sess, gw, gvc, hp, threshold, l1_shrk, seed, defer=False):
        """Apply the gradients on this shard (FTRL on w, AdaGrad on V)."""
        if sess.slots.shape[0]:
            self.store.difacto_push(sess.slots, sess.hdr_own, gw, gvc, hp, threshold, l1_shrk,
                                    seed)
