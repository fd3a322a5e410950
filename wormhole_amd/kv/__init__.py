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
from .cpu_store import CpuKVStore


def make_store(cap, vcap, dim, device):
    device = torch.device(device)
    if device.type == "cuda":
        return _native.hip().KVStore(int(cap), int(vcap), int(dim), device.index or 0)
    return CpuKVStore(cap, vcap, dim)


class Session:
    """Per-minibatch exchange state (keys sent once, splits reused)."""

    __slots__ = ("send", "recv", "keys", "slots", "hdr_own", "vsend", "vrecv", "m")

    def __init__(self, send, recv, keys):
        self.send = send
        self.recv = recv
        self.keys = keys
        self.slots = None
        self.hdr_own = None  # owner-side pull header (owner vidx numbering)
        self.vsend = None    # embedding rows this rank sent per peer in the pull
        self.vrecv = None    # ... and received per peer
        self.m = None        # device int64 [1]: embedding rows in the local model

    def segments(self):
        b = 0
        for n in self.recv:
            yield b, b + n
            b += n


class ShardedKV:
    def __init__(self, store, comm, nshard=None):
        self.store = store
        self.comm = comm
        # keys are owned by the first `nshard` ranks (the conf's -s S servers)
        self.nshard = comm.size if nshard is None else max(1, min(int(nshard), comm.size))
        self.push_count = 0  # number of push requests applied (SGD's t)

    def open(self, uniq, owner_cnt, insert):
        send = [int(x) for x in (owner_cnt.tolist() if hasattr(owner_cnt, "tolist") else owner_cnt)]
        send += [0] * (self.comm.size - len(send))
        if self.comm.size == 1:
            sess = Session(send, send, uniq)
        else:
            recv = self.comm.exchange_counts(send)
            sess = Session(send, recv, self.comm.all_to_all_v(uniq, send, recv))
        sess.slots = self.store.find(sess.keys, insert)
        return sess

    def _to_owner(self, sess, x):
        return x if self.comm.size == 1 else self.comm.all_to_all_v(x, sess.send, sess.recv)

    def _to_worker(self, sess, x):
        return x if self.comm.size == 1 else self.comm.all_to_all_v(x, sess.recv, sess.send)

    # ---------------------------------------------------------------- linear
    def linear_pull(self, sess):
        return self._to_worker(sess, self.store.linear_pull(sess.slots))

    def linear_push(self, sess, grad, algo, alpha, beta, l1, l2):
        g = self._to_owner(sess, grad.reshape(-1).contiguous())
        for a, b in sess.segments():
            self.push_count += 1
            eta = (beta + float(self.push_count) ** 0.5) / alpha
            if b > a:
                self.store.linear_push(sess.slots[a:b], g[a:b], algo, alpha, beta, l1, l2, eta)

    # --------------------------------------------------------------- difacto
    def difacto_push_cnt(self, sess, cnt, hp, threshold, l1_shrk, seed):
        c = self._to_owner(sess, cnt)
        for a, b in sess.segments():
            if b > a:
                self.store.difacto_push_cnt(sess.slots[a:b], c[a:b], hp, threshold, l1_shrk, seed)

    def difacto_pull(self, sess, l1_shrk):
        """Returns (hdr [U, 2], vc [mcap, vstride]) in the worker's key order;
        sess.m holds the live embedding-row count on the device."""
        hdr, vc, vpos = self.store.difacto_pull(sess.slots, l1_shrk)
        sess.hdr_own = hdr
        if self.comm.size == 1:
            sess.m = vpos[-1:]
            return hdr, vc
        # per-peer embedding rows: vpos at the receive-segment boundaries
        bounds = [0]
        for n in sess.recv:
            bounds.append(bounds[-1] + n)
        vb = vpos[torch.tensor(bounds, dtype=torch.int64, device=vpos.device)].tolist()
        sess.vrecv = [vb[i + 1] - vb[i] for i in range(len(sess.recv))]  # owner -> worker
        sess.vsend = self.comm.exchange_counts(sess.vrecv)
        hdr_w = self.comm.all_to_all_v(hdr, sess.recv, sess.send)
        vc_w = self.comm.all_to_all_v(vc[:vb[-1]], sess.vrecv, sess.vsend)
        sess.m = ops.vidx_renumber(hdr_w)
        return hdr_w, vc_w

    def difacto_push(self, sess, gw, gvc, hp, threshold, l1_shrk, seed):
        if self.comm.size == 1:
            g, gv = gw, gvc
        else:
            g = self.comm.all_to_all_v(gw.contiguous(), sess.send, sess.recv)
            gv = self.comm.all_to_all_v(gvc[:sum(sess.vsend)].contiguous(), sess.vsend,
                                        sess.vrecv)
        for a, b in sess.segments():
            if b > a:
                self.store.difacto_push(sess.slots[a:b], sess.hdr_own[a:b], g[a:b], gv, hp,
                                        threshold, l1_shrk, seed)
