"""Collective communication: RCCL over xGMI on GPUs (torch.distributed backend
"nccl" IS RCCL on ROCm), gloo on CPU.  One process per GPU.

Replaces both of the reference's communication substrates:

* rabit (BSP allreduce / broadcast; SURVEY §2.6 call sites) -> :meth:`allreduce`,
  :meth:`broadcast`, :meth:`allgather_object`.
* ps-lite KVWorker push/pull (ZPull/ZPush/ZVPull/ZVPush) -> :meth:`all_to_all_v`,
  used by :class:`wormhole_amd.kv.ShardedKV` (keys sent once per minibatch,
  values/gradients reuse the same splits = ps-lite's KEY_CACHING).
"""
import datetime
import os

import torch
import torch.distributed as dist


# rank / local rank as set by the launchers (tracker/dmlc_*.py): torchrun and
# dmlc_local/ssh set RANK / LOCAL_RANK; under dmlc_mpi the MPI launcher's own
# variables name the rank; under dmlc_sge the (1-based) array task id does.
_RANK_VARS = ("RANK", "DMLC_TASK_ID", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "PMIX_RANK",
              "SLURM_PROCID")
_LOCAL_VARS = ("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
               "SLURM_LOCALID")


_RCCL_SEQ = 0  # native communicators made so far (the store key of each id)


def env_rank():
    for v in _RANK_VARS:
        if v in os.environ:
            return int(os.environ[v])
    if "SGE_TASK_ID" in os.environ and os.environ["SGE_TASK_ID"].isdigit():
        return int(os.environ["SGE_TASK_ID"]) - 1
    return 0


def env_world():
    return int(os.environ.get("WORLD_SIZE", os.environ.get("DMLC_NUM_WORKER", "1")))


def env_local_rank():
    for v in _LOCAL_VARS:
        if v in os.environ:
            return int(os.environ[v])
    return 0


def same_gpu_rccl(rank):
    """Let several RCCL ranks share one GPU (a rehearsal of the multi-GPU
    data plane on a one-GPU box). RCCL refuses two ranks of one host on the
    same device; with a host id of its own per rank (``NCCL_HOSTID``, which
    RCCL hashes in place of the host name) every rank looks like a node of
    its own, and the ranks talk through RCCL's network transport over the
    loopback interface (sockets, host-staged) instead of xGMI peer access.
    The transfers are slow, but every RCCL call of the multi-rank path --
    grouped per-peer ncclSend / ncclRecv on the step's three communicators,
    c10d's collectives -- runs for real. Must run before the first RCCL
    call of the process."""
    os.environ["NCCL_HOSTID"] = "wh-same-gpu-rank-%d" % int(rank)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")


class _Done:
    def wait(self):
        pass


class _Keep:
    """A pending collective plus the input it reads."""

    def __init__(self, work, keep):
        self.work = work
        self.keep = keep

    def wait(self):
        if self.work is not None:
            self.work.wait()
        self.work, self.keep = None, None


class _Reqs:
    """Pending point-to-point group; keeps the send buffers alive."""

    def __init__(self, reqs, keep):
        self.reqs = reqs
        self.keep = keep

    def wait(self):
        for r in self.reqs:
            r.wait()
        self.reqs, self.keep = [], None


class Comm:
    """A process group handle.  ``size == 1`` needs no torch.distributed."""

    def __init__(self, device=None, backend=None, init=True, timeout_s=600):
        self.rank = env_rank()
        self.size = env_world()
        if device is None:
            device = torch.device("cpu")
        self.device = torch.device(device)
        if backend is None:
            backend = os.environ.get("WH_COMM_BACKEND") or (
                "nccl" if self.device.type == "cuda" else "gloo")
        self.backend = backend
        # gloo with GPU tensors (a rehearsal of the multi-rank GPU code paths
        # with several ranks sharing one GPU, which RCCL refuses): tensors are
        # staged through host memory around every transfer
        self.stage = backend == "gloo" and self.device.type == "cuda"
        self.pg = None
        self._rccl = None  # the native exchange's own communicator (rccl())
        # ps-lite COMPRESSING filter (msg_compression): LZ4 per peer chunk on
        # HOST transfers (gloo between CPU ranks; not the staged multi-rank GPU
        # rehearsal, whose payloads are device rows staged per step). Device
        # transfers over RCCL/xGMI stay raw (docs/linear.md msg_compression).
        self.compress = False
        if self.size > 1 and init:
            if backend == "nccl" and os.environ.get("WH_BENCH_SAME_GPU") == "1":
                same_gpu_rccl(self.rank)
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29500")
                kw = dict(backend=backend, rank=self.rank, world_size=self.size,
                          timeout=datetime.timedelta(seconds=timeout_s))
                if backend == "nccl":
                    kw["device_id"] = self.device
                dist.init_process_group(**kw)
            self.pg = dist.group.WORLD
            self.rank = dist.get_rank()
            self.size = dist.get_world_size()

    # ------------------------------------------------------ native RCCL
    def rccl(self, tag="c23"):
        """This group's own RCCL communicator ``tag`` (csrc/bind/rccl_comm.h
        RcclComm: grouped ncclSend / ncclRecv per peer, driven from C++ by
        the multi-shard step, which keeps one per exchange class: RCCL runs a
        communicator's operations in issue order). Created on first use by
        every rank at the same point: rank 0 makes the id and passes it
        through the c10d store."""
        if self._rccl is None:
            self._rccl = {}
        c = self._rccl.get(tag)
        if c is None:
            from .. import _native
            hip = _native.hip()
            if self.backend != "nccl" or self.device.type != "cuda":
                raise RuntimeError("Comm.rccl: needs the nccl backend on a GPU")
            global _RCCL_SEQ
            _RCCL_SEQ += 1
            key = "wh_rccl_uid_%d_%s" % (_RCCL_SEQ, tag)
            if self.size == 1:
                uid = hip.RcclComm.unique_id()
            else:
                store = dist.distributed_c10d._get_default_store()
                if self.rank == 0:
                    uid = hip.RcclComm.unique_id()
                    store.set(key, uid)
                else:
                    uid = store.get(key)
            c = self._rccl[tag] = hip.RcclComm(bytes(uid), self.size, self.rank,
                                               self.device.index)
        return c

    def _close_rccl(self):
        for c in (self._rccl or {}).values():
            c.close()
        self._rccl = None

    # ----------------------------------------------------------- basics
    def barrier(self):
        if self.size > 1:
            if self.backend == "nccl" and self.device.type == "cuda":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def allreduce(self, t, op="sum"):
        if self.size == 1:
            return t
        o = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
             "min": dist.ReduceOp.MIN}[op]
        if self.stage and t.is_cuda:
            h = t.cpu()
            dist.all_reduce(h, op=o)
            t.copy_(h)
            return t
        dist.all_reduce(t, op=o)
        return t

    def broadcast(self, t, root=0):
        if self.size > 1:
            if self.stage and t.is_cuda:
                h = t.cpu()
                dist.broadcast(h, src=root)
                t.copy_(h)
            else:
                dist.broadcast(t, src=root)
        return t

    def allgather_object(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj)
        return out

    def allgather(self, t):
        if self.size == 1:
            return [t]
        if self.stage and t.is_cuda:
            h = t.cpu()
            out = [torch.empty_like(h) for _ in range(self.size)]
            dist.all_gather(out, h)
            return [o.to(t.device) for o in out]
        out = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(out, t)
        return out

    # ----------------------------------------------------- all-to-all-v
    def exchange_counts(self, send_counts):
        """send_counts: python list (len size) -> recv_counts list."""
        if self.size == 1:
            return list(send_counts)
        s = torch.tensor(send_counts, dtype=torch.int64,
                         device="cpu" if self.stage else self.device)
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s)
        return r.tolist()

    def set_compression(self, on):
        """Enable the LZ4 filter (applies to host transfers only)."""
        self.compress = bool(on) and self.backend == "gloo" and self.device.type == "cpu"

    def _a2a_lz4(self, x, send_rows, recv_rows):
        """all_to_all_v of a CPU tensor with every peer chunk LZ4-compressed
        (ps-lite COMPRESSING, learn/linear/async_sgd.h:290-301): the signed
        compressed sizes are exchanged first, then the packed bytes."""
        from .. import _native
        host = _native.host()
        x = x.contiguous()
        row = x.element_size()
        for d in x.shape[1:]:
            row *= int(d)
        sb = [int(r) * row for r in send_rows]
        rb = [int(r) * row for r in recv_rows]
        packed, csz = host.lz4_pack(x.view(-1).view(torch.uint8) if x.numel() else
                                    torch.empty(0, dtype=torch.uint8), sb)
        rcsz = torch.empty(self.size, dtype=torch.int64)
        dist.all_to_all_single(rcsz, torch.tensor(csz, dtype=torch.int64))
        rc = rcsz.tolist()
        got = torch.empty(sum(abs(c) for c in rc), dtype=torch.uint8)
        dist.all_to_all_single(got, packed.contiguous(), [abs(c) for c in rc],
                               [abs(c) for c in csz])
        out = torch.empty((sum(recv_rows),) + tuple(x.shape[1:]), dtype=x.dtype)
        host.lz4_unpack(got, rc, rb, out.view(-1).view(torch.uint8) if out.numel() else
                        torch.empty(0, dtype=torch.uint8))
        return out

    def all_to_all_v(self, x, send_rows, recv_rows):
        """Row-wise all-to-all-v: rank p receives send_rows[p] rows of x from
        this rank.  x may be 1-D or 2-D [rows, width]."""
        if self.size == 1:
            return x
        if self.stage and x.is_cuda:
            return self.all_to_all_v(x.cpu(), send_rows, recv_rows).to(x.device)
        if self.compress and not x.is_cuda:
            return self._a2a_lz4(x, send_rows, recv_rows)
        width = x[0].numel() if x.dim() > 1 and x.shape[0] > 0 else (
            x.shape[1] if x.dim() > 1 else 1)
        shape = (sum(recv_rows),) + tuple(x.shape[1:])
        out = torch.empty(shape, dtype=x.dtype, device=x.device)
        if x.dim() == 1:
            dist.all_to_all_single(out, x.contiguous(), recv_rows, send_rows)
        else:
            dist.all_to_all_single(out.view(-1), x.contiguous().view(-1),
                                   [r * width for r in recv_rows],
                                   [s * width for s in send_rows])
        return out

    def all_to_all_v_async(self, x, send_rows, recv_rows):
        """:meth:`all_to_all_v` without blocking the current stream: returns
        (out, work); ``work.wait()`` orders the CURRENT stream (at the time
        of the wait) after the transfer, so independent kernels queued in
        between overlap it. RCCL runs it on the process group's own stream,
        which waits for the current stream's queued work at issue time."""
        if self.size == 1:
            return x, _Done()
        if (self.stage and x.is_cuda) or (self.compress and not x.is_cuda):
            return self.all_to_all_v(x, send_rows, recv_rows), _Done()
        x = x.contiguous()
        width = 1
        for d in x.shape[1:]:
            width *= int(d)
        out = torch.empty((sum(recv_rows),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        # (issued even when this rank moves nothing: a collective every rank
        # must join; skipping it here would hang the peers)
        work = dist.all_to_all_single(out.view(-1), x.view(-1),
                                      [r * width for r in recv_rows],
                                      [s_ * width for s_ in send_rows], async_op=True)
        return out, _Keep(work, x)

    def all_to_all_v_multi(self, items, async_op=False):
        """Several row-wise all-to-all-v exchanges issued back to back, one
        RCCL all-to-all-v per tensor (RCCL runs each as one grouped
        send/recv over every xGMI peer link at once; the collectives queue on
        the same stream, so the tensors' transfers pipeline). items:
        [(x, send_rows, recv_rows), ...]. async_op: return (outputs, handle)
        and leave the wait to the caller (handle.wait() orders the current
        stream after the transfers); the inputs must stay alive until then."""
        if self.size == 1:
            outs = [x for x, _, _ in items]
            return (outs, _Done()) if async_op else outs
        if self.stage and any(x.is_cuda for x, _, _ in items):
            dev = [x.device for x, _, _ in items]
            outs = self.all_to_all_v_multi([(x.cpu(), s, r) for x, s, r in items])
            outs = [o.to(d) for o, d in zip(outs, dev)]
            return (outs, _Done()) if async_op else outs
        if self.compress and not any(x.is_cuda for x, _, _ in items):
            outs = [self.all_to_all_v(x, s_, r) for x, s_, r in items]
            return (outs, _Done()) if async_op else outs
        outs, reqs, keep = [], [], []
        for x, send, recv in items:
            x = x.contiguous()
            keep.append(x)
            out = torch.empty((sum(recv),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            outs.append(out)
            width = 1
            for d in x.shape[1:]:
                width *= int(d)
            if x.numel() == 0 and out.numel() == 0 and width == 0:
                continue
            req = dist.all_to_all_single(out.view(-1), x.view(-1),
                                         [r * width for r in recv], [s_ * width for s_ in send],
                                         async_op=async_op)
            if async_op:
                reqs.append(req)
        if async_op:
            return outs, _Reqs(reqs, keep)
        return outs

    def exchange_counts_dev(self, send_dev):
        """Device-side count exchange: send_dev int64 [size] -> recv int64
        [size] on the device (no host synchronisation)."""
        if self.size == 1:
            return send_dev.clone()
        if self.stage and send_dev.is_cuda:
            return self.exchange_counts_dev(send_dev.cpu()).to(send_dev.device)
        r = torch.empty_like(send_dev)
        dist.all_to_all_single(r, send_dev.contiguous())
        return r

    def finalize(self):
        self._close_rccl()
        if self.size > 1 and dist.is_initialized():
            # every rank is past its last collective before any tears the
            # group down (a gloo rank whose peer closed its sockets early
            # could abort in a transport thread: seen under CPU overload)
            self.barrier()
            if self.backend == "gloo":
                # gloo's barrier work holds the group's earlier works (and
                # so their tensors); the worker thread drops them just after
                # the barrier completes, and a tensor freed there takes the
                # GIL. Were the interpreter already finalising, that thread
                # would be ended mid-unwind and abort the process: give it
                # the GIL for a moment first (bin/_launch.py skips the
                # teardown altogether for the apps)
                import time
                time.sleep(0.05)
            dist.destroy_process_group()


class LoopbackComm(Comm):
    """``nshard`` virtual ranks in ONE process: every exchange is the
    identity (peer q sends this rank exactly what this rank sends q), so the
    multi-shard parameter-server code path -- owner grouping, packed records,
    row-aligned regions, multi-segment owner kernels, the pipelined step --
    runs end to end on a single GPU with no transport underneath. Used to
    measure that path's device and host overhead on one GPU (``bench.py
    --loopback P``); it owns every shard itself, so its table holds the whole
    key space like a 1-rank run."""

    def __init__(self, nshard, device=None, rccl=False):
        self.rank = 0
        self.size = int(nshard)
        self.device = torch.device(device if device is not None else "cpu")
        self.backend = "loopback"
        self.stage = False
        self.pg = None
        self._rccl = None
        self.compress = False
        # rccl=True: every exchange still moves this process's own bytes, but
        # through a real RCCL all-to-all on a 1-rank process group (async work
        # handles, the process group's stream, input lifetimes: exactly the
        # calls Comm makes over xGMI), so the RCCL stream semantics of the
        # multi-shard step are exercised on a one-GPU box, where RCCL refuses
        # two ranks on one device.
        self.rccl_on = bool(rccl) and self.device.type == "cuda"
        if self.rccl_on:
            if not dist.is_initialized():
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29531")
                dist.init_process_group(backend="nccl", rank=0, world_size=1,
                                        device_id=self.device)
            assert dist.get_world_size() == 1, "rccl loopback needs a 1-rank group"
            self.pg = dist.group.WORLD
            self.backend = "loopback-rccl"

    def rccl(self, tag="c23"):
        """A 1-rank RCCL communicator ``tag``: the native step moves the P-1
        virtual peers' segments as one send / recv pair to self (the own
        segment a device copy)."""
        if not self.rccl_on:
            raise RuntimeError("LoopbackComm.rccl: built without rccl=True")
        if self._rccl is None:
            self._rccl = {}
        c = self._rccl.get(tag)
        if c is None:
            from .. import _native
            hip = _native.hip()
            c = self._rccl[tag] = hip.RcclComm(bytes(hip.RcclComm.unique_id()), 1, 0,
                                               self.device.index)
        return c

    def _a2a(self, x, async_op):
        """Identity exchange through RCCL (1-rank all-to-all = self copy)."""
        x = x.contiguous()
        out = torch.empty_like(x)
        if x.numel() == 0:
            return out, _Done()
        work = dist.all_to_all_single(out.view(-1), x.view(-1), async_op=async_op)
        return out, (_Keep(work, x) if async_op else _Done())

    def barrier(self):
        pass

    def allreduce(self, t, op="sum"):
        return t

    def broadcast(self, t, root=0):
        return t

    def allgather_object(self, obj):
        return [obj] * self.size

    def allgather(self, t):
        return [t] * self.size

    def exchange_counts(self, send_counts):
        return list(send_counts)

    def all_to_all_v(self, x, send_rows, recv_rows):
        assert list(send_rows) == list(recv_rows), "loopback exchange must be symmetric"
        if self.rccl_on and x.is_cuda:
            return self._a2a(x, False)[0]
        return x

    def all_to_all_v_async(self, x, send_rows, recv_rows):
        assert list(send_rows) == list(recv_rows), "loopback exchange must be symmetric"
        if self.rccl_on and x.is_cuda:
            return self._a2a(x, True)
        return x, _Done()

    def all_to_all_v_multi(self, items, async_op=False):
        if self.rccl_on:
            outs, hs = [], []
            for x, s, r in items:
                assert list(s) == list(r), "loopback exchange must be symmetric"
                o, h = self._a2a(x, async_op)
                outs.append(o)
                hs.append(h)
            return (outs, _Reqs(hs, None)) if async_op else outs
        outs = [self.all_to_all_v(x, s, r) for x, s, r in items]
        return (outs, _Done()) if async_op else outs

    def exchange_counts_dev(self, send_dev):
        if self.rccl_on and send_dev.is_cuda:
            return self._a2a(send_dev, False)[0]
        return send_dev.clone()

    def finalize(self):
        self._close_rccl()
        if self.rccl_on and dist.is_initialized():
            dist.destroy_process_group()
