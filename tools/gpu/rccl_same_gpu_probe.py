#!/usr/bin/env python3
"""Probe: can several RCCL ranks share one GPU through RCCL's network
transport (a host id of its own per rank, ``WH_BENCH_SAME_GPU=1``)? Each
stage prints a line, so a hang names where it stopped.

    timeout -k 10 120 python tools/gpu/rccl_same_gpu_probe.py [NRANKS]
"""
import os
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def _say(rank, msg):
    print("[probe %d %.1fs] %s" % (rank, time.time() - _T0, msg), flush=True)


_T0 = time.time()


def _main(rank, world, port, lazy):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0", WH_BENCH_SAME_GPU="1")
    import torch.distributed as dist
    from wormhole_amd.parallel.comm import same_gpu_rccl
    torch.cuda.set_device(0)
    same_gpu_rccl(rank)
    _say(rank, "env NCCL_HOSTID=%s IFNAME=%s" % (os.environ["NCCL_HOSTID"],
                                                  os.environ.get("NCCL_SOCKET_IFNAME")))
    kw = {} if lazy else {"device_id": torch.device("cuda", 0)}
    dist.init_process_group("nccl", rank=rank, world_size=world, **kw)
    _say(rank, "process group up (lazy=%s)" % lazy)
    t = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    _say(rank, "c10d all_reduce -> %s" % t.tolist())
    from wormhole_amd import _native
    hip = _native.hip()
    store = dist.distributed_c10d._get_default_store()
    if rank == 0:
        store.set("probe_uid", bytes(hip.RcclComm.unique_id()))
    uid = store.get("probe_uid")
    c = hip.RcclComm(bytes(uid), world, rank, 0)
    _say(rank, "own RcclComm up")
    x = torch.full((world * 3, 4), float(rank), device="cuda")
    y = c.a2av(x, [3] * world, [3] * world)
    torch.cuda.synchronize()
    _say(rank, "a2av ok: %s" % y[:, 0].tolist())
    c.close()
    dist.destroy_process_group()
    _say(rank, "done")


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    lazy = len(sys.argv) > 2 and sys.argv[2] == "lazy"
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_main, args=(world, port, lazy), nprocs=world, join=True)
