"""Entry point of the parameter-server learners (bin/linear.dmlc,
bin/difacto.dmlc): ``<bin> <conf|none> [key=value ...]``.

Role comes from the launcher environment (tracker/dmlc_local.py):
``DMLC_ROLE`` = scheduler | worker (servers are folded into the workers: each
worker owns one parameter shard).  Without a launcher the binary runs a
1-worker job in-process (scheduler thread + worker), which is what
``dmlc_local.py -n 1 -s 1`` would do.
"""
import os
import sys
import threading
import time

import torch


def _device():
    want = os.environ.get("WH_DEVICE", "auto")
    if want == "cpu":
        return torch.device("cpu")
    if want == "auto" and not torch.cuda.is_available():
        return torch.device("cpu")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = torch.cuda.device_count()
    idx = local % max(n, 1)
    torch.cuda.set_device(idx)
    return torch.device("cuda", idx)


def _conf_cls(kind):
    from ..config import schema
    return schema.LinearConfig if kind == "linear" else schema.DifactoConfig


def latest_checkpoint(model_out, nshard):
    """Newest iteration k whose periodic save completed on every shard (each
    worker seals its shard with ``<model_out>_iter-<k>_part-<r>.ok`` once
    the shard and its resume state are written), or -1."""
    import re
    from ..utils import fs
    seen = {}
    for f in fs.glob(str(model_out) + "_iter-*_part-*.ok"):
        m = re.match(r".*_iter-(\d+)_part-(\d+)\.ok$", f)
        if m:
            seen.setdefault(int(m.group(1)), set()).add(int(m.group(2)))
    done = [k for k, parts in seen.items() if parts >= set(range(nshard))]
    return max(done) if done else -1


def scheduler_conf(kind, conf, nshard=1):
    """The fields the native scheduler (csrc/host/scheduler.cc) reads.

    On a restarted job (launcher ``--max-restart``: WH_RESTART_ATTEMPT > 0)
    with periodic saves, training resumes after the newest sealed
    checkpoint instead of starting over (reference: reload with model_in /
    load_iter, learn/solver/minibatch_solver.h:96-109)."""
    d = {"app": kind}
    attempt = int(os.environ.get("WH_RESTART_ATTEMPT", "0") or 0)
    if attempt > 0 and conf.model_out and int(conf.save_iter or 0) > 0:
        k = latest_checkpoint(conf.model_out, nshard)
        if k >= 0:
            d.update(model_in=conf.model_out, load_iter=k, resume=True)
    for k in ("train_data", "val_data", "data_format", "model_in", "model_out", "predict_out",
              "max_data_pass", "save_iter", "load_iter", "num_parts_per_file", "print_sec",
              "local_data"):
        v = getattr(conf, k, None)
        if v is not None and k not in d:
            d[k] = v
    if kind == "difacto":
        d["early_stop"] = bool(conf.early_stop)
        d["min_objv_decr"] = float(conf.min_objv_decr)
        if conf.has("max_objv"):
            d["max_objv"] = float(conf.max_objv)
    return d


def run_scheduler(host, kind, conf, nw, ns, van):
    """The native scheduler (GIL released while it runs); a short grace period
    lets the workers read the final exit command before the van closes."""
    host.run_scheduler(scheduler_conf(kind, conf, ns), nw, ns, van)
    time.sleep(0.2)


def _learner(kind, conf, comm, device, nshard, max_key=0):
    cap = int(os.environ.get("WH_KV_CAP", 1 << (24 if device.type == "cuda" else 16)))
    vcap = int(os.environ.get("WH_KV_VCAP", 1 << (20 if device.type == "cuda" else 14)))
    if kind == "linear":
        from ..models.linear import LinearLearner
        lr = LinearLearner(conf, comm, device, cap=cap, nshard=nshard)
    else:
        from ..models.difacto import DifactoLearner
        lr = DifactoLearner(conf, comm, device, cap=cap, vcap=vcap, nshard=nshard)
    lr.max_key = int(max_key)
    return lr


def split_system_flags(argv):
    """Separate ps-lite system flags (gflags style ``-name=value`` /
    ``--name=value`` / ``-name value``) from the conf file and its
    ``key=value`` overrides. Known: ``max_key`` (fold feature ids into
    [0, max_key), reference learn/base/localizer.h:108-115)."""
    flags, rest = {}, []
    i = 0
    while i < len(argv):
        a = argv[i]
        if a.startswith("-") and len(a) > 1 and not a[1:2].isdigit():
            name = a.lstrip("-")
            if "=" in name:
                name, val = name.split("=", 1)
            elif i + 1 < len(argv):
                i += 1
                val = argv[i]
            else:
                raise SystemExit("flag %s needs a value" % a)
            if name != "max_key":
                raise SystemExit("unknown system flag -%s" % name)
            flags[name] = int(val)
        else:
            rest.append(a)
        i += 1
    return flags, rest


def main(kind, argv):
    from .. import _native, config
    from ..parallel.comm import Comm
    from ..solver.ps import Worker

    sysflags, argv = split_system_flags(list(argv))
    if len(argv) < 1:
        print("usage: %s.dmlc <conf|none> [key=value ...]" % kind, file=sys.stderr)
        return 1
    conf = config.load(_conf_cls(kind), argv[0], argv[1:])
    if kind == "difacto" and conf.early_stop and not conf.val_data:
        raise SystemExit("early stop needs validation dataset")
    role = os.environ.get("DMLC_ROLE")
    nw = int(os.environ.get("DMLC_NUM_WORKER", "1"))
    ns = int(os.environ.get("DMLC_NUM_SERVER", "1"))
    nshard = max(1, min(ns, nw))
    host = _native.host()
    if role is None:
        # standalone: scheduler in a thread, one worker here
        van_s = host.Van()
        port = van_s.listen(0)
        err = []

        def run_sched():
            try:
                run_scheduler(host, kind, conf, 1, 1, van_s)
            except Exception as e:  # pragma: no cover - surfaced below
                err.append(e)
        th = threading.Thread(target=run_sched, daemon=True)
        th.start()
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("RANK", "0")
        dev = _device()
        comm = Comm(dev)
        van = host.Van()
        van.connect("127.0.0.1", port, "worker-0")
        Worker(conf, kind, _learner(kind, conf, comm, dev, 1, sysflags.get("max_key", 0)), comm,
               van, 1, kind).serve()
        th.join()
        van.close()
        van_s.close()
        if err:
            raise err[0]
        return 0
    uri = os.environ.get("DMLC_PS_ROOT_URI", "127.0.0.1")
    port = int(os.environ["DMLC_PS_ROOT_PORT"])
    if role == "scheduler":
        van = host.Van()
        van.listen(port)
        run_scheduler(host, kind, conf, nw, nshard, van)
        van.close()
        return 0
    if role == "server":
        # parameter shards live inside the workers; a server process has nothing to do
        return 0
    dev = _device()
    comm = Comm(dev)
    van = host.Van()
    van.connect(uri, port, "worker-%d" % comm.rank)
    try:
        Worker(conf, kind, _learner(kind, conf, comm, dev, nshard, sysflags.get("max_key", 0)),
               comm, van, nshard, kind).serve()
    finally:
        van.close()
        comm.finalize()
    return 0
