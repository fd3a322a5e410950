#!/usr/bin/env python3
"""Local job launcher, compatible with dmlc-core's ``tracker/dmlc_local.py``
command line (SURVEY §2.2 "dmlc-core tracker"):

    dmlc_local.py -n W [-s S] <binary> <args...>

* ``-s S > 0``  parameter-server job (linear, difacto): one scheduler process
  + W worker processes.  Parameter shards live inside the first S workers
  (the ps-lite server group is folded into the GPU workers), so no separate
  server processes are started.
* ``-s 0``      BSP / allreduce job (lbfgs, fm, kmeans, xgboost): W identical
  ranks.

Every worker gets the torch.distributed rendezvous (RANK, WORLD_SIZE,
LOCAL_RANK, MASTER_ADDR=127.0.0.1, MASTER_PORT) and the DMLC_* role
variables; worker i is pinned to GPU i mod #GPUs via LOCAL_RANK.  The
launcher monitors the children: the first failure terminates the job
(process groups), and ``--max-restart K`` relaunches a failed job up to K
times with WH_RESTART_ATTEMPT set: BSP ranks resume from their
last versioned checkpoint; a parameter-server job resumes after the newest
``save_iter`` checkpoint sealed on every shard (its scheduler loads it as
model_in / load_iter and continues with the next pass).
"""
import argparse
import os
import signal
import subprocess
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tracker_common import job_env, normalize_cmd  # noqa: E402


def launch_once(args, cmd, attempt):
    n, s = args.num_workers, args.num_servers
    base = dict(os.environ)
    base.update(job_env(n, s, "127.0.0.1", attempt=attempt))
    base["LOCAL_WORLD_SIZE"] = str(n)
    procs = []

    def spawn(role, rank):
        env = dict(base)
        env["DMLC_ROLE"] = role
        if role == "worker":
            env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "DMLC_TASK_ID": str(rank),
                        "DMLC_WORKER_ID": str(rank)})
        p = subprocess.Popen(cmd, env=env, start_new_session=True)
        procs.append((role, rank, p))

    if s > 0:
        spawn("scheduler", -1)
    for r in range(n):
        spawn("worker", r)

    rc = 0
    alive = list(procs)
    try:
        while alive:
            time.sleep(0.05)
            nxt = []
            for role, rank, p in alive:
                code = p.poll()
                if code is None:
                    nxt.append((role, rank, p))
                elif code != 0 and rc == 0:
                    rc = code
                    print("[tracker] %s %s exited with code %d; stopping the job" % (
                        role, "" if rank < 0 else rank, code), file=sys.stderr, flush=True)
            alive = nxt
            if rc != 0:
                break
    except KeyboardInterrupt:
        rc = 130
    if rc != 0:
        for _, _, p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for _, _, p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return rc


def main(argv=None):
    ap = argparse.ArgumentParser(description="local launcher for wormhole_amd jobs")
    ap.add_argument("-n", "--num-workers", type=int, required=True)
    ap.add_argument("-s", "--num-servers", type=int, default=0)
    ap.add_argument("--max-restart", type=int, default=0,
                    help="relaunch a failed job up to this many times (BSP: from the last "
                         "checkpoint; PS: after the last sealed save_iter checkpoint)")
    ap.add_argument("command", nargs=argparse.REMAINDER)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing the binary to run")
    cmd = normalize_cmd(args.command)
    attempt = 0
    while True:
        rc = launch_once(args, cmd, attempt)
        if rc == 0 or attempt >= args.max_restart:
            return rc
        attempt += 1
        print("[tracker] restarting the job (attempt %d)" % attempt, file=sys.stderr, flush=True)


if __name__ == "__main__":
    sys.exit(main())
