#!/usr/bin/env python3
"""Multi-host launcher over ssh (dmlc-core ``dmlc_ssh.py`` command line):

    dmlc_ssh.py -n W [-s S] -H hostfile [--gpus-per-host G] <binary> <args...>

Worker rank r runs on host ``hosts[r // G]`` (hosts listed once per line in
the host file) with ``LOCAL_RANK = r % G`` (its GPU), started through
``ssh host 'cd <cwd> && env ... <cmd>'``; the job's working directory must be
the same path on every host (shared file system). For a PS job (-s S > 0)
the scheduler runs on this machine. ``--dry-run`` prints the commands.
"""
import argparse
import os
import shlex
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tracker_common import add_common_args, host_ip, job_env, normalize_cmd, read_hosts  # noqa: E402


def plan(args):
    hosts = read_hosts(args.hostfile)
    g = args.gpus_per_host
    if args.num_workers > len(hosts) * g:
        raise SystemExit("%d workers need %d hosts at %d GPUs each; host file has %d" % (
            args.num_workers, (args.num_workers + g - 1) // g, g, len(hosts)))
    root = args.host_ip or host_ip()
    env = job_env(args.num_workers, args.num_servers, root)
    cmd = normalize_cmd(args.command)
    cwd = os.getcwd()
    jobs = []
    if args.num_servers > 0:
        e = dict(env, DMLC_ROLE="scheduler")
        jobs.append(("local", e, cmd))
    for r in range(args.num_workers):
        e = dict(env, DMLC_ROLE="worker", RANK=str(r), DMLC_TASK_ID=str(r),
                 DMLC_WORKER_ID=str(r), LOCAL_RANK=str(r % g), LOCAL_WORLD_SIZE=str(g))
        remote = "cd %s && env %s %s" % (
            shlex.quote(cwd), " ".join("%s=%s" % (k, shlex.quote(v)) for k, v in sorted(e.items())),
            " ".join(shlex.quote(c) for c in cmd))
        jobs.append((hosts[r // g], e, ["ssh", "-o", "StrictHostKeyChecking=no", hosts[r // g],
                                        remote]))
    return jobs


def main(argv=None):
    ap = argparse.ArgumentParser(description="ssh launcher for wormhole_amd jobs")
    ap.add_argument("-H", "--hostfile", required=True)
    ap.add_argument("--gpus-per-host", type=int, default=8)
    ap.add_argument("--host-ip", default=None, help="address workers use to reach this host")
    ap.add_argument("--dry-run", action="store_true")
    add_common_args(ap)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing the binary to run")
    jobs = plan(args)
    if args.dry_run:
        for host, _, cmd in jobs:
            print("%s: %s" % (host, " ".join(cmd)))
        return 0
    procs = []
    for host, env, cmd in jobs:
        e = dict(os.environ, **env) if host == "local" else None
        procs.append(subprocess.Popen(cmd, env=e))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
