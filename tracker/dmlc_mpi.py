#!/usr/bin/env python3
"""MPI launcher (dmlc-core ``dmlc_mpi.py`` command line; SURVEY §2.4: MPI is
only a process launcher here, no MPI collectives are used):

    dmlc_mpi.py -n W [-s S] [-H hostfile] <binary> <args...>

Runs ``mpirun -n W [--hostfile H] -x VAR ... <cmd>``; each worker takes its
rank from the MPI launcher (OMPI_COMM_WORLD_RANK / PMI_RANK) and its GPU from
the local rank. For a PS job (-s S > 0) the scheduler runs on this machine.
``--dry-run`` prints the command instead of running it.
"""
import argparse
import os
import shutil
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tracker_common import add_common_args, host_ip, job_env, normalize_cmd  # noqa: E402


def mpirun_cmd(args, env, cmd):
    mpirun = shutil.which("mpirun") or "mpirun"
    c = [mpirun, "-n", str(args.num_workers)]
    if args.hostfile:
        c += ["--hostfile", args.hostfile]
    for k in sorted(env):
        c += ["-x", "%s=%s" % (k, env[k])]
    c += ["-x", "DMLC_ROLE=worker"]
    return c + cmd


def main(argv=None):
    ap = argparse.ArgumentParser(description="MPI launcher for wormhole_amd jobs")
    ap.add_argument("-H", "--hostfile", default=None)
    ap.add_argument("--host-ip", default=None)
    ap.add_argument("--dry-run", action="store_true")
    add_common_args(ap)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing the binary to run")
    root = args.host_ip or (host_ip() if args.hostfile else "127.0.0.1")
    env = job_env(args.num_workers, args.num_servers, root)
    cmd = normalize_cmd(args.command)
    workers = mpirun_cmd(args, env, cmd)
    if args.dry_run:
        if args.num_servers > 0:
            print("local: DMLC_ROLE=scheduler " + " ".join(cmd))
        print(" ".join(workers))
        return 0
    if not shutil.which("mpirun"):
        raise SystemExit("dmlc_mpi.py: mpirun not found on PATH")
    sched = None
    if args.num_servers > 0:
        sched = subprocess.Popen(cmd, env=dict(os.environ, DMLC_ROLE="scheduler", **env))
    rc = subprocess.call(workers)
    if sched is not None:
        rc = sched.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
