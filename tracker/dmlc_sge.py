#!/usr/bin/env python3
"""Sun Grid Engine launcher (dmlc-core ``dmlc_sge.py`` command line):

    dmlc_sge.py -n W [-s S] [-q queue] [--jobname NAME] <binary> <args...>

Submits one SGE array job of W tasks (``qsub -t 1-W``); task i runs worker
rank i-1 (``SGE_TASK_ID``, see wormhole_amd.parallel.comm.env_rank). The
rendezvous address is this machine, where a PS job's scheduler also runs.
``--dry-run`` prints the job script instead of submitting it.
"""
import argparse
import os
import shlex
import shutil
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tracker_common import add_common_args, host_ip, job_env, normalize_cmd  # noqa: E402


def job_script(args, env, cmd):
    lines = ["#!/bin/bash", "#$ -S /bin/bash", "#$ -cwd", "#$ -N %s" % args.jobname,
             "#$ -t 1-%d" % args.num_workers]
    if args.queue:
        lines.append("#$ -q %s" % args.queue)
    if args.log_dir:
        lines += ["#$ -o %s" % args.log_dir, "#$ -e %s" % args.log_dir]
    for k in sorted(env):
        lines.append("export %s=%s" % (k, shlex.quote(env[k])))
    lines.append("export DMLC_ROLE=worker")
    lines.append("export RANK=$((SGE_TASK_ID - 1)) DMLC_TASK_ID=$((SGE_TASK_ID - 1))")
    lines.append(" ".join(shlex.quote(c) for c in cmd))
    return "\n".join(lines) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser(description="SGE launcher for wormhole_amd jobs")
    ap.add_argument("-q", "--queue", default=None)
    ap.add_argument("--jobname", default="wormhole")
    ap.add_argument("--log-dir", default=None)
    ap.add_argument("--host-ip", default=None)
    ap.add_argument("--dry-run", action="store_true")
    add_common_args(ap)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing the binary to run")
    env = job_env(args.num_workers, args.num_servers, args.host_ip or host_ip())
    cmd = normalize_cmd([os.path.abspath(args.command[0])] + args.command[1:])
    script = job_script(args, env, cmd)
    if args.dry_run:
        sys.stdout.write(script)
        return 0
    if not shutil.which("qsub"):
        raise SystemExit("dmlc_sge.py: qsub not found on PATH")
    sched = None
    if args.num_servers > 0:
        sched = subprocess.Popen(cmd, env=dict(os.environ, DMLC_ROLE="scheduler", **env))
    with tempfile.NamedTemporaryFile("w", suffix=".sh", delete=False) as f:
        f.write(script)
    rc = subprocess.call(["qsub", "-sync", "y", f.name])
    if sched is not None:
        rc = sched.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
