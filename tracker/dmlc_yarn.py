#!/usr/bin/env python3
"""YARN launcher (dmlc-core ``dmlc_yarn.py`` command line, e.g. the xgboost
guide's ``dmlc_yarn.py -n 4 --vcores 2 bin/xgboost.dmlc conf k=v``):

    dmlc_yarn.py -n W [-s S] [--vcores C] [--memory MB] [--ngpus G] <binary> <args...>

YARN containers are started by dmlc-core's ApplicationMaster jar
(``$DMLC_YARN_JAR``, ``hadoop jar ... -cmd ...``); every container receives
the job environment of tracker_common.job_env plus ``DMLC_ROLE=worker`` and
takes its rank from ``DMLC_TASK_ID``. A PS job's scheduler runs here.
``--dry-run`` prints the submission command.
"""
import argparse
import os
import shlex
import shutil
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tracker_common import add_common_args, host_ip, job_env, normalize_cmd  # noqa: E402


def yarn_cmd(args, env, cmd):
    jar = os.environ.get("DMLC_YARN_JAR", "dmlc-yarn.jar")
    c = ["hadoop", "jar", jar, "org.apache.hadoop.yarn.dmlc.Client",
         "-nworker", str(args.num_workers), "-vcores", str(args.vcores),
         "-memory", str(args.memory), "-ngpus", str(args.ngpus), "-jobname", args.jobname]
    for k in sorted(env):
        c += ["-env", "%s=%s" % (k, env[k])]
    c += ["-env", "DMLC_ROLE=worker", "-cmd", " ".join(shlex.quote(x) for x in cmd)]
    return c


def main(argv=None):
    ap = argparse.ArgumentParser(description="YARN launcher for wormhole_amd jobs")
    ap.add_argument("--vcores", type=int, default=1)
    ap.add_argument("--memory", type=int, default=4096)
    ap.add_argument("--ngpus", type=int, default=1)
    ap.add_argument("--jobname", default="wormhole")
    ap.add_argument("--host-ip", default=None)
    ap.add_argument("--dry-run", action="store_true")
    add_common_args(ap)
    args = ap.parse_args(argv)
    if not args.command:
        ap.error("missing the binary to run")
    env = job_env(args.num_workers, args.num_servers, args.host_ip or host_ip())
    cmd = normalize_cmd(args.command)
    sub = yarn_cmd(args, env, cmd)
    if args.dry_run:
        print(" ".join(sub))
        return 0
    if not shutil.which("hadoop"):
        raise SystemExit("dmlc_yarn.py: hadoop not found on PATH (set DMLC_YARN_JAR too)")
    sched = None
    if args.num_servers > 0:
        sched = subprocess.Popen(cmd, env=dict(os.environ, DMLC_ROLE="scheduler", **env))
    rc = subprocess.call(sub)
    if sched is not None:
        rc = sched.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
