"""Shared pieces of the job launchers (dmlc-core tracker protocol).

Every launcher gives each process the same environment contract:

* ``DMLC_ROLE`` = scheduler | worker, ``DMLC_NUM_WORKER`` / ``DMLC_NUM_SERVER``,
  ``DMLC_PS_ROOT_URI`` / ``DMLC_PS_ROOT_PORT`` (the scheduler's control-plane
  address), ``DMLC_TRACKER_URI``;
* the torch.distributed rendezvous: ``MASTER_ADDR`` / ``MASTER_PORT``,
  ``WORLD_SIZE``; ``RANK`` / ``LOCAL_RANK`` where the launcher knows them, else
  the worker derives them from the launcher's own variables
  (``OMPI_COMM_WORLD_RANK``, ``PMI_RANK``, ``SGE_TASK_ID``; see
  :func:`wormhole_amd.parallel.comm.env_rank`).

PS jobs (``-s S > 0``) run the scheduler on the launching machine; every worker
process owns a GPU and a parameter shard (the ps-lite server group is folded
into the workers), so no separate server processes are started.
"""
import os
import socket
import sys


def free_port():
    s = socket.socket()
    s.bind(("", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def host_ip(default="127.0.0.1"):
    """An address of this machine other hosts can reach (best effort)."""
    try:
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        s.connect(("10.255.255.255", 1))
        ip = s.getsockname()[0]
        s.close()
        return ip
    except OSError:
        return default


def normalize_cmd(cmd):
    """Run Python app entry points (bin/*.dmlc python scripts) with this
    interpreter; native tools and shell wrappers run as they are."""
    cmd = list(cmd)
    if cmd and os.path.isfile(cmd[0]):
        try:
            with open(cmd[0], "rb") as f:
                first = f.readline()
        except OSError:
            first = b""
        if cmd[0].endswith(".py") or (first.startswith(b"#!") and b"python" in first):
            cmd = [sys.executable] + cmd
    return cmd


def job_env(num_workers, num_servers, root_uri, ps_port=None, master_port=None, attempt=0):
    env = {
        "DMLC_NUM_WORKER": str(num_workers),
        "DMLC_NUM_SERVER": str(num_servers),
        "DMLC_PS_ROOT_URI": root_uri,
        "DMLC_PS_ROOT_PORT": str(ps_port or free_port()),
        "DMLC_TRACKER_URI": root_uri,
        "MASTER_ADDR": root_uri,
        "MASTER_PORT": str(master_port or free_port()),
        "WORLD_SIZE": str(num_workers),
        "WH_RESTART_ATTEMPT": str(attempt),
        "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    }
    return env


def read_hosts(path):
    hosts = []
    for line in open(path):
        line = line.split("#")[0].strip()
        if line:
            hosts.append(line.split()[0].split(":")[0])
    if not hosts:
        raise SystemExit("host file %s lists no hosts" % path)
    return hosts


def add_common_args(ap):
    ap.add_argument("-n", "--num-workers", type=int, required=True)
    ap.add_argument("-s", "--num-servers", type=int, default=0)
    ap.add_argument("command", nargs="...")
