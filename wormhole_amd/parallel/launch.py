"""Self-launch of the multi-GPU benchmarks: one process per GPU.

``python bench.py --gpus N`` with no launcher around it (``WORLD_SIZE``
unset) starts N ranks itself -- ``torch.distributed.run --nproc-per-node N``
on 127.0.0.1 as a child process, the same launch the driver uses -- and exits
with the launcher's code. The parent never touches the GPU (counting devices
does not initialise HIP); it only checks that N devices are visible, so a
1-GPU box fails fast with a clear error instead of hanging in RCCL init.
Each rank then verifies its world (:func:`verify_world`): the group has
exactly N members and, on GPUs, no two ranks share a device (RCCL would
refuse that at init time anyway, with a much less helpful message).

Reference: the tracker launches W worker processes
(``tracker/dmlc_local.py -n W``, /root/reference/README.md:43).
"""
import os
import signal
import socket
import subprocess
import sys


def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
    finally:
        s.close()


def launched():
    """True inside a launcher-started rank (torchrun / dmlc trackers)."""
    return "WORLD_SIZE" in os.environ


def visible_gpus():
    """Devices this process could use, without initialising HIP."""
    import torch
    return torch.cuda.device_count()


def self_launch(script, argv, nproc, device="cuda", timeout_s=3600):
    """Run ``script argv`` as ``nproc`` ranks under torch.distributed.run and
    return its exit code (never hangs past ``timeout_s``: the whole process
    group is killed and 124 returned). Rank 0's stdout (the JSON line)
    passes straight through."""
    if device == "cuda" and os.environ.get("WH_BENCH_SAME_GPU") != "1":
        n = visible_gpus()
        if n < nproc:
            sys.stderr.write(
                "error: --gpus %d needs %d visible GPUs, only %d device%s visible "
                "(HIP_VISIBLE_DEVICES=%s)\n" % (nproc, nproc, n, "" if n == 1 else "s",
                                                os.environ.get("HIP_VISIBLE_DEVICES", "<unset>")))
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), script] + list(argv)
    env = dict(os.environ)
    env["WH_SELF_LAUNCHED"] = "1"
    env.setdefault("OMP_NUM_THREADS", "4")
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        sys.stderr.write("error: %d-rank run exceeded %d s; killing it\n" % (nproc, timeout_s))
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        p.wait()
        return 124
    except KeyboardInterrupt:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait()
        return 130


def verify_world(comm, expect, same_gpu_ok=False):
    """Inside a rank: the group has ``expect`` members and (GPU ranks) every
    rank drives a distinct device. Returns the per-rank device ids."""
    if comm.size != expect:
        raise SystemExit("rank %d: world size %d != --gpus %d" % (comm.rank, comm.size, expect))
    dev = comm.device
    ident = None
    if dev.type == "cuda":
        import torch
        pr = torch.cuda.get_device_properties(dev)
        ident = "%s:%x:%x:%x" % (pr.uuid, pr.pci_domain_id, pr.pci_bus_id, pr.pci_device_id)
    ids = comm.allgather_object(ident)
    if dev.type == "cuda" and not same_gpu_ok and len(set(ids)) != len(ids):
        raise SystemExit("rank %d: ranks share a GPU: %s" % (comm.rank, ids))
    return ids
