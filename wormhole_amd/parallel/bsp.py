"""BSP (rabit-style) engine on RCCL / gloo (SURVEY §2.2 "rabit", §5.3-5.4).

Reference API used by the rabit apps (lbfgs, fm, kmeans, xgboost):
Init/Finalize, GetRank/GetWorldSize, Allreduce<Sum|Max>(buf, n[, lazy_fn]),
Broadcast, LoadCheckPoint -> version, CheckPoint, LazyCheckPoint,
TrackerPrintf.  Re-expressed:

* collectives are torch.distributed (RCCL over xGMI on GPUs, gloo on CPU);
* the lazy prepare function of Allreduce is kept in the signature (it is
  skipped when the result was restored from a checkpoint);
* fault tolerance is checkpoint-restart: ``checkpoint()`` writes a versioned
  snapshot (global state once by rank 0, local state per rank) under
  ``$WH_CKPT_DIR``; a relaunched job (tracker ``--max-restart``) gets the
  latest complete version back from ``load_checkpoint()``.  RCCL
  communicators cannot shrink in place, so this replaces rabit's in-memory
  replicated replay.
"""
import glob
import os
import sys

import torch

from .comm import Comm


class BSP:
    def __init__(self, device=None, ckpt_dir=None, job="job"):
        if device is None:
            device = torch.device("cpu")
        self.comm = Comm(device)
        self.device = torch.device(device)
        self.rank = self.comm.rank
        self.world = self.comm.size
        self.ckpt_dir = ckpt_dir if ckpt_dir is not None else os.environ.get("WH_CKPT_DIR", "")
        self.job = job
        self.version = 0
        if self.ckpt_dir:
            os.makedirs(self.ckpt_dir, exist_ok=True)

    # -------------------------------------------------------- collectives
    def allreduce(self, t, op="sum", prepare=None):
        if prepare is not None:
            prepare()
        return self.comm.allreduce(t, op)

    def allreduce_scalar(self, v, op="sum", dtype=torch.float64):
        t = torch.tensor([v], dtype=dtype, device=self.comm.device)
        self.comm.allreduce(t, op)
        return t.item()

    def broadcast(self, t, root=0):
        return self.comm.broadcast(t, root)

    def barrier(self):
        self.comm.barrier()

    def tracker_print(self, msg):
        if self.rank == 0:
            sys.stdout.write(msg if msg.endswith("\n") else msg + "\n")
            sys.stdout.flush()

    # --------------------------------------------------------- checkpoint
    def _path(self, kind, version, rank=None):
        r = "" if rank is None else ".r%d" % rank
        return os.path.join(self.ckpt_dir, "%s.%s%s.v%d.pt" % (self.job, kind, r, version))

    def load_checkpoint(self):
        """Returns (version, global_state, local_state); version 0 = fresh."""
        if not self.ckpt_dir:
            return 0, None, None
        best = 0
        for f in glob.glob(os.path.join(self.ckpt_dir, "%s.global.v*.pt" % self.job)):
            try:
                best = max(best, int(f.rsplit(".v", 1)[1][:-3]))
            except ValueError:
                pass
        # every rank must agree on a version whose files all exist
        ok = best > 0 and os.path.exists(self._path("local", best, self.rank))
        v = int(self.allreduce_scalar(best if ok else 0, "min", torch.int64))
        if v == 0:
            return 0, None, None
        g = torch.load(self._path("global", v), map_location="cpu", weights_only=True)
        lp = self._path("local", v, self.rank)
        loc = torch.load(lp, map_location="cpu", weights_only=True) if os.path.exists(lp) else None
        self.version = v
        return v, g, loc

    def checkpoint(self, global_state, local_state=None):
        self.version += 1
        if not self.ckpt_dir:
            return self.version
        if local_state is not None:
            torch.save(local_state, self._path("local", self.version, self.rank))
        else:
            torch.save({}, self._path("local", self.version, self.rank))
        self.barrier()
        if self.rank == 0:
            tmp = self._path("global", self.version) + ".tmp"
            torch.save(global_state, tmp)
            os.replace(tmp, self._path("global", self.version))
            for old in range(1, self.version - 1):
                for f in glob.glob(os.path.join(self.ckpt_dir, "%s.*.v%d.pt" % (self.job, old))):
                    try:
                        os.remove(f)
                    except OSError:
                        pass
        self.barrier()
        return self.version

    def lazy_checkpoint(self, global_state):
        return self.checkpoint(global_state, None)

    def finalize(self):
        self.comm.finalize()


def fault_point(rank, version):
    """WH_FAULT=die:<rank>:<version>: exit right after checkpoint `version`
    on the first launch (fault-injection for the restart tests)."""
    spec = os.environ.get("WH_FAULT", "")
    if not spec.startswith("die:") or os.environ.get("WH_RESTART_ATTEMPT", "0") != "0":
        return
    _, r, v = spec.split(":")
    if int(r) == rank and int(v) == version:
        sys.stderr.write("[rank %d] WH_FAULT: dying after checkpoint %d\n" % (rank, version))
        sys.stderr.flush()
        os._exit(17)
