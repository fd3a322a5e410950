"""Helper of test_deterministic_gpu.py: train a few DiFacto steps in a fresh
process (the mode is read once per process) and print a digest of the
progress sums and the whole model (sorted by key)."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from wormhole_amd import _native  # noqa: E402
from wormhole_amd.config.schema import DifactoConfig, Embedding  # noqa: E402
from wormhole_amd.data.synthetic import CRITEO_TB_CARD  # noqa: E402
from wormhole_amd.kv.checkpoint import _gather, _numpy  # noqa: E402
from wormhole_amd.models.difacto import DifactoLearner  # noqa: E402
from wormhole_amd.parallel.comm import Comm  # noqa: E402

dev = torch.device("cuda", 0)
hip = _native.hip()
card = torch.tensor(CRITEO_TB_CARD, dtype=torch.int64, device=dev)
emb = Embedding(dim=16, threshold=4)
lr = DifactoLearner(DifactoConfig(minibatch=20000, embedding=[emb]), Comm(dev, init=False), dev,
                    cap=1 << 22, vcap=1 << 18, seed=3)
data = [hip.synth_criteo(20000, 5, s, card) for s in range(6)]
for s, (k, l, o) in enumerate(data):
    nb = (data[s + 1][0], data[s + 1][2], None) if s + 1 < len(data) else None
    lr.process(k, o, None, l, 0, 0, next_batch=nb)
prog = lr.take_progress()
snap = _numpy(_gather(lr.store, "difacto"))
order = np.argsort(snap["keys"].astype(np.uint64))
h = hashlib.sha256()
h.update(np.array(prog, dtype=np.float64).tobytes())
for name in ("keys", "w", "z", "sq", "cnt"):
    h.update(np.ascontiguousarray(snap[name][order]).tobytes())
hv = snap["has_v"][order]
vrow_rank = np.cumsum(snap["has_v"]) - 1  # V rows in slot order -> reorder by key
vidx = vrow_rank[order][hv]
h.update(np.ascontiguousarray(snap["V"][vidx]).tobytes())
h.update(np.ascontiguousarray(snap["VG"][vidx]).tobytes())
# the linear model's single-GPU native step with the look-ahead localize (in
# deterministic mode: the hash localize, finished on the compute stream)
from wormhole_amd.config.schema import LinearConfig  # noqa: E402
from wormhole_amd.models.linear import LinearLearner  # noqa: E402
lin = LinearLearner(LinearConfig(minibatch=20000), Comm(dev, init=False), dev, cap=1 << 22)
for s, (k, l, o) in enumerate(data):
    nb = (data[s + 1][0], data[s + 1][2], None) if s + 1 < len(data) else None
    lin.process(k, o, None, l, 0, 0, next_batch=nb)
lin.flush()
lp = lin.take_progress()
ls = _numpy(_gather(lin.store, "linear"))
lo = np.argsort(ls["keys"].astype(np.uint64))
h.update(np.array(lp, dtype=np.float64).tobytes())
for name in ("keys", "w"):
    h.update(np.ascontiguousarray(ls[name][lo]).tobytes())
print("DIGEST", h.hexdigest(), "LOSS %.9g" % (prog[0] / prog[5]))
