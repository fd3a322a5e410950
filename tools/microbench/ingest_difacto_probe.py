"""DiFacto steps fed by the device ingest iterator (text or CRB blocks), in
one process (no tracker): ms per step, to find a format-dependent slowdown."""
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
from bench_e2e import criteo_text  # noqa: E402
from wormhole_amd import _native  # noqa: E402
from wormhole_amd.config.schema import DifactoConfig, Embedding  # noqa: E402
from wormhole_amd.data.device_text import DeviceTextIter  # noqa: E402
from wormhole_amd.models.difacto import DifactoLearner  # noqa: E402
from wormhole_amd.parallel.comm import Comm  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "crb"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1000000
shuf = int(sys.argv[3]) if len(sys.argv) > 3 else 10
work = "/tmp/ingest_probe"
os.makedirs(work, exist_ok=True)
txt = os.path.join(work, "a.txt")
if not os.path.exists(txt):
    open(txt, "wb").write(criteo_text(rows, 3))
path = txt
if fmt == "crb":
    path = os.path.join(work, "a.crb")
    if not os.path.exists(path):
        subprocess.run([os.path.join(ROOT, "bin", "convert.dmlc"), "-data_in", txt, "-data_out",
                        path, "-format_in", "criteo", "-format_out", "crb"], check=True)
dev = torch.device("cuda", 0)
host = _native.host()
emb = Embedding(dim=64, threshold=100)
lr = DifactoLearner(DifactoConfig(minibatch=100000, embedding=[emb]), Comm(dev, init=False), dev,
                    cap=1 << 22, vcap=1 << 18, seed=1)
it = DeviceTextIter(host, path, 0, 1, fmt, 100000, 100000 * shuf, 1.0, 7, dev)
batches = []
while (b := it.next()) is not None:
    a = b.to_main(dev) if hasattr(b, "to_main") else b
    batches.append(a)
torch.cuda.synchronize()
print("batches", len(batches), "rows", [int(a[3].numel()) for a in batches[:6]],
      "dtypes", [(x.dtype, tuple(x.shape), x.is_contiguous()) if x is not None else None
                 for x in batches[0]])
for rep in range(2):
    torch.cuda.synchronize()
    t = time.time()
    for i, (k, o, v, l) in enumerate(batches):
        nb = batches[i + 1][:3] if i + 1 < len(batches) else None
        lr.process(k, o, v, l, 0, 0, next_batch=nb)
    lr.flush()
    torch.cuda.synchronize()
    dt = time.time() - t
    print("%s rep %d: %.2f ms per step, %.1f M ex/s" % (fmt, rep, dt / len(batches) * 1e3,
                                                       sum(a[3].numel() for a in batches) / dt / 1e6))
