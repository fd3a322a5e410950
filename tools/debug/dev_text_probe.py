"""Exercise DeviceTextIter (shuffled and not) on generated Criteo text with
a stack dump on a stall (debug aid for the producer thread)."""
import faulthandler
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "benchmarks"))
from bench_e2e import criteo_text  # noqa: E402
from wormhole_amd import _native  # noqa: E402
from wormhole_amd.data.device_text import DeviceTextIter  # noqa: E402

faulthandler.dump_traceback_later(60, exit=True)
p = "/tmp/dtp.txt"
open(p, "wb").write(criteo_text(1_000_000, 3))
host = _native.host()
dev = torch.device("cuda", 0)
for shuf in (0, 10 * 100000):
    t0 = time.time()
    it = DeviceTextIter(host, p, 0, 1, "criteo", 100000, shuf, 1.0, 5, dev)
    n = 0
    while True:
        b = it.next()
        if b is None:
            break
        keys, off, val, lab = b.to_main(dev)
        n += lab.numel()
        print("shuf", shuf, "rows", n, "%.3f s" % (time.time() - t0), flush=True)
    torch.cuda.synchronize()
    print("done", shuf, n, flush=True)
