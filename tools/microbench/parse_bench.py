"""Device Criteo parse of one 100k-line text batch, repeated (kernel-time
study under rocprofv3; prints ms per parse)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))
from bench_e2e import criteo_text  # noqa: E402
from wormhole_amd import _native  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
hip = _native.hip()
text = torch.frombuffer(bytearray(criteo_text(n, 7)), dtype=torch.uint8).cuda()
for _ in range(3):
    hip.parse_criteo(text, n, True)
torch.cuda.synchronize()
t = time.time()
for _ in range(reps):
    keys, label, off = hip.parse_criteo(text, n, True)
torch.cuda.synchronize()
dt = (time.time() - t) / reps
print("rows %d bytes %d: %.3f ms per parse, %.1f M rows/s, %.1f GB/s, nnz %d" % (
    n, text.numel(), dt * 1e3, n / dt / 1e6, text.numel() / dt / 1e9, keys.numel()))
