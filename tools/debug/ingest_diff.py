"""Where device Criteo keys differ from the host parser's (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_ingest import _criteo_text
from wormhole_amd import _native

host, hip = _native.host(), _native.hip()
data = _criteo_text(2000, 2)
keys_h, off_h, _, lab_h, _ = host.parse_text(data, "criteo")
t = torch.frombuffer(bytearray(data + b"\n"), dtype=torch.uint8)
k, lab, off = hip.parse_criteo(t.cuda(), 2000, True)
k, lab, off = k.cpu(), lab.cpu(), off.cpu()
print("nnz", k.numel(), keys_h.numel(), "offs equal", torch.equal(off, off_h),
      "labels equal", torch.equal(lab, lab_h))
lines = [ln.rstrip(b"\r") for ln in data.split(b"\n") if ln]
bad = 0
for r in range(2000):
    a, b = int(off_h[r]), int(off_h[r + 1])
    c, d = int(off[r]), int(off[r + 1])
    if b - a != d - c or not torch.equal(keys_h[a:b], k[c:d]):
        bad += 1
        if bad <= 5:
            f = lines[r].split(b"\t")
            print("row", r, "nfields", len(f), "host n", b - a, "dev n", d - c)
            hk = {int(x) >> 54: int(x) for x in keys_h[a:b]}
            dk = {int(x) >> 54: int(x) for x in k[c:d]}
            for fi in sorted(set(hk) | set(dk)):
                if hk.get(fi) != dk.get(fi):
                    print("  field", fi, "len", len(f[fi + 1]) if fi + 1 < len(f) else None,
                          hk.get(fi), dk.get(fi))
print("bad rows", bad)
