"""Device-side Criteo ingest (csrc/hip/ingest.hip + the host TextBatches
batcher): keys, labels and row offsets must be bit-identical to the host
parser (csrc/host/parsers.cc ParseCriteo, whose CityHash64 keys follow
learn/base/criteo_parser.h:64-86)."""
import os
import random

import pytest
import torch

from wormhole_amd import _native


def _criteo_text(nlines, seed):
    """Lines that exercise the tokenizer: empty and missing fields, every
    CityHash64 length class (0-16, 17-32, 33-64, >64 bytes), CRLF endings,
    empty lines, a final line without a newline."""
    rng = random.Random(seed)
    alpha = "0123456789abcdefXYZ_-."
    out = []
    for i in range(nlines):
        f = [rng.choice(["0", "1"])]
        nf = 39 if rng.random() < 0.9 else rng.randrange(0, 45)
        for k in range(nf):
            r = rng.random()
            if r < 0.1:
                f.append("")
            elif r < 0.8:
                f.append("".join(rng.choice(alpha) for _ in range(rng.randrange(1, 12))))
            else:
                n = rng.choice([17, 24, 32, 33, 48, 64, 65, 100, 200])
                f.append("".join(rng.choice(alpha) for _ in range(n)))
        line = "\t".join(f)
        out.append(line + ("\r\n" if i % 7 == 3 else "\n"))
        if i % 11 == 5:
            out.append("\n")
    text = "".join(out)
    return text[:-1].encode()  # the last line ends without a newline


def _batches(path, mb, pinned):
    tb = _native.host().TextBatches(str(path), 0, 1, mb, pinned)
    res = []
    while True:
        b = tb.next()
        if b is None:
            return res
        res.append(b)


def test_text_batches_cut_whole_lines(tmp_path):
    data = _criteo_text(300, 1)
    p = tmp_path / "d.txt"
    p.write_bytes(data)
    bs = _batches(p, 16, False)
    joined = b"".join(bytes(t.numpy()) for t, _ in bs)
    assert joined == data + b"\n"
    nonempty = [ln for ln in data.split(b"\n") if ln]
    assert sum(n for _, n in bs) == len(nonempty) == 300
    for t, n in bs[:-1]:
        assert n == 16 and bytes(t[-1:].numpy()) == b"\n"


@pytest.mark.gpu
def test_device_criteo_parse_matches_host_parser(tmp_path):
    host = _native.host()
    hip = _native.hip()
    data = _criteo_text(2000, 2)
    p = tmp_path / "d.txt"
    p.write_bytes(data)
    keys_h, off_h, _, lab_h, _ = host.parse_text(data, "criteo")
    keys, labs, offs = [], [], [0]
    for t, n in _batches(p, 137, True):
        k, lab, off = hip.parse_criteo(t.cuda(), n, True)
        assert off.numel() == n + 1 and lab.numel() == n
        keys.append(k.cpu())
        labs.append(lab.cpu())
        offs.extend((off[1:].cpu() + offs[-1]).tolist())
    assert torch.equal(torch.cat(keys), keys_h)
    assert torch.equal(torch.cat(labs), lab_h)
    assert offs == off_h.tolist()
    # criteo_test: no label column, every field a feature
    t = torch.frombuffer(bytearray(data + b"\n"), dtype=torch.uint8)
    keys_t, off_t, _, lab_t, _ = host.parse_text(data, "criteo_test")
    k, lab, off = hip.parse_criteo(t.cuda(), 2000, False)
    assert torch.equal(k.cpu(), keys_t) and torch.equal(off.cpu(), off_t)
    assert float(lab.abs().sum()) == 0.0


@pytest.mark.gpu
def test_ps_worker_device_parse_trains_like_host_parse(tmp_path):
    """The same linear job on Criteo text with the device parser and with the
    host parser learns the same model (same keys, same row order)."""
    import subprocess
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = tmp_path / "train.txt"
    p.write_bytes(_criteo_text(20000, 3))
    models = []
    for dp in ("1", "0"):
        conf = tmp_path / ("c%s.conf" % dp)
        conf.write_text('train_data = "%s"\ndata_format = "criteo"\nmax_data_pass = 1\n'
                        'minibatch = 1000\nmodel_out = "%s/m%s"\n' % (p, tmp_path, dp))
        env = dict(os.environ, WH_DEVICE_PARSE=dp)
        r = subprocess.run([sys.executable, os.path.join(root, "tracker", "dmlc_local.py"), "-n",
                            "1", "-s", "1", os.path.join(root, "bin", "linear.dmlc"), str(conf)],
                           capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
        assert r.returncode == 0, r.stderr[-3000:]
        rec = np.fromfile(str(tmp_path / ("m%s_part-0" % dp)),
                          dtype=np.dtype([("k", "<u8"), ("w", "<f4")]))
        models.append(np.sort(rec, order="k"))
    a, b = models
    assert len(a) > 1000 and np.array_equal(a["k"], b["k"])
    np.testing.assert_allclose(a["w"], b["w"], rtol=1e-4, atol=1e-6)
