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
    host parser learns the same model (same keys, same row order: without a
    shuffle buffer the device path reads each part with ONE reader, in the
    host parser's order, whatever WH_TEXT_READERS says)."""
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
                        'minibatch = 1000\nrand_shuffle = 0\nmodel_out = "%s/m%s"\n'
                        % (p, tmp_path, dp))
        env = dict(os.environ, WH_DEVICE_PARSE=dp, WH_TEXT_READERS="4")
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


def _libsvm_text(nlines, seed, values=True, weights=True):
    rng = random.Random(seed)
    fmts = [lambda: "%d" % rng.randrange(0, 100), lambda: "%.6g" % rng.uniform(-1e3, 1e3),
            lambda: "%.3e" % rng.uniform(-1, 1), lambda: "%.9f" % rng.random(),
            lambda: "%.17g" % rng.lognormvariate(0, 20), lambda: "0.%s" % ("0" * rng.randrange(12)
                                                                         + "37")]
    out = []
    for i in range(nlines):
        lab = rng.choice(["1", "-1", "+1", "0", "0.5"])
        if weights and i % 5 == 2:
            lab += ":%g" % rng.uniform(0.1, 3)
        toks = [lab]
        for _ in range(rng.randrange(0, 150 if i % 9 == 0 else 12)):
            idx = str(rng.randrange(0, 1 << rng.choice([8, 20, 40])))
            if values and rng.random() < 0.7:
                idx += ":" + rng.choice(fmts)()
            toks.append(idx)
        sep = "\t" if i % 4 == 1 else " "
        out.append(sep.join(toks) + (" \r\n" if i % 6 == 3 else "\n"))
    return "".join(out).encode()


@pytest.mark.gpu
@pytest.mark.parametrize("values,weights", [(True, True), (False, False)])
def test_device_libsvm_parse_matches_host_parser(tmp_path, values, weights):
    host = _native.host()
    hip = _native.hip()
    data = _libsvm_text(3000, 4, values, weights)
    keys_h, off_h, val_h, lab_h, w_h = host.parse_text(data, "libsvm")
    t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    keys, lab, off, val, w = hip.parse_libsvm(t.cuda(), 3000)
    assert torch.equal(off.cpu(), off_h)
    assert torch.equal(keys.cpu(), keys_h)
    assert torch.equal(lab.cpu(), lab_h)
    assert (val is None) == (val_h is None) and (w is None) == (w_h is None)
    if val is not None:
        bad = (val.cpu() != val_h).nonzero()
        assert bad.numel() == 0, (bad[:5], val.cpu()[bad[:5]], val_h[bad[:5]])
    if w is not None:
        assert torch.equal(w.cpu(), w_h)


@pytest.mark.gpu
def test_device_shuffle_buffer_is_a_permutation_and_neg_sampling_drops_negatives(tmp_path):
    """rand_shuffle on the device: every row of the part exactly once,
    minibatches of exactly `mb` rows (spanning shuffle blocks), a different
    order than the file; neg_sampling keeps ~that share of the negatives."""
    from wormhole_amd.data.device_text import DeviceTextIter
    host = _native.host()
    dev = torch.device("cuda")
    data = _criteo_text(5000, 5)
    p = tmp_path / "d.txt"
    p.write_bytes(data)
    keys_h, off_h, _, lab_h, _ = host.parse_text(data, "criteo")
    rows_h = [tuple(keys_h[off_h[i]:off_h[i + 1]].tolist()) + (float(lab_h[i]),)
              for i in range(5000)]
    it = DeviceTextIter(host, str(p), 0, 1, "criteo", 300, 300 * 4, 1.0, 7, dev)
    rows, sizes = [], []
    while True:
        b = it.next()
        if b is None:
            break
        keys, off, val, lab = [x.cpu() if x is not None else None for x in b.to_main(dev)]
        assert val is None
        sizes.append(lab.numel())
        rows += [tuple(keys[off[i]:off[i + 1]].tolist()) + (float(lab[i]),)
                 for i in range(lab.numel())]
    assert sorted(rows) == sorted(rows_h) and rows != rows_h
    assert sizes[:-1] == [300] * (len(sizes) - 1)
    # no shuffle buffer: the part's sub-range readers, round-robin; every
    # row once, each reader's rows in file order
    it = DeviceTextIter(host, str(p), 0, 1, "criteo", 300, 0, 1.0, 7, dev)
    rows = []
    while True:
        b = it.next()
        if b is None:
            break
        keys, off, val, lab = [x.cpu() if x is not None else None for x in b.to_main(dev)]
        rows += [tuple(keys[off[i]:off[i + 1]].tolist()) + (float(lab[i]),)
                 for i in range(lab.numel())]
    assert sorted(rows) == sorted(rows_h)
    assert rows[:300] == rows_h[:300]  # the first batch: sub-range 0's first lines
    # a part shorter than a minibatch: one partial batch, then None, repeatedly
    it = DeviceTextIter(host, str(p), 3, 20, "criteo", 1000, 4000, 1.0, 7, dev)
    b = it.next()
    assert b is not None and 0 < b.to_main(dev)[3].numel() < 1000
    assert it.next() is None and it.next() is None
    it = DeviceTextIter(host, str(p), 0, 1, "criteo", 300, 0, 0.25, 7, dev)
    labs = []
    while True:
        b = it.next()
        if b is None:
            break
        labs.append(b.to_main(dev)[3].cpu())
    labs = torch.cat(labs)
    npos, nneg = int((lab_h > 0).sum()), int((lab_h <= 0).sum())
    assert int((labs > 0).sum()) == npos
    assert abs(int((labs <= 0).sum()) - 0.25 * nneg) < 0.05 * nneg


@pytest.mark.gpu
@pytest.mark.parametrize("shuf", [0, 1200])
def test_device_crb_blocks_match_host_records(tmp_path, shuf):
    """CRB input on a GPU worker: records decoded by the host reader threads,
    minibatches (and, with a shuffle buffer, the permutation) on the device.
    Unshuffled: the same minibatches as the host iterator; shuffled: every
    row of the part exactly once, in another order."""
    from wormhole_amd.data.device_text import DeviceTextIter, applies
    host = _native.host()
    dev = torch.device("cuda")
    data = _criteo_text(3000, 9)
    keys_h, off_h, _, lab_h, _ = host.parse_text(data, "criteo")
    p = tmp_path / "d.crb"
    w = host.RecordIOWriter(str(p))
    for a in range(0, 3000, 700):  # several records, not aligned to the minibatch
        b = min(a + 700, 3000)
        o = off_h[a:b + 1] - off_h[a]
        w.write(host.crb_encode(keys_h[off_h[a]:off_h[b]], o, None, lab_h[a:b], None))
    w.close()
    assert applies("crb", str(p), dev)
    rows_h = [tuple(keys_h[off_h[i]:off_h[i + 1]].tolist()) + (float(lab_h[i]),)
              for i in range(3000)]
    it = DeviceTextIter(host, str(p), 0, 1, "crb", 500, shuf, 1.0, 3, dev)
    rows, sizes = [], []
    while True:
        bt = it.next()
        if bt is None:
            break
        keys, off, val, lab = [x.cpu() if x is not None else None for x in bt.to_main(dev)]
        sizes.append(lab.numel())
        rows += [tuple(keys[off[i]:off[i + 1]].tolist()) + (float(lab[i]),)
                 for i in range(lab.numel())]
    assert sizes[:-1] == [500] * (len(sizes) - 1)
    if shuf:
        assert sorted(rows) == sorted(rows_h) and rows != rows_h
    else:
        assert rows == rows_h


def test_crb_truncated_record_is_an_error(tmp_path):
    """A CRB part cut inside its last record (a partial copy, a writer that
    died) is an error when read, not a silently shorter pass. (Parts are read
    through a shared mapping: files must not change while being read.)"""
    host = _native.host()
    data = _criteo_text(1200, 4)
    keys_h, off_h, _, lab_h, _ = host.parse_text(data, "criteo")
    p = tmp_path / "t.crb"
    w = host.RecordIOWriter(str(p))
    for a in range(0, 1200, 400):
        b = a + 400
        w.write(host.crb_encode(keys_h[off_h[a]:off_h[b]], off_h[a:b + 1] - off_h[a], None,
                                lab_h[a:b], None))
    w.close()
    full = p.read_bytes()
    it = host.MinibatchIter(str(p), 0, 1, "crb", 300, 0, 1.0, 1, False)
    n = 0
    while True:
        b = it.next()
        if b is None:
            break
        n += int(b[3].numel())
    assert n == 1200
    p.write_bytes(full[:len(full) - 100])  # inside the third record
    it = host.MinibatchIter(str(p), 0, 1, "crb", 300, 0, 1.0, 1, False)
    with pytest.raises(Exception, match="truncated"):
        while it.next() is not None:
            pass
