"""Native host runtime: config parser, codecs, I/O splits, parsers,
workload pool, control-plane transport, CPU localizer (CPU only)."""
import os
import struct
import threading
import time

import numpy as np
import pytest
import torch

from wormhole_amd import _native, config
from wormhole_amd.config.schema import DifactoConfig, LinearConfig
from wormhole_amd.ops import ref

REF = "/root/reference/learn"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "learn", "data")


@pytest.fixture(scope="module")
def host():
    return _native.host()


# ------------------------------------------------------------------ config
def test_conf_reference_files_parse():
    lc = config.load(LinearConfig, os.path.join(ROOT, "learn/linear/guide/demo.conf"))
    assert lc.train_data == "learn/data/agaricus.txt.train"
    assert lc.max_data_pass == 3 and lc.algo == 3 and lc.loss == 2 and lc.lambda_l1 == 1.0
    dc = config.load(DifactoConfig, os.path.join(ROOT, "learn/difacto/guide/demo.conf"))
    assert dc.embedding[0].dim == 5 and dc.embedding[0].threshold == 5
    assert dc.model_out == "./agaricus_model"


def test_conf_argv_overrides_and_enums():
    c = config.load(LinearConfig, os.path.join(ROOT, "learn/linear/guide/demo.conf"),
                    ["max_data_pass=7", "algo=SGD", "loss = SQUARE_HINGE", 'model_out="x y"'])
    assert c.max_data_pass == 7 and c.algo == 1 and c.loss == 4 and c.model_out == "x y"
    assert c.has("max_data_pass") and not c.has("lr_beta")
    c = config.load(LinearConfig, "none", ["lambda_l1:4", "lr_eta = .1"])
    assert c.lambda_l1 == 4.0 and abs(c.lr_eta - 0.1) < 1e-9


def test_conf_unknown_key_is_fatal():
    # the reference criteo.conf carries a stale `max_delay` key
    with pytest.raises(ValueError, match="max_delay"):
        config.load(DifactoConfig, os.path.join(ROOT, "learn/difacto/guide/criteo.conf"),
                    ["max_delay = 1"])
    c = config.load(DifactoConfig, os.path.join(ROOT, "learn/difacto/guide/criteo.conf"))
    assert c.embedding[0].dim == 50 and c.minibatch == 100000 and c.data_format == "crb"
    with pytest.raises(ValueError):
        config.load(LinearConfig, "none", ["no_such_key=1"])


def test_conf_nested_and_comments(host):
    items = host.parse_conf('# c\nembedding {\n dim: 50 # x\n threshold = 100 }\nlr_eta = .01\n'
                            'train_data = "s3://a/b_.*" ')
    assert items[0][0] == "embedding" and items[0][1] == "m"
    assert ("dim", "t", "50") in items[0][2]
    assert items[2] == ("train_data", "s", "s3://a/b_.*")
    with pytest.raises(Exception):
        host.parse_conf("embedding { dim = 5 ")


# ----------------------------------------------------------------- codecs
def test_cityhash64_known_values(host):
    assert host.cityhash64(b"") == 0x9AE16A3B2F90404F  # k2, the empty-string hash
    # every length class exercises a different code path; hashes must be stable
    vals = [host.cityhash64(bytes(range(n))) for n in (3, 7, 15, 30, 60, 100, 200)]
    assert len(set(vals)) == len(vals)
    assert host.cityhash64(b"68fd1e64") == host.cityhash64(b"68fd1e64")


@pytest.mark.parametrize("kind", ["rand", "ties", "const", "wide", "tiny", "nonfinite", "negzero"])
def test_host_auc_matches_oracle(host, kind):
    """The host AUC (csrc/host/auc_host.h: bucketed fast path, radix path for
    non-finite scores) equals the plain-PyTorch oracle bit for bit: ties
    broken by index, -0 == +0, one class -> 1."""
    g = torch.Generator().manual_seed(len(kind))
    for n in (1, 2, 7, 999, 20000, 100000):
        py = {"rand": lambda: torch.sigmoid(torch.randn(n, generator=g) * 3),
              "ties": lambda: torch.randint(0, 5, (n,), generator=g).float() / 4,
              "const": lambda: torch.full((n,), 0.5),
              "wide": lambda: torch.randn(n, generator=g) * 1e4,
              "tiny": lambda: torch.rand(n, generator=g) * 1e-30,
              "nonfinite": lambda: torch.where(torch.rand(n, generator=g) < 0.02,
                                               torch.tensor(float("nan")), torch.randn(n, generator=g)),
              "negzero": lambda: torch.where(torch.rand(n, generator=g) < 0.5, torch.tensor(-0.0),
                                             torch.rand(n, generator=g))}[kind]()
        for p in (0.0, 0.3, 1.0):
            lab = (torch.rand(n, generator=g) < p).float()
            assert host.auc_exact(py, lab) == float(ref.auc(py, lab)), (n, p)


@pytest.mark.parametrize("n", [0, 1, 13, 100, 65536 + 7, 300000])
def test_lz4_roundtrip(host, n):
    rng = np.random.default_rng(n)
    a = rng.integers(0, 4, n, dtype=np.uint8).tobytes()  # compressible
    b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # incompressible
    for d in (a, b, (b"abcdefgh" * (n // 8 + 1))[:n]):
        c = host.lz4_compress(d)
        assert host.lz4_decompress(c, len(d)) == d
    if n > 1000:
        assert len(host.lz4_compress(a)) < len(a)


@pytest.mark.parametrize("period", [1, 2, 3, 5, 7])
def test_lz4_short_offset_runs(host, period):
    """Matches whose offset is shorter than 8 bytes (the decoder's period-
    stepping copy): long periodic runs between literals, lengths that end
    on and off the 8-byte step."""
    rng = np.random.default_rng(period)
    parts = []
    for run in (9, 16, 17, 63, 64, 1000, 4099):
        pat = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
        parts.append(rng.integers(0, 256, 11, dtype=np.uint8).tobytes())
        parts.append((pat * (run // period + 1))[:run])
    d = b"".join(parts) + b"tail-literals!"
    c = host.lz4_compress(d)
    assert len(c) < len(d)
    assert host.lz4_decompress(c, len(d)) == d


def test_lz4_decodes_reference_format(host):
    # hand-built LZ4 block: literal "abcd", match (offset 4, len 8), literals "xyz12"
    blk = bytes([0x44]) + b"abcd" + bytes([4, 0]) + bytes([0x50]) + b"xyz12"
    assert host.lz4_decompress(blk, 17) == b"abcdabcdabcdxyz12"


def test_recordio_roundtrip_with_embedded_magic(host, tmp_path):
    magic = struct.pack("<I", 0xCED7230A)
    recs = [b"hello", b"", b"ab" + magic + b"cd" + magic, magic * 3, os.urandom(1001)]
    p = str(tmp_path / "r.rec")
    w = host.RecordIOWriter(p)
    for r in recs * 50:
        w.write(r)
    w.close()
    got = []
    for k in range(4):
        got += host.read_recordio(p, k, 4)
    assert got == recs * 50


def test_crb_roundtrip(host):
    keys = torch.tensor([1, 2, 3, 2 ** 62, 5], dtype=torch.int64)
    off = torch.tensor([0, 2, 2, 5], dtype=torch.int64)
    lab = torch.tensor([1.0, 0.0, 1.0])
    b = host.crb_encode(keys, off, None, lab)
    k2, o2, v2, l2, w2 = host.crb_decode(b)
    assert torch.equal(k2, keys) and torch.equal(o2, off) and torch.equal(l2, lab)
    assert v2 is None and w2 is None
    val = torch.tensor([1.0, 0.5, 2.0, 1.0, 3.0])
    b = host.crb_encode(keys, off, val, lab)
    assert torch.equal(host.crb_decode(b)[2], val)
    assert struct.unpack_from("<i", b, 0)[0] == 1196140743


# ------------------------------------------------------------------ splits
def test_text_split_partitions_lines(host):
    path = os.path.join(DATA, "agaricus.txt.train")
    whole = open(path, "rb").read()
    for n in (1, 2, 3, 7, 16):
        parts = [host.read_text_split(path, k, n) for k in range(n)]
        assert b"".join(parts) == whole, n


def test_match_file(host):
    got = host.match_file(os.path.join(DATA, "agaricus.txt.t.*"))
    assert sorted(os.path.basename(g) for g in got) == ["agaricus.txt.test", "agaricus.txt.train"]
    assert host.match_file(os.path.join(DATA, "nothing_here_.*")) == []


# ----------------------------------------------------------------- parsers
def test_libsvm_parser(host):
    keys, off, val, lab, w = host.parse_text(b"1 3:1 10:2.5\n0 7:1\n\n1 1:1 2:1 3:1\n", "libsvm")
    assert lab.tolist() == [1, 0, 1]
    assert off.tolist() == [0, 2, 3, 6]
    assert keys.tolist() == [3, 10, 7, 1, 2, 3]
    assert val.tolist() == [1, 2.5, 1, 1, 1, 1]
    k2, o2, v2, l2, _ = host.parse_text(b"1 3 4\n0 5:1\n", "libsvm")
    assert v2 is None and k2.tolist() == [3, 4, 5]


def test_criteo_parser(host):
    ints = "\t".join(["1", "", "5"] + [""] * 10)
    cats = "\t".join(["68fd1e64", "", "80e26c9b"] + [""] * 23)
    line = ("1\t" + ints + "\t" + cats + "\n").encode()
    keys, off, val, lab, _ = host.parse_text(line * 2, "criteo")
    assert lab.tolist() == [1.0, 1.0] and off.tolist() == [0, 4, 8]
    k = keys.numpy().view(np.uint64)
    fields = (k >> np.uint64(54)).tolist()
    assert fields[:4] == [0, 2, 13, 15]
    h = host.cityhash64(b"68fd1e64")
    assert int(k[2]) == ((h >> 10) | (13 << 54))
    keys_t, off_t, _, lab_t, _ = host.parse_text((ints + "\t" + cats + "\n").encode(), "criteo_test")
    assert lab_t.tolist() == [0.0] and torch.equal(keys_t, keys[:4])


def test_adfea_parser(host):
    txt = b"100 1 1 5:2 9:3\n101 1 0 7:1\n"
    keys, off, val, lab, _ = host.parse_text(txt, "adfea")
    assert lab.tolist() == [1.0, 0.0] and off.tolist() == [0, 2, 3]
    k = keys.numpy().view(np.uint64)
    assert int(k[0]) == ((5 >> 10) | (2 << 54))


def test_minibatch_iter_covers_file(host):
    path = os.path.join(DATA, "agaricus.txt.train")
    total = 0
    for k in range(3):
        it = host.MinibatchIter(path, k, 3, "libsvm", 500)
        while (b := it.next()) is not None:
            assert b[3].numel() <= 500
            total += b[3].numel()
    assert total == 6513
    # shuffle buffer + negative down-sampling keeps every positive
    it = host.MinibatchIter(path, 0, 1, "libsvm", 100, 1000, 0.5, 3)
    pos = neg = 0
    while (b := it.next()) is not None:
        pos += int((b[3] > 0).sum())
        neg += int((b[3] <= 0).sum())
    lab = host.load_split(path, 0, 1, "libsvm")[3]
    assert pos == int((lab > 0).sum())
    assert 0.3 * int((lab <= 0).sum()) < neg < 0.7 * int((lab <= 0).sum())


def test_crb_file_split_via_minibatch_iter(host, tmp_path):
    path = os.path.join(DATA, "agaricus.txt.train")
    keys, off, val, lab, _ = host.load_split(path, 0, 1, "libsvm")
    p = str(tmp_path / "a.crb")
    w = host.RecordIOWriter(p)
    for r0 in range(0, 6513, 1000):
        r1 = min(r0 + 1000, 6513)
        o = off[r0:r1 + 1] - off[r0]
        w.write(host.crb_encode(keys[off[r0]:off[r1]], o, None, lab[r0:r1]))
    w.close()
    rows = 0
    for k in range(2):
        it = host.MinibatchIter(p, k, 2, "crb", 777)
        while (b := it.next()) is not None:
            rows += b[3].numel()
    assert rows == 6513


@pytest.mark.parametrize("with_val", [False, True])
@pytest.mark.parametrize("rows", [777, 2000, 100000])
def test_block_iter_matches_minibatch_iter(host, tmp_path, with_val, rows):
    """BlockIter (CRB records decoded in parallel straight into the block
    tensors; parsed text chunks copied into them) yields the same blocks as
    MinibatchIter without a shuffle buffer: same rows in file order (records
    straddling blocks split), same CSR, weights, values dropped when all are
    1."""
    path = os.path.join(DATA, "agaricus.txt.train")
    keys, off, val, lab, _ = host.load_split(path, 0, 1, "libsvm")
    g = torch.Generator().manual_seed(3)
    v = (torch.rand(keys.numel(), generator=g) + 0.5) if with_val else None
    p = str(tmp_path / "a.crb")
    w = host.RecordIOWriter(p)
    for r0 in range(0, 6513, 1000):
        r1 = min(r0 + 1000, 6513)
        o = off[r0:r1 + 1] - off[r0]
        w.write(host.crb_encode(keys[off[r0]:off[r1]], o,
                                v[off[r0]:off[r1]] if with_val else None, lab[r0:r1],
                                (lab[r0:r1] + 2.0) if with_val else None))
    w.close()
    for k in range(2):
        a = host.MinibatchIter(p, k, 2, "crb", rows)
        b = host.BlockIter(p, k, 2, "crb", rows, pinned=False)
        n = 0
        while True:
            x, y = a.next(), b.next()
            assert (x is None) == (y is None)
            if x is None:
                break
            n += 1
            for i in range(5):
                assert (x[i] is None) == (y[i] is None), i
                if x[i] is not None:
                    assert torch.equal(x[i], y[i]), i
        assert n >= 1
    # text chunks too (the host parser's blocks)
    a = host.MinibatchIter(path, 0, 1, "libsvm", rows)
    b = host.BlockIter(path, 0, 1, "libsvm", rows, pinned=False)
    while (x := a.next()) is not None:
        y = b.next()
        assert torch.equal(x[0], y[0]) and torch.equal(x[1], y[1]) and torch.equal(x[3], y[3])
    assert b.next() is None


# -------------------------------------------------------------- localize
@pytest.mark.parametrize("nshard", [1, 4])
def test_localize_cpu_matches_reference(host, nshard):
    g = torch.Generator().manual_seed(nshard)
    keys = torch.randint(0, 500, (4000,), generator=g) * 7919 + 3
    off = torch.arange(0, 4001, 40)
    val = torch.rand(4000, generator=g)
    got = host.localize_cpu(keys, off, val, nshard)
    exp = ref.localize(keys, off, val, nshard)
    for a, b in zip(got, exp):
        assert torch.equal(a.to(b.dtype), b)


# ------------------------------------------------------------ workload pool
def test_workload_pool_dispatch_and_reset(host):
    pool = host.WorkloadPool(False, 0, 2.0, 5.0, 10, 0.0)
    pool.add(["a", "b"], 3)
    got = []
    while (a := pool.get("w0")) is not None:
        got.append(a)
        pool.finish("w0")
    assert sorted(got) == [(f, k, 3) for f in "ab" for k in range(3)]
    assert pool.is_finished() and pool.num_finished == 6
    pool = host.WorkloadPool(True, 7, 2.0, 5.0, 10, 0.0)
    pool.add(["a"], 4)
    a0 = pool.get("w0")
    a1 = pool.get("w1")
    pool.reset("w0")  # w0 died: its part goes back to the pool
    seen = {a1}
    pool.finish("w1")
    while (a := pool.get("w1")) is not None:
        seen.add(a)
        pool.finish("w1")
    assert a0 in seen and len(seen) == 4 and pool.is_finished()


def test_workload_pool_straggler_requeue(host):
    pool = host.WorkloadPool(False, 0, 2.0, 0.05, 2, 0.0)
    pool.add(["f"], 5)
    for _ in range(2):
        pool.get("fast")
        pool.finish("fast")
    slow = pool.get("slow")
    time.sleep(0.3)
    pool.remove_straggler()
    assert pool.num_requeued == 1
    again = pool.get("fast")
    assert again == slow  # the straggler's part is handed out again


def test_workload_pool_node_affinity(host):
    pool = host.WorkloadPool(False, 0, 2.0, 5.0, 10, 0.0)
    pool.add(["local_a"], 2, "w0")
    assert pool.get("w1") is None
    assert pool.get("w0")[0] == "local_a"


# ---------------------------------------------------------------------- van
def test_van_messaging_and_failure_notice(host):
    srv = host.Van()
    port = srv.listen(0)
    clients = []
    for i in range(3):
        c = host.Van()
        c.connect("127.0.0.1", port, "worker-%d" % i)
        clients.append(c)
    for i, c in enumerate(clients):
        c.send("scheduler", b"hi %d" % i)
    got = sorted(srv.recv(5.0) for _ in range(3))
    assert [g[1] for g in got] == [b"hi 0", b"hi 1", b"hi 2"]
    assert srv.send("worker-1", b"x" * 100000)
    assert clients[1].recv(5.0) == ("scheduler", b"x" * 100000)
    clients[2].close()  # a dead peer is reported to the scheduler
    t0 = time.time()
    msg = None
    while time.time() - t0 < 5:
        m = srv.recv(0.5)
        if m and m[1] == b"__closed__":
            msg = m
            break
    assert msg == ("worker-2", b"__closed__")
    for c in clients[:2]:
        c.close()
    srv.close()


def test_parallel_parser_is_ordered(tmp_path, monkeypatch):
    """Chunks parsed by many threads come out in file order: the minibatches
    do not depend on the parser thread count."""
    import random
    from wormhole_amd import _native
    host = _native.host()
    rnd = random.Random(3)
    path = tmp_path / "c.txt"
    with open(path, "w") as f:
        for i in range(40000):
            ints = [str(rnd.randint(0, 99)) if rnd.random() > 0.2 else "" for _ in range(13)]
            cats = ["%08x" % rnd.getrandbits(32) if rnd.random() > 0.1 else "" for _ in range(26)]
            f.write("\t".join([str(i % 2)] + ints + cats) + "\n")
    outs = []
    for nt in ("1", "7"):
        monkeypatch.setenv("WH_PARSE_THREADS", nt)
        it = host.MinibatchIter(str(path), 0, 1, "criteo", 1000, 0, 1.0, 0)
        got = []
        while True:
            r = it.next()
            if r is None:
                break
            got.append([t.clone() if t is not None else None for t in r[:4]])
        outs.append(got)
        full = host.load_split(str(path), 0, 1, "criteo")
        outs.append([[full[0], full[1], full[2], full[3]]])
    a, b = outs[0], outs[2]
    assert len(a) == len(b) == 40
    def same(u, v):
        return (u is None and v is None) or (u is not None and v is not None and torch.equal(u, v))
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            assert same(u, v)
    for u, v in zip(outs[1][0], outs[3][0]):
        assert same(u, v)


@pytest.mark.parametrize("period", [1, 2, 3, 5, 7, 8, 9, 12, 15, 16, 17, 24, 40])
def test_lz4_roundtrip_repeats(host, period):
    """Short-offset matches and the decoder's fast loop: periodic runs of
    every offset class, and CRB-like index sections (8-byte hashed keys
    drawn with repeats, one short sequence per key)."""
    rng = np.random.default_rng(period)
    unit = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
    runs = []
    for i in range(60):
        runs.append(unit * int(rng.integers(1, 40)))
        runs.append(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8).tobytes())
    for d in (b"".join(runs), (unit * 5000)[:31337]):
        c = host.lz4_compress(d)
        assert host.lz4_decompress(c, len(d)) == d
    keys = rng.integers(0, 2**63, 64 + period * 10, dtype=np.int64)
    pick = np.minimum(rng.pareto(1.1, 50000) * 3, keys.size - 1).astype(np.int64)
    d = keys[pick].tobytes()
    c = host.lz4_compress(d)
    assert len(c) < len(d)
    assert host.lz4_decompress(c, len(d)) == d
