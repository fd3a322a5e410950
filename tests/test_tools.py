"""Native data conversion tools (reference learn/tool/convert.cc, text2crb.cc)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")
TRAIN = os.path.join(ROOT, "learn", "data", "agaricus.txt.train")


def _rows(path):
    out = []
    for line in open(path):
        t = line.split()
        out.append((float(t[0]), [int(x.split(":")[0]) for x in t[1:]]))
    return out


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(os.path.join(BIN, "native", "convert")):
        import build_native
        build_native.build()


def test_convert_libsvm_crb_roundtrip(tmp_path):
    crb, txt = str(tmp_path / "a.crb"), str(tmp_path / "a.txt")
    subprocess.run([os.path.join(BIN, "convert.dmlc"), "-data_in", TRAIN, "-data_out", crb,
                    "-format_in", "libsvm", "-format_out", "crb"], check=True)
    subprocess.run([os.path.join(BIN, "convert.dmlc"), "--data_in=" + crb, "--data_out=" + txt,
                    "--format_in=crb", "--format_out=libsvm"], check=True)
    assert _rows(txt) == _rows(TRAIN)
    # the CRB file reads back through the native minibatch iterator too
    from wormhole_amd import _native
    it = _native.host().MinibatchIter(crb, 0, 1, "crb", 100000, 0, 1.0, 0)
    n = 0
    while True:
        b = it.next()
        if b is None:
            break
        n += b[3].numel()  # (keys, offset, val, label, weight)
    assert n == 6513


def test_convert_parts_and_stdio(tmp_path):
    base = str(tmp_path / "p")
    # tiny part size: one part per 4 MB parse chunk -> a single part here
    subprocess.run([os.path.join(BIN, "text2crb.dmlc"), TRAIN, base, "libsvm", "0"], check=True)
    assert os.path.exists(base + "-part_00")
    r = subprocess.run([os.path.join(BIN, "convert.dmlc"), "-format_out", "libsvm"],
                       input=open(TRAIN, "rb").read(), capture_output=True, check=True)
    lines = r.stdout.decode().splitlines()
    assert len(lines) == 6513 and lines[0].split()[0] == "1"


def test_convert_criteo_hashes_fields(tmp_path):
    src = tmp_path / "c.tsv"
    ints = "\t".join(str(i) for i in range(13))
    cats = "\t".join("%08x" % (i * 7919) for i in range(26))
    src.write_text("1\t%s\t%s\n0\t%s\t%s\n" % (ints, cats, ints, cats))
    out = str(tmp_path / "c.txt")
    subprocess.run([os.path.join(BIN, "convert.dmlc"), "-data_in", str(src), "-data_out", out,
                    "-format_in", "criteo", "-format_out", "libsvm"], check=True)
    rows = _rows(out)
    assert [r[0] for r in rows] == [1.0, 0.0]
    fields = sorted(k >> 54 for k in rows[0][1])
    assert fields == sorted(set(fields)) and len(fields) >= 26
