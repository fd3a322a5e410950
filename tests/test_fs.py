"""URI resolution (dmlc Stream/FileSystem surface, doc/common/input.rst):
local / file:// paths, and remote schemes served through the mount named by
WH_FS_MOUNT_<SCHEME> -- identical in the native runtime and in Python."""
import os

import pytest

from wormhole_amd import _native
from wormhole_amd.utils import fs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "learn", "data", "agaricus.txt.train")


def test_resolve_rules(monkeypatch):
    host = _native.host()
    monkeypatch.setenv("WH_FS_MOUNT_HDFS", "/mnt/hdfs")
    monkeypatch.setenv("WH_FS_MOUNT_S3", "/mnt/s3")
    cases = {
        "a/b.txt": "a/b.txt",
        "file:///tmp/x": "/tmp/x",
        "hdfs://nn:9000/user/a/part-0": "/mnt/hdfs/user/a/part-0",
        "s3://bucket/key/x": "/mnt/s3/bucket/key/x",
    }
    for uri, local in cases.items():
        assert fs.resolve(uri) == local, uri
        assert host.resolve_path(uri) == local, uri
    monkeypatch.delenv("WH_FS_MOUNT_S3")
    with pytest.raises(OSError, match="WH_FS_MOUNT_S3"):
        fs.resolve("s3://bucket/key")
    with pytest.raises(RuntimeError, match="WH_FS_MOUNT_S3"):
        host.resolve_path("s3://bucket/key")


def test_remote_scheme_reads_through_mount(monkeypatch, tmp_path):
    host = _native.host()
    monkeypatch.setenv("WH_FS_MOUNT_HDFS", os.path.dirname(os.path.dirname(DATA)))
    uri = "hdfs://namenode:8020/data/agaricus.txt.train"
    assert host.file_size(uri) == os.path.getsize(DATA)
    got = host.match_file("hdfs://namenode:8020/data/agaricus.txt.t")
    assert any(g.endswith("agaricus.txt.train") for g in got)
    text = b"".join(host.read_text_split(uri, 0, 1)) if isinstance(
        host.read_text_split(uri, 0, 1), list) else host.read_text_split(uri, 0, 1)
    assert len(text) > 0
    monkeypatch.setenv("WH_FS_MOUNT_S3", str(tmp_path))
    with fs.open_uri("s3://bucket/out/model_part-0", "w") as f:
        f.write("ok")
    assert (tmp_path / "bucket" / "out" / "model_part-0").read_text() == "ok"
