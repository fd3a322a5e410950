"""PS model shard files (reference layouts): save/load round trip
of the DiFacto and linear stores, and reading a reference-style interleaved
DiFacto shard."""
import struct

import numpy as np
import torch

from wormhole_amd.kv import checkpoint
from wormhole_amd.kv.cpu_store import CpuKVStore
from wormhole_amd.ops import ref


def _trained_store(dim=4):
    st = CpuKVStore(1 << 10, 1 << 8, dim)
    g = torch.Generator().manual_seed(0)
    keys = torch.unique(torch.randint(0, 1 << 40, (300,), generator=g))
    hp = [0.05, 1.0, 0.01, 0.1, 0.02, 1.0, 0.5, 0.01]
    for _ in range(4):
        s = st.find(keys, True)
        st.difacto_push_cnt(s, torch.randint(1, 4, (keys.numel(),), generator=g).float(), hp, 3,
                            False, 7)
        hdr, vc, _ = st.difacto_pull(s, False)
        gvc = torch.randn(vc.shape[0], vc.shape[1], generator=g)
        st.difacto_push(s, hdr, torch.randn(keys.numel(), generator=g), gvc, hp, 3, False, 7)
    return st, keys


def test_difacto_roundtrip(tmp_path):
    st, keys = _trained_store()
    n = checkpoint.save_difacto(st, str(tmp_path / "m"))
    assert n > 0
    st2 = CpuKVStore(1 << 10, 1 << 8, 4)
    assert checkpoint.load_difacto(st2, str(tmp_path / "m")) == n
    a = st.difacto_pull(st.find(keys, False), False)
    b = st2.difacto_pull(st2.find(keys, False), False)
    w_live = a[0][:, 0] != 0
    assert torch.equal(a[0][w_live, 0], b[0][w_live, 0])
    va, vb = ref.hdr_vidx(a[0]), ref.hdr_vidx(b[0])
    assert torch.equal(va >= 0, vb >= 0)
    assert torch.allclose(a[1][va[va >= 0].long()], b[1][vb[vb >= 0].long()])


def test_reference_interleaved_shard(tmp_path):
    dim = 3
    out = bytearray()
    out += struct.pack("<Qi", 5, 1) + struct.pack("<fIff", 0.5, 0, 1.0, 2.0)
    out += struct.pack("<Qi", 7, dim + 1) + np.array([1, 2, 3, 4], "<f4").tobytes()
    out += np.array([9, 8, 7, 6, 5], "<f4").tobytes()
    out += struct.pack("<Qi", 9, 1) + struct.pack("<fIff", -0.5, 0, 3.0, 4.0)
    (tmp_path / "ref").write_bytes(bytes(out))
    st = CpuKVStore(1 << 8, 1 << 6, dim)
    assert checkpoint.load_difacto(st, str(tmp_path / "ref")) == 3
    hdr, vc, _ = st.difacto_pull(st.find(torch.tensor([5, 7, 9]), False), False)
    assert hdr[:, 0].tolist() == [0.5, 1.0, -0.5]
    v = ref.hdr_vidx(hdr)
    assert v[0] == -1 and v[2] == -1 and vc[v[1]][:dim].tolist() == [2.0, 3.0, 4.0]


def test_linear_roundtrip(tmp_path):
    st = CpuKVStore(1 << 10, 0, 0)
    keys = torch.arange(1, 200) * 7919
    s = st.find(keys, True)
    st.linear_push(s, torch.randn(keys.numel()), 3, 0.1, 1.0, 0.1, 0.0, 1.0)
    checkpoint.save_linear(st, str(tmp_path / "l"))
    st2 = CpuKVStore(1 << 10, 0, 0)
    checkpoint.load_linear(st2, str(tmp_path / "l"))
    assert torch.equal(st.linear_pull(st.find(keys, False)), st2.linear_pull(st2.find(keys, False)))


def test_async_saver_host_store(tmp_path):
    st, _ = _trained_store()
    checkpoint.save_difacto(st, str(tmp_path / "a"))
    sv = checkpoint.AsyncSaver()
    sv.save("difacto", st, str(tmp_path / "b"))
    sv.join()
    assert (tmp_path / "a").read_bytes() == (tmp_path / "b").read_bytes()
    lin = CpuKVStore(1 << 10, 0, 0)
    lin.find(torch.arange(5), True)
    checkpoint.save_linear(lin, str(tmp_path / "l1"))
    sv.save("linear", lin, str(tmp_path / "l2"))
    assert (tmp_path / "l1").read_bytes() == (tmp_path / "l2").read_bytes()
