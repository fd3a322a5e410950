"""ps-lite COMPRESSING filter (msg_compression) on host transfers: LZ4 per
peer chunk of an all-to-all-v (parallel/comm.py ``_a2a_lz4``, native
``lz4_pack`` / ``lz4_unpack``). Lossless: every exchange must return exactly
what the raw exchange returns, for compressible, incompressible and empty
chunks (reference filter: learn/linear/async_sgd.h:290-301)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def test_lz4_pack_roundtrip():
    from wormhole_amd import _native
    host = _native.host()
    g = torch.Generator().manual_seed(3)
    parts = [torch.zeros(4096, dtype=torch.uint8),                         # compressible
             torch.randint(0, 256, (5000,), dtype=torch.uint8, generator=g),  # incompressible
             torch.empty(0, dtype=torch.uint8),                             # empty
             torch.arange(3000, dtype=torch.int64).view(torch.uint8)]       # structured
    src = torch.cat(parts)
    sizes = [p.numel() for p in parts]
    packed, csz = host.lz4_pack(src, sizes)
    assert csz[0] > 0 and csz[0] < 4096          # shrunk
    assert csz[1] == -5000                       # stored raw
    assert csz[2] == 0
    assert packed.numel() == sum(abs(c) for c in csz) < src.numel()
    out = torch.empty_like(src)
    host.lz4_unpack(packed, csz, sizes, out)
    assert torch.equal(out, src)
    bad = packed.clone()
    bad[:8] = 255
    with pytest.raises(Exception):
        host.lz4_unpack(bad, csz, sizes, torch.empty_like(src))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    from wormhole_amd.parallel.comm import Comm
    comm = Comm("cpu")
    g = torch.Generator().manual_seed(11 + rank)
    send = [(rank + 1) * (p + 1) * 7 % 13 for p in range(world)]
    recv = comm.exchange_counts(send)
    xs = [torch.randn(sum(send), 16, generator=g),                         # floats
          torch.randint(0, 1 << 62, (sum(send),), generator=g),            # hashed ids
          torch.zeros(sum(send), 64),                                      # zero rows
          torch.arange(sum(send), dtype=torch.int32) // 3]                 # repeats
    comm.set_compression(False)
    raw = [comm.all_to_all_v(x, send, recv) for x in xs]
    raw_multi = comm.all_to_all_v_multi([(x, send, recv) for x in xs])
    comm.set_compression(True)
    assert comm.compress
    lz = [comm.all_to_all_v(x, send, recv) for x in xs]
    lz_multi, h = comm.all_to_all_v_multi([(x, send, recv) for x in xs], async_op=True)
    h.wait()
    out, w = comm.all_to_all_v_async(xs[0], send, recv)
    w.wait()
    for a, b, c, d in zip(raw, lz, raw_multi, lz_multi):
        assert a.dtype == b.dtype and torch.equal(a, b) and torch.equal(c, d) and torch.equal(a, c)
    assert torch.equal(out, raw[0])
    comm.barrier()
    open(os.path.join(out_dir, "r%d" % rank), "w").write("ok")
    comm.finalize()


def test_lz4_all_to_all_v_matches_raw(tmp_path):
    mp.spawn(_main, args=(3, _free_port(), str(tmp_path)), nprocs=3, join=True)
    for r in range(3):
        assert (tmp_path / ("r%d" % r)).read_text() == "ok"
