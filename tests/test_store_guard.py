"""Overflow-safe parameter store (kv.StoreGuard, KVStore.grow / grow_v):
the table grows on the device before it passes the load bound, in-flight
slot ids are remapped, and any lost key or embedding row is a hard error."""
import pytest
import torch

from wormhole_amd.kv import CpuKVStore, StoreError, StoreGuard


def test_guard_raises_on_lost_keys_cpu():
    st = CpuKVStore(cap=1 << 10, vcap=16, dim=4)
    g = StoreGuard(st)
    g.before_open(10)
    st.find(torch.arange(10), True)
    g.after_open()
    g.read()  # fine
    st.add_stat(2, 3)  # three failed inserts
    g.after_open()
    with pytest.raises(StoreError, match="3 failed inserts"):
        g.before_open(1)


def test_guard_grows_cpu_store():
    st = CpuKVStore(cap=1 << 6, vcap=4, dim=4)
    g = StoreGuard(st)
    for b in range(5):
        keys = torch.arange(b * 50, b * 50 + 50)
        g.before_open(keys.numel())
        assert st.find(keys, True).min() >= 0
        g.after_open()
    g.read()
    assert g.grows >= 1 and st.cap >= (250 / 0.7)
    assert g.vgrows >= 1 and st.vcap >= 2 * 50


@pytest.mark.gpu
def test_device_store_overflow_is_reported():
    from wormhole_amd.kv import make_store
    st = make_store(1 << 10, 16, 4, "cuda")
    g = StoreGuard(st)
    keys = torch.randint(0, 1 << 60, (4000,), device="cuda")
    slot = st.find(keys, True)  # bypasses the guard's growth: overfills 1024 slots
    g.after_open()
    with pytest.raises(StoreError, match="failed inserts"):
        g.read()
    assert int((slot >= 0).sum()) == 1024


@pytest.mark.gpu
def test_device_store_grows_and_remaps():
    from wormhole_amd import _native
    from wormhole_amd.kv import make_store
    st = make_store(1 << 10, 64, 8, "cuda")
    g = StoreGuard(st)
    gen = torch.Generator().manual_seed(0)
    allk, held = [], None
    for b in range(12):
        keys = torch.randint(0, 1 << 62, (3000,), generator=gen).cuda()
        remapped = []
        g.before_open(keys.numel(), lambda r: remapped.append(r))
        if held is not None and remapped:
            held = (held[0], remapped[-1][held[1].long()])  # in-flight slot ids follow the rehash
        slot = st.find(keys, True)
        g.after_open()
        assert int((slot < 0).sum()) == 0
        st.w[slot.long()] = keys.float()  # a value to follow through the rehash
        allk.append(keys)
        held = (keys, slot)
    g.read()
    assert g.grows >= 3 and st.cap >= 36000 / 0.7
    k = torch.cat(allk)
    slot = st.find(k, False)
    assert int((slot < 0).sum()) == 0
    assert torch.equal(st.w[slot.long()], k.float())
    # the slot ids held across growths still address their keys
    assert torch.equal(st.keys[held[1].long()], held[0])
    s = st.summary().tolist()
    assert s[0] == k.unique().numel() and s[1] == 0


@pytest.mark.parametrize("nshard", [1, 2])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_shrinking_minibatch_keeps_room_for_the_inflight_push(device, nshard):
    """with l1_shrk a key's embedding row is allocated by the PUSH
    that first makes w non-zero. A large minibatch followed by a small one:
    the guard must reserve V rows for the large minibatch's push still in
    flight, not only for the small coming open."""
    from wormhole_amd.config.schema import DifactoConfig, Embedding
    from wormhole_amd.models.difacto import DifactoLearner
    from wormhole_amd.parallel.comm import Comm, LoopbackComm
    dev = torch.device(device)
    emb = Embedding(dim=4, threshold=0)
    conf = DifactoConfig(embedding=[emb], lambda_l1=1e-6, l1_shrk=True, lr_eta=0.5)
    comm = Comm(dev, init=False) if nshard == 1 else LoopbackComm(nshard, dev)
    lr = DifactoLearner(conf, comm, dev, cap=1 << 12, vcap=64, seed=1)
    g = torch.Generator().manual_seed(0)

    def batch(rows, nkeys, base):
        keys = torch.randint(0, nkeys, (rows * 4,), generator=g) + base
        off = torch.arange(0, rows * 4 + 1, 4)
        label = (torch.rand(rows, generator=g) > 0.5).float()
        return keys.to(dev), off.to(dev), label.to(dev)
    for k, (rows, nkeys) in enumerate([(20, 60), (30, 90), (600, 2000), (5, 10), (5, 10),
                                       (5, 10)]):
        keys, off, label = batch(rows, nkeys, 100000 * k)
        lr.process(keys, off, None, label, 0, 0)
    lr.flush()
    lr.kv.guard.after_open()
    lr.kv.guard.read()  # raises StoreError on any dropped embedding row
    assert lr.kv.guard.vgrows >= 1 and lr.store.vcap > 64
