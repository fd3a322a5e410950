"""ps-lite ``-max_key`` system flag: feature ids are folded into [0, max_key)
before localization (reference learn/base/localizer.h:108-115)."""
import numpy as np
import pytest
import torch

from wormhole_amd import ops
from wormhole_amd.apps.ps_app import split_system_flags


def test_split_system_flags():
    f, rest = split_system_flags(["demo.conf", "-max_key=1000", "lr_eta=0.1"])
    assert f == {"max_key": 1000} and rest == ["demo.conf", "lr_eta=0.1"]
    f, rest = split_system_flags(["--max_key", "77", "demo.conf"])
    assert f == {"max_key": 77} and rest == ["demo.conf"]
    with pytest.raises(SystemExit):
        split_system_flags(["demo.conf", "-bogus=1"])


def test_key_mod_uint64_semantics():
    keys = torch.tensor([5, 1 << 62, -1, -(1 << 40)], dtype=torch.int64)
    got = ops.key_mod(keys, 1000).tolist()
    exp = [int(np.uint64(np.int64(k).view(np.uint64)) % np.uint64(1000)) for k in keys.tolist()]
    assert got == exp


def test_linear_learner_folds_keys():
    from wormhole_amd.config.schema import LinearConfig
    from wormhole_amd.models.linear import LinearLearner
    from wormhole_amd.parallel.comm import Comm
    lr = LinearLearner(LinearConfig(minibatch=64), Comm(torch.device("cpu"), init=False), "cpu",
                       cap=1 << 12)
    lr.max_key = 50
    g = torch.Generator().manual_seed(0)
    keys = torch.randint(0, 1 << 50, (640,), generator=g)
    off = torch.arange(0, 641, 10, dtype=torch.int64)
    label = (torch.rand(64, generator=g) < 0.5).float()
    lr.process(keys, off, None, label, 0, 0)
    lr.flush()
    occ = lr.store.occupied().long()
    stored = lr.store.keys[occ]
    assert stored.numel() <= 50 and bool((stored >= 0).all()) and bool((stored < 50).all())


@pytest.mark.gpu
def test_key_mod_gpu():
    keys = torch.tensor([5, 1 << 62, -1, -(1 << 40), 123456789], dtype=torch.int64)
    assert ops.key_mod(keys.cuda(), 997).cpu().tolist() == ops.key_mod(keys, 997).tolist()
