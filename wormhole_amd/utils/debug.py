"""Debug strings for arrays and minibatches (reference learn/base/debug.h:9-43,
``DebugStr``): ``[n]: a0 a1 a2 a3 a4 ... a(n-5) .. a(n-1)`` -- the first and
last ``m`` entries of long arrays.  Implemented natively (csrc/host/common.h)."""
from .. import _native


def debug_str(t, m=5):
    """Debug string of a 1-D tensor (any device; copied to host)."""
    import torch
    if not torch.is_tensor(t):
        t = torch.as_tensor(t)
    return _native.host().debug_str(t, m)


def debug_str_block(keys, offset, val, label):
    """Debug string of a CSR minibatch (label / offset / index [/ value])."""
    return _native.host().debug_str_block(keys, offset, val, label)
