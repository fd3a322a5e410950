"""Hot ops.  GPU tensors run the hand-written gfx950 HIP kernels
(``wormhole_amd._hip``); CPU tensors run the PyTorch reference
(:mod:`wormhole_amd.ops.ref`).  There is no silent fallback: a GPU tensor
with the HIP extension missing raises.
"""
from .. import _native
from . import ref

LOSS_SQUARE, LOSS_LOGIT, LOSS_SQUARE_HINGE = ref.LOSS_SQUARE, ref.LOSS_LOGIT, ref.LOSS_SQUARE_HINGE


def _gpu(t):
    return t.is_cuda


def vstride_for(dim):
    return ref.vstride_for(dim)


def localize(keys, offset, val=None, nshard=1):
    """Unique feature ids of a minibatch (grouped by owner shard), per-id
    counts, the nnz->local-id map and the per-id occurrence lists (CSC)."""
    if _gpu(keys):
        return _native.hip().localize(keys, offset, val, nshard)
    return _native.host().localize_cpu(keys, offset, val, nshard)


def fm_forward(offset, lid, val, pulled, vstride, label, loss, met):
    if _gpu(pulled):
        return _native.hip().fm_forward(offset, lid, val, pulled, vstride, label, loss, met)
    return ref.fm_forward(offset, lid, val, pulled, vstride, label, loss, met)


def fm_backward(csc_off, csc_row, csc_val, dual, xv, pulled, vstride):
    if _gpu(dual):
        return _native.hip().fm_backward(csc_off, csc_row, csc_val, dual, xv, pulled, vstride)
    return ref.fm_backward(csc_off, csc_row, csc_val, dual, xv, pulled, vstride)


def fm_grad_post(grad, vstride, dim, clip, dropout, seed, normalize):
    if vstride == 0 or (clip <= 0 and dropout <= 0 and not normalize):
        return
    if _gpu(grad):
        return _native.hip().fm_grad_post(grad, vstride, dim, clip, dropout, seed, normalize)
    import torch
    g = grad.view(-1, vstride + 4)
    flag = g[:, 1] != 0
    gv = g[:, 4:4 + dim]
    if clip > 0:
        gv.clamp_(-clip, clip)
    if dropout > 0:
        gen = torch.Generator().manual_seed(int(seed) & 0x7fffffff)
        drop = torch.rand(gv.shape, generator=gen) > 1 - dropout
        gv[drop] = 0
    gv[~flag] = 0
    if normalize:
        n2 = float((gv.double() ** 2).sum())
        if n2 >= 1e-10:
            gv /= n2 ** 0.5


def spmv(offset, col, val, x):
    """y = X x for CSR X (columns are dense local ids; col < 0 skipped)."""
    if _gpu(x):
        return _native.hip().spmv(offset, col, val, x)
    import torch
    nrows = offset.numel() - 1
    rows = torch.repeat_interleave(torch.arange(nrows), offset[1:] - offset[:-1])
    c = col.long()
    m = c >= 0
    v = val if (val is not None and val.numel()) else torch.ones(c.numel())
    return torch.zeros(nrows, dtype=x.dtype).index_add_(0, rows[m], v[m] * x[c[m]])


def spmv_t(csc_off, csc_row, csc_val, p):
    """y = X^T p using the per-column occurrence lists of `localize`."""
    if _gpu(p):
        return _native.hip().spmv_t(csc_off, csc_row, csc_val, p)
    import torch
    ncol = csc_off.numel() - 1
    key = torch.repeat_interleave(torch.arange(ncol), csc_off[1:] - csc_off[:-1])
    v = csc_val if (csc_val is not None and csc_val.numel()) else torch.ones(csc_row.numel())
    return torch.zeros(ncol, dtype=p.dtype).index_add_(0, key, v * p[csc_row.long()])


def auc(py, label):
    if _gpu(py):
        return _native.hip().auc(py, label)
    return ref.auc(py, label)
