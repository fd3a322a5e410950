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


def auc(py, label):
    if _gpu(py):
        return _native.hip().auc(py, label)
    return ref.auc(py, label)
