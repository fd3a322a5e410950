"""Hot ops.  GPU tensors run the hand-written gfx950 HIP kernels
(``wormhole_amd._hip``); CPU tensors run the PyTorch reference
(:mod:`wormhole_amd.ops.ref`).  There is no silent fallback: a GPU tensor
with the HIP extension missing raises.
"""
import torch

from .. import _native
from . import ref

LOSS_SQUARE, LOSS_LOGIT, LOSS_SQUARE_HINGE = ref.LOSS_SQUARE, ref.LOSS_LOGIT, ref.LOSS_SQUARE_HINGE


def _gpu(t):
    return t.is_cuda


make_hdr = ref.make_hdr
hdr_vidx = ref.hdr_vidx


def vstride_for(dim):
    return ref.vstride_for(dim)


def localize(keys, offset, val=None, nshard=1, hint=0, exchange=None):
    """Unique feature ids of a minibatch (grouped by owner shard), per-id
    counts, the nnz->local-id map and the per-id occurrence lists (CSC).
    hint: expected number of unique ids (e.g. the previous minibatch's); it
    sizes the GPU scratch table (a wrong hint costs a retry, never a result).

    exchange (multi-rank, see ShardedKV.count_exchange): the owner counts are
    exchanged with the peers inside localize, before its one host read; then
    an 8th result, the list of key counts received from each rank, is
    returned."""
    if _gpu(keys):
        out = _native.hip().localize(keys, offset, val, nshard, int(hint), exchange)
        if exchange is None:
            return tuple(out[:7])
        return tuple(out[:7]) + (out[7][0::2].tolist(),)
    out = tuple(_native.host().localize_cpu(keys, offset, val, nshard))
    if exchange is None:
        return out
    oc = out[2]
    dev = torch.cat([oc.to(torch.int64), torch.zeros(1, dtype=torch.int64)])
    return out + (exchange(dev)[0::2].tolist(),)


class _CpuJob:
    def __init__(self, args):
        self.args = args

    def finish(self):
        return localize(*self.args)


def localize_begin(keys, offset, val=None, nshard=1, hint=0, exchange=None):
    """Start localizing a minibatch (hash insert, owner counts, count exchange,
    async read of the counts); :func:`localize_finish` completes it with the
    same results as :func:`localize`. Beginning minibatch i+1 before training
    minibatch i hides the one host read of the counts behind i's kernels."""
    if _gpu(keys):
        return _native.hip().LocalizeJob(keys, offset, val, nshard, int(hint), exchange)
    return _CpuJob((keys, offset, val, nshard, hint, exchange))


def localize_finish(job):
    out = job.finish()
    if isinstance(job, _CpuJob) or len(out) == 7:
        return tuple(out)
    if out[7].numel() == 0:
        return tuple(out[:7])
    return tuple(out[:7]) + (out[7][0::2].tolist(),)


def fm_forward(offset, lid, val, w_or_hdr, vc, vstride, label, loss, met):
    """difacto: w_or_hdr = pull header [U, 2] {w, vidx}, vc = [m, vstride]
    embedding rows; linear (vstride == 0): w_or_hdr = w [U], vc = None."""
    if _gpu(w_or_hdr):
        return _native.hip().fm_forward(offset, lid, val, w_or_hdr, vc, vstride, label, loss, met)
    return ref.fm_forward(offset, lid, val, w_or_hdr, vc, vstride, label, loss, met)


def fm_backward(csc_off, csc_row, csc_val, dual, xv, w_or_hdr, vc, vstride):
    """Returns (gw [U], gvc [like vc])."""
    if _gpu(dual):
        return _native.hip().fm_backward(csc_off, csc_row, csc_val, dual, xv, w_or_hdr, vc,
                                         vstride)
    return ref.fm_backward(csc_off, csc_row, csc_val, dual, xv, w_or_hdr, vc, vstride)


def fm_backward_plan(csc_off, csc_row, hdr, vc_rows, nrows, vstride):
    """GPU: phase 1 of :func:`fm_backward` on the current stream -- the
    planning that needs no dual (chunk lists, V-chunk bucketing), so it can
    overlap the forward; :func:`fm_backward_run` finishes it."""
    return _native.hip().fm_backward_plan(csc_off, csc_row, hdr, int(vc_rows), int(nrows),
                                          int(vstride))


def fm_backward_run(plan, csc_off, csc_row, csc_val, dual, xv, hdr, vc, vstride):
    """Phase 2 of :func:`fm_backward` (dual / xv dependent); (gw, gvc)."""
    return _native.hip().fm_backward_run(plan, csc_off, csc_row, csc_val, dual, xv, hdr, vc,
                                         vstride)


def fm_grad_post(gvc, m, dim, clip, dropout, seed, normalize):
    """Clip / dropout / normalise the first m (device int64 [1]) rows of the
    embedding gradient gvc [mcap, vstride] (learn/difacto/loss.h:131-155)."""
    if gvc.numel() == 0 or (clip <= 0 and dropout <= 0 and not normalize):
        return
    if _gpu(gvc):
        return _native.hip().fm_grad_post(gvc, m, dim, clip, dropout, seed, normalize)
    import torch
    gv = gvc[:int(m.reshape(-1)[0]), :dim]
    if clip > 0:
        gv.clamp_(-clip, clip)
    if dropout > 0:
        gen = torch.Generator().manual_seed(int(seed) & 0x7fffffff)
        drop = torch.rand(gv.shape, generator=gen) > 1 - dropout
        gv[drop] = 0
    if normalize:
        n2 = float((gv.double() ** 2).sum())
        if n2 >= 1e-10:
            gv /= n2 ** 0.5


def vidx_renumber(hdr):
    """Renumber a received pull header's vidx column into local compact order
    (exclusive scan of vidx >= 0); returns m as an int64 [1] tensor."""
    if _gpu(hdr):
        return _native.hip().vidx_renumber(hdr)
    import torch
    v = ref.hdr_vidx(hdr)
    has = v >= 0
    pos = torch.cumsum(has.to(torch.int64), 0) - has.to(torch.int64)
    hdr.view(torch.int32).view(-1, 2)[:, 1] = torch.where(has, pos, -1).to(torch.int32)
    return has.sum().reshape(1).to(torch.int64)


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
        auc_join(py)  # the AUC workspace is shared with queued auc_acc calls
        return _native.hip().auc(py, label)
    return ref.auc(py, label)





def auc_acc(py, label, auc_sum):
    """auc_sum (float64 [1]) += exact AUC of the minibatch, on the device.

    The AUC chain (min/max, bucket, one-block scan, place, count: ~60 us of
    small, latency-bound launches) runs on a side stream owned by the native
    layer (it waits for the current stream first), overlapped with the
    backward pass that follows on the compute stream; :func:`auc_join` makes
    the current stream wait for it before ``auc_sum`` is read or reset."""
    if py.numel() == 0:  # an empty step of a lockstep rank: no minibatch, no AUC term
        return auc_sum
    if _gpu(py):
        _native.hip().auc_acc_side(py, label, auc_sum)
        return auc_sum
    auc_sum += ref.auc(py, label)
    return auc_sum


def auc_join(auc_sum):
    """Order the current stream after every queued :func:`auc_acc`."""
    if auc_sum.is_cuda:
        _native.hip().auc_join(auc_sum)


def quant_rows(x, nb, seed):
    """fixed_bytes payload filter: [rows, w] float32 -> uint8 records."""
    if _gpu(x):
        return _native.hip().quant_rows(x.contiguous(), int(nb), int(seed))
    return ref.quant_rows(x, nb, seed)


def dequant_rows(q, w, nb):
    if _gpu(q):
        return _native.hip().dequant_rows(q.contiguous(), int(w), int(nb))
    return ref.dequant_rows(q, w, nb)


def ps_qpack(x, desc_h, desc_d, rows, W, nb, seed):
    """Multi-shard exchange payload filter (fixed_bytes): float regions ->
    uint8 wire rows (see csrc/hip/quant.hip qregion). desc_h: the host copy
    of the per-peer table (bounds-checked by the caller), desc_d: the same
    on x's device."""
    if _gpu(x):
        return _native.hip().ps_qpack(x=x.contiguous(), desc=desc_d, rows=int(rows), W=int(W),
                                      nb=int(nb), seed=int(seed))
    return ref.ps_qpack(x, desc_h, rows, W, nb, seed)


def ps_qunpack(q, desc_h, desc_d, W, nb, out):
    if _gpu(q):
        _native.hip().ps_qunpack(q=q.contiguous(), desc=desc_d, W=int(W), nb=int(nb), out=out)
        return out
    return ref.ps_qunpack(q, desc_h, W, nb, out)


def trunc_u8(c):
    """feature counts -> uint8, saturating (the count push's TRUNCATE filter)."""
    if _gpu(c) and c.dtype == torch.int32:
        return _native.hip().trunc_u8(c.contiguous())
    return ref.trunc_u8(c)


def key_mod(keys, max_key):
    """Fold 64-bit feature ids into [0, max_key) (uint64 modulo): the ps-lite
    ``max_key`` flag as applied by the reference Localizer
    (learn/base/localizer.h:108-115)."""
    if _gpu(keys):
        return _native.hip().key_mod(keys.contiguous(), int(max_key))
    import numpy as np
    k = keys.contiguous().numpy().view(np.uint64) % np.uint64(max_key)
    return torch.from_numpy(k.view(np.int64).copy())


def ps_unpack(rbuf, U, segS, segHS, vrecv):
    """Worker side of the multi-shard pull (kv/psx.py): (hdr [U, 2], rows [1])."""
    if _gpu(rbuf):
        return tuple(_native.hip().ps_unpack(rbuf, int(U), segS, segHS, vrecv))
    return ref.ps_unpack(rbuf, U, segS, segHS, vrecv)


def ps_pack_gw(gw, gbuf, segS, segHS, vrecv):
    """gw [U] into the header rows of the multi-shard push buffer (in place)."""
    if _gpu(gw):
        return _native.hip().ps_pack_gw(gw, gbuf, segS, segHS, vrecv)
    return ref.ps_pack_gw(gw, gbuf, segS, segHS, vrecv)


def ps_records(uniq, ucnt=None):
    """12-byte key records {lo, hi, count} int32 [U, 3] of the key exchange."""
    if _gpu(uniq):
        return _native.hip().ps_records(uniq, ucnt)
    return ref.ps_records(uniq, ucnt)


def ps_c0(owner_cnt, vcnt, P, flag):
    """C0 count-exchange buffers (send [4P], payload [S+1+5P]) from the owner
    counts [S+1] over S <= P shards; see kv/psx.py."""
    if _gpu(owner_cnt):
        return tuple(_native.hip().ps_c0(owner_cnt, vcnt, int(P), int(flag)))
    return ref.ps_c0(owner_cnt, vcnt, P, flag)
