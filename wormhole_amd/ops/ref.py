"""Plain-PyTorch reference implementations of every hot op.

These are (a) the numerics oracle for the HIP kernel tests and (b) the
execution path for CPU tensors (the reference's CPU plumbing configuration,
e.g. ``dmlc_local.py -n 2 -s 1 bin/linear.dmlc demo.conf`` on a machine with
no GPU).  They follow the reference formulas literally:

* localize      learn/base/localizer.h:96-221
* FM forward    learn/difacto/loss.h:53-94
* FM backward   learn/difacto/loss.h:102-158
* linear losses learn/linear/loss.h:92-157
* AUC           learn/base/binary_class_evaluation.h:17-38
"""
import math

import numpy as np
import torch

LOSS_SQUARE, LOSS_LOGIT, LOSS_SQUARE_HINGE = 1, 2, 4
_M64 = (1 << 64) - 1


def _u64(x):
    return x & _M64


def mix64b_int(x):
    x = _u64(x)
    x ^= x >> 33
    x = _u64(x * 0xff51afd7ed558ccd)
    x ^= x >> 33
    x = _u64(x * 0xc4ceb9fe1a85ec53)
    x ^= x >> 33
    return x


def owner_of(keys, nshard):
    """Shard owner of each int64-encoded uint64 key (matches wh::owner_of)."""
    if nshard <= 1:
        return torch.zeros(keys.numel(), dtype=torch.int64, device=keys.device)
    # vectorised uint64 arithmetic (numpy wraps modulo 2^64 like the device)
    x = keys.detach().cpu().numpy().astype(np.int64).view(np.uint64).copy()
    s33 = np.uint64(33)
    x ^= x >> s33
    x *= np.uint64(0xff51afd7ed558ccd)
    x ^= x >> s33
    x *= np.uint64(0xc4ceb9fe1a85ec53)
    x ^= x >> s33
    own = (x % np.uint64(nshard)).astype(np.int64)
    return torch.from_numpy(own).to(keys.device)


def localize(keys, offset, val=None, nshard=1):
    """Map feature ids to local ids grouped by owner; build the CSC.

    Returns (uniq, ucnt, owner_cnt, lid, csc_off, csc_row, csc_val) with the
    same meaning as the HIP ``_hip.localize``.  Within an owner bucket ids are
    sorted by key (the HIP version uses table order; tests compare sets).
    """
    nnz = keys.numel()
    dev = keys.device
    uniq, inv, cnt = torch.unique(keys, sorted=True, return_inverse=True, return_counts=True)
    own = owner_of(uniq, nshard)
    order = torch.argsort(own * (1 << 0), stable=True)  # stable: keeps key order per owner
    uniq = uniq[order]
    cnt = cnt[order]
    rank = torch.empty_like(order)
    rank[order] = torch.arange(order.numel(), device=dev)
    lid = rank[inv].to(torch.int32)
    owner_cnt = torch.bincount(own, minlength=nshard).cpu()
    nrows = offset.numel() - 1
    rows = torch.repeat_interleave(torch.arange(nrows, device=dev), offset[1:] - offset[:-1])
    perm = torch.argsort(lid.long(), stable=True)
    csc_off = torch.zeros(uniq.numel() + 1, dtype=torch.int64, device=dev)
    csc_off[1:] = torch.cumsum(cnt, 0)
    csc_row = rows[perm].to(torch.int32)
    csc_val = val[perm] if val is not None and val.numel() else torch.empty(0, device=dev)
    return uniq, cnt.to(torch.int32), owner_cnt, lid, csc_off, csc_row, csc_val


def _loss(loss, label, py):
    if loss == LOSS_SQUARE:
        d = py - label
        return 0.5 * d * d, d
    y = torch.where(label > 0, 1.0, -1.0).to(py.dtype)
    if loss == LOSS_SQUARE_HINGE:
        t = torch.clamp(1 - y * py, min=0)
        return t * t, -2 * y * t
    return torch.nn.functional.softplus(-y * py), -y / (1 + torch.exp(y * py))


def hdr_vidx(hdr):
    """int32 view of the vidx column of a [U, 2] float32 pull header."""
    return hdr.contiguous().view(torch.int32).view(-1, 2)[:, 1]


def make_hdr(w, vidx):
    """[U, 2] float32 pull header {w, bit-cast int32 vidx}."""
    h = torch.empty(w.numel(), 2, dtype=torch.float32, device=w.device)
    h[:, 0] = w
    h.view(torch.int32)[:, 1] = vidx.to(torch.int32)
    return h


def fm_forward(offset, lid, val, w_or_hdr, vc, vstride, label, loss, met):
    """Returns (py, dual, xv); accumulates {objv, objv_w, correct, n} into met.

    difacto: w_or_hdr = hdr [U, 2] {w, vidx}, vc = [m, vstride] embedding rows
    (vidx = -1: no embedding); linear (vstride == 0): w_or_hdr = w [U]."""
    nrows = offset.numel() - 1
    dev = w_or_hdr.device
    rows = torch.repeat_interleave(torch.arange(nrows, device=dev), offset[1:] - offset[:-1])
    lid = lid.long()
    x = val if (val is not None and val.numel()) else torch.ones(lid.numel(), device=dev)
    if vstride == 0:
        w = w_or_hdr.reshape(-1)
        py = torch.zeros(nrows, device=dev).index_add_(0, rows, x * w[lid])
        wsum = py
        xv = torch.empty(0, device=dev)
    else:
        w = w_or_hdr[:, 0]
        vid = hdr_vidx(w_or_hdr).long()
        has = vid >= 0
        V = torch.zeros(w.numel(), vstride, device=dev)
        if bool(has.any()):
            V[has] = vc.reshape(-1, vstride)[vid[has]]
        wsum = torch.zeros(nrows, device=dev).index_add_(0, rows, x * w[lid])
        xv = torch.zeros(nrows, vstride, device=dev).index_add_(0, rows, x[:, None] * V[lid])
        xxvv = torch.zeros(nrows, vstride, device=dev).index_add_(
            0, rows, (x * x)[:, None] * V[lid] * V[lid])
        py = wsum + 0.5 * (xv * xv - xxvv).sum(1)
    objv, dual = _loss(loss, label, py)
    objw, _ = _loss(loss, label, wsum)
    correct = ((label > 0) & (py > 0)) | ((label <= 0) & (py <= 0))
    met[0] += objv.double().sum().to(met.device)
    met[1] += objw.double().sum().to(met.device)
    met[2] += correct.double().sum().to(met.device)
    met[3] += float(nrows)
    if met.numel() >= 5 and nrows > 0:  # per-minibatch accuracy, flipped below 0.5
        acc = float(correct.double().sum()) / nrows
        met[4] += acc if acc > 0.5 else 1.0 - acc
    return py, dual, xv.reshape(-1)


def fm_backward(csc_off, csc_row, csc_val, dual, xv, w_or_hdr, vc, vstride):
    """Returns (gw [U], gvc [like vc]); gvc rows follow the header vidx."""
    U = csc_off.numel() - 1
    dev = dual.device
    cnt = csc_off[1:] - csc_off[:-1]
    key = torch.repeat_interleave(torch.arange(U, device=dev), cnt)
    rows = csc_row.long()
    x = csc_val if (csc_val is not None and csc_val.numel()) else torch.ones(rows.numel(), device=dev)
    dx = dual[rows] * x
    gw = torch.zeros(U, device=dev).index_add_(0, key, dx)
    if vstride == 0:
        return gw, torch.empty(0, device=dev)
    vid = hdr_vidx(w_or_hdr).long()
    has = vid >= 0
    vcr = vc.reshape(-1, vstride)
    gvc = torch.zeros(vcr.shape[0], vstride, device=dev)
    if not bool(has.any()):
        return gw, gvc
    xvr = xv.reshape(-1, vstride)
    acc = torch.zeros(U, vstride, device=dev).index_add_(0, key, dx[:, None] * xvr[rows])
    xxp = torch.zeros(U, device=dev).index_add_(0, key, dx * x)
    gvc[vid[has]] = acc[has] - xxp[has, None] * vcr[vid[has]]
    return gw, gvc


def auc(py, label):
    """Exact AUC with the reference's rank-sum convention (>= 0.5)."""
    n = py.numel()
    order = torch.argsort(py, stable=True)
    lab = (label[order] > 0).double()
    cum = torch.cumsum(lab, 0) - lab  # positives strictly before
    tp = float(lab.sum())
    if tp == 0 or tp == n:
        return torch.ones(1, dtype=torch.float64, device=py.device)
    area = float((cum * (1 - lab)).sum()) / (tp * (n - tp))
    return torch.tensor([max(area, 1 - area)], dtype=torch.float64, device=py.device)


def l1l2_solve(z, eta, l1, l2):
    out = (z - torch.sign(z) * l1) / (eta + l2)
    return torch.where(z.abs() <= l1, torch.zeros_like(z), out)


def vstride_for(dim):
    if dim == 0:
        return 0
    q = (dim + 3) // 4
    p = 1
    while p < q:
        p <<= 1
    return 4 * p


def sigmoid(x):
    return 1.0 / (1.0 + math.exp(-x))


# ----------------------------------------------------------- payload filter
def quant_record_bytes(w, nb):
    return (4 + w * nb + 3) // 4 * 4


def _qmax(nb):
    return float((1 << (8 * nb - 1)) - 1)


def quant_rows(x, nb, seed):
    """fixed_bytes filter (csrc/hip/quant.hip): rows of w floats -> uint8
    records {float scale, w signed nb-byte ints}, unbiased random rounding."""
    import numpy as np
    from ..kv.cpu_store import uhash01
    xn = x.detach().cpu().numpy().astype(np.float32)
    rows, w = xn.shape
    lim = _qmax(nb)
    m = np.abs(xn).max(axis=1) if w else np.zeros(rows, np.float32)
    scale = np.where(m > 0, m / np.float32(lim), np.float32(1.0)).astype(np.float32)
    inv = (np.float32(1.0) / scale).astype(np.float32)
    r = np.arange(rows, dtype=np.uint64)[:, None]
    c = np.arange(w, dtype=np.uint64)[None, :]
    u = uhash01(seed, r, c)
    q = np.clip(np.floor(xn * inv[:, None] + u), -lim, lim).astype(np.int64)
    rec = quant_record_bytes(w, nb)
    out = np.zeros((rows, rec), dtype=np.uint8)
    out[:, :4] = scale.view(np.uint8).reshape(rows, 4)
    uq = (q & ((1 << (8 * nb)) - 1)).astype(np.uint64)
    for b in range(nb):
        out[:, 4 + b:4 + w * nb:nb] = ((uq >> np.uint64(8 * b)) & np.uint64(0xff)).astype(np.uint8)
    return torch.from_numpy(out)


def dequant_rows(q, w, nb):
    import numpy as np
    qn = q.cpu().numpy()
    rows = qn.shape[0]
    scale = qn[:, :4].copy().view(np.float32).reshape(rows)
    u = np.zeros((rows, w), dtype=np.int64)
    for b in range(nb):
        u |= qn[:, 4 + b:4 + w * nb:nb].astype(np.int64) << (8 * b)
    sign = 1 << (8 * nb - 1)
    v = (u ^ sign) - sign
    return torch.from_numpy((v.astype(np.float32) * scale[:, None]).astype(np.float32))


def trunc_u8(c):
    return c.clamp(0, 255).to(torch.uint8)


def ps_qpack(x, desc, rows, W, nb, seed):
    """Region payload filter of the multi-shard exchange (oracle of
    csrc/hip/quant.hip k_qregion_pack): desc int64 [P, 6] {sf, a, vf, nf, sq,
    ha} per peer -> uint8 [rows, R] wire rows."""
    import numpy as np
    from ..kv.cpu_store import uhash01
    xf = x.detach().reshape(-1).cpu().numpy().astype(np.float32)
    d = np.asarray(desc, dtype=np.int64).reshape(-1, 6)
    R = quant_record_bytes(W, nb)
    out = np.zeros((rows, R), dtype=np.uint8)
    lim = _qmax(nb)
    for sf, a, vf, nf, sq, ha in d.tolist():
        if ha:  # raw words: the exact part, zero-padded to whole rows
            raw = np.zeros(ha * (R // 4), dtype=np.float32)
            raw[:a] = xf[sf:sf + a]
            out[sq:sq + ha] = raw.view(np.uint8).reshape(ha, R)
        nr = -(-nf // W)
        if not nr:
            continue
        blk = np.zeros(nr * W, dtype=np.float32)
        blk[:nf] = xf[sf + vf:sf + vf + nf]
        blk = blk.reshape(nr, W)
        valid = (np.arange(nr * W).reshape(nr, W) < nf)
        m = np.abs(blk).max(axis=1)
        scale = np.where(m > 0, m / np.float32(lim), np.float32(1.0)).astype(np.float32)
        inv = (np.float32(1.0) / scale).astype(np.float32)
        r0 = sq + ha
        rr = np.arange(r0, r0 + nr, dtype=np.uint64)[:, None]
        cc = np.arange(W, dtype=np.uint64)[None, :]
        u = uhash01(seed, rr, cc)
        q = np.clip(np.floor(blk * inv[:, None] + u), -lim, lim).astype(np.int64)
        q = np.where(valid, q, 0)
        rec = out[r0:r0 + nr]
        rec[:, :4] = scale.view(np.uint8).reshape(nr, 4)
        uq = (q & ((1 << (8 * nb)) - 1)).astype(np.uint64)
        for bb in range(nb):
            rec[:, 4 + bb:4 + W * nb:nb] = ((uq >> np.uint64(8 * bb)) & np.uint64(0xff)).astype(
                np.uint8)
    return torch.from_numpy(out)


def ps_qunpack(q, desc, W, nb, out):
    """Inverse of :func:`ps_qpack` into the float layout ``out`` (in place)."""
    import numpy as np
    qn = q.cpu().numpy()
    d = np.asarray(desc, dtype=np.int64).reshape(-1, 6)
    R = quant_record_bytes(W, nb)
    of = out.view(-1)
    for sf, a, vf, nf, sq, ha in d.tolist():
        if a:
            raw = np.ascontiguousarray(qn[sq:sq + ha]).reshape(-1).view(np.float32)
            of[sf:sf + a] = torch.from_numpy(raw[:a].copy())
        nr = -(-nf // W)
        if not nr:
            continue
        rec = qn[sq + ha:sq + ha + nr]
        scale = np.ascontiguousarray(rec[:, :4]).view(np.float32).reshape(nr)
        u = np.zeros((nr, W), dtype=np.int64)
        for bb in range(nb):
            u |= rec[:, 4 + bb:4 + W * nb:nb].astype(np.int64) << (8 * bb)
        sh = 64 - 8 * nb
        iv = (u << sh) >> sh
        vals = (iv.astype(np.float32) * scale[:, None]).reshape(-1)[:nf]
        of[sf + vf:sf + vf + nf] = torch.from_numpy(vals.astype(np.float32))
    return out


# ------------------------------------------------- multi-shard exchange (psx)
def ps_unpack(rbuf, U, segS, segHS, vrecv):
    """Worker side of the P-shard pull (oracle of psx.hip k_ps_unpack):
    hdr [U, 2] {w, row of the key's embedding inside rbuf or -1}, rows [1]."""
    vs = rbuf.shape[1]
    S = [int(x) for x in segS.tolist()]
    HS = [int(x) for x in segHS.tolist()]
    vr = [int(x) for x in vrecv.tolist()]
    flat = rbuf.reshape(-1)
    hdr = torch.zeros(U, 2, dtype=torch.float32)
    hv = hdr.view(torch.int32)
    VS = 0
    for q in range(len(S) - 1):
        a, b = S[q], S[q + 1]
        base = (HS[q] + VS) * vs
        pairs = flat[base:base + 2 * (b - a)].reshape(-1, 2)
        j = pairs.contiguous().view(torch.int32)[:, 1]
        hdr[a:b, 0] = pairs[:, 0]
        hv[a:b, 1] = torch.where(j >= 0, HS[q + 1] + VS + j, torch.full_like(j, -1))
        VS += vr[q]
    return hdr, torch.tensor([HS[-1] + VS], dtype=torch.int64)


def ps_pack_gw(gw, gbuf, segS, segHS, vrecv):
    """gw [U] into the header rows of the push buffer (in place)."""
    vs = gbuf.shape[1]
    S = [int(x) for x in segS.tolist()]
    HS = [int(x) for x in segHS.tolist()]
    vr = [int(x) for x in vrecv.tolist()]
    flat = gbuf.view(-1)
    VS = 0
    for q in range(len(S) - 1):
        a, b = S[q], S[q + 1]
        base = (HS[q] + VS) * vs
        flat[base:base + (b - a)] = gw[a:b]
        VS += vr[q]


def ps_records(uniq, ucnt=None):
    U = uniq.numel()
    rec = torch.empty(U, 3, dtype=torch.int32)
    rec[:, 0:2] = uniq.contiguous().view(torch.int32).view(U, 2)
    rec[:, 2] = ucnt if ucnt is not None else 0
    return rec


def ps_c0(owner_cnt, vcnt, P, flag):
    """Oracle of psx.hip k_ps_c0: send[4p..] = {keys for p (0 when p >= S),
    overflow flag, V rows for p, has-data flag}; payload = [owner_cnt (S+1) |
    4P receive slot | vcnt P]."""
    S = owner_cnt.numel() - 1
    send = torch.zeros(P, 4, dtype=torch.int64)
    send[:S, 0] = owner_cnt[:S]
    send[:, 1] = owner_cnt[S]
    v = vcnt if vcnt is not None else torch.zeros(P, dtype=torch.int64)
    send[:, 2] = v
    send[:, 3] = int(flag)
    payload = torch.zeros(S + 1 + 5 * P, dtype=torch.int64)
    payload[:S + 1] = owner_cnt
    payload[S + 1 + 4 * P:] = v
    return send.reshape(-1), payload
