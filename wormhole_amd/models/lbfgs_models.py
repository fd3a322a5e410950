"""L-BFGS learners on a device-resident data split:

* linear / logistic regression (reference learn/lbfgs-linear/{linear.h,lbfgs.cc})
* factorization machine, order 2 (reference learn/lbfgs-fm/{fm.h,fm.cc})

On the GPU the linear objective runs on csrc/hip/glm.hip over a plan of the
split prepared once (:class:`_GLMPlan`): one fused pass for margin + loss
(+ pred - label), one segmented CSC pass for X^T (pred - label) written
straight into the global gradient.

Each rank loads ``RowBlockIter(data, rank, world)`` (its byte-range split of
the libsvm file) ONCE into HBM, localizes it once (unique feature ids + the
per-feature CSC), and then every objective/gradient evaluation is one fused
device pass: SpMV / FM-forward for the margins, elementwise loss, SpMV^T /
FM-backward for the gradient (no atomics).

Model file: ``"binf"`` + raw ModelParam{f32 base_score; u64
num_feature; i32 loss_type; i32 reserved[16]} (88 bytes incl. padding) +
f32 weights.  Linear: ``w[F] | bias``.  FM: ``w[F] | V[F x nfactor] | bias``;
the reference reads the FM bias from ``weight[num_feature]`` (= V[0][0]) but
writes its gradient to the last slot; here the bias is
consistently the last slot.
"""
import math
import struct

import torch

from .. import ops
from ..utils.fs import open_uri  # noqa: E402

_PARAM_FMT = "<f4xQi16i4x"  # 88 bytes, matches the padded C++ struct


class _ModelParam:
    def __init__(self):
        self.base_score = 0.5
        self.num_feature = 0
        self.loss_type = 1

    def set_param(self, name, val):
        if name == "base_score":
            self.base_score = float(val)
        elif name == "num_feature":
            self.num_feature = int(val)
        elif name == "objective":
            if val == "linear":
                self.loss_type = 0
            elif val == "logistic":
                self.loss_type = 1
            else:
                raise ValueError("unknown objective type " + val)

    def init_base_score(self):
        if not 0.0 < self.base_score < 1.0:
            raise ValueError("base_score must be in (0,1) for logistic loss")
        self.base_score = -math.log(1.0 / self.base_score - 1.0)

    def pack(self):
        return struct.pack(_PARAM_FMT, self.base_score, self.num_feature, self.loss_type,
                           *([0] * 16))

    def unpack(self, b):
        v = struct.unpack(_PARAM_FMT, b)
        self.base_score, self.num_feature, self.loss_type = float(v[0]), int(v[1]), int(v[2])

    def state(self):
        return {"base_score": self.base_score, "num_feature": self.num_feature,
                "loss_type": self.loss_type}

    def load(self, d):
        self.base_score = d["base_score"]
        self.num_feature = d["num_feature"]
        self.loss_type = d["loss_type"]


def margin_to_loss(loss_type, label, margin):
    if loss_type == 1:
        nlogprob = torch.where(margin > 0, torch.log1p(torch.exp(-margin)),
                               -margin + torch.log1p(torch.exp(margin)))
        return label * nlogprob + (1.0 - label) * (margin + nlogprob)
    d = margin - label
    return 0.5 * d * d


def margin_to_pred(loss_type, margin):
    return torch.sigmoid(margin) if loss_type == 1 else margin


class _SplitData:
    """One rank's split, resident on the device and localized once."""

    def __init__(self, keys, offset, val, label, device):
        self.device = device
        self.offset = offset.to(device)
        self.label = label.to(device)
        self.val = val.to(device) if val is not None else None
        keys = keys.to(device)
        (self.uniq, _ucnt, _oc, self.lid, self.csc_off, self.csc_row,
         csc_val) = ops.localize(keys, self.offset, self.val, 1)
        self.csc_val = csc_val if (csc_val is not None and csc_val.numel()) else None
        self.nrows = self.offset.numel() - 1
        self.max_col = int(keys.max().item()) + 1 if keys.numel() else 0


# rows per block of the X^T stream: the 2 MB of pred - label a block gathers
# from stays in an XCD's 4 MB L2
_XTG_ROW_BLOCK_SHIFT = 19


class _GLMPlan:
    """The split, prepared once for the glm.hip passes:

    * ``gcol``: the CSR entries' global weight index (-1: id >= num_feature)
    * the X^T stream: the valid entries ordered (row block, global id), rows
      ascending inside, as runs of one (block, id) each -- ``crow`` /
      ``cval`` per entry, the run-start bits ``hb``, the run of every
      1024-entry wave's first entry ``col0``; and per id (``cgid``) its runs
      in block order (``rlist`` [``coff[c]``, ``coff[c + 1]``)), summed by
      the reduce."""

    def __init__(self, d, F):
        from .. import _native
        self.hip = _native.hip()
        self.F = F
        dev = d.uniq.device
        uniq = d.uniq
        ucol = torch.where(uniq < F, uniq, torch.full_like(uniq, -1)).to(torch.int32)
        lid = d.lid.long()
        self.gcol = torch.where(lid >= 0, ucol[lid.clamp_min(0)],
                                torch.full_like(d.lid, -1)).to(torch.int32).contiguous()
        self.label = d.label.float().contiguous()
        self.none_i32 = torch.empty(0, dtype=torch.int32, device=dev)
        nrows = d.offset.numel() - 1
        gid = self.gcol.long()
        rows = torch.repeat_interleave(torch.arange(nrows, device=dev),
                                       d.offset[1:] - d.offset[:-1], output_size=gid.numel())
        keep = gid >= 0
        rows, gid = rows[keep], gid[keep]
        key = ((rows >> _XTG_ROW_BLOCK_SHIFT) << 31) | gid
        key, perm = torch.sort(key, stable=True)
        self.crow = rows[perm].to(torch.int32)
        self.cval = d.val[keep][perm].contiguous() if d.val is not None else None
        del rows, gid
        nnz = key.numel()
        starts = torch.ones(nnz, dtype=torch.bool, device=dev)
        if nnz > 1:
            starts[1:] = key[1:] != key[:-1]
        run_off = torch.nonzero(starts).view(-1)
        rgid = key[run_off] & ((1 << 31) - 1)
        self.nruns = run_off.numel()
        # each id's runs in block order: the reduce of the run sums
        rk, rperm = torch.sort(rgid, stable=True)
        cst = torch.ones(rk.numel(), dtype=torch.bool, device=dev)
        if rk.numel() > 1:
            cst[1:] = rk[1:] != rk[:-1]
        cpos = torch.nonzero(cst).view(-1)
        self.cgid = rk[cpos].to(torch.int32)
        self.coff = torch.cat([cpos, torch.tensor([rk.numel()], device=dev, dtype=torch.int64)])
        self.rlist = rperm.to(torch.int32)
        del rk, rperm, rgid
        run_off = torch.cat([run_off, torch.tensor([nnz], device=dev, dtype=torch.int64)])
        self.hb = self.hip.glm_heads(run_off, nnz)
        waves = (nnz + 1023) // 1024
        pos = torch.arange(waves, device=dev, dtype=torch.int64) * 1024
        self.col0 = (torch.searchsorted(run_off, pos, right=True) - 1).to(torch.int32)


class LinearObjective:
    def __init__(self, bsp, data, device):
        self.bsp = bsp
        self.device = device
        self.d = data
        self.param = _ModelParam()
        self.reg_L2 = 0.0
        self.model_in = None
        self.loaded = None

    def set_param(self, name, val):
        self.param.set_param(name, val)
        if name == "reg_L2":
            self.reg_L2 = float(val)

    def num_weights(self):
        return self.param.num_feature + 1

    def init_num_dim(self):
        if self.model_in is None:
            ndim = int(self.bsp.allreduce_scalar(self.d.max_col, "max", torch.int64))
            self.param.num_feature = max(ndim, self.param.num_feature)
        return self.num_weights()

    def init_model(self, n):
        if self.model_in is None:
            self.param.init_base_score()
            return torch.zeros(n, dtype=torch.float32)
        return self.loaded.clone()

    def save_state(self):
        return self.param.state()

    def load_state(self, s):
        self.param.load(s)

    # ------------------------------------------------------------- math
    def _feat(self):
        F = self.param.num_feature
        valid = self.d.uniq < F
        idx = torch.where(valid, self.d.uniq, torch.zeros_like(self.d.uniq))
        return valid, idx

    def _plan(self):
        F = self.param.num_feature
        p = getattr(self, "_glm", None)
        if p is None or p.F != F:
            p = self._glm = _GLMPlan(self.d, F)
        return p

    def _glm_fwd(self, mode, w):
        p = self._plan()
        return p.hip.glm_fwd(mode, self.d.offset, p.gcol, self.d.val, w.contiguous(), p.F,
                             float(self.param.base_score), p.label if mode != 2 else None,
                             int(self.param.loss_type))

    def margin(self, w):
        F = self.param.num_feature
        if w.is_cuda:
            return self._glm_fwd(2, w)[0]
        valid, idx = self._feat()
        wu = torch.where(valid, w[idx], torch.zeros((), device=w.device))
        return ops.spmv(self.d.offset, self.d.lid, self.d.val, wu.contiguous()) + (
            self.param.base_score + w[F])

    def eval(self, w):
        F = self.param.num_feature
        if w.is_cuda:  # margin + loss in one pass (glm.hip k_glm_fwd)
            m, sums = self._glm_fwd(3, w)
            # the accepted point of a line search is the next gradient's: its
            # margins are kept for calc_grad (one SpMV per iteration saved)
            self._mcache = (w, w._version, self.param.num_feature, m)
            val = float(sums[0])
        else:
            val = float(margin_to_loss(self.param.loss_type, self.d.label, self.margin(w)).sum(
                dtype=torch.float64))
        if self.bsp.rank == 0 and self.reg_L2 != 0.0:
            val += 0.5 * self.reg_L2 * float((w[:F].double() ** 2).sum())
        if math.isnan(val):
            raise RuntimeError("nan occurs")
        return val

    def calc_grad(self, w):
        F = self.param.num_feature
        if w.is_cuda:  # pred - label, then X^T of it (glm.hip)
            mc = getattr(self, "_mcache", None)
            p = self._plan()
            if mc is not None and mc[0] is w and mc[1] == w._version and mc[2] == F:
                g, sums = p.hip.glm_grad_from_margin(mc[3], p.label, int(self.param.loss_type))
            else:
                g, sums = self._glm_fwd(1, w)
            self._mcache = None
            grad = torch.zeros_like(w)
            S = torch.zeros(p.nruns, dtype=torch.float32, device=w.device)
            p.hip.glm_xtg(p.crow, p.cval, p.hb, p.col0, p.none_i32, g, S)
            p.hip.glm_runs_reduce(p.coff, p.rlist, S, p.cgid, grad)
            grad[F:F + 1].copy_(sums[1:2])
            if self.bsp.rank == 0 and self.reg_L2 != 0.0:
                grad[:F] += self.reg_L2 * w[:F]
            return grad
        pred = margin_to_pred(self.param.loss_type, self.margin(w))
        g = (pred - self.d.label).contiguous()
        gu = ops.spmv_t(self.d.csc_off, self.d.csc_row, self.d.csc_val, g)
        valid, idx = self._feat()
        grad = torch.zeros_like(w)
        grad.index_copy_(0, idx[valid], gu[valid])  # (unique ids: a scatter, no atomics)
        grad[F] = g.sum()
        if self.bsp.rank == 0 and self.reg_L2 != 0.0:
            grad[:F] += self.reg_L2 * w[:F]
        return grad

    def predict(self, w):
        return margin_to_pred(self.param.loss_type, self.margin(w))

    # ------------------------------------------------------------- I/O
    def save_model(self, path, w):
        with open_uri(path, "wb") as f:
            f.write(b"binf")
            f.write(self.param.pack())
            f.write(w.detach().float().cpu().numpy().tobytes())

    def load_model(self, path):
        with open_uri(path, "rb") as f:
            if f.read(4) != b"binf":
                raise ValueError("invalid model file")
            self.param.unpack(f.read(struct.calcsize(_PARAM_FMT)))
            import numpy as np
            self.loaded = torch.from_numpy(np.frombuffer(f.read(), dtype="<f4").copy())
        self.model_in = path
        if self.loaded.numel() != self.num_weights():
            raise ValueError("model size mismatch")


class FMObjective(LinearObjective):
    def __init__(self, bsp, data, device):
        super().__init__(bsp, data, device)
        self.nfactor = 10
        self.reg_L2_V = 0.0
        self.fm_random = 0.01

    def set_param(self, name, val):
        super().set_param(name, val)
        if name == "nfactor":
            self.nfactor = int(val)
        elif name == "reg_L2_V":
            self.reg_L2_V = float(val)
        elif name == "fm_random":
            self.fm_random = float(val)

    def num_weights(self):
        return self.param.num_feature * (self.nfactor + 1) + 1

    def init_model(self, n):
        if self.model_in is None:
            self.param.init_base_score()
            if self.bsp.rank == 0:
                g = torch.Generator().manual_seed(0)
                return torch.randn(n, generator=g) * self.fm_random
            return torch.zeros(n, dtype=torch.float32)
        return self.loaded.clone()

    def _pulled(self, w):
        """The FM weights in the variable-length pull layout of the fused FM
        kernels: hdr {w, vidx} per local feature, vc = its V rows (vidx = i)."""
        F, k = self.param.num_feature, self.nfactor
        vs = ops.vstride_for(k)
        valid, idx = self._feat()
        U = idx.numel()
        zero = torch.zeros((), device=w.device)
        vidx = torch.where(valid, torch.arange(U, device=w.device), torch.full_like(idx, -1))
        hdr = ops.make_hdr(torch.where(valid, w[idx], zero), vidx)
        V = w[F:F + F * k].view(F, k)
        vc = torch.zeros(U, vs, dtype=torch.float32, device=w.device)
        vc[:, :k] = torch.where(valid[:, None], V[idx], zero)
        return hdr, vc, vs

    def _forward(self, w):
        hdr, vc, vs = self._pulled(w)
        met = torch.zeros(4, dtype=torch.float64, device=w.device)
        py, _dual, xv = ops.fm_forward(self.d.offset, self.d.lid, self.d.val, hdr, vc, vs,
                                       self.d.label, 1, met)
        F, k = self.param.num_feature, self.nfactor
        return py + (self.param.base_score + w[F * (k + 1)]), (hdr, vc), vs, xv

    def margin(self, w):
        return self._forward(w)[0]

    def eval(self, w):
        F, k = self.param.num_feature, self.nfactor
        fw = self._forward(w)
        # (kept for a gradient at the same weights: the accepted line-search
        # point's forward is not run twice)
        self._fcache = (w, w._version, F, fw)
        val = float(margin_to_loss(self.param.loss_type, self.d.label, fw[0]).sum(
            dtype=torch.float64))
        if self.bsp.rank == 0:
            if self.reg_L2 != 0.0:
                val += 0.5 * self.reg_L2 * float((w[:F].double() ** 2).sum())
            if self.reg_L2_V != 0.0:
                val += 0.5 * self.reg_L2_V * float((w[F:F * (k + 1)].double() ** 2).sum())
        if math.isnan(val):
            raise RuntimeError("nan occurs")
        return val

    def calc_grad(self, w):
        F, k = self.param.num_feature, self.nfactor
        fc = getattr(self, "_fcache", None)
        self._fcache = None
        if fc is not None and fc[0] is w and fc[1] == w._version and fc[2] == F:
            margin, (hdr, vc), vs, xv = fc[3]
        else:
            margin, (hdr, vc), vs, xv = self._forward(w)
        g = (margin_to_pred(self.param.loss_type, margin) - self.d.label).contiguous()
        gw, gvc = ops.fm_backward(self.d.csc_off, self.d.csc_row, self.d.csc_val, g, xv, hdr, vc,
                                  vs)
        valid, idx = self._feat()
        grad = torch.zeros_like(w)
        grad.index_add_(0, idx[valid], gw[valid])
        gV = grad[F:F + F * k].view(F, k)
        gV.index_add_(0, idx[valid], gvc[valid][:, :k])
        grad[F * (k + 1)] = g.sum()
        if self.bsp.rank == 0:
            if self.reg_L2 != 0.0:
                grad[:F] += self.reg_L2 * w[:F]
            if self.reg_L2_V != 0.0:
                grad[F:F * (k + 1)] += self.reg_L2_V * w[F:F * (k + 1)]
        return grad
