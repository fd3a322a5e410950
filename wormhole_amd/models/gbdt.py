"""Distributed histogram GBDT: the xgboost learner the
reference wraps (bin/xgboost.dmlc, learn/xgboost/), built from scratch on
HIP kernels + RCCL.

Algorithm (xgboost "hist" semantics, row split ``dsplit=row``):

* quantile cuts per feature from rank-local order statistics that are
  all-gathered and merged (<= max_bin cuts; features with few distinct values
  get one bin per value); values are binned once into a uint8 matrix
  (255 = missing) that stays resident in HBM;
* per level, LDS-privatised (g, h) histograms are built only for the smaller
  child of every split (the sibling is parent - child), allreduced over the
  ranks (RCCL), and scanned for the best split of every node: gain
  G_L^2/(H_L+lambda) + G_R^2/(H_R+lambda) - G^2/(H+lambda) with L1 ``alpha``,
  ``min_child_weight`` on both children, and both default directions for
  missing values;
* rows are stably partitioned per node on the device;
* the grown tree is pruned bottom-up with ``gamma`` (xgboost's prune updater)
  and leaves store eta * weight; training margins are updated from the final
  leaf segments, other sets by a device tree walk.
"""
import math
import os
import struct

import numpy as np
import torch

from .. import _native
from ..utils.fs import open_uri  # noqa: E402

RT_EPS = 1e-6
MISSING_BIN = 255
_HIST32_ROWS = 8192  # rows per int32 LDS pass of the GPU histogram
# Alternate device paths, kept as the tests' cross-checks (process-wide, the
# same on every rank):
HIST32 = True  # int32 LDS histogram passes (False: int64 sums throughout)
LEAF_WALK_LDS = True  # the LDS-resident tree walk when it fits (False: global walk)
DEFER_TREES = True  # device trees: host lists one tree later (False: read every tree at once)
HOST_GROWER = False  # the per-level host grower instead of the device level loop


# ------------------------------------------------------------------ params
class GBDTParam:
    ALIASES = {"learning_rate": "eta", "min_split_loss": "gamma", "reg_lambda": "lambda",
               "reg_alpha": "alpha", "n_estimators": "num_round"}

    def __init__(self):
        self.booster = "gbtree"
        self.objective = "reg:linear"
        self.eta = 0.3
        self.gamma = 0.0
        self.min_child_weight = 1.0
        self.max_depth = 6
        self.reg_lambda = 1.0
        self.alpha = 0.0
        self.base_score = 0.5
        self.max_bin = 256
        self.subsample = 1.0
        self.colsample_bytree = 1.0
        self.seed = 0
        self.eval_metric = []
        self.silent = 0

    def set(self, name, val):
        name = self.ALIASES.get(name, name)
        if name == "lambda":
            self.reg_lambda = float(val)
        elif name in ("eta", "gamma", "min_child_weight", "alpha", "base_score", "subsample",
                      "colsample_bytree"):
            setattr(self, name, float(val))
        elif name in ("max_depth", "max_bin", "seed", "silent"):
            setattr(self, name, int(val))
        elif name in ("objective", "booster"):
            setattr(self, name, val)
        elif name == "eval_metric":
            self.eval_metric.append(val)
        else:
            return False
        return True

    def calc_gain(self, G, H):
        g = _threshold_l1(G, self.alpha)
        out = g * g / (H + self.reg_lambda)
        return torch.where(H < self.min_child_weight, torch.zeros_like(out), out)

    def calc_weight(self, G, H):
        if H < self.min_child_weight:
            return 0.0
        g = G
        if self.alpha > 0:
            g = G - self.alpha if G > self.alpha else (G + self.alpha if G < -self.alpha else 0.0)
        return -g / (H + self.reg_lambda)


def _h2d(t, dev):
    """Host -> device without a synchronous pageable copy: the per-level
    tables (segments, split descriptions, hist tasks) go through pinned
    memory, asynchronously on the current stream."""
    dev = torch.device(dev)
    if dev.type != "cuda":
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def _threshold_l1(G, alpha):
    if alpha == 0:
        return G
    return torch.where(G > alpha, G - alpha, torch.where(G < -alpha, G + alpha, torch.zeros_like(G)))


# ---------------------------------------------------------------- objective
class Objective:
    def __init__(self, name):
        if name not in ("binary:logistic", "reg:logistic", "reg:linear", "reg:squarederror",
                        "binary:logitraw"):
            raise ValueError("unknown objective " + name)
        self.name = name
        self.logistic = name in ("binary:logistic", "reg:logistic", "binary:logitraw")

    def prob_to_margin(self, base):
        if self.logistic:
            if not 0.0 < base < 1.0:
                raise ValueError("base_score must be in (0,1) for logistic loss")
            return -math.log(1.0 / base - 1.0)
        return base

    def gpair(self, margin, label, weight):
        if margin.is_cuda and margin.dtype == torch.float32 and label.dtype == torch.float32:
            # one launch; the root statistics ride along (gpair_stats)
            gp, st = _native.hip().gbdt_gpair(margin.contiguous(), label.contiguous(),
                                              weight.contiguous() if weight is not None else None,
                                              bool(self.logistic))
            gp._wh_stats = st
            return gp
        if self.logistic:
            p = torch.sigmoid(margin)
            g = p - label
            h = torch.clamp(p * (1.0 - p), min=1e-16)
        else:
            g = margin - label
            h = torch.ones_like(margin)
        if weight is not None:
            g, h = g * weight, h * weight
        return torch.stack([g, h], 1).float().contiguous()

    def pred(self, margin):
        if self.name in ("binary:logistic", "reg:logistic"):
            return torch.sigmoid(margin)
        return margin

    def default_metric(self):
        return "error" if self.name == "binary:logistic" else "rmse"


def gpair_stats(gpair):
    """(sum g, sum h) in fp64 and (max |g|, max |h|) of a gradient-pair
    tensor: the ones the fused GPU gradient kernel computed alongside it,
    else reduced here."""
    st = getattr(gpair, "_wh_stats", None)
    if st is not None:
        return st[:2].clone(), st[2:4].float()
    if gpair.shape[0] == 0:
        z = torch.zeros(2, dtype=torch.float64, device=gpair.device)
        return z, z.float()
    return gpair.double().sum(0), gpair.abs().amax(0).float()


def eval_metric(name, pred, label, weight, bsp):
    """Globally reduced metric (xgboost CLI names)."""
    w = weight if weight is not None else torch.ones_like(label)
    if name == "error":
        s = (((pred > 0.5).float() != (label > 0.5).float()).float() * w).sum()
        v = torch.stack([s.double(), w.sum().double()])
        bsp.allreduce(v)
        return float(v[0] / v[1])
    if name == "logloss":
        p = pred.clamp(1e-16, 1 - 1e-16)
        s = (-(label * torch.log(p) + (1 - label) * torch.log(1 - p)) * w).sum()
        v = torch.stack([s.double(), w.sum().double()])
        bsp.allreduce(v)
        return float(v[0] / v[1])
    if name == "rmse":
        s = (((pred - label) ** 2) * w).sum()
        v = torch.stack([s.double(), w.sum().double()])
        bsp.allreduce(v)
        return math.sqrt(float(v[0] / v[1]))
    if name == "auc":
        from .. import ops
        parts = bsp.comm.allgather_object((pred.cpu(), label.cpu())) if bsp.world > 1 else [
            (pred.cpu(), label.cpu())]
        p = torch.cat([a for a, _ in parts])
        lab = torch.cat([b for _, b in parts])
        return float(ops.ref.auc(p, lab))
    raise ValueError("unknown eval_metric " + name)


# ------------------------------------------------------------------- data
class DMatrix:
    """A rank's rows as a dense device matrix with NaN = missing."""

    def __init__(self, keys, offset, val, label, weight, ncol, device):
        n = offset.numel() - 1
        self.n = n
        self.ncol = int(ncol)
        self.device = device
        X = torch.full((n, self.ncol), float("nan"), dtype=torch.float32, device=device)
        if keys.numel():
            rows = torch.repeat_interleave(torch.arange(n), offset[1:] - offset[:-1]).to(device)
            k = keys.to(device)
            m = k < self.ncol
            v = val.to(device) if val is not None else torch.ones(keys.numel(), device=device)
            X[rows[m], k[m]] = v[m]
        self.X = X
        self.label = label.to(device).float()
        self.weight = weight.to(device).float() if weight is not None else None
        self.B = None

    @staticmethod
    def from_dense(X, label, device):
        d = DMatrix.__new__(DMatrix)
        d.n, d.ncol = X.shape
        d.device = device
        d.X = X.to(device).float().contiguous()
        d.label = label.to(device).float()
        d.weight = None
        d.B = None
        return d

    def predict_tree(self, tree, margin):
        return tree.predict_margin(self.X, margin)


class CSRMatrix:
    """A rank's rows kept sparse (libsvm data with a wide feature space:
    a dense n x ncol matrix would not fit). Row feature ids are sorted
    ascending within each row; a feature a row does not store is missing
    (default direction), exactly as NaN in the dense matrix."""

    sparse = True

    def __init__(self, keys, offset, val, label, weight, ncol, device):
        n = offset.numel() - 1
        self.n, self.ncol, self.device = n, int(ncol), device
        off = offset.to(torch.int64)
        k = keys.to(torch.int64)
        v = val.float() if val is not None and val.numel() else None
        if k.numel():
            rows = torch.repeat_interleave(torch.arange(n, dtype=torch.int64), off[1:] - off[:-1])
            order = torch.argsort(rows * (self.ncol + 1) + k.clamp(0, self.ncol), stable=True)
            k = k[order]
            v = v[order] if v is not None else None
        self.row_off = off.to(device).contiguous()
        self.fid = k.to(torch.int32).to(device).contiguous()
        self.val = v.to(device).contiguous() if v is not None else None
        self.label = label.to(device).float()
        self.weight = weight.to(device).float() if weight is not None else None
        self.gbin = None

    def entry_rows(self):
        return torch.repeat_interleave(torch.arange(self.n, device=self.device),
                                       self.row_off[1:] - self.row_off[:-1])

    def predict_tree(self, tree, margin):
        if self.n == 0:
            return margin
        if self.device.type == "cuda":
            _native.hip().gbdt_predict_csr(self.row_off, self.fid, self.val,
                                           *tree.device_arrays(self.device), margin)
            return margin
        return tree.predict_margin(self.dense_cpu(), margin)

    def dense_cpu(self):
        """(CPU reference path only: small matrices)"""
        X = torch.full((self.n, self.ncol), float("nan"))
        rows = self.entry_rows().cpu()
        ok = self.fid.cpu().long() < self.ncol
        X[rows[ok], self.fid.cpu().long()[ok]] = (self.val.cpu()[ok] if self.val is not None
                                                  else torch.ones(int(ok.sum())))
        return X


def make_dmatrix(keys, offset, val, label, weight, ncol, device, sparse=None):
    """Dense device matrix, or CSR when asked (sparse=True) or when the dense
    form would be large and mostly missing (auto: sparse=None)."""
    n = offset.numel() - 1
    if sparse is None:
        cells = n * max(int(ncol), 1)
        sparse = int(ncol) > 4096 or (cells > (1 << 28) and keys.numel() < cells // 8)
    if sparse:
        return CSRMatrix(keys, offset, val, label, weight, ncol, device)
    return DMatrix(keys, offset, val, label, weight, ncol, device)


class Cuts:
    def __init__(self, values, offsets):
        self.values = values  # float32 [total]
        self.offsets = offsets  # int32 [F + 1]

    @property
    def nbin_max(self):
        o = self.offsets.tolist()
        return max(b - a for a, b in zip(o, o[1:])) if len(o) > 1 else 1

    @staticmethod
    def build(dm, max_bin, bsp, hess=None, nsummary=None):
        """Hessian-weighted quantile sketch (xgboost's WQSketch semantics):
        every stored value weighs its row's hessian (x instance weight; the
        hessian at the base margin when not given), cuts split each
        feature's weight evenly. Each rank summarises its values into <= 4 x
        max_bin weighted points per feature; the summaries are all-gathered
        and merged by the same weighted quantile rule."""
        max_bin = min(int(max_bin), 255)
        nsummary = nsummary or 4 * max_bin
        w_row = hess if hess is not None else torch.ones(dm.n, device=dm.device)
        if dm.weight is not None:
            w_row = w_row * dm.weight
        w_row = w_row.float()
        if getattr(dm, "sparse", False):
            fid, v, w = dm.fid.long(), (dm.val if dm.val is not None else
                                        torch.ones(dm.fid.numel(), device=dm.device)), None
            w = w_row[dm.entry_rows()] if dm.n else torch.zeros(0, device=dm.device)
            ok = (fid >= 0) & (fid < dm.ncol)
            sf, sv, sw = Cuts._summary(fid[ok], v[ok].float(), w[ok], dm.ncol, nsummary)
        else:
            F = dm.ncol
            parts = []
            for j in range(F):
                col = dm.X[:, j]
                ok = ~torch.isnan(col)
                parts.append((torch.full((int(ok.sum()),), j, dtype=torch.int64,
                                         device=dm.device), col[ok], w_row[ok]))
            sf, sv, sw = Cuts._summary(torch.cat([p[0] for p in parts]),
                                       torch.cat([p[1] for p in parts]),
                                       torch.cat([p[2] for p in parts]), F, nsummary)
        local = (sf.cpu(), sv.double().cpu(), sw.double().cpu())
        gathered = bsp.comm.allgather_object(local) if bsp.world > 1 else [local]
        f_all = torch.cat([g[0] for g in gathered])
        v_all = torch.cat([g[1] for g in gathered])
        w_all = torch.cat([g[2] for g in gathered])
        order = torch.argsort(f_all * 0 + v_all, stable=True)
        order = order[torch.argsort(f_all[order], stable=True)]
        f_all, v_all, w_all = f_all[order], v_all[order], w_all[order]
        return Cuts._cuts_from_sorted(f_all, v_all, w_all, dm.ncol, max_bin)

    @staticmethod
    def _segsum(w, ids, nseg):
        """Sums of w over runs of equal, nondecreasing ids in [0, nseg): by
        prefix-sum differences -- a GPU index_add over sorted ids piles
        every row of a run onto one fp64 atomic address (seconds at 11M x 28)."""
        cnt = torch.bincount(ids, minlength=nseg)
        cwp = torch.zeros(w.numel() + 1, dtype=torch.float64, device=w.device)
        torch.cumsum(w.double(), 0, out=cwp[1:])
        end = torch.cumsum(cnt, 0)
        return cwp[end] - cwp[end - cnt]

    @staticmethod
    def _summary(fid, v, w, ncol, m):
        """Per feature: the distinct values when there are <= m, else m
        weighted quantile points each carrying its bucket's weight."""
        if fid.numel() == 0:
            z = torch.zeros(0)
            return z.long(), z, z
        order = torch.argsort(v, stable=True)
        order = order[torch.argsort(fid[order], stable=True)]
        fid, v, w = fid[order], v[order].double(), w[order].double()
        # merge equal (feature, value) runs
        new = torch.ones(fid.numel(), dtype=torch.bool, device=fid.device)
        new[1:] = (fid[1:] != fid[:-1]) | (v[1:] != v[:-1])
        grp = torch.cumsum(new.long(), 0) - 1
        ng = int(grp[-1]) + 1
        fid, v = fid[new], v[new]
        w = Cuts._segsum(w, grp, ng)
        cnt = torch.bincount(fid, minlength=ncol)
        start = torch.cumsum(cnt, 0) - cnt
        big = cnt[fid] > m
        if bool(big.any()):
            cw = torch.cumsum(w, 0)
            fw = Cuts._segsum(w, fid, ncol)
            base = cw[start[fid]] - w[start[fid]]
            q = ((cw - base) / fw[fid].clamp_min(1e-300) * m).floor().clamp(max=m - 1)
            key = fid * (m + 1) + q.long()
            keep_bkt = torch.ones_like(new[: fid.numel()])
            keep_bkt[1:] = key[1:] != key[:-1]
            # a big feature keeps the last value of each weight bucket with
            # the bucket's weight; small features keep every value
            last = torch.ones_like(keep_bkt)
            last[:-1] = key[1:] != key[:-1]
            bid = torch.cumsum(keep_bkt.long(), 0) - 1
            bw = Cuts._segsum(w, bid, int(bid[-1]) + 1)
            keep = ~big | last
            wout = torch.where(big, bw[bid], w)
            return fid[keep], v[keep], wout[keep]
        return fid, v, w

    @staticmethod
    def _cuts_from_sorted(fid, v, w, ncol, max_bin):
        vals, offs = [], [0]
        fid, v, w = fid.long(), v.double(), w.double()
        cnt = torch.bincount(fid, minlength=ncol).tolist() if fid.numel() else [0] * ncol
        pos = 0
        for j in range(ncol):
            c = cnt[j]
            if c:
                vals.extend(Cuts._feature_cuts(v[pos:pos + c], w[pos:pos + c], max_bin))
            pos += c
            offs.append(len(vals))
        return Cuts(torch.tensor(vals, dtype=torch.float32), torch.tensor(offs, dtype=torch.int32))

    @staticmethod
    def _feature_cuts(v, w, max_bin):
        if v.numel() == 0:
            return []
        order = torch.argsort(v)
        v, w = v[order].double(), w[order]
        uniq, inv = torch.unique_consecutive(v, return_inverse=True)
        uw = torch.zeros(uniq.numel(), dtype=torch.float64).index_add_(0, inv, w)
        last = float(uniq[-1])
        top = last + abs(last) + 1.0
        if uniq.numel() <= max_bin:
            cuts = uniq[1:].tolist() + [top]
        else:
            cw = torch.cumsum(uw, 0)
            total = float(cw[-1])
            cuts = []
            for b in range(1, max_bin):
                target = total * b / max_bin
                i = int(torch.searchsorted(cw, torch.tensor([target], dtype=torch.float64)))
                i = min(i + 1, uniq.numel() - 1)
                c = float(uniq[i])
                if not cuts or c > cuts[-1]:
                    cuts.append(c)
            cuts.append(top)
        return [float(np.float32(c)) for c in cuts]

    def bin(self, dm):
        if getattr(dm, "sparse", False):
            if dm.device.type == "cuda":
                return _native.hip().gbdt_bin_csr(dm.fid, dm.val, dm.ncol,
                                                  self.values.to(dm.device),
                                                  self.offsets.to(dm.device))
            fid = dm.fid.long()
            v = dm.val if dm.val is not None else torch.ones(fid.numel())
            o = self.offsets.tolist()
            g = torch.full((fid.numel(),), -1, dtype=torch.int32)
            for j in range(dm.ncol):
                m = fid == j
                if o[j + 1] > o[j] and bool(m.any()):
                    c = self.values[o[j]:o[j + 1]]
                    b = torch.searchsorted(c, v[m], right=True).clamp(max=c.numel() - 1)
                    g[m] = (b + o[j]).to(torch.int32)
            return g
        if dm.X.is_cuda:
            return _native.hip().gbdt_bin(dm.X, self.values.to(dm.device),
                                          self.offsets.to(dm.device))
        out = torch.full(dm.X.shape, MISSING_BIN, dtype=torch.uint8)
        o = self.offsets.tolist()
        for j in range(dm.ncol):
            c = self.values[o[j]:o[j + 1]]
            col = dm.X[:, j]
            ok = ~torch.isnan(col)
            b = torch.searchsorted(c, col[ok], right=True).clamp(max=c.numel() - 1)
            out[ok, j] = b.to(torch.uint8)
        return out


# ------------------------------------------------------------------- tree
class RegTree:
    def __init__(self):
        self.feat, self.bin, self.cond, self.defl = [], [], [], []
        self.left, self.right, self.parent = [], [], []
        self.leaf, self.gain, self.cover, self.base_weight = [], [], [], []

    def add(self, parent):
        i = len(self.feat)
        self.feat.append(-1), self.bin.append(0), self.cond.append(0.0), self.defl.append(0)
        self.left.append(-1), self.right.append(-1), self.parent.append(parent)
        self.leaf.append(0.0), self.gain.append(0.0), self.cover.append(0.0)
        self.base_weight.append(0.0)
        return i

    def is_leaf(self, i):
        return self.feat[i] < 0

    def depth(self, i):
        d = 0
        while self.parent[i] >= 0:
            i = self.parent[i]
            d += 1
        return d

    def device_arrays(self, device):
        f = torch.tensor(self.feat, dtype=torch.int32, device=device)
        return (f, torch.tensor(self.cond, dtype=torch.float32, device=device),
                torch.tensor(self.left, dtype=torch.int32, device=device),
                torch.tensor(self.right, dtype=torch.int32, device=device),
                torch.tensor(self.defl, dtype=torch.uint8, device=device),
                torch.tensor(self.leaf, dtype=torch.float32, device=device))

    def predict_margin(self, X, margin):
        if X.is_cuda:
            _native.hip().gbdt_predict(X, *self.device_arrays(X.device), margin)
            return margin
        node = torch.zeros(X.shape[0], dtype=torch.long)
        feat = torch.tensor(self.feat)
        cond = torch.tensor(self.cond)
        left, right = torch.tensor(self.left), torch.tensor(self.right)
        defl = torch.tensor(self.defl, dtype=torch.bool)
        leaf = torch.tensor(self.leaf)
        for _ in range(64):
            f = feat[node]
            active = f >= 0
            if not bool(active.any()):
                break
            v = X[torch.arange(X.shape[0]), f.clamp(min=0)]
            go_left = torch.where(torch.isnan(v), defl[node], v < cond[node])
            nxt = torch.where(go_left, left[node], right[node])
            node = torch.where(active, nxt, node)
        margin += leaf[node]
        return margin

    # -------------------------------------------------------------- dump
    def dump(self, fmap=None, with_stats=False):
        out = []

        def rec(i, depth):
            pad = "\t" * depth
            if self.is_leaf(i):
                s = "%s%d:leaf=%s" % (pad, i, _fmt(self.leaf[i]))
                if with_stats:
                    s += ",cover=%s" % _fmt(self.cover[i])
                out.append(s)
                return
            f = self.feat[i]
            name, typ = (fmap[f] if fmap and f < len(fmap) else ("f%d" % f, "q"))
            if typ == "i":
                # indicator: "yes" is the branch a present feature (value 1) takes
                yes, no = (self.left[i], self.right[i]) if 1.0 < self.cond[i] else (
                    self.right[i], self.left[i])
                s = "%s%d:[%s] yes=%d,no=%d" % (pad, i, name, yes, no)
            elif typ == "int":
                s = "%s%d:[%s<%d] yes=%d,no=%d" % (pad, i, name, int(math.ceil(self.cond[i])),
                                                   self.left[i], self.right[i])
            else:
                s = "%s%d:[%s<%s] yes=%d,no=%d" % (pad, i, name, _fmt(self.cond[i]),
                                                   self.left[i], self.right[i])
            if typ != "i":
                s += ",missing=%d" % (self.left[i] if self.defl[i] else self.right[i])
            if with_stats:
                s += ",gain=%s,cover=%s" % (_fmt(self.gain[i]), _fmt(self.cover[i]))
            out.append(s)
            rec(self.left[i], depth + 1)
            rec(self.right[i], depth + 1)
        rec(0, 0)
        return "\n".join(out) + "\n"



class _DeviceTree(RegTree):
    """A tree grown by the device level loop whose host lists are built on
    first use (models/gbdt.py TreeBuilder._build_native, defer): the node
    table is copied to pinned host memory right away, behind the tree's
    kernels, and renumbered breadth-first (``gbdt_tree_from_nodes``) when an
    attribute is first read -- by the builder one tree later, or by whoever
    reads the model first. Until then it holds no lists."""

    def __init__(self, nodes, cut_lists):  # noqa: D401 (no RegTree lists yet)
        host = torch.empty(nodes.shape, dtype=nodes.dtype, pin_memory=True)
        host.copy_(nodes, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.__dict__["_pend"] = (host, ev, cut_lists, nodes)

    def materialize(self):
        pend = self.__dict__.pop("_pend", None)
        if pend is None:
            return self
        host, ev, (cut_vals, cut_off), _ = pend
        ev.synchronize()
        RegTree.__init__(self)
        (feat, bin_, cond, defl, left, right, parent, gain, cover, bw, leaf,
         _segs) = _native.hip().gbdt_tree_from_nodes(host, cut_vals, cut_off)
        self.feat, self.bin, self.cond, self.defl = list(feat), list(bin_), list(cond), list(defl)
        self.left, self.right, self.parent = list(left), list(right), list(parent)
        self.gain, self.cover, self.base_weight = list(gain), list(cover), list(bw)
        self.leaf = list(leaf)
        TreeBuilder._compact(self)
        return self

    def __getattr__(self, name):  # only for attributes not set yet
        if name.startswith("__") or "_pend" not in self.__dict__:
            raise AttributeError(name)
        self.materialize()
        return object.__getattribute__(self, name)

    def __getstate__(self):
        self.materialize()
        return self.__dict__

def _fmt(x):
    return "%g" % x


def load_fmap(path):
    names = []
    for line in open_uri(path):
        parts = line.rstrip("\n").split("\t")
        if len(parts) < 3:
            continue
        fid = int(parts[0])
        while len(names) <= fid:
            names.append(("f%d" % len(names), "q"))
        names[fid] = (parts[1], parts[2])
    return names


# ------------------------------------------------------ histogram exchange
class HistExchange:
    """Feature-sharded histogram exchange of the multi-rank dense grower
    (xgboost's row split, ``dsplit=row``, allreduces every
    level's histograms, learn/xgboost/mushroom.hadoop.conf:33).

    Rank r owns the contiguous feature slice ``ranges[r]``. A level's built
    histograms -- the rank-local partial sums [S, F, nbin, 2] -- go out as
    ONE all-to-all-v of feature-major rows (each peer receives its slice
    only) and are summed locally in rank order: a reduce-scatter by feature,
    (P-1)/P of the histogram bytes per rank on the wire where a ring
    allreduce moves 2(P-1)/P. Each rank keeps only its slice of the node
    histograms (sibling subtraction included), searches splits over its
    features, and the per-slot best candidates [S, 6] are all-gathered and
    reduced by gain (ties: lowest rank = lowest feature index, the same
    winner as a row-major argmax over all features on one rank). Trees are
    identical to the allreduce grower's (``WH_GBDT_XCHG=allreduce`` keeps
    that path): on the GPU the histograms are exact fixed-point sums, so the
    reduction order cannot matter."""

    def __init__(self, bsp, F):
        self.comm = bsp.comm
        self.P, self.rank = bsp.world, bsp.rank
        per = -(-F // self.P) if F else 0
        self.ranges = [(min(F, r * per), min(F, (r + 1) * per)) for r in range(self.P)]
        self.lo, self.hi = self.ranges[self.rank]
        self.sent = 0  # bytes this rank sent to its peers (histograms + candidates)

    @staticmethod
    def mode(bsp, dense):
        if bsp.world <= 1 or not dense:
            return None
        return None if os.environ.get("WH_GBDT_XCHG", "rs") == "allreduce" else "rs"

    def reduce_scatter(self, h):
        """h [S, F, nbin, 2] local partials -> [S, Fr, nbin, 2] global sums
        of this rank's features."""
        S, F = int(h.shape[0]), int(h.shape[1])
        rest = tuple(h.shape[2:])
        width = S
        for d in rest:
            width *= int(d)
        x = h.transpose(0, 1).reshape(F, width)  # feature-major rows
        send = [hi - lo for lo, hi in self.ranges]
        fr = self.hi - self.lo
        out = self.comm.all_to_all_v(x, send, [fr] * self.P)
        self.sent += (F - fr) * width * x.element_size()
        acc = out[0:fr].clone()
        for q in range(1, self.P):  # rank order: deterministic on the CPU path too
            acc += out[q * fr:(q + 1) * fr]
        return acc.view((fr, S) + rest).transpose(0, 1).contiguous()

    def pick(self, cand):
        """cand [S, 6] {gain, feature (global), bin, dir, GL, HL}: this
        rank's best per slot -> the best over all ranks."""
        cand = cand.contiguous()
        allc = torch.stack(self.comm.allgather(cand))  # [P, S, 6]
        self.sent += (self.P - 1) * cand.numel() * cand.element_size()
        r = torch.argmax(allc[:, :, 0], 0)  # first maximum: lowest rank on ties
        return allc.gather(0, r[None, :, None].expand(1, cand.shape[0], cand.shape[1]))[0]


# ---------------------------------------------------------------- builder
class TreeBuilder:
    """Depth-wise histogram tree growth on one DMatrix split per rank."""

    def __init__(self, param, bsp, dm, cuts, B):
        self.p = param
        self.bsp = bsp
        self.dm = dm
        self.cuts = cuts
        self.B = B.contiguous()
        self.F = dm.ncol
        self.nbin = max(1, cuts.nbin_max)
        self.gpu = B.is_cuda
        self._native = None  # grower choice, made collectively at the first build()
        self.device = B.device
        # features per LDS histogram block: int64 (g, h) per bin in <= 160 KB
        fg = max(1, (160 * 1024) // (self.nbin * 16))
        fg = min(fg, 64)
        if fg >= 4:
            fg -= fg % 4  # 4-aligned groups let the kernel load 4 bins per dword
        self.fgroups = [(j, min(fg, self.F - j)) for j in range(0, self.F, fg)]
        self.max_fcnt = max(c for _, c in self.fgroups) if self.fgroups else 1
        o = cuts.offsets.tolist()
        nb = torch.tensor([b - a for a, b in zip(o, o[1:])])
        self.bin_mask = torch.arange(self.nbin)[None, :] < nb[:, None]  # [F, nbin]
        self.valid_mask = self.bin_mask.clone()
        self._nglobal = None
        self._valid_dev = None
        self._Bc = None
        mode = HistExchange.mode(bsp, True)
        self.xchg = HistExchange(bsp, self.F) if mode else None
        self.ar_sent = 0  # allreduced histogram bytes per rank (ring model: 2 (P-1) / P)

    def _hist_scale(self, gpair):
        """Fixed-point scales {2^eg, 2^eh} of the GPU histograms: the largest
        powers of two with (global rows) * max|g| * 2^eg <= 2^61, so no node's
        int64 sum can overflow on any rank (see csrc/hip/gbdt.hip).  Unless
        WH_GBDT_HIST=64, a third entry R selects the int32 LDS histograms:
        every row is rounded to 2^-17 of max|g| (|q| <= 2^30 / R) and blocks
        sum <= R rows at a time with 32-bit LDS atomics, ~2x the rate of the
        int64 ones.  The rounding is the same in every block, so histograms
        stay exact sums of the rounded rows (identical for any chunking)."""
        if self._nglobal is None:
            self._nglobal = max(1, int(self.bsp.allreduce_scalar(self.dm.n)))
        m = gpair_stats(gpair)[1] if self.dm.n else torch.zeros(2, device=self.device)
        m = m.float().contiguous()
        self.bsp.allreduce(m, op="max")
        r32 = _HIST32_ROWS if HIST32 else 0
        if m.is_cuda:  # one launch (csrc/hip/gbdt.hip k_qscale), same formula as below
            return _native.hip().gbdt_qscale(m, float(self._nglobal), r32)
        e = torch.floor(torch.log2(2.0 ** 61 / (self._nglobal * m.double().clamp_min(1e-30))))
        if r32:
            # int32 LDS sums of <= R rows: |q| <= 2^30 / R per row (k_hist W32)
            e32 = torch.floor(torch.log2(2.0 ** 30 / (_HIST32_ROWS * m.double().clamp_min(1e-30))))
            e = torch.minimum(e, e32)
            rows = torch.full((1,), float(_HIST32_ROWS), dtype=torch.float64, device=e.device)
            return torch.cat([torch.pow(2.0, e.clamp(-60, 100)), rows]).float()
        scale = torch.pow(2.0, e.clamp(-60, 100))
        return scale.float()

    def sample_features(self, gen):
        """colsample_bytree: restrict this tree's candidate features."""
        self.valid_mask = self.bin_mask.clone()
        if self.p.colsample_bytree < 1.0 and self.F > 0:
            k = max(1, int(round(self.p.colsample_bytree * self.F)))
            keep = torch.randperm(self.F, generator=gen)[:k]
            m = torch.zeros(self.F, dtype=torch.bool)
            m[keep] = True
            self.valid_mask &= m[:, None]

    # ----------------------------------------------------------- histograms
    def _build_hist(self, ridx, gpair, segs, slots, nslot):
        """segs: list of (beg, end) local row ranges; slots: output slot of each."""
        hist = torch.zeros(nslot, self.F, self.nbin, 2, dtype=torch.float64, device=self.device)
        if self.gpu:
            # ~512 row chunks per call (two rounds of the 256 resident
            # 1024-thread blocks); partials are summed per (slot, group)
            total = sum(max(0, e - b) for b, e in segs)
            chunk = max(8192, -(-total // 512))
            G = len(self.fgroups)
            tasks, red = [], []
            for (b, e), s in zip(segs, slots):
                if e <= b:
                    continue
                t0, nch = len(tasks), 0
                for r in range(b, e, chunk):
                    nch += 1
                    for fb, fc in self.fgroups:
                        tasks.append((s, fb, fc, r, min(e, r + chunk)))
                for g, (fb, fc) in enumerate(self.fgroups):
                    red.append((s, fb, fc, t0 + g, nch, G))
            if tasks:
                both = torch.tensor(tasks, dtype=torch.int32).reshape(-1)
                both = torch.cat([both, torch.tensor(red, dtype=torch.int32).reshape(-1)])
                both = _h2d(both, self.device)
                t = both[:5 * len(tasks)].view(-1, 5)
                rd = both[5 * len(tasks):].view(-1, 6)
                _native.hip().gbdt_hist(B=self.B, nbin=self.nbin, ridx=ridx, gpair=gpair,
                                        qscale=self._qscale, tasks=t, red=rd,
                                        max_fcnt=self.max_fcnt, hist=hist)
        else:
            for (b, e), s in zip(segs, slots):
                if e <= b:
                    continue
                rows = ridx[b:e].long()
                bins = self.B[rows].long()  # [r, F]
                gh = gpair[rows].double()  # [r, 2]
                ok = bins != MISSING_BIN
                flat = (torch.arange(self.F)[None, :] * self.nbin + bins.clamp(max=self.nbin - 1))
                for c in range(2):
                    val = gh[:, c][:, None].expand_as(flat)[ok]
                    hist[s].view(-1, 2)[:, c].index_add_(0, flat[ok], val)
        return hist

    # -------------------------------------------------------- split search
    def _find_splits(self, hist, totals):
        """hist [S, F, nbin, 2] (global); totals [S, 2] -> per slot best split.
        On the GPU: the fused split-search kernels (csrc/hip/gbdt.hip
        k_split_feat / k_split_node: scan + gain + argmax in two launches
        instead of ~40 elementwise ops per level); the torch form below is
        their reference. With a feature-sharded exchange, hist holds this
        rank's feature slice only: the local best goes through
        :meth:`HistExchange.pick`."""
        x = getattr(self, "xchg", None)
        if x is None:
            return self._find_splits_local(hist, totals, self.valid_mask, 0)
        S = hist.shape[0]
        if x.hi > x.lo:
            bg, bf, bb, bd, bL = self._find_splits_local(hist, totals,
                                                         self.valid_mask[x.lo:x.hi], x.lo)
            cand = torch.cat([bg[:, None].double(), (bf + x.lo)[:, None].double(),
                              bb[:, None].double(), bd[:, None].double(), bL.double()], 1)
        else:  # (more ranks than features: this rank owns none)
            cand = torch.zeros(S, 6, dtype=torch.float64)
            cand[:, 0] = -float("inf")
        out = x.pick(cand.to(self.device)).cpu()
        return out[:, 0], out[:, 1].long(), out[:, 2].long(), out[:, 3].long(), out[:, 4:6]

    def _find_splits_local(self, hist, totals, valid, lo):
        if hist.is_cuda and hist.shape[0] > 0 and hist.shape[2] <= 1024:
            p = self.p
            if self._valid_dev is None or self._valid_dev[0] is not self.valid_mask:
                self._valid_dev = (self.valid_mask,
                                   self.valid_mask.to(hist.device).contiguous())
            vd = self._valid_dev[1][lo:lo + hist.shape[1]].contiguous()
            out = _native.hip().gbdt_split(hist.double().contiguous(),
                                           totals.double().contiguous(), vd,
                                           float(p.alpha), float(p.reg_lambda),
                                           float(p.min_child_weight)).cpu()
            return (out[:, 0], out[:, 1].long(), out[:, 2].long(), out[:, 3].long(),
                    out[:, 4:6])
        return self._find_splits_ref(hist, totals, valid)

    def _find_splits_ref(self, hist, totals, valid=None):
        if valid is None:
            valid = self.valid_mask
        p = self.p
        cum = hist.cumsum(2)
        present = cum[:, :, -1, :]
        tot = totals[:, None, None, :]
        miss = (totals[:, None, :] - present)[:, :, None, :]
        G, H = totals[:, 0], totals[:, 1]
        parent_gain = p.calc_gain(G, H)[:, None, None]
        best = []
        cands = []
        for defl in (0, 1):
            L = cum + (miss if defl else 0.0)
            R = tot - L
            ok = (L[..., 1] >= p.min_child_weight) & (R[..., 1] >= p.min_child_weight)
            gain = p.calc_gain(L[..., 0], L[..., 1]) + p.calc_gain(R[..., 0], R[..., 1]) - parent_gain
            gain = torch.where(ok, gain, torch.full_like(gain, -float("inf")))
            cands.append((gain, L))
        gain = torch.stack([c[0] for c in cands], -1)  # [S, F, nbin, 2dir]
        # thresholds past a feature's own bin count, and features dropped by
        # colsample_bytree, are not candidates
        gain = torch.where(valid.to(gain.device)[None, :, :, None], gain,
                           torch.full_like(gain, -float("inf")))
        S = gain.shape[0]
        flat = gain.reshape(S, -1)
        arg = flat.argmax(1)
        bg = flat.gather(1, arg[:, None])[:, 0]
        d = arg % 2
        rest = arg // 2
        b = rest % self.nbin
        f = rest // self.nbin
        Lall = torch.stack([cands[0][1], cands[1][1]], 3)  # [S, F, nbin, 2dir, 2]
        Ls = Lall[torch.arange(S, device=arg.device), f, b, d]  # [S, 2]
        # one device->host transfer for the whole level
        out = torch.cat([bg[:, None].double(), f[:, None].double(), b[:, None].double(),
                         d[:, None].double(), Ls.double()], 1).cpu()
        return out[:, 0], out[:, 1].long(), out[:, 2].long(), out[:, 3].long(), out[:, 4:6]

    # ----------------------------------------------------------------- build
    def build(self, gpair, margin):
        if getattr(self, "_native", None) is None:
            # every rank must take the same grower (their allreduce sequences
            # differ): native only if every rank can, decided once, together
            ok = self.gpu and self.dm.n > 0 and not getattr(self.dm, "sparse", False)
            self._native = bool(self.bsp.allreduce_scalar(1.0 if ok else 0.0, "min") > 0)
        if self._native:
            return self._build_native(gpair, margin)
        return self._build_py(gpair, margin)

    def _build_native(self, gpair, margin):
        """The level loop in C++ (``_hip.gbdt_grow``): one host sync per
        level, device-derived child segments, fused sibling subtraction.
        Same tree as :meth:`_build_py` (which stays the CPU path and the
        reference)."""
        p = self.p
        n = self.dm.n
        tot = gpair_stats(gpair)[0]
        self.bsp.allreduce(tot)
        self._qscale = self._hist_scale(gpair)
        if self._Bc is None:
            self._Bc = self.B.t().contiguous()
        if self._valid_dev is None or self._valid_dev[0] is not self.valid_mask:
            self._valid_dev = (self.valid_mask, self.valid_mask.to(self.device).contiguous())
        if not hasattr(self, "_cut_lists"):
            self._cut_lists = (self.cuts.values.tolist(), self.cuts.offsets.tolist())
        ar = self._allreduce_hist if self.bsp.world > 1 else None
        # the level loop on the device (one host read per tree) unless the
        # per-level host grower is asked for (HOST_GROWER, or trees deeper
        # than the device loop's heap numbering)
        host = HOST_GROWER or p.max_depth > 10
        kw = dict(B=self.B, Bc=self._Bc, ridx0=self._iota(n), gpair=gpair, qscale=self._qscale,
                  valid=self._valid_dev[1], nbin=self.nbin, fgroups=self.fgroups,
                  max_fcnt=self.max_fcnt, cut_vals=self._cut_lists[0],
                  cut_off=self._cut_lists[1], eta=float(p.eta), alpha=float(p.alpha),
                  reg_lambda=float(p.reg_lambda), min_child_weight=float(p.min_child_weight),
                  max_depth=int(p.max_depth), rt_eps=RT_EPS, allreduce=ar)
        # deferred: the tree stays a device node table, the margins are
        # walked from it on the device, and its host lists are built one tree
        # later (no GPU idle between trees); needs the row walk and no
        # pruning (gamma <= 0: every accepted split has gain > RT_EPS)
        defer = not host and self._walks(n) and p.gamma <= 0 and DEFER_TREES
        if host:  # (the per-level host grower allreduces whole histograms)
            out = _native.hip().gbdt_grow(root_tot=tot.cpu().tolist(), **kw)
        else:  # root totals as a device tensor: no host wait
            x = self.xchg
            out = _native.hip().gbdt_grow_dev(
                root_tot=tot.contiguous(), **kw,
                reduce_scatter=x.reduce_scatter if x is not None else None,
                pick=x.pick if x is not None else None, f_lo=x.lo if x is not None else 0,
                walk=self._walks(n), defer=defer)
        if defer:
            nodes = out[0]
            _native.hip().gbdt_walk_heap(self.B, nodes, margin, lds=LEAF_WALK_LDS)
            tree = _DeviceTree(nodes, self._cut_lists)
            prev, self._pending = getattr(self, "_pending", None), tree
            if prev is not None:
                prev.materialize()  # (its copy finished during this tree's levels)
            return tree
        (feat, bin_, cond, defl, left, right, parent, gain, cover, bw, leaf, segs, ridx) = out
        tree = RegTree()
        tree.feat, tree.bin, tree.cond, tree.defl = list(feat), list(bin_), list(cond), list(defl)
        tree.left, tree.right, tree.parent = list(left), list(right), list(parent)
        tree.gain, tree.cover, tree.base_weight = list(gain), list(cover), list(bw)
        tree.leaf = list(leaf)
        self._finish(tree, ridx, margin, n, {nd: (b, e) for nd, b, e in segs})
        return tree

    def _iota(self, n):
        """0..n-1 as int32 on the device (the grower only reads it)."""
        t = getattr(self, "_iota_t", None)
        if t is None or t.numel() != n:
            t = self._iota_t = torch.arange(n, dtype=torch.int32, device=self.device)
        return t

    def _build_py(self, gpair, margin):
        p = self.p
        n = self.dm.n
        dev = self.device
        tree = RegTree()
        root = tree.add(-1)
        ridx = torch.arange(n, dtype=torch.int32, device=dev)
        tot = gpair_stats(gpair)[0] if n else torch.zeros(2, dtype=torch.float64, device=dev)
        self.bsp.allreduce(tot)
        totals = {root: tot.cpu()}
        seg = {root: (0, n)}
        done = {}  # finished leaves -> their final ridx segment
        if self.gpu:
            self._qscale = self._hist_scale(gpair)
        hist_root = self._reduce_hist(self._build_hist(ridx, gpair, [seg[root]], [0], 1))
        H_front = hist_root  # [len(frontier), F, nbin, 2], frontier order
        frontier = [root]
        cuts_v = self.cuts.values.tolist()
        cuts_o = self.cuts.offsets.tolist()
        for depth in range(p.max_depth + 1):
            if not frontier:
                break
            for nd in frontier:
                G, H = float(totals[nd][0]), float(totals[nd][1])
                tree.cover[nd] = H
                tree.base_weight[nd] = p.calc_weight(G, H)
                tree.leaf[nd] = p.eta * tree.base_weight[nd]
            if depth == p.max_depth:
                break
            S = len(frontier)
            H_all = H_front
            T_all = _h2d(torch.stack([totals[nd] for nd in frontier]), H_all.device)
            bg, bf, bb, bd, bL = self._find_splits(H_all, T_all)
            split_nodes = []
            for k, nd in enumerate(frontier):
                if float(bg[k]) > RT_EPS:
                    f, b = int(bf[k]), int(bb[k])
                    tree.feat[nd] = f
                    tree.bin[nd] = b
                    tree.cond[nd] = cuts_v[cuts_o[f] + b]
                    tree.defl[nd] = int(bd[k])
                    tree.gain[nd] = float(bg[k])
                    l, r = tree.add(nd), tree.add(nd)
                    tree.left[nd], tree.right[nd] = l, r
                    totals[l] = bL[k].double()
                    totals[r] = (totals[nd] - bL[k]).double()
                    split_nodes.append(nd)
            if not split_nodes:
                break
            # ---- partition rows of the split nodes
            nnode = len(tree.feat)
            node_feat = torch.full((nnode,), -1, dtype=torch.int32)
            node_bin = torch.zeros(nnode, dtype=torch.int32)
            node_defl = torch.zeros(nnode, dtype=torch.uint8)
            seg_beg = torch.zeros(nnode, dtype=torch.int32)
            seg_end = torch.zeros(nnode, dtype=torch.int32)
            for nd in split_nodes:
                node_feat[nd] = tree.feat[nd]
                node_bin[nd] = tree.bin[nd]
                node_defl[nd] = tree.defl[nd]
            for nd, (b, e) in seg.items():
                seg_beg[nd], seg_end[nd] = b, e
            pos_node = self._pos_node(seg, n)
            ridx, nleft = self._partition(ridx, pos_node, node_feat, node_bin, node_defl,
                                          seg_beg, seg_end)
            nleft = nleft.tolist()
            new_frontier = []
            build_segs, build_slots, small, big = [], [], [], []
            for nd in split_nodes:
                b, e = seg.pop(nd)
                l, r = tree.left[nd], tree.right[nd]
                seg[l] = (b, b + nleft[nd])
                seg[r] = (b + nleft[nd], e)
                new_frontier += [l, r]
                # build the child with the smaller GLOBAL hessian, derive the other
                s_, g_ = (l, r) if float(totals[l][1]) <= float(totals[r][1]) else (r, l)
                small.append(s_)
                big.append(g_)
                build_segs.append(seg[s_])
                build_slots.append(len(build_slots))
            for nd in frontier:
                if nd not in split_nodes and nd in seg:
                    done[nd] = seg.pop(nd)  # finished leaf: its rows are final
            hsmall = self._reduce_hist(self._build_hist(ridx, gpair, build_segs, build_slots,
                                                        len(build_slots)))
            # sibling subtraction for every split node at once; the new
            # frontier is [l, r] per split node, in split order
            fpos = {nd: i for i, nd in enumerate(frontier)}
            par = _h2d(torch.tensor([fpos[nd] for nd in split_nodes], dtype=torch.int64),
                       H_front.device)
            hbig = H_front.index_select(0, par) - hsmall
            small_is_left = _h2d(torch.tensor([small[k] == tree.left[nd]
                                               for k, nd in enumerate(split_nodes)]),
                                 H_front.device)
            sil = small_is_left.view(-1, *([1] * (hsmall.dim() - 1)))
            hl = torch.where(sil, hsmall, hbig)
            hr = torch.where(sil, hbig, hsmall)
            H_front = torch.stack([hl, hr], 1).reshape(-1, *H_front.shape[1:])
            frontier = new_frontier
        # margins of the training rows from the final leaf segments
        done.update(seg)
        self._finish(tree, ridx, margin, n, done)
        return tree

    def _reduce_hist(self, h):
        """Rank partials -> global histograms: allreduced (all features), or
        this rank's feature slice (:class:`HistExchange`)."""
        if getattr(self, "xchg", None) is not None:
            return self.xchg.reduce_scatter(h)
        self._allreduce_hist(h)
        return h

    def _allreduce_hist(self, h):
        P = self.bsp.world
        if P > 1:
            self.ar_sent += 2 * (P - 1) * h.numel() * h.element_size() // P
        self.bsp.allreduce(h)

    def hist_bytes(self):
        """Histogram-exchange bytes this rank has sent to its peers so far
        (all-to-all bytes + candidates, or the ring model of the allreduce)."""
        return self.ar_sent + (self.xchg.sent if self.xchg is not None else 0)

    def _pos_node(self, seg, n):
        """Node id of every ridx position (-1 for rows of finished leaves),
        expanded on the device from the segment list."""
        ids, lens = [], []
        cur = 0
        for nd, (b, e) in sorted(seg.items(), key=lambda kv: kv[1][0]):
            if b > cur:
                ids.append(-1), lens.append(b - cur)
            ids.append(nd), lens.append(e - b)
            cur = e
        if cur < n:
            ids.append(-1), lens.append(n - cur)
        dev = self.device
        if self.gpu and ids:
            begs, acc = [], 0
            for ln in lens:
                begs.append(acc)
                acc += ln
            seg = _h2d(torch.tensor([begs, ids], dtype=torch.int32), dev)
            return _native.hip().gbdt_seg_fill(seg[0].contiguous(), seg[1].contiguous(), n)
        return torch.repeat_interleave(torch.tensor(ids, dtype=torch.int32, device=dev),
                                       torch.tensor(lens, dtype=torch.int64, device=dev),
                                       output_size=n)

    def _partition(self, ridx, pos_node, node_feat, node_bin, node_defl, seg_beg, seg_end):
        dev = self.device
        if self.gpu:
            nleft = torch.zeros(node_feat.numel(), dtype=torch.int32, device=dev)
            pk = _h2d(torch.stack([node_feat, node_bin, node_defl.to(torch.int32), seg_beg,
                                   seg_end]), dev)  # one host->device copy
            if self._Bc is None:  # feature-major copy for the partition gathers
                self._Bc = self.B.t().contiguous()
            out = _native.hip().gbdt_partition(self.B, ridx, pos_node, pk[0], pk[1],
                                               pk[2].to(torch.uint8), pk[3], pk[4], nleft,
                                               self._Bc)
            return out, nleft.cpu()
        out = ridx.clone()
        nleft = torch.zeros(node_feat.numel(), dtype=torch.int32)
        for nd in range(node_feat.numel()):
            f = int(node_feat[nd])
            if f < 0:
                continue
            b, e = int(seg_beg[nd]), int(seg_end[nd])
            rows = ridx[b:e].long()
            bins = self.B[rows, f].long()
            left = torch.where(bins == MISSING_BIN, torch.full_like(bins, int(node_defl[nd])),
                               (bins <= int(node_bin[nd])).long()).bool()
            nl = int(left.sum())
            out[b:b + nl] = ridx[b:e][left]
            out[b + nl:e] = ridx[b:e][~left]
            nleft[nd] = nl
        return out, nleft

    def _prune(self, tree):
        """xgboost prune updater: collapse splits whose loss_chg < gamma."""
        self._prune_mark(tree)
        self._compact(tree)

    def _prune_mark(self, tree):
        """The collapse itself, node ids unchanged (see :meth:`_compact`)."""
        if self.p.gamma <= 0:  # accepted splits have gain > RT_EPS > 0: nothing to prune
            return
        changed = True
        while changed:
            changed = False
            for i in range(len(tree.feat)):
                if tree.is_leaf(i):
                    continue
                l, r = tree.left[i], tree.right[i]
                if tree.is_leaf(l) and tree.is_leaf(r) and tree.gain[i] < self.p.gamma:
                    tree.feat[i] = -1
                    tree.leaf[i] = self.p.eta * tree.base_weight[i]
                    changed = True

    def _walks(self, n):
        """True when :meth:`_finish` adds the leaf values by walking each
        row's bins (the dense GPU matrix): the grower may then skip the last
        level's partition and histograms."""
        B = getattr(self, "B", None)
        return bool(n and self.gpu and B is not None and B.dim() == 2 and B.shape[0] == n
                    and B.dtype == torch.uint8 and not getattr(self.dm, "sparse", False))

    def _finish(self, tree, ridx, margin, n, leaf_segs):
        """Prune, then add the leaf values to the training margins from the
        final (pre-prune) leaf segments, then renumber: a pruned-away
        subtree's rows take the value of its nearest ancestor that is a leaf
        after pruning, looked up BEFORE the BFS renumbering changes ids."""
        self._prune_mark(tree)
        B = getattr(self, "B", None)
        if self._walks(n):
            # walk the pruned tree per row on its bins (a pruned-away
            # subtree's rows stop at its collapsed root, whose leaf value
            # _prune_mark set): coalesced, instead of a scatter by ridx
            # the six node arrays in ONE upload (six small copies cost ~20 us
            # of queue time each between the level loop and the walk)
            import numpy as np
            nn = len(tree.feat)
            h = np.empty(6 * nn, dtype=np.int32)
            for q, v in enumerate((tree.feat, tree.bin, tree.left, tree.right, tree.defl)):
                h[q * nn:(q + 1) * nn] = v
            h[5 * nn:].view(np.float32)[:] = tree.leaf
            d = torch.from_numpy(h).to(self.device, non_blocking=True)
            _native.hip().gbdt_leaf_walk(
                B, d[:nn], d[nn:2 * nn], d[4 * nn:5 * nn].to(torch.uint8), d[2 * nn:3 * nn],
                d[3 * nn:4 * nn], d[5 * nn:].view(torch.float32), margin, lds=LEAF_WALK_LDS)
        elif n and self.gpu:
            val = torch.zeros(len(tree.feat), dtype=torch.float32)
            for nd in leaf_segs:
                a, top = nd, nd
                while tree.parent[a] >= 0:
                    a = tree.parent[a]
                    if tree.is_leaf(a):
                        top = a
                val[nd] = tree.leaf[top]
            pos = self._pos_node(leaf_segs, n)
            _native.hip().gbdt_leaf_add(ridx, pos, val.to(self.device), margin)
        self._compact(tree)
        if n and not self.gpu:
            self.dm.predict_tree(tree, margin)

    @staticmethod
    def _compact(tree):
        """Renumber reachable nodes in BFS order (like xgboost's node ids)."""
        order = [0]
        k = 0
        while k < len(order):
            i = order[k]
            if not tree.is_leaf(i):
                order += [tree.left[i], tree.right[i]]
            k += 1
        remap = {old: new for new, old in enumerate(order)}
        t = RegTree()
        for old in order:
            t.add(remap.get(tree.parent[old], -1) if tree.parent[old] >= 0 else -1)
        for old in order:
            i = remap[old]
            t.feat[i] = tree.feat[old]
            t.bin[i], t.cond[i], t.defl[i] = tree.bin[old], tree.cond[old], tree.defl[old]
            t.leaf[i], t.gain[i], t.cover[i] = tree.leaf[old], tree.gain[old], tree.cover[old]
            t.base_weight[i] = tree.base_weight[old]
            if not tree.is_leaf(old):
                t.left[i], t.right[i] = remap[tree.left[old]], remap[tree.right[old]]
        tree.__dict__.update(t.__dict__)
        tree._remap = remap


class CSRTreeBuilder(TreeBuilder):
    """Tree growth on a :class:`CSRMatrix`: the same depth-wise level loop
    (smaller-child histograms, sibling subtraction, both default directions)
    over compact [slots][total bins][2] histograms -- no F x max_bin padding
    and no dense n x F bin matrix."""

    def __init__(self, param, bsp, dm, cuts, gbin):
        self.p, self.bsp, self.dm, self.cuts = param, bsp, dm, cuts
        self.gbin = gbin
        self.F = dm.ncol
        self.device = dm.device
        self.gpu = dm.device.type == "cuda"
        self.tb = int(cuts.offsets[-1]) if cuts.offsets.numel() else 0
        self.cut_off = cuts.offsets.to(self.device).contiguous()
        self.fvalid = None
        self._nglobal = None
        self._rows = None
        self.xchg = None  # compact global-bin histograms: allreduced (HistExchange is dense-only)
        self.ar_sent = 0

    def sample_features(self, gen):
        self.fvalid = None
        if self.p.colsample_bytree < 1.0 and self.F > 0:
            k = max(1, int(round(self.p.colsample_bytree * self.F)))
            keep = torch.randperm(self.F, generator=gen)[:k]
            m = torch.zeros(self.F, dtype=torch.uint8)
            m[keep] = 1
            self.fvalid = m.to(self.device)

    def _build_hist(self, ridx, gpair, segs, slots, nslot):
        if self.gpu:
            chunk, tasks = 16384, []
            for (b, e), sl in zip(segs, slots):
                for r in range(b, e, chunk):
                    tasks += [sl, r, min(e, r + chunk)]
            t = _h2d(torch.tensor(tasks or [0, 0, 0], dtype=torch.int32), self.device)
            return _native.hip().gbdt_hist_csr(self.dm.row_off, self.gbin, ridx, gpair,
                                               self._qscale, t, chunk if tasks else 0, self.tb,
                                               nslot)
        hist = torch.zeros(nslot, self.tb, 2, dtype=torch.float64)
        if self._rows is None:
            self._rows = self.dm.entry_rows()
        for (b, e), sl in zip(segs, slots):
            if e <= b:
                continue
            inseg = torch.zeros(self.dm.n, dtype=torch.bool)
            inseg[ridx[b:e].long()] = True
            m = inseg[self._rows] & (self.gbin >= 0)
            gb = self.gbin[m].long()
            gh = gpair[self._rows[m]].double()
            for c in range(2):
                hist[sl, :, c].index_add_(0, gb, gh[:, c])
        return hist

    def _find_splits(self, hist, totals):
        p = self.p
        if self.gpu:
            out = _native.hip().gbdt_split_csr(hist.contiguous(), totals.double().contiguous(),
                                               self.cut_off, self.fvalid, float(p.alpha),
                                               float(p.reg_lambda),
                                               float(p.min_child_weight)).cpu()
            return (out[:, 0], out[:, 1].long(), out[:, 2].long(), out[:, 3].long(),
                    out[:, 4:6])
        # reference: per feature scans over its compact bins
        o = self.cuts.offsets.tolist()
        S = hist.shape[0]
        res = torch.zeros(S, 6, dtype=torch.float64)
        for s_ in range(S):
            TG, TH = float(totals[s_, 0]), float(totals[s_, 1])
            parent = float(p.calc_gain(torch.tensor(TG), torch.tensor(TH)))
            best = (-float("inf"), 0, 0, 0, 0.0, 0.0)
            for f in range(self.F):
                if o[f + 1] <= o[f] or (self.fvalid is not None and not int(self.fvalid[f])):
                    continue
                hb = hist[s_, o[f]:o[f + 1]]
                cum = hb.cumsum(0)
                mg, mh = TG - float(cum[-1, 0]), TH - float(cum[-1, 1])
                for b in range(hb.shape[0]):
                    for d in (0, 1):
                        GL = float(cum[b, 0]) + (mg if d else 0.0)
                        HL = float(cum[b, 1]) + (mh if d else 0.0)
                        GR, HR = TG - GL, TH - HL
                        if not (HL >= p.min_child_weight and HR >= p.min_child_weight):
                            continue
                        g = (float(p.calc_gain(torch.tensor(GL), torch.tensor(HL))) +
                             float(p.calc_gain(torch.tensor(GR), torch.tensor(HR))) - parent)
                        if g > best[0]:
                            best = (g, f, b, d, GL, HL)
            res[s_] = torch.tensor(best, dtype=torch.float64)
        return res[:, 0], res[:, 1].long(), res[:, 2].long(), res[:, 3].long(), res[:, 4:6]

    def _partition(self, ridx, pos_node, node_feat, node_bin, node_defl, seg_beg, seg_end):
        if self.gpu:
            nleft = torch.zeros(node_feat.numel(), dtype=torch.int32, device=self.device)
            pk = _h2d(torch.stack([node_feat, node_bin, node_defl.to(torch.int32), seg_beg,
                                   seg_end]), self.device)
            out = _native.hip().gbdt_partition_csr(self.dm.row_off, self.dm.fid, self.gbin,
                                                   self.cut_off, ridx, pos_node, pk[0], pk[1],
                                                   pk[2].to(torch.uint8), pk[3], pk[4], nleft)
            return out, nleft.cpu()
        if self._rows is None:
            self._rows = self.dm.entry_rows()
        out = ridx.clone()
        nleft = torch.zeros(node_feat.numel(), dtype=torch.int32)
        o = self.cuts.offsets
        for nd in range(node_feat.numel()):
            f = int(node_feat[nd])
            if f < 0:
                continue
            b, e = int(seg_beg[nd]), int(seg_end[nd])
            rows = ridx[b:e].long()
            lb = torch.full((self.dm.n,), -1, dtype=torch.long)
            m = self.dm.fid.long() == f
            lb[self._rows[m]] = self.gbin[m].long() - int(o[f])
            v = lb[rows]
            left = torch.where(v < 0, torch.full_like(v, int(node_defl[nd])),
                               (v <= int(node_bin[nd])).long()).bool()
            nl = int(left.sum())
            out[b:b + nl] = ridx[b:e][left]
            out[b + nl:e] = ridx[b:e][~left]
            nleft[nd] = nl
        return out, nleft


def make_builder(param, bsp, dm, cuts, B):
    if getattr(dm, "sparse", False):
        return CSRTreeBuilder(param, bsp, dm, cuts, B)
    return TreeBuilder(param, bsp, dm, cuts, B)


# ---------------------------------------------------------------- booster
class Booster:
    MAGIC = b"WHGB"

    def __init__(self, param, num_feature):
        self.param = param
        self.num_feature = int(num_feature)
        self.trees = []
        self.obj = Objective(param.objective)
        self.base_margin = self.obj.prob_to_margin(param.base_score)

    def predict_margin(self, dm, ntree_limit=0):
        margin = torch.full((dm.n,), self.base_margin, dtype=torch.float32, device=dm.device)
        trees = self.trees[:ntree_limit] if ntree_limit else self.trees
        for t in trees:
            dm.predict_tree(t, margin)
        return margin

    def save(self, path):
        p = self.param
        with open_uri(path, "wb") as f:
            f.write(self.MAGIC)
            hdr = ("%s|%g|%d|%d" % (p.objective, p.base_score, self.num_feature,
                                     len(self.trees))).encode()
            f.write(struct.pack("<I", len(hdr)) + hdr)
            for t in self.trees:
                n = len(t.feat)
                f.write(struct.pack("<I", n))
                arr = np.zeros(n, dtype=[("feat", "<i4"), ("cond", "<f4"), ("left", "<i4"),
                                         ("right", "<i4"), ("defl", "<i4"), ("leaf", "<f4"),
                                         ("gain", "<f4"), ("cover", "<f4")])
                for k in ("feat", "cond", "left", "right", "defl", "leaf", "gain", "cover"):
                    arr[k] = getattr(t, k)
                f.write(arr.tobytes())

    @staticmethod
    def load(path, param):
        with open_uri(path, "rb") as f:
            if f.read(4) != Booster.MAGIC:
                raise ValueError("invalid model file " + path)
            (ln,) = struct.unpack("<I", f.read(4))
            objective, base, nf, ntree = f.read(ln).decode().split("|")
            param.objective = objective
            param.base_score = float(base)
            b = Booster(param, int(nf))
            for _ in range(int(ntree)):
                (n,) = struct.unpack("<I", f.read(4))
                arr = np.frombuffer(f.read(32 * n), dtype=[
                    ("feat", "<i4"), ("cond", "<f4"), ("left", "<i4"), ("right", "<i4"),
                    ("defl", "<i4"), ("leaf", "<f4"), ("gain", "<f4"), ("cover", "<f4")])
                t = RegTree()
                for k in ("feat", "cond", "left", "right", "defl", "leaf", "gain", "cover"):
                    setattr(t, k, [x.item() for x in arr[k]])
                t.parent = [-1] * n
                for i in range(n):
                    if t.feat[i] >= 0:
                        t.parent[t.left[i]] = i
                        t.parent[t.right[i]] = i
                t.bin = [0] * n
                t.base_weight = [0.0] * n
                b.trees.append(t)
        return b

    def dump(self, fmap=None, with_stats=False):
        return "".join("booster[%d]:\n%s" % (i, t.dump(fmap, with_stats))
                       for i, t in enumerate(self.trees))
