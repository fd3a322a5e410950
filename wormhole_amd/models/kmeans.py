"""Distributed spherical k-means (reference learn/kmeans/kmeans.cc).

Each rank keeps its data split resident in HBM -- densified, plus the MFMA
fragment-packed copy, or as CSR rows for wide sparse input (:class:`KMeansCSR`,
chosen by :func:`use_sparse`) -- so one iteration is: pack C -> fused MFMA X.C^T +
row argmax -> per-cluster sum/count with row-contiguous atomics -> one
allreduce of K x (F+1) floats (RCCL) -> mean + L2 normalise -> checkpoint.

Assignment precision (MI355X): for F <= 128 the scores come from the bf16
MFMA as a three-product hi/lo split (bf16 x 3, 16x the fp32 MFMA rate) with
a proven error bound; every row whose best two scores are closer than twice
the bound is re-scored in exact fp32, so the argmax is the exact fp32 one.
WH_KMEANS_PREC=fp32 selects the plain fp32 MFMA kernel.

Deviations from the reference (fixed): a zero-norm
centroid row is skipped instead of aborting the normalisation of the rest,
and an empty cluster keeps its previous centroid (with a warning) instead of
exit(-1).
"""
import os

import torch

from .. import _native
from ..utils.fs import open_uri  # noqa: E402


def densify(keys, offset, val, nrows, ncol, device):
    X = torch.zeros(nrows, ncol, dtype=torch.float32, device=device)
    if keys.numel():
        rows = torch.repeat_interleave(torch.arange(nrows, device=device),
                                       (offset[1:] - offset[:-1]).to(device))
        v = val.to(device) if val is not None else torch.ones(keys.numel(), device=device)
        X.index_put_((rows, keys.to(device)), v, accumulate=True)
    return X


def normalize_rows(C):
    n = C.double().norm(dim=1)
    scale = torch.where(n < 1e-6, torch.ones_like(n), 1.0 / n).to(C.dtype)
    return C * scale[:, None]


class KMeans:
    def __init__(self, bsp, X, k):
        self.bsp = bsp
        self.X = X.contiguous()
        self.n, self.f = X.shape
        self.k = int(k)
        self.device = X.device
        self.gpu = X.is_cuda
        self.split = (self.gpu and 1 <= self.f <= 128 and
                      os.environ.get("WH_KMEANS_PREC", "split") != "fp32")
        self.Xp = self.xnorm = None
        if self.split:
            self.Xp, self.xnorm = _native.hip().kmeans_pack_x3(self.X)
        elif self.gpu:
            self.Xp = _native.hip().kmeans_pack_x(self.X)
        self.C = None
        self.rescored = None  # device count of near-tie rows re-scored in fp32 (last assign)
        self._empty_host = None  # pinned count of empty clusters of the last step
        self._empty_ev = None

    def init_centroids(self, seed=0):
        """Reference InitCentroids: every rank draws num_cluster random rows of
        its data (same srand(0) sequence), centroid i comes from a random rank."""
        g = torch.Generator().manual_seed(seed)
        if self.n == 0:
            raise RuntimeError("dataset is empty")
        idx = torch.randint(0, self.n, (self.k,), generator=g)
        cand = self.X[idx.to(self.device)].contiguous()
        parts = self.bsp.comm.allgather(cand) if self.bsp.world > 1 else [cand]
        proc = torch.randint(0, self.bsp.world, (self.k,), generator=g).tolist()
        C = torch.stack([parts[p][i] for i, p in enumerate(proc)])
        self.C = normalize_rows(C)

    def assign(self):
        if self.split:
            hip = _native.hip()
            C = self.C.contiguous()
            a, _, self.rescored = hip.kmeans_assign_x3(self.Xp, self.xnorm, self.X,
                                                       hip.kmeans_pack_c3(C), C)
            return a
        if self.gpu:
            hip = _native.hip()
            Cp = hip.kmeans_pack_c(self.C.contiguous())
            a, _ = hip.kmeans_assign(self.Xp, self.n, self.f, Cp, self.k)
            return a
        s = self.X.double() @ self.C.double().t()
        return s.argmax(1).to(torch.int32)

    def accumulate(self, a):
        if self.gpu:
            return _native.hip().kmeans_accum(self.X, a, self.k)
        sums = torch.zeros(self.k, self.f + 1, dtype=torch.float32)
        sums[:, : self.f].index_add_(0, a.long(), self.X)
        sums[:, self.f].index_add_(0, a.long(), torch.ones(self.n))
        return sums

    def step(self):
        a = self.assign()
        sums = self.accumulate(a)
        self.bsp.allreduce(sums)  # rabit::Allreduce<Sum>(temp, K*(F+1), lazy_fn)
        if self.gpu:  # mean + normalise + empty count in one launch
            self.C, n_empty = _native.hip().kmeans_update(sums, self.C.contiguous())
            self._warn_empty(n_empty)
            return a
        cnt = sums[:, self.f]
        empty = cnt == 0
        self._warn_empty(empty.sum())
        newC = sums[:, : self.f] / torch.where(empty, torch.ones_like(cnt), cnt)[:, None]
        newC = torch.where(empty[:, None], self.C, newC)
        self.C = normalize_rows(newC)
        return a

    def _warn_empty(self, n_empty):
        """The reference's zero-size-cluster warning without a host sync per
        iteration: the count goes to pinned memory asynchronously and is
        reported one iteration later (and by :meth:`flush_warnings`)."""
        self.flush_warnings()
        if self.gpu:
            if self._empty_host is None:
                self._empty_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
            self._empty_host.copy_(n_empty.reshape(1), non_blocking=True)
            self._empty_ev = torch.cuda.Event()
            self._empty_ev.record()
        elif int(n_empty):
            self._print_empty(int(n_empty))

    def _print_empty(self, n):
        self.bsp.tracker_print("Warning: found %d zero size cluster(s), maybe too less number "
                               "of datapoints? keeping their previous centroids" % n)

    def flush_warnings(self):
        if self._empty_ev is not None:
            self._empty_ev.synchronize()
            self._empty_ev = None
            if int(self._empty_host[0]):
                self._print_empty(int(self._empty_host[0]))

    def objective(self, a=None):
        """Mean cosine similarity of rows to their centroid (diagnostic)."""
        if a is None:
            a = self.assign()
        xn = self.X.norm(dim=1).clamp_min(1e-12)
        s = (self.X * self.C[a.long()]).sum(1) / xn
        tot = torch.tensor([float(s.sum()), float(self.n)], dtype=torch.float64,
                           device=self.bsp.comm.device)
        self.bsp.allreduce(tot)
        return float(tot[0] / tot[1])

    def save_text(self, path):
        with open_uri(path, "w") as f:
            for row in self.C.cpu().tolist():
                f.write(" ".join("%g" % v for v in row) + "\n")


# Dense input above this many bytes per rank, or wider than this with fewer
# non-zeros than this fraction, is clustered in CSR form (KMeansCSR).
_DENSE_MAX_BYTES = 4 << 30
_SPARSE_MIN_WIDTH = 4096
_SPARSE_MAX_DENSITY = 0.05


def use_sparse(nrows, ncol, nnz):
    """Auto choice of the input form (``WH_KMEANS_INPUT=dense|sparse``
    overrides): CSR when the dense split would be large, or wide and
    sparse."""
    mode = os.environ.get("WH_KMEANS_INPUT", "auto")
    if mode in ("dense", "sparse"):
        return mode == "sparse"
    dense = nrows * ncol * 4
    density = nnz / max(1, nrows * ncol)
    return dense > _DENSE_MAX_BYTES or (ncol > _SPARSE_MIN_WIDTH and density < _SPARSE_MAX_DENSITY)


class KMeansCSR(KMeans):
    """Spherical k-means on CSR rows (the reference's form: Cos() walks a
    libsvm Row<unsigned>, learn/kmeans/kmeans.cc:108-130, and only the K x F
    centroids are dense). The split never densifies: assignment reads the
    centroids through their transpose Ct [F, Kp] (csrc/hip/kmeans.hip
    k_assign_csr, double accumulation, ties to the smaller cluster like the
    reference's strict `>`), accumulation scatters each row into its
    cluster's K x (F+1) sum row (k_accum_csr), then the same allreduce and
    centroid update as the dense path."""

    def __init__(self, bsp, keys, offset, val, ncol, k, device):
        self.bsp = bsp
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.off = offset.to(self.device, torch.int64).contiguous()
        self.n = self.off.numel() - 1
        self.f = int(ncol)
        self.k = int(k)
        self.col = keys.to(self.device, torch.int32).contiguous()
        if self.col.numel():
            lo, hi = int(self.col.min()), int(self.col.max())
            if lo < 0 or hi >= self.f:
                raise ValueError("kmeans: feature id %d outside [0, %d)" % (hi if hi >= self.f
                                                                          else lo, self.f))
        self.val = None
        if val is not None and val.numel():
            v = val.to(self.device, torch.float32).contiguous()
            if not bool((v == 1).all()):
                self.val = v
        self.split = False
        self.Xp = self.xnorm = None
        self.C = None
        self.Ct = None
        self.rescored = None
        self._empty_host = None
        self._empty_ev = None
        self.X = None  # (never densified)

    def _rows_dense(self, idx):
        """Dense copies of the given local rows only (centroid init)."""
        out = torch.zeros(len(idx), self.f, dtype=torch.float32, device=self.device)
        off = self.off.cpu().tolist()
        for i, r in enumerate(idx):
            a, b = off[r], off[r + 1]
            if b > a:
                v = self.val[a:b] if self.val is not None else torch.ones(b - a, device=self.device)
                out[i].index_add_(0, self.col[a:b].long(), v)
        return out

    def init_centroids(self, seed=0):
        g = torch.Generator().manual_seed(seed)
        if self.n == 0:
            raise RuntimeError("dataset is empty")
        idx = torch.randint(0, self.n, (self.k,), generator=g).tolist()
        cand = self._rows_dense(idx).contiguous()
        parts = self.bsp.comm.allgather(cand) if self.bsp.world > 1 else [cand]
        proc = torch.randint(0, self.bsp.world, (self.k,), generator=g).tolist()
        C = torch.stack([parts[p][i] for i, p in enumerate(proc)])
        self.C = normalize_rows(C)

    def _transposed(self):
        kp = -(-self.k // 4) * 4
        Ct = torch.zeros(self.f, kp, dtype=torch.float32, device=self.device)
        Ct[:, :self.k] = self.C.t()
        return Ct

    def assign(self):
        if self.gpu:
            return _native.hip().kmeans_assign_csr(offset=self.off, col=self.col, val=self.val,
                                                   Ct=self._transposed(), K=self.k)
        X = torch.sparse_csr_tensor(self.off, self.col.long(),
                                    self.val.double() if self.val is not None else
                                    torch.ones(self.col.numel(), dtype=torch.float64),
                                    size=(self.n, self.f))
        s = (X @ self.C.double().t())
        return s.argmax(1).to(torch.int32)

    def accumulate(self, a):
        if self.gpu:
            return _native.hip().kmeans_accum_csr(offset=self.off, col=self.col, val=self.val,
                                                  assign=a, K=self.k, F=self.f)
        sums = torch.zeros(self.k, self.f + 1, dtype=torch.float32)
        rows = torch.repeat_interleave(torch.arange(self.n), self.off[1:] - self.off[:-1])
        cl = a.long()[rows]
        v = self.val if self.val is not None else torch.ones(self.col.numel())
        sums.view(-1).index_add_(0, cl * (self.f + 1) + self.col.long(), v.float())
        sums[:, self.f].index_add_(0, a.long(), torch.ones(self.n))
        return sums

    def objective(self, a=None):
        """Mean cosine similarity of rows to their centroid (diagnostic)."""
        if a is None:
            a = self.assign()
        rows = torch.repeat_interleave(torch.arange(self.n, device=self.device),
                                       self.off[1:] - self.off[:-1])
        v = self.val if self.val is not None else torch.ones(self.col.numel(),
                                                             device=self.device)
        dot = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        dot.index_add_(0, rows, (v * self.C[a.long()[rows], self.col.long()]).double())
        nrm = torch.zeros(self.n, dtype=torch.float64, device=self.device)
        nrm.index_add_(0, rows, (v * v).double())
        s = dot / nrm.sqrt().clamp_min(1e-12)
        tot = torch.tensor([float(s.sum()), float(self.n)], dtype=torch.float64,
                           device=self.bsp.comm.device)
        self.bsp.allreduce(tot)
        return float(tot[0] / tot[1])
