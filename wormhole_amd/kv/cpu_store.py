"""Host (CPU) parameter store with the same interface and update math as the
device store ``wormhole_amd._hip.KVStore``.

Used for the GPU-free plumbing configuration and as the oracle of the fused
update kernels in tests.  Update rules follow the reference handles:
linear SGD/AdaGrad/FTRL (learn/linear/async_sgd.h:71-180) and DiFacto
FTRL-w + AdaGrad-V with lazy V allocation (learn/difacto/async_sgd.h:214-296).
"""
import numpy as np
import torch

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xbf58476d1ce4e5b9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94d049bb133111eb)
        x = x ^ (x >> np.uint64(31))
    return x


def uhash01(seed, a, b):
    """Same counter-based uniform as wh::uhash01 (device)."""
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        inner = _mix64(a * np.uint64(0x9e3779b97f4a7c15) + b)
        h = _mix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ inner)
    return (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def _vstride(dim):
    if dim == 0:
        return 0
    q, p = (dim + 3) // 4, 1
    while p < q:
        p <<= 1
    return 4 * p


class CpuKVStore:
    def __init__(self, cap=1 << 16, vcap=1 << 14, dim=0, device=None):
        self.dim = int(dim)
        self.vstride = _vstride(self.dim)
        self.cap = int(cap)
        self.vcap = int(vcap) if dim > 0 else 0
        self._index = {}
        n = 0
        self._keys = np.zeros(64, dtype=np.int64)
        self._w = np.zeros(64, dtype=np.float32)
        self._z = np.zeros(64, dtype=np.float32)
        self._sq = np.zeros(64, dtype=np.float32)
        self._cnt = np.zeros(64, dtype=np.uint32)
        self._vrow = np.full(64, -1, dtype=np.int32)
        self._V = np.zeros((16, max(self.vstride, 1)), dtype=np.float32)
        self._VG = np.zeros((16, max(self.vstride, 1)), dtype=np.float32)
        self._n = n
        self._vnext = 0
        self._stats = np.zeros(8, dtype=np.int64)

    # ---------------------------------------------------------------- views
    @property
    def keys(self):
        return torch.from_numpy(self._keys[: self._n].copy())

    @property
    def w(self):
        return torch.from_numpy(self._w[: self._n].copy())

    @property
    def z(self):
        return torch.from_numpy(self._z[: self._n].copy())

    @property
    def sq(self):
        return torch.from_numpy(self._sq[: self._n].copy())

    @property
    def cnt(self):
        return torch.from_numpy(self._cnt[: self._n].astype(np.int32))

    @property
    def vrow(self):
        return torch.from_numpy(self._vrow[: self._n].copy())

    @property
    def V(self):
        return torch.from_numpy(self._V[: self._vnext].copy())

    @property
    def VG(self):
        return torch.from_numpy(self._VG[: self._vnext].copy())

    @property
    def vnext(self):
        return torch.tensor([self._vnext], dtype=torch.int32)

    @property
    def stats(self):
        return torch.from_numpy(self._stats.copy())  # a copy (like the device store)

    def reset_stats(self, i0, i1):
        self._stats[i0:i1] = 0

    def add_stat(self, i, v):
        self._stats[i] += int(v)

    def occupied(self):
        return torch.arange(self._n, dtype=torch.int32)

    # ---------------------------------------------------------------- index
    def _grow(self, need):
        cur = self._keys.shape[0]
        if need <= cur:
            return
        new = max(need, cur * 2)
        for name, fill in (("_keys", 0), ("_w", 0), ("_z", 0), ("_sq", 0), ("_cnt", 0),
                           ("_vrow", -1)):
            a = getattr(self, name)
            b = np.full(new, fill, dtype=a.dtype)
            b[:cur] = a
            setattr(self, name, b)

    def _grow_v(self, need):
        cur = self._V.shape[0]
        if need <= cur:
            return
        new = max(need, cur * 2)
        for name in ("_V", "_VG"):
            a = getattr(self, name)
            b = np.zeros((new, a.shape[1]), dtype=np.float32)
            b[:cur] = a
            setattr(self, name, b)

    def find(self, keys, insert):
        ks = keys.cpu().numpy().astype(np.int64)
        out = np.empty(ks.shape[0], dtype=np.int32)
        idx = self._index
        for i, k in enumerate(ks.tolist()):
            s = idx.get(k)
            if s is None:
                if insert:
                    if self._n >= self.cap:
                        self._stats[2] += 1
                        s = -1
                    else:
                        s = self._n
                        self._grow(s + 1)
                        self._keys[s] = k
                        idx[k] = s
                        self._n += 1
                        self._stats[4] += 1
                else:
                    s = -1
            out[i] = s
        return torch.from_numpy(out)

    # ------------------------------------------------------------- loading
    def load_entries(self, keys, cols):
        s = self.find(keys, True).numpy()
        if (s < 0).any():
            raise RuntimeError("parameter table full while loading the model")
        for name, val in cols.items():
            getattr(self, "_" + name)[s] = val.numpy()

    def load_v(self, keys, V, VG):
        s = self.find(keys, True).numpy()
        for i, slot in enumerate(s.tolist()):
            row = self._vnext
            self._vnext += 1
            self._grow_v(row + 1)
            self._vrow[slot] = row
            self._V[row] = 0
            self._V[row, : V.shape[1]] = V[i].numpy()
            self._VG[row] = 0
            self._VG[row, : VG.shape[1]] = VG[i].numpy()

    # --------------------------------------------------------------- linear
    @staticmethod
    def _solve(z, eta, l1, l2):
        out = (z - np.sign(z) * l1) / (eta + l2)
        return np.where(np.abs(z) <= l1, 0.0, out).astype(np.float32)

    def _count_delta(self, old, new):
        self._stats[0] += int(((old == 0) & (new != 0)).sum()) - int(((old != 0) & (new == 0)).sum())

    def linear_pull(self, slot):
        s = slot.cpu().numpy()
        out = np.where(s >= 0, self._w[np.maximum(s, 0)], 0.0).astype(np.float32)
        return torch.from_numpy(out)

    def linear_push(self, slot, grad, algo, alpha, beta, l1, l2, sgd_eta):
        s = slot.cpu().numpy()
        g = grad.cpu().numpy().reshape(-1)[: s.shape[0]].astype(np.float32)
        m = s >= 0
        s, g = s[m], g[m]
        old = self._w[s].copy()
        f32 = np.float32
        if algo == 1:
            new = self._solve(f32(sgd_eta) * old - g, f32(sgd_eta), f32(l1), f32(l2))
        elif algo == 2:
            sq = np.sqrt(self._sq[s] * self._sq[s] + g * g).astype(np.float32)
            self._sq[s] = sq
            eta = (sq + f32(beta)) / f32(alpha)
            new = self._solve(eta * old - g, eta, f32(l1), f32(l2))
        elif algo == 4:  # DiFacto's FTRL on w (learn/difacto/async_sgd.h:262-286)
            gg = (g + f32(l2) * old).astype(np.float32)
            cg = self._sq[s]
            cg_new = np.sqrt(cg * cg + gg * gg).astype(np.float32)
            self._sq[s] = cg_new
            z = (self._z[s] - (gg - (cg_new - cg) / f32(alpha) * old)).astype(np.float32)
            self._z[s] = z
            eta = (f32(beta) + cg_new) / f32(alpha)
            new = np.where((z <= f32(l1)) & (z >= -f32(l1)), f32(0),
                           np.where(z > 0, z - f32(l1), z + f32(l1)) / eta).astype(np.float32)
        else:
            sq0 = self._sq[s]
            sq = np.sqrt(sq0 * sq0 + g * g).astype(np.float32)
            self._sq[s] = sq
            sigma = (sq - sq0) / f32(alpha)
            z = self._z[s] + g - sigma * old
            self._z[s] = z
            new = self._solve(-z, (f32(beta) + sq) / f32(alpha), f32(l1), f32(l2))
        self._w[s] = new
        self._count_delta(old, new)

    # -------------------------------------------------------------- difacto
    def _alloc_v(self, s, seed, v_init):
        row = self._vnext
        self._vnext += 1
        if row >= self.vcap:
            self._stats[3] += 1
            return -1
        self._grow_v(row + 1)
        self._vrow[s] = row
        d = np.arange(self.vstride, dtype=np.uint64)
        u = uhash01(seed, np.uint64(np.int64(self._keys[s]).view(np.uint64)), d)
        v = ((u * np.float32(2) - np.float32(1)) * np.float32(v_init)).astype(np.float32)
        v[self.dim:] = 0
        self._V[row] = v
        self._VG[row] = 0
        self._stats[1] += self.dim
        return row

    def difacto_push_cnt(self, slot, cnt, h, threshold, l1_shrk, seed):
        s_all = slot.cpu().numpy()
        c_all = cnt.cpu().numpy()
        for s, c in zip(s_all.tolist(), c_all.tolist()):
            if s < 0:
                continue
            self._cnt[s] = np.uint32(int(self._cnt[s]) + int(c))
            if (self.vstride > 0 and self._cnt[s] > threshold and self._vrow[s] < 0
                    and (not l1_shrk or self._w[s] != 0)):
                self._alloc_v(s, seed, h[7])

    def difacto_open_pull(self, keys, insert, cnt, h, threshold, l1_shrk, seed, direct=False):
        """find + (optional) count push + pull, like the HIP store's fused op
        (always the compact pull: ``direct`` is a device-path layout)."""
        slot = self.find(keys, insert)
        if cnt is not None:
            self.difacto_push_cnt(slot, cnt, h, threshold, l1_shrk, seed)
        hdr, vc, vpos = self.difacto_pull(slot, l1_shrk)
        return slot, hdr, vc, vpos

    def difacto_pull(self, slot, l1_shrk):
        """Variable-length pull: (hdr [n, 2] {w, vidx bits}, vc [m, vstride],
        vpos int64 [n+1]) -- the layout of the HIP store (vc is exact here)."""
        s_all = slot.cpu().numpy()
        n = s_all.shape[0]
        w = np.zeros(n, dtype=np.float32)
        vid = np.full(n, -1, dtype=np.int32)
        rows = []
        for i, s in enumerate(s_all.tolist()):
            if s < 0:
                continue
            w[i] = self._w[s]
            row = self._vrow[s] if self.vstride > 0 else -1
            if l1_shrk and w[i] == 0:
                row = -1
            if row >= 0:
                vid[i] = len(rows)
                rows.append(row)
        hdr = np.zeros((n, 2), dtype=np.float32)
        hdr[:, 0] = w
        hdr.view(np.int32)[:, 1] = vid
        vc = (self._V[np.array(rows, dtype=np.int64)] if rows
              else np.zeros((0, max(self.vstride, 1)), dtype=np.float32))
        flag = (vid >= 0).astype(np.int64)
        vpos = np.zeros(n + 1, dtype=np.int64)
        vpos[1:] = np.cumsum(flag)
        return torch.from_numpy(hdr), torch.from_numpy(vc.copy()), torch.from_numpy(vpos)

    def difacto_push(self, slot, hdr, gw, gvc, h, threshold, l1_shrk, seed):
        """gw [n] for every key; gvc[vidx_i] for keys whose pull header
        (this shard's numbering) had an embedding row."""
        alpha, beta, l1, l2, v_alpha, v_beta, v_l2, v_init = [np.float32(x) for x in h]
        s_all = slot.cpu().numpy()
        gw_all = gw.cpu().numpy().reshape(-1)
        vid_all = hdr.cpu().contiguous().numpy().view(np.int32).reshape(-1, 2)[:, 1]
        gv_all = gvc.cpu().numpy().reshape(-1, max(self.vstride, 1)) if gvc.numel() else None
        for i, s in enumerate(s_all.tolist()):
            if s < 0:
                continue
            g = np.float32(gw_all[i])
            w = self._w[s]
            g = np.float32(g + l2 * w)
            cg = self._sq[s]
            cg_new = np.float32(np.sqrt(cg * cg + g * g))
            self._sq[s] = cg_new
            z = np.float32(self._z[s] - (g - (cg_new - cg) / alpha * w))
            self._z[s] = z
            if -l1 <= z <= l1:
                nw = np.float32(0)
            else:
                eta = (beta + cg_new) / alpha
                nw = np.float32((z - l1 if z > 0 else z + l1) / eta)
            self._w[s] = nw
            if w == 0 and nw != 0:
                self._stats[0] += 1
                if self.vstride > 0 and self._cnt[s] > threshold and self._vrow[s] < 0:
                    self._alloc_v(s, seed, v_init)
            elif w != 0 and nw == 0:
                self._stats[0] -= 1
            if self.vstride > 0 and vid_all[i] >= 0:
                row = self._vrow[s]
                if row >= 0:
                    v = self._V[row]
                    cgv = self._VG[row]
                    gv = gv_all[vid_all[i]].astype(np.float32) + v_l2 * v
                    cgv[:] = np.sqrt(cgv * cgv + gv * gv)
                    v -= v_alpha / (cgv + v_beta) * gv

    # ----------------------------------------------- multi-shard (psx) ops
    def ps_open(self, keys, use_cnt, segS, segHS, rows_cap, insert, chains, h, threshold,
                l1_shrk, seed):
        """Owner side of a P-shard minibatch (host oracle of psx.hip ps_open):
        segments in peer order, each one find/insert + count push (the lane
        whose add crosses the threshold allocates) + variable-length pull
        into the row-aligned reply buffer. Returns (slot, vpos, chain, head,
        rbuf, vcnt); chain / head are unused on the host (duplicates are
        applied in peer order by ps_push)."""
        if keys.dtype == torch.int32:
            rec = keys.reshape(-1, 3).numpy()
            ks = (rec[:, 0].astype(np.int64) & 0xFFFFFFFF) | (rec[:, 1].astype(np.int64) << 32)
            cnt = rec[:, 2].astype(np.int64) if use_cnt else None
        else:
            ks = keys.numpy().astype(np.int64)
            cnt = None
        n = ks.shape[0]
        S = [int(x) for x in segS.tolist()]
        HS = [int(x) for x in segHS.tolist()]
        P = len(S) - 1
        vs = self.vstride
        slot = self.find(torch.from_numpy(ks), insert).numpy()
        if vs == 0:  # linear: the reply is w, one float per key
            w = np.where(slot >= 0, self._w[np.maximum(slot, 0)], 0).astype(np.float32)
            return (torch.from_numpy(slot.astype(np.int32)), torch.zeros(n + 1, dtype=torch.int64),
                    torch.zeros(n, dtype=torch.int32), torch.ones(n, dtype=torch.uint8),
                    torch.from_numpy(w), torch.zeros(P, dtype=torch.int64))
        w = np.zeros(n, dtype=np.float32)
        rows = np.full(n, -1, dtype=np.int64)
        for i in range(n):
            s = int(slot[i])
            if s < 0:
                continue
            if cnt is not None:
                old = int(self._cnt[s])
                new = old + int(cnt[i])
                self._cnt[s] = np.uint32(new)
                if (vs > 0 and old <= threshold < new and self._vrow[s] < 0
                        and (not l1_shrk or self._w[s] != 0)):
                    self._alloc_v(s, seed, h[7])
            w[i] = self._w[s]
            r = int(self._vrow[s]) if vs > 0 else -1
            if l1_shrk and w[i] == 0:
                r = -1
            rows[i] = r
        flag = (rows >= 0).astype(np.int64)
        vpos = np.zeros(n + 1, dtype=np.int64)
        vpos[1:] = np.cumsum(flag)
        rbuf = np.zeros((rows_cap, max(vs, 1)), dtype=np.float32)
        vcnt = np.zeros(P, dtype=np.int64)
        for p in range(P):
            a, b = S[p], S[p + 1]
            vs0 = int(vpos[a])
            vcnt[p] = int(vpos[b]) - vs0
            flat = rbuf.reshape(-1)
            base = (HS[p] + vs0) * vs
            for i in range(a, b):
                j = int(vpos[i] - vs0) if rows[i] >= 0 else -1
                flat[base + 2 * (i - a)] = w[i]
                flat[base + 2 * (i - a) + 1:base + 2 * (i - a) + 2].view(np.int32)[0] = j
                if rows[i] >= 0:
                    rbuf[HS[p + 1] + int(vpos[i])] = self._V[rows[i]]
        return (torch.from_numpy(slot.astype(np.int32)), torch.from_numpy(vpos),
                torch.zeros(n, dtype=torch.int32), torch.ones(n, dtype=torch.uint8),
                torch.from_numpy(rbuf), torch.from_numpy(vcnt))

    def ps_push(self, slot, vpos, chain, head, segS, segHS, gbuf, h, threshold, l1_shrk, seed):
        """Owner side push of a P-shard minibatch: every peer's segment in
        peer order (ps-lite server: one request at a time)."""
        S = [int(x) for x in segS.tolist()]
        HS = [int(x) for x in segHS.tolist()]
        vs = self.vstride
        vp = vpos.numpy()
        flat = gbuf.reshape(-1).numpy()
        for p in range(len(S) - 1):
            a, b = S[p], S[p + 1]
            if b <= a:
                continue
            vs0 = int(vp[a])
            gw = flat[(HS[p] + vs0) * vs + np.arange(b - a)]
            vid = np.where(vp[a + 1:b + 1] > vp[a:b], vp[a:b] - vs0, -1).astype(np.int32)
            hdr = np.zeros((b - a, 2), dtype=np.float32)
            hdr.view(np.int32)[:, 1] = vid
            nv = int(vp[b] - vs0)
            gv = gbuf.reshape(-1, max(vs, 1))[HS[p + 1] + vs0:HS[p + 1] + vs0 + nv]
            self.difacto_push(slot[a:b], torch.from_numpy(hdr), torch.from_numpy(gw.copy()),
                              gv.contiguous(), h, threshold, l1_shrk, seed)

    def ps_push_linear(self, slot, chain, head, segS, g, algo, alpha, beta, l1, l2, t0):
        """Linear owner push of a P-shard minibatch: segment p (peer p's
        request) in peer order; SGD's request counter t = t0 + p + 1."""
        S = [int(x) for x in segS.tolist()]
        for p in range(len(S) - 1):
            a, b = S[p], S[p + 1]
            if b > a:
                eta = (beta + (t0 + p + 1) ** 0.5) / alpha
                self.linear_push(slot[a:b], g[a:b], algo, alpha, beta, l1, l2, eta)

    def grow(self, newcap):
        """Host table: capacity bookkeeping only (slots never move)."""
        if newcap <= self.cap:
            raise ValueError("grow: new capacity must be larger")
        self.cap = int(newcap)
        return torch.arange(self._keys.shape[0], dtype=torch.int32)

    def grow_v(self, newvcap):
        if newvcap <= self.vcap:
            raise ValueError("grow_v: new capacity must be larger")
        self.vcap = int(newvcap)

    def summary(self):
        return torch.tensor([self._n, self._stats[2], self._stats[3], self._vnext],
                            dtype=torch.int64)
