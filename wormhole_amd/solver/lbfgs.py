"""Distributed vector-free OWL-QN L-BFGS (reference learn/solver/lbfgs.h:56-663,
SURVEY C22).

The 2m+1 history vectors (m weight deltas s, m gradient deltas y, and the
steepest-descent direction) are sharded by parameter range: each rank keeps
only its ``[range_begin, range_end)`` slice in device memory (8-aligned,
lbfgs.h:126-136).  Per iteration the ranks compute the <= 5n new partial dot
products with ONE batched device reduction, allreduce them (<= 50 doubles),
run the scalar two-loop recursion on the (2m+1)^2 dot basis, build their
direction slice as one skinny GEMV (coef[2m+1] @ H[2m+1, nsub]) and
all-gather the slices (the reference allreduces a zero-padded full vector).
Backtracking Armijo line search; OWL-QN pseudo-gradient and sign fixing for
L1.  State is checkpointed every iteration through :class:`BSP`.
"""
import math

import torch

from .. import _native


class LBFGSSolver:
    def __init__(self, bsp, obj):
        self.bsp = bsp
        self.obj = obj
        self.device = obj.device
        self.reg_L1 = 0.0
        self.max_linesearch_iter = 100
        self.linesearch_backoff = 0.5
        self.linesearch_c1 = 1e-4
        self.min_lbfgs_iter = 5
        self.max_lbfgs_iter = 500
        self.lbfgs_stop_tol = 1e-5
        self.size_memory = 10
        self.num_dim = 0
        self.silent = False

    def set_param(self, name, val):
        conv = {"num_dim": int, "size_memory": int, "reg_L1": float, "lbfgs_stop_tol": float,
                "linesearch_backoff": float, "max_linesearch_iter": int,
                "max_lbfgs_iter": int, "min_lbfgs_iter": int, "linesearch_c1": float}
        if name in conv:
            setattr(self, name, conv[name](val))

    # ----------------------------------------------------------- indexing
    def _map(self, i):
        m = self.size_memory
        if i == 2 * m:
            return i
        if i < m:
            return (i + self.offset) % m
        return (i + self.offset) % m + m

    def _dot_idx(self, i, j):
        if i > j:
            i, j = j, i
        return self._map(i), self._map(j)

    def dotbuf(self, i, j):
        a, b = self._dot_idx(i, j)
        return self.data[a, b]

    def _set_dotbuf(self, i, j, v):
        a, b = self._dot_idx(i, j)
        self.data[a, b] = v

    def H(self, i):
        return self.hist[self._map(i), : self.nsub]

    # --------------------------------------------------------------- init
    def init(self):
        bsp = self.bsp
        version, g, loc = bsp.load_checkpoint()
        if version == 0:
            self.num_dim = int(self.obj.init_num_dim())
        else:
            print("restart from version=%d" % version, flush=True)
            self.size_memory = int(g["size_memory"])
            self.num_dim = int(g["num_dim"])
        nproc, rank = bsp.world, bsp.rank
        step = (self.num_dim + nproc - 1) // nproc
        step = (step + 7) // 8 * 8
        self.step = step
        self.rb = min(rank * step, self.num_dim)
        self.re = min((rank + 1) * step, self.num_dim)
        self.nsub = self.re - self.rb
        m = self.size_memory
        dev = self.device
        # rows padded to a multiple of 4 floats (16-byte rows for the
        # history kernels); the padding stays zero
        self.hist = torch.zeros(2 * m + 1, (self.nsub + 3) // 4 * 4, dtype=torch.float32,
                                device=dev)
        if version == 0:
            self.num_iteration = 0
            self.offset = 0
            self.num_useful = 0
            self.data = torch.zeros(2 * m + 1, 2 * m + 1, dtype=torch.float64)
            self.weight = self.obj.init_model(self.num_dim).to(dev)
            bsp.broadcast(self.weight, 0)
            self.old_objval = self.eval(self.weight)
            self.init_objval = self.old_objval
            if not self.silent:
                bsp.tracker_print(
                    "L-BFGS solver starts, num_dim=%d, init_objval=%g, size_memory=%d, "
                    "RAM-approx=%d" % (self.num_dim, self.init_objval, m,
                                       4 * 3 * self.num_dim + 4 * (2 * m + 1) * self.nsub))
        else:
            self.num_iteration = int(g["num_iteration"])
            self.init_objval = float(g["init_objval"])
            self.old_objval = float(g["old_objval"])
            self.offset = int(g["offset"])
            self.data = g["data"].clone()
            self.weight = g["weight"].to(dev)
            self.obj.load_state(g["obj"])
            self.num_useful = int(loc["num_useful"])
            for i in range(self.num_useful):
                self.H(i).copy_(loc["s"][i].to(dev))
                self.H(i + m).copy_(loc["y"][i].to(dev))

    def _state(self):
        m = self.size_memory
        g = {"size_memory": m, "num_iteration": self.num_iteration, "num_dim": self.num_dim,
             "init_objval": self.init_objval, "old_objval": self.old_objval,
             "offset": self.offset, "data": self.data.clone(),
             "weight": self.weight.detach().cpu().clone(), "obj": self.obj.save_state()}
        loc = {"num_useful": self.num_useful,
               "s": torch.stack([self.H(i).cpu() for i in range(self.num_useful)])
               if self.num_useful else torch.zeros(0),
               "y": torch.stack([self.H(i + m).cpu() for i in range(self.num_useful)])
               if self.num_useful else torch.zeros(0)}
        return g, loc

    # ---------------------------------------------------------- iteration
    def eval(self, w, l1norm=None):
        """l1norm: |w|_1 when the caller already has it (the fused step)."""
        val = self.bsp.allreduce_scalar(float(self.obj.eval(w)))
        if self.reg_L1 != 0.0:
            if l1norm is None:
                l1norm = float(w.abs().sum(dtype=torch.float64))
            val += l1norm * self.reg_L1
        return val

    def update_one_iter(self):
        g = self.obj.calc_grad(self.weight)
        self.bsp.allreduce(g)
        d, vdot = self.find_change_direction(g, self.weight)
        new_w, it = self.backtrack_line_search(d, self.weight, vdot)
        if it >= self.max_linesearch_iter:
            raise RuntimeError("line search failed")
        self.weight = new_w
        if self.num_iteration > self.min_lbfgs_iter:
            if self.old_objval - self.new_objval < self.lbfgs_stop_tol * self.init_objval:
                return True
        if not self.silent:
            self.bsp.tracker_print(
                "[%d] L-BFGS: linesearch finishes in %d rounds, new_objval=%g, improvment=%g" % (
                    self.num_iteration, it, self.new_objval, self.old_objval - self.new_objval))
        self.old_objval = self.new_objval
        # (the state -- weights and the history slices -- is copied to the
        # host only when checkpoints are written: 1.4 GB per iteration at
        # 2^24 weights)
        v = self.bsp.checkpoint(*self._state()) if self.bsp.ckpt_dir else self.bsp.checkpoint(None)
        from ..parallel.bsp import fault_point
        fault_point(self.bsp.rank, v)
        return False

    def run(self):
        self.init()
        while self.num_iteration < self.max_lbfgs_iter:
            if self.update_one_iter():
                break
        if not self.silent:
            nz = int((self.weight != 0).sum())
            self.bsp.tracker_print("L-BFGS: finishes at iteration %d, %d/%d active weights" % (
                self.num_iteration, nz, self.num_dim))
        return self.weight

    # ------------------------------------------------------------ OWL-QN
    def set_l1_dir(self, grad, weight):
        l1 = self.reg_L1
        if grad.is_cuda:  # csrc/hip/lbfgs.hip k_owlqn_dir
            return _native.hip().owlqn_dir(grad.contiguous(), weight.contiguous(), float(l1))
        if l1 == 0.0:
            return -grad
        d = torch.where(weight > 0, -grad - l1, torch.where(weight < 0, -grad + l1, torch.zeros_like(grad)))
        zero = weight == 0
        d = torch.where(zero & (grad < -l1), -grad - l1, d)
        d = torch.where(zero & (grad > l1), -grad + l1, d)
        return d

    def fix_dir_l1_sign(self, d, steep):
        if self.reg_L1 != 0.0:
            d = torch.where(d * steep <= 0, torch.zeros_like(d), d)
        return d

    def fix_weight_l1_sign(self, new_w, w):
        if self.reg_L1 != 0.0:
            new_w = torch.where(new_w * w < 0, torch.zeros_like(new_w), new_w)
        return new_w

    def find_change_direction(self, grad, weight):
        m = self.size_memory
        n = self.num_useful
        rb, re = self.rb, self.re
        gsub = grad[rb:re]
        if n != 0:
            y_last = self.H(m + n - 1)
            torch.sub(gsub, y_last, out=y_last)  # y_{n-1} = g_new - g_old
            if gsub.is_cuda:  # written in place into the history row
                _native.hip().owlqn_dir(gsub.contiguous(), weight[rb:re].contiguous(),
                                        float(self.reg_L1), self.H(2 * m))
            else:
                self.H(2 * m).copy_(self.set_l1_dir(gsub, weight[rb:re]))
            idx = []
            for j in range(n):
                idx += [(j, 2 * m), (j, n - 1), (j, m + n - 1)]
            for j in range(n):
                idx += [(m + j, 2 * m), (m + j, m + n - 1)]
            # all new partial dots in ONE batched reduction, then one allreduce
            tmp = self._history_dots(idx)
            self.bsp.allreduce(tmp)
            tmp = tmp.cpu()
            pa, pb = zip(*(self._dot_idx(a, b) for a, b in idx))
            self.data[list(pa), list(pb)] = tmp.to(self.data.dtype)
            # two-loop recursion on the dot basis (vector-free), in plain
            # floats over the logical dot matrix (0-d tensor arithmetic here
            # cost milliseconds of host time per iteration)
            R = 2 * m + 1
            phys = self.data.tolist()
            mp = [self._map(i) for i in range(R)]
            D = [[phys[mp[min(i, j)]][mp[max(i, j)]] for j in range(R)] for i in range(R)]
            alpha = [0.0] * n
            delta = [0.0] * R
            delta[2 * m] = 1.0
            for j in range(n - 1, -1, -1):
                vsum = sum(delta[k] * D[k][j] for k in range(R))
                alpha[j] = vsum / D[j][m + j]
                delta[m + j] -= alpha[j]
            scale = D[n - 1][m + n - 1] / D[m + n - 1][m + n - 1]
            delta = [x * scale for x in delta]
            for j in range(n):
                vsum = sum(delta[k] * D[k][m + j] for k in range(R))
                beta = vsum / D[j][m + j]
                delta[j] += alpha[j] - beta
            steep = self.H(2 * m)
            if self.hist.is_cuda:
                # d = sum delta_k H_k in the reference's AddScale order (y rows,
                # the steepest direction, s rows), sign fix + dot: ONE pass
                # over the history (lbfgs.hip k_dir_fix_dot)
                order = list(range(m, m + n)) + [2 * m] + list(range(n))
                dirsub, v = _native.hip().dir_fix_dot(
                    self.hist, [self._map(k) for k in order], [delta[k] for k in order],
                    self._map(2 * m), self.reg_L1 != 0.0, self.nsub)
                vdot = -float(v)
            else:
                coef = torch.zeros(2 * m + 1, dtype=torch.float32)
                for k in list(range(n)) + list(range(m, m + n)) + [2 * m]:
                    coef[self._map(k)] = delta[k]
                dirsub = coef.to(self.device) @ self.hist[:, : self.nsub]  # skinny GEMV
                dirsub = self.fix_dir_l1_sign(dirsub, steep)
                vdot = -float((dirsub * steep).sum(dtype=torch.float64))
            d = self._allgather_dir(dirsub)
            vdot = self.bsp.allreduce_scalar(vdot)
        else:
            d = self.set_l1_dir(grad, weight)
            vdot = -float((d * d).sum(dtype=torch.float64))
        if n < m:
            n += 1
        else:
            self.offset = (self.offset + 1) % m
        self.num_useful = n
        self.H(m + n - 1).copy_(gsub)
        return d, vdot

    def _history_dots(self, idx):
        """fp64 <H_a, H_b> for the (a, b) index pairs of FindChangeDirection.
        Every pair's b is one of three probe rows (the steepest direction and
        the newest s / y), so on the GPU all rows are dotted with the probes
        in one pass (lbfgs.hip k_hist_dots) and the pairs picked out."""
        ia = [self._map(a) for a, _ in idx]
        ib = [self._map(b) for _, b in idx]
        if not self.hist.is_cuda:
            a, b = torch.tensor(ia), torch.tensor(ib)
            return (self.hist[a] * self.hist[b]).sum(1, dtype=torch.float64)
        probes = sorted(set(ib))
        if len(probes) <= 4:
            out = _native.hip().hist_dots(self.hist, probes)
            col = {p: k for k, p in enumerate(probes)}
            sel = torch.tensor([a * len(probes) + col[b] for a, b in zip(ia, ib)],
                               device=self.device)
            return out.view(-1)[sel]
        return _native.hip().multi_dot(self.hist[:, : self.nsub].contiguous(),
                                       torch.tensor(ia, device=self.device).int(),
                                       torch.tensor(ib, device=self.device).int())

    def _allgather_dir(self, dirsub):
        if self.bsp.world == 1:
            return dirsub
        pad = torch.zeros(self.step, dtype=dirsub.dtype, device=dirsub.device)
        pad[: dirsub.numel()] = dirsub
        parts = self.bsp.comm.allgather(pad)
        return torch.cat(parts)[: self.num_dim]

    def backtrack_line_search(self, d, w, vdot):
        if not vdot < 0.0:
            raise RuntimeError("not a descent direction (dot=%g)" % vdot)
        alpha = 1.0
        backoff = self.linesearch_backoff
        if self.num_iteration == 0:
            alpha = 1.0 / math.sqrt(-vdot)
            backoff = 0.1
        it = 0
        old_val = self.old_objval
        c1 = self.linesearch_c1
        new_w = None
        while True:
            it += 1
            if it >= self.max_linesearch_iter:
                return new_w, it
            if w.is_cuda:  # step + sign fix + |w|_1 in one pass (k_owlqn_step)
                new_w, l1 = _native.hip().owlqn_step(w.contiguous(), d.contiguous(), alpha,
                                                     self.reg_L1 != 0.0)
                new_val = self.eval(new_w, float(l1) if self.reg_L1 != 0.0 else None)
            else:
                new_w = self.fix_weight_l1_sign(w + d * alpha, w)
                new_val = self.eval(new_w)
            if new_val - old_val <= c1 * vdot * alpha:
                self.new_objval = new_val
                break
            alpha *= backoff
        torch.sub(new_w[self.rb:self.re], w[self.rb:self.re], out=self.H(self.num_useful - 1))
        self.num_iteration += 1
        return new_w, it
