"""DiFacto: distributed factorization machines with frequency-adaptive
embeddings (reference learn/difacto/).

Per minibatch (reference AsyncWorker::ProcessMinibatch,
learn/difacto/async_sgd.h:363-425), re-expressed on the GPU:

  localize (device hash)  ->  key all-to-all  ->  [pass 0: push feature
  counts; owner allocates V lazily for keys with cnt > threshold]  ->  pull
  w / V (variable length: V only where allocated and, with l1_shrk, w != 0)
  ->  fused FM forward + loss + metrics  ->  AUC  ->  fused FM backward
  ->  gradient clip / dropout / normalisation  ->  push  ->  owner applies
  FTRL on w and AdaGrad on V in one fused kernel.
"""

import os

import torch

from .. import ops
from ._pipeline import begin_next, localize_current
from ..kv import ShardedKV, make_store
from ..utils import trace

TRAIN, VAL, PRED = 0, 1, 2


class DifactoLearner:
    def __init__(self, conf, comm, device, cap=1 << 22, vcap=1 << 20, seed=0, nshard=None):
        self.conf = conf
        self.comm = comm
        self.device = torch.device(device)
        emb = conf.embedding[0] if conf.embedding else None
        self.dim = emb.dim if emb is not None else 0
        self.emb = emb
        self.vstride = ops.vstride_for(self.dim)
        self.store = make_store(cap, vcap, self.dim, self.device)
        self.kv = ShardedKV(self.store, comm, nshard, fixed_bytes=getattr(conf, "fixed_bytes", 0),
                            seed=seed)
        # ps-lite COMPRESSING filter on the pushes / pulls (host transfers)
        if hasattr(comm, "set_compression"):
            comm.set_compression(getattr(conf, "msg_compression", False))
        self.seed = seed
        self.l1_shrk = bool(conf.l1_shrk)
        if emb is not None:
            v_alpha = emb.lr_eta if emb.has("lr_eta") else conf.lr_eta
            v_beta = emb.lr_beta if emb.has("lr_beta") else conf.lr_beta
            self.hp = [conf.lr_eta, conf.lr_beta, conf.lambda_l1, conf.lambda_l2,
                       v_alpha, v_beta, emb.lambda_l2, emb.init_scale]
            self.threshold = int(emb.threshold)
        else:
            self.hp = [conf.lr_eta, conf.lr_beta, conf.lambda_l1, conf.lambda_l2,
                       conf.lr_eta, conf.lr_beta, 0.0, 0.01]
            self.threshold = 0
        # device-side progress accumulators (read only when printing)
        self.met = torch.zeros(4, dtype=torch.float64, device=self.device)
        self.auc_sum = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.n_mb = 0
        self.max_key = 0  # set from the -max_key system flag (apps/ps_app.py)
        self._job = None  # (keys, localize job) begun for the next minibatch
        self.uhint = 0  # unique ids of the previous minibatch (localize table size)
        # overlap each push's all-to-all with the next minibatch's localize
        # (same semantics: the push is applied before the next lookup)
        self.defer_push = True
        self.step = 0
        self.last_sizes = None
        self.loss = ops.LOSS_LOGIT
        # True after a process() call in which no rank had data (the pass is
        # over; kv/psx.py reads it from the count exchange's flags)
        self.last_empty = False
        # P > 1 ranks: the lean pipelined exchange (kv/psx.py), whatever the
        # number of server shards S <= P, with or without the fixed_bytes
        # payload filter and embedding.
        # One shard on the GPU: the FM kernels read the V rows in place in the
        # table's slab instead of a pulled copy (kv.difacto_open_pull direct)
        # -- unless the embedding gradients are post-processed (clipping /
        # dropout / normalisation walk the compact gradient rows).
        post = emb is not None and (emb.grad_clipping > 0 or emb.dropout > 0
                                    or bool(emb.grad_normalization))
        self.direct_pull = (self.device.type == "cuda" and comm.size == 1 and self.vstride > 0
                            and not post)
        self.psx = None
        if comm.size > 1:
            from ..kv.psx import Psx
            self.psx = Psx(self)
        # one shard on the GPU: the whole minibatch in one native call
        # (csrc/bind/difacto_step.inl; WH_DIFACTO_NATIVE=0 keeps this
        # module's op-by-op step, the test oracle)
        self._nat = None
        if (self.psx is None and self.device.type == "cuda" and self.vstride > 0
                and os.environ.get("WH_DIFACTO_NATIVE", "1") != "0"):
            from .. import _native
            e = emb
            self._nat = _native.hip().DifactoStep(
                store=self.store, hp=[float(x) for x in self.hp], threshold=self.threshold,
                l1_shrk=self.l1_shrk, seed=int(seed), loss=int(self.loss),
                post=[float(e.grad_clipping), float(e.dropout),
                      1.0 if e.grad_normalization else 0.0, float(self.dim)],
                max_load=float(self.kv.guard.max_load), direct=self.direct_pull)

    def psx_linear_hp(self):
        """Embedding-free model on the multi-shard step's linear wire format:
        the owner applies DiFacto's FTRL on w (push algo 4,
        learn/difacto/async_sgd.h:262-286)."""
        c = self.conf
        return 4, float(c.lr_eta), float(c.lr_beta), float(c.lambda_l1), float(c.lambda_l2)

    # ------------------------------------------------------------------ step
    def process(self, keys, offset, val, label, wtype=TRAIN, data_pass=0, next_batch=None):
        """One minibatch. Returns predictions (py) for PRED, else None."""
        train = wtype == TRAIN
        if self.psx is not None:
            if train:
                self.psx.train(keys, offset, val, label, data_pass, next_batch)
                self.last_empty = self.psx.last_empty
                return None
            py = self.psx.evaluate(keys, offset, val, label)
            self.last_empty = self.psx.last_empty
            return py if wtype == PRED else None
        self.last_empty = offset.numel() <= 1 and self.comm.size == 1
        if self._nat is not None and not self.max_key:
            nk = no = nv = None
            ready = 0
            if next_batch is not None:
                nk, no, nv = next_batch[:3]
                if len(next_batch) > 3 and next_batch[3] is not None:
                    ready = next_batch[3].cuda_event
            py, u, m = self._nat.step(keys=keys, offset=offset, val=val, label=label,
                                      train=train, data_pass=int(data_pass), met=self.met,
                                      auc_sum=self.auc_sum, step=self.step, next_keys=nk,
                                      next_offset=no, next_val=nv, ready=ready)
            self.last_sizes = (u, m)
            if label.numel():
                self.n_mb += 1
            self.step += 1
            return py if wtype == PRED else None
        with trace.span("localize"):
            loc = localize_current(self, keys, offset, val)
        uniq, ucnt, owner_cnt, lid, csc_off, csc_row, csc_val = loc[:7]
        self.uhint = uniq.numel()
        push_cnt = train and data_pass == 0 and self.dim > 0
        with trace.span("pull"):
            sess, hdr, vc = self.kv.difacto_open_pull(
                uniq, owner_cnt, train, ucnt if push_cnt else None, self.hp, self.threshold,
                self.l1_shrk, self.seed, recv=loc[7] if len(loc) > 7 else None,
                direct=self.direct_pull)
        self.last_sizes = (uniq.numel(), sess.m)  # (unique keys, embedding rows; device)
        # The next minibatch's localize begins right AFTER this pull's launch
        # (the host reaches the pull sooner after its count read; the job's
        # count read still comes well before the next call needs it)
        if next_batch is not None:
            begin_next(self, next_batch, uniq.numel())
        if self.vstride == 0:  # no embedding: a plain linear model over w
            hdr, vc = hdr[:, 0].contiguous(), None
        with trace.span("forward"):
            py, dual, xv = ops.fm_forward(offset, lid, val, hdr, vc, self.vstride, label,
                                          ops.LOSS_LOGIT, self.met)
            if not train:  # (a training step's AUC follows its backward)
                ops.auc_acc(py, label, self.auc_sum)
        if label.numel():
            self.n_mb += 1
        if train:
            with trace.span("backward"):
                gw, gvc = ops.fm_backward(csc_off, csc_row, csc_val, dual, xv, hdr, vc,
                                          self.vstride)
                if self.emb is not None and self.vstride > 0:
                    ops.fm_grad_post(gvc, sess.m, self.dim, self.emb.grad_clipping,
                                     self.emb.dropout, self.seed + 7919 * self.step + 1,
                                     bool(self.emb.grad_normalization))
            # the AUC side stream starts behind the backward, so its kernels
            # overlap the push / next open rather than the backward planning
            ops.auc_acc(py, label, self.auc_sum)
            with trace.span("push"):
                self.kv.difacto_push(sess, gw, gvc, self.hp, self.threshold, self.l1_shrk,
                                     self.seed, defer=self.defer_push)
        self.step += 1
        return py if wtype == PRED else None

    # -------------------------------------------------------------- progress
    def flush(self):
        """Complete the last minibatch's deferred push (before reading the
        model: progress counters, save, end of pass, end of a timed run)."""
        if self.psx is not None:
            self.psx.flush()
        if self._nat is not None:  # (its guard's growth counts, for the reports)
            g = self.kv.guard
            g.grows, g.vgrows = max(g.grows, self._nat.grows), max(g.vgrows, self._nat.vgrows)
        self.kv.flush()

    def take_progress(self):
        """Progress vector in the reference layout (learn/difacto/progress.h):
        [objv, auc, objv_w, copc, count, new_ex, new_w, new_V]; resets.

        Local only: it may run at different minibatches on different ranks
        (the worker reports on its own clock), so it must not issue
        collectives -- minibatches still in the multi-shard pipeline are
        counted by the next report; the end of a pass flushes first."""
        self.kv.flush()
        ops.auc_join(self.auc_sum)
        m = self.met.tolist()
        a = float(self.auc_sum.item())
        st = self.store.stats
        st_l = st.tolist()
        prog = [m[0], a, m[1], 0.0, float(self.n_mb), m[3], float(st_l[0]), float(st_l[1])]
        self.met.zero_()
        self.auc_sum.zero_()
        self.n_mb = 0
        self.store.reset_stats(0, 2)
        return prog
