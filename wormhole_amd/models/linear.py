"""Linear models trained by asynchronous-style minibatch SGD / AdaGrad / FTRL
with an L1/L2 proximal step (reference learn/linear/).

Per minibatch (reference AsgdWorker::ProcessMinibatch,
learn/linear/async_sgd.h:240-288): localize -> key all-to-all -> pull w ->
fused SpMV forward + loss + dual + metrics -> AUC -> segmented SpMV^T
backward -> push -> owner applies the fused proximal update.
"""
import torch

from .. import ops
from ._pipeline import localize_pipelined
from ..kv import ShardedKV, make_store
from ..parallel.comm import LoopbackComm
from ..utils import trace

TRAIN, VAL, PRED = 0, 1, 2
# one GPU, one shard: the localize-free native step (per-tile de-duplication,
# csrc/bind/hip_ops.cc LinearStep) up to ~15k Criteo rows; False keeps the
# localize path at every size (the tests' cross-check of the two)
DIRECT_STEP = True


class LinearLearner:
    def __init__(self, conf, comm, device, cap=1 << 22, seed=0, nshard=None):
        self.conf = conf
        self.comm = comm
        self.device = torch.device(device)
        self.store = make_store(cap, 0, 0, self.device)
        self.kv = ShardedKV(self.store, comm, nshard)
        # ps-lite COMPRESSING filter on the pushes / pulls (host transfers)
        if hasattr(comm, "set_compression"):
            comm.set_compression(getattr(conf, "msg_compression", False))
        self.seed = seed
        self.alpha = conf.lr_eta
        self.beta = conf.lr_beta
        # [objv, -, correct, count, sum of per-minibatch accuracies flipped
        # below 0.5] (learn/base/binary_class_evaluation.h:40-51 +
        # learn/linear/loss.h:85), all summed by the forward kernel
        self.met = torch.zeros(5, dtype=torch.float64, device=self.device)
        self.auc_sum = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.n_mb = 0
        self.max_key = 0  # set from the -max_key system flag (apps/ps_app.py)
        self._job = None  # (keys, localize job) begun for the next minibatch
        self.uhint = 0  # unique ids of the previous minibatch (localize table size)
        # overlap each push's all-to-all with the next minibatch's localize
        # (same semantics: the push is applied before the next lookup)
        self.defer_push = True
        # the attributes the multi-shard step reads (kv/psx.py)
        self.loss = conf.loss
        self.hp = [0.0] * 8   # (no embedding: DiFacto's hyper-parameters unused)
        self.threshold = 0
        self.l1_shrk = False
        self.emb = None
        self.dim = 0
        self.step = 0
        self.last_sizes = None
        self.last_empty = False
        # P > 1 ranks: the lean pipelined exchange (kv/psx.py) over S <= P
        # server shards: keys out, w back, gradients out, one owner launch
        self.psx = None
        if comm.size > 1:
            from ..kv.psx import Psx
            self.psx = Psx(self)
        # one GPU, one shard: the whole step is one native call
        # (csrc/bind/hip_ops.cc LinearStep) -- at the reference's minibatch
        # of 10000 rows the Python glue of the step cost more host time than
        # the GPU work it launches
        self._native = None
        if (self.device.type == "cuda" and comm.size == 1 and self.kv.nshard == 1
                and not isinstance(comm, LoopbackComm)):
            from .. import _native
            self._native = _native.hip().LinearStep(
                store=self.store, algo=int(conf.algo), alpha=conf.lr_eta, beta=conf.lr_beta,
                l1=conf.lambda_l1, l2=conf.lambda_l2, loss=int(conf.loss),
                max_load=self.kv.guard.max_load, direct=DIRECT_STEP)

    def _localize(self, keys, offset, val, next_batch):
        return localize_pipelined(self, keys, offset, val, next_batch)

    def psx_linear_hp(self):
        """Owner update of the multi-shard step (kv/psx.py): the conf's
        SGD / AdaGrad / FTRL (learn/linear/async_sgd.h:71-180)."""
        c = self.conf
        return int(c.algo), float(self.alpha), float(self.beta), float(c.lambda_l1), float(
            c.lambda_l2)

    def process(self, keys, offset, val, label, wtype=TRAIN, data_pass=0, next_batch=None):
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
        if self._native is not None and not self.max_key:
            nk = no = nv = None
            ready = 0
            if next_batch is not None:
                nk, no, nv = next_batch[:3]
                if len(next_batch) > 3 and next_batch[3] is not None:
                    ready = next_batch[3].cuda_event
            py = self._native.step(keys, offset, val, label, train, self.met, self.auc_sum,
                                   nk, no, nv, ready)
            if label.numel():
                self.n_mb += 1
            return py if wtype == PRED else None
        with trace.span("localize"):
            loc = self._localize(keys, offset, val, next_batch)
        uniq, ucnt, owner_cnt, lid, csc_off, csc_row, csc_val = loc[:7]
        self.uhint = uniq.numel()
        with trace.span("pull"):
            sess = self.kv.open(uniq, owner_cnt, insert=train,
                                recv=loc[7] if len(loc) > 7 else None)
            w = self.kv.linear_pull(sess)
        with trace.span("forward"):
            py, dual, _ = ops.fm_forward(offset, lid, val, w, None, 0, label, self.conf.loss,
                                         self.met)
            ops.auc_acc(py, label, self.auc_sum)
        if label.numel():
            self.n_mb += 1
        if train:
            with trace.span("backward"):
                grad, _ = ops.fm_backward(csc_off, csc_row, csc_val, dual, None, w, None, 0)
            with trace.span("push"):
                self.kv.linear_push(sess, grad, self.conf.algo, self.alpha, self.beta,
                                    self.conf.lambda_l1, self.conf.lambda_l2,
                                    defer=self.defer_push)
        return py if wtype == PRED else None

    def flush(self):
        """Complete the last minibatch's deferred push (before reading the
        model: progress counters, save, end of pass, end of a timed run)."""
        if self.psx is not None:
            self.psx.flush()
        if self._native is not None:
            self._native.reset()  # (a localize begun for a minibatch never trained)
            self._native.guard_sync()  # a failed insert raises here at the latest
            self.kv.guard.grows = self._native.grows
        self.kv.flush()

    def take_progress(self):
        """Reference layout (learn/linear/progress.h): [objv, acc, auc, count,
        new_ex, new_w]; accuracy is the per-minibatch-mean convention.

        Local only (no collectives: a worker reports on its own clock);
        minibatches still in the multi-shard pipeline count in the next
        report, and the end of a pass flushes first."""
        self.kv.flush()
        ops.auc_join(self.auc_sum)
        m = self.met.tolist()
        a = float(self.auc_sum.item())
        st = self.store.stats
        new_w = float(st.tolist()[0])
        self.store.reset_stats(0, 1)
        prog = [m[0], m[4], a, float(self.n_mb), m[3], new_w]
        self.met.zero_()
        self.auc_sum.zero_()
        self.n_mb = 0
        return prog
