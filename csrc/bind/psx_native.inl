// Native driver of the pipelined multi-shard parameter-server step
// (included by hip_ops.cc after LinearStep; the Python twin, kept as the
// test oracle, is wormhole_amd/kv/psx.py Psx.train).
//
// Reference per-minibatch flow: learn/difacto/async_sgd.h:372-424 (push the
// feature counts -> ZVPull(w, V) -> compute -> ZVPush(gw, gV)) and
// learn/linear/async_sgd.h:240-301 (ZPull w -> gradient -> ZPush), with
// max_concurrency minibatches in flight. A call of PsxStep::train enqueues
// what Psx.train does -- the same four collectives C0..C3 and phases -- but
// from C++: the Python step spent ~300 us of host time per call at the
// reference's minibatch of 10000 rows (~40 Python-level operations and
// stream switches), more than the GPU work it launched. Streams: DiFacto
// runs the compute stream S, the localize stream ls, the count side stream
// cs and the exchange stream xs; the linear step runs everything on S (at
// 10 000 rows host API calls bound the step, and each cross-stream edge
// costs an event record and a wait for an overlap worth less).
//
// Transport (kTx*):
//   kTxRccl     our own RCCL communicator (csrc/bind/rccl_comm.h): every
//               exchange is one grouped ncclSend / ncclRecv per peer on the
//               issuing stream (a 1-rank communicator with P virtual peers
//               in the one-GPU --loopback-rccl rehearsal);
//   kTxStaged   a gloo process group with the ranks sharing one GPU (RCCL
//               refuses two ranks on one device): device -> host, gloo
//               all-to-all-v, host -> device, synchronously; the multi-
//               process correctness rehearsal of the RCCL path;
//   kTxIdentity P virtual shards in one process, no transfer (--loopback).

#include <condition_variable>
#include <thread>
#include <unistd.h>

namespace {

enum PsxTx { kTxIdentity = 0, kTxRccl = 1, kTxStaged = 2 };

struct PsxEv {  // a HIP event shared by an exchange and the watchdog's log
  hipEvent_t e = nullptr;
  explicit PsxEv(bool timing = false) {
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&e, timing ? hipEventDefault : hipEventDisableTiming));
  }
  PsxEv(const PsxEv&) = delete;
  PsxEv& operator=(const PsxEv&) = delete;
  ~PsxEv() {
    if (e) (void)hipEventDestroy(e);
  }
};
using PsxEvP = std::shared_ptr<PsxEv>;

struct PsxWork {  // an issued exchange and the tensor it reads
  Tensor keep;
  PsxEvP ev;  // end of the transfer on the exchange stream
  bool pending = false;
  PsxWork() = default;
  PsxWork(const PsxWork&) = delete;
  PsxWork& operator=(const PsxWork&) = delete;
  void wait() {  // the current stream waits for the transfer
    if (pending)
      WH_HIP_CHECK_HOST(hipStreamWaitEvent(c10::hip::getCurrentHIPStream().stream(), ev->e, 0));
    pending = false;
    keep = Tensor();
  }
};

// ------------------------------------------------------------ watchdog
// A multi-rank step that stops making progress -- a peer that never posts
// its half of an exchange, a transport error, mismatched collectives --
// would otherwise hang until an outer launcher kills the job, with no
// record of what stalled. The watchdog thread watches the step's host side:
// while a PsxStep call is running, the host must pass a phase mark (an
// exchange issued, a host read returned) at least every `deadline` seconds,
// and no RCCL communicator of the step may report an asynchronous error.
// On a breach it prints the rank, the step, the phase the host is blocked
// in and the recent exchanges -- class C0..C3, step, issuing stream, rows
// per peer, and whether each has completed on the device -- then aborts the
// communicators and ends the process with exit status 3 (a plain exit, no
// re-exec). WH_RCCL_TIMEOUT_S sets the deadline (default 120 s).
//
// (ps-lite's van dies on a lost peer through its heartbeat timeout; c10d's
// own watchdog covers the collectives issued through torch.distributed.)
struct PsxXLog {
  int cls = -1;
  int64_t step = -1;
  const char* stream = "";
  std::vector<int64_t> send, recv;
  PsxEvP ev;  // completion on the issuing stream (null: not tracked)
};

class PsxWatchdog {
 public:
  static constexpr int kExit = 3;
  PsxWatchdog(int rank, double deadline_s, std::vector<std::shared_ptr<RcclComm>> comms)
      : rank_(rank), deadline_(deadline_s), comms_(std::move(comms)) {
    beat_ = now();
    th_ = std::thread([this] { run(); });
  }
  PsxWatchdog(const PsxWatchdog&) = delete;
  PsxWatchdog& operator=(const PsxWatchdog&) = delete;
  ~PsxWatchdog() {
    {
      std::lock_guard<std::mutex> l(m_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  double deadline() const { return deadline_; }

  // a PsxStep call begins / ends (the deadline applies in between only: the
  // host may legitimately spend any time elsewhere, e.g. reading input)
  void enter(const char* call, int64_t step) {
    std::lock_guard<std::mutex> l(m_);
    depth_++;
    phase_ = call;
    cls_ = -1;
    step_ = step;
    beat_ = now();
  }
  void leave() {
    std::lock_guard<std::mutex> l(m_);
    depth_ = std::max(0, depth_ - 1);
    beat_ = now();
  }
  // the host passed a mark: `what` (of exchange class cls, -1 none)
  void phase(const char* what, int cls, int64_t step) {
    std::lock_guard<std::mutex> l(m_);
    phase_ = what;
    cls_ = cls;
    step_ = step;
    beat_ = now();
  }
  void log(PsxXLog&& x) {
    std::lock_guard<std::mutex> l(m_);
    ring_[ri_ % kLog] = std::move(x);
    ++ri_;
  }

 private:
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static std::string rows(const std::vector<int64_t>& v) {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) s += (i ? "," : "") + std::to_string(v[i]);
    return s + "]";
  }
  void run() {
    std::unique_lock<std::mutex> l(m_);
    while (!stop_) {
      cv_.wait_for(l, std::chrono::milliseconds(200));
      if (stop_ || depth_ == 0) continue;
      std::string why;
      for (size_t i = 0; i < comms_.size() && why.empty(); ++i) {
        const std::string e = comms_[i] ? comms_[i]->async_error_str() : std::string();
        if (!e.empty() && e.find("in progress") == std::string::npos)
          why = "RCCL communicator " + std::to_string(i) + " reports an asynchronous error: " + e;
      }
      const double idle = now() - beat_;
      if (why.empty() && idle > deadline_) {
        char b[160];
        std::snprintf(b, sizeof b, "no progress for %.1f s (deadline %.0f s, WH_RCCL_TIMEOUT_S)",
                      idle, deadline_);
        why = b;
      }
      if (!why.empty()) fail(why, idle);  // (holds the lock: the owner stays blocked)
    }
  }
  [[noreturn]] void fail(const std::string& why, double idle) {
    std::fprintf(stderr, "[psx watchdog] rank %d: %s\n", rank_, why.c_str());
    std::fprintf(stderr,
                 "[psx watchdog] rank %d: host blocked in '%s'%s%s of step %lld for %.1f s\n",
                 rank_, phase_, cls_ >= 0 ? " of C" : "",
                 cls_ >= 0 ? std::to_string(cls_).c_str() : "", (long long)step_, idle);
    const int64_t n = std::min<int64_t>(ri_, kLog);
    for (int64_t i = ri_ - n; i < ri_; ++i) {
      const PsxXLog& x = ring_[i % kLog];
      const char* st = "issued";
      if (x.ev) st = hipEventQuery(x.ev->e) == hipSuccess ? "done" : "PENDING";
      std::fprintf(stderr,
                   "[psx watchdog] rank %d:   C%d of step %lld on %s: send rows %s recv rows %s "
                   "-- %s\n",
                   rank_, x.cls, (long long)x.step, x.stream, rows(x.send).c_str(),
                   rows(x.recv).c_str(), st);
    }
    // (ncclCommAbort can itself wait on a stuck proxy or kernel: it gets a
    // thread of its own and a few seconds; the exit does not wait longer)
    auto fin = std::make_shared<std::atomic<bool>>(false);
    auto comms = comms_;
    std::thread([comms, fin] {
      for (auto& c : comms)
        if (c) c->abort();
      fin->store(true);
    }).detach();
    for (int i = 0; i < 100 && !fin->load(); ++i)
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    std::fprintf(stderr, "[psx watchdog] rank %d: communicators %s, exiting with status %d\n",
                 rank_, fin->load() ? "aborted" : "abort still pending after 5 s", kExit);
    std::fflush(stderr);
    std::fflush(stdout);
    ::_exit(kExit);
  }

  static constexpr int kLog = 16;
  const int rank_;
  const double deadline_;
  std::vector<std::shared_ptr<RcclComm>> comms_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
  int depth_ = 0;
  const char* phase_ = "";
  int cls_ = -1;
  int64_t step_ = 0;
  double beat_ = 0;
  PsxXLog ring_[kLog];
  int64_t ri_ = 0;
  std::thread th_;
};

// WH_FAULT=xstall:<rank>:<step>: that rank stops before its first exchange
// of that step and never posts it (the peers' watchdogs must catch it)
void parse_xstall(int64_t rank, int64_t* step) {
  *step = -1;
  const char* f = std::getenv("WH_FAULT");
  long long r = -1, s = -1;
  if (f && std::sscanf(f, "xstall:%lld:%lld", &r, &s) == 2 && r == rank) *step = s;
}

struct PsxSt {  // one minibatch in flight (kv/psx.py _Step)
  bool train = false, use_cnt = false, have_v = false;
  int64_t U = 0, seed_step = 0;
  std::vector<int64_t> send, recv, Hw, Ho, vown, vrecv;
  Tensor label, uniq, ucnt, lid, offset, val, csc_off, csc_row, csc_val;
  Tensor tabs, segS_w, segHS_w, segS_o, segHS_o, vrecv_d;
  Tensor keys_o, slot, vpos, chain, head, rbuf, vcnt;
  Tensor rrecv, hdr, rows, py, dual, xv, gpush, gvc;
  // fixed_bytes filter: the receiving side's region table (device) and float
  // extent of C2 / C3's wire rows (q2_desc / q3_desc undefined: exact floats)
  Tensor q2_desc, q3_desc;
  int64_t q2_ext = 0, q3_ext = 0;
  // C2 / C3 wait for these only: the open's and the backward's ends on S
  // (the step's own pair from PsxStep::sev_, recorded once each)
  hipEvent_t ev_open = nullptr, ev_grad = nullptr;
  hipEvent_t own_open = nullptr, own_grad = nullptr;
  PsxWork w_c1, w_c2, w_c3;
};
using PsxStP = std::shared_ptr<PsxSt>;

int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
int64_t vsum(const std::vector<int64_t>& v) { return std::accumulate(v.begin(), v.end(), (int64_t)0); }

// kTxStaged's host all-to-all-v: row-wise alltoall_base over a (gloo)
// process group, exposed for a multi-rank CPU test.
Tensor c10d_rows(const c10::intrusive_ptr<c10d::ProcessGroup>& g, const Tensor& x,
                 const std::vector<int64_t>& send_rows, const std::vector<int64_t>& recv_rows) {
  Tensor xc = x.contiguous();
  int64_t width = 1;
  for (int64_t d = 1; d < xc.dim(); ++d) width *= xc.size(d);
  std::vector<int64_t> shape(xc.sizes().begin(), xc.sizes().end());
  shape[0] = vsum(recv_rows);
  Tensor out = torch::empty(shape, xc.options());
  Tensor of = out.view({-1}), xf = xc.view({-1});
  std::vector<int64_t> rs, ss;
  for (int64_t r : recv_rows) rs.push_back(r * width);
  for (int64_t r : send_rows) ss.push_back(r * width);
  auto w = g->alltoall_base(of, xf, rs, ss);
  if (w) w->wait();
  return out;
}

}  // namespace

class PsxStep {
 public:
  // tx: the transport (PsxTx); pg: the gloo process group of kTxStaged;
  // rccl: the communicator of kTxRccl (P ranks, or 1 for the loopback
  // rehearsal); lin_hp: (algo, alpha, beta, l1, l2) of the linear wire
  // format's owner push; hp / threshold / l1_shrk / seed: DiFacto's
  // (kv/psx.py reads the same from the learner); met / auc_sum: the
  // learner's device progress accumulators.
  PsxStep(KVStore* store, int64_t P, int64_t S, int64_t rank, int64_t tx, py::object pg,
          py::object rccl, bool linear, std::vector<double> lin_hp, std::vector<double> hp,
          int64_t threshold, bool l1_shrk, int64_t seed, int64_t loss, Tensor met, Tensor auc_sum,
          int64_t tau, double max_load, int64_t cu_reserve, std::vector<int64_t> filt,
          std::vector<double> post)
      : store_(store), P_(P), S_(S), rank_(rank), linear_(linear), lin_hp_(std::move(lin_hp)),
        hp_(std::move(hp)), threshold_(threshold), l1_shrk_(l1_shrk), seed_(seed), loss_(loss),
        met_(std::move(met)), auc_sum_(std::move(auc_sum)), tau_(tau), max_load_(max_load) {
    TORCH_CHECK(P >= 2 && S >= 1 && S <= P && rank >= 0 && rank < P, "PsxStep: bad P / S / rank");
    TORCH_CHECK(lin_hp_.size() == 5 && hp_.size() == 8, "PsxStep: hyper-parameter sizes");
    // filt = (fixed_bytes, filter seed): ps-lite's FIXING_FLOAT filter on the
    // exchanged floats (kv/psx.py _QFilter); post = (grad_clipping, dropout,
    // grad_normalization, dim): the embedding-gradient post-processing
    TORCH_CHECK(filt.size() == 2 && post.size() == 4, "PsxStep: filt = (nb, seed), post = "
                "(clip, dropout, normalize, dim)");
    qnb_ = (int)filt[0];
    qseed_ = filt[1];
    TORCH_CHECK(qnb_ >= 0 && qnb_ <= 3, "PsxStep: fixed_bytes must be 0..3");
    clip_ = post[0];
    dropout_ = post[1];
    gnorm_ = post[2] != 0.0;
    pdim_ = (int64_t)post[3];
    post_on_ = !linear && (clip_ > 0 || dropout_ > 0 || gnorm_);
    TORCH_CHECK(tau >= 0 && tau <= kMaxTau, "PsxStep: tau (max_concurrency - 1) must be 0..",
                kMaxTau);
    vs_ = store->vstride();
    TORCH_CHECK(linear_ == (vs_ == 0), "PsxStep: the linear wire format is the vstride-0 store");
    TORCH_CHECK(tx >= kTxIdentity && tx <= kTxStaged, "PsxStep: unknown transport");
    tx_ = (PsxTx)tx;
    if (tx_ == kTxStaged) {
      TORCH_CHECK(!pg.is_none(), "PsxStep: the staged transport needs a process group");
      pg_ = pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>();
      TORCH_CHECK(pg_->getSize() == P && pg_->getRank() == rank,
                  "PsxStep: the process group must have P ranks");
    } else if (tx_ == kTxRccl) {
      // (c0, c1, c23): RCCL runs every operation of ONE communicator in issue
      // order, whatever stream it was issued on, so the count exchange C0 and
      // the keys C1 -- both on the path to the next open -- get
      // communicators of their own instead of queueing behind the big pull /
      // push transfers C2 / C3 of earlier minibatches. One communicator for
      // all three is accepted too (tests).
      TORCH_CHECK(!rccl.is_none(), "PsxStep: the RCCL transport needs a communicator");
      if (py::isinstance<py::sequence>(rccl)) {
        auto seq = rccl.cast<py::sequence>();
        TORCH_CHECK(seq.size() == 3, "PsxStep: rccl = (c0, c1, c23) communicators");
        rccl_c0_ = seq[0].cast<std::shared_ptr<RcclComm>>();
        rccl_c1_ = seq[1].cast<std::shared_ptr<RcclComm>>();
        rccl_ = seq[2].cast<std::shared_ptr<RcclComm>>();
      } else {
        rccl_ = rccl_c0_ = rccl_c1_ = rccl.cast<std::shared_ptr<RcclComm>>();
      }
      for (const auto& c : {rccl_c0_, rccl_c1_, rccl_})
        TORCH_CHECK((c->size() == P && c->rank() == rank) || c->size() == 1,
                    "PsxStep: the communicators must have P ranks (or 1: loopback rehearsal)");
    }
    dev_ = store->slots_.device().index();
    for (const auto& c : {rccl_c0_, rccl_c1_, rccl_})
      TORCH_CHECK(!c || c->device() == dev_, "PsxStep: communicator on another device");
    c10::DeviceGuard g(store->slots_.device());
    // streams of our own (as Python's torch.cuda.Stream()): the pool's
    // round-robin streams are shared with other users, and a localize queued
    // behind a collective on a shared stream serialises the step. The linear
    // step keeps every phase on the compute stream (see the file comment).
    one_ = sx_ = linear_;
    if (!one_) {
      ls_h_ = own_stream(dev_, kStreamPsxLs);
      ls_ = c10::hip::getStreamFromExternal(ls_h_, dev_);
    }
    if (!sx_) {
      cs_h_ = own_stream(dev_, kStreamPsxCs);
      xs_h_ = own_stream(dev_, kStreamPsxXs);
      cs_ = c10::hip::getStreamFromExternal(cs_h_, dev_);
      xs_ = c10::hip::getStreamFromExternal(xs_h_, dev_);
    }
    for (auto& e : ring_) WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : gev_) WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& p : sev_)
      for (auto& e : p) WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (tx_ == kTxRccl) wh::fm_set_cu_reserve((int)cu_reserve);
    const int64_t dflt = std::max<int64_t>(4 * (P + 1) + P, 64);
    for (int i = 0; i < kPins; ++i) {
      pins_[i] = torch::empty({dflt}, torch::TensorOptions().dtype(torch::kInt64).pinned_memory(true));
      WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&pin_ev_[i], hipEventDisableTiming));
    }
    parse_xstall(rank_, &fault_step_);
    if (tx_ != kTxIdentity) {  // (the identity transport cannot stall on a peer)
      const char* t = std::getenv("WH_RCCL_TIMEOUT_S");
      const double dl = t && std::atof(t) > 0 ? std::atof(t) : 120.0;
      std::vector<std::shared_ptr<RcclComm>> cs;
      if (tx_ == kTxRccl) cs = {rccl_c0_, rccl_c1_, rccl_};
      wd_ = std::make_unique<PsxWatchdog>((int)rank_, dl, cs);
    }
    xt_on_ = tx_ == kTxRccl;
    if (timing_on("comm")) xt_every_ = 1;  // WH_TIMING=comm: every exchange timed
    if (qnb_) {
      qW_ = linear_ ? 64 : std::max(vs_, 1);
      qR_ = (4 + qW_ * qnb_ + 3) / 4 * 4;  // ops/ref.py quant_record_bytes
    }
  }

  ~PsxStep() {
    wd_.reset();
    if (timing_) timing_->print();
    job_.reset();
    (void)hipDeviceSynchronize();
    for (auto& e : ring_) (void)hipEventDestroy(e);
    for (auto& e : gev_) (void)hipEventDestroy(e);
    for (auto& p : sev_)
      for (auto& e : p) (void)hipEventDestroy(e);
    for (auto& e : pin_ev_) (void)hipEventDestroy(e);
  }

  // One training minibatch (Psx.train). Returns (has_data, minibatches
  // forwarded, unique keys, embedding rows) of the step whose forward ran.
  py::tuple train(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                  const Tensor& label, int64_t data_pass, const c10::optional<Tensor>& nkeys,
                  const c10::optional<Tensor>& noffset, const c10::optional<Tensor>& nval,
                  int64_t ready) {
    c10::DeviceGuard g(keys.device());
    WdCall wc(wd_.get(), "train", step_);
    // WH_TIMING=step: host us per phase, printed every 1000 calls: s0 job,
    // s1 count read (the host WAIT), s2 tables + C2/C3 issue, s3 localize
    // finish + next begin + C1, s4 reply (forward), s5 owner push, s6 open,
    // s7 C0 of the next job, s8 backward
    HostTimer ht(timing_.get());
    ht_ = timing_ ? &ht : nullptr;
    set_streams();
    fwd_mb_ = 0;
    ensure_job(keys, offset, val);
    ht.mark(0);
    std::vector<int64_t> send, recv;
    const bool empty = counts(send, recv);
    ht.mark(1);
    if (empty) {
      finish_job();
      return py::make_tuple(false, 0, 0, 0);
    }
    PsxStP prev = pull_;
    if (prev && !prev->have_v) vcount_exchange(*prev);
    PsxStP st = new_step(send, recv, label, true, data_pass, prev.get());
    // the open's chain buffer, prepared by the last push before it
    const int64_t n_open = vsum(recv);
    Tensor prep = torch::empty({std::max<int64_t>(n_open, 1)},
                               torch::TensorOptions().dtype(torch::kInt32).device(torch::kCUDA, dev_));
    bool prepped = false;
    // (C2, C3 and C1 stay three RCCL launches: grouped into one, RCCL split
    // the group's several operations per peer over serialised launches and
    // C1, which the open waits for, landed only behind the big C2 / C3 --
    // measured 74 vs 92 M ex/s on the loopback rehearsal)
    if (prev) c2(*prev);
    // the newest push (its backward ran at the end of the previous call)
    if (!pushes_.empty() && pushes_.back()->gvc.defined()) c3(*pushes_.back());
    ht.mark(2);
    set_loc(*st, finish_job(), offset, val);
    const bool early = nkeys.has_value() && nkeys->defined();
    if (early) begin(*nkeys, *noffset, nval, st, ready, true);
    c1(*st);
    ht.mark(3);
    if (prev) {
      reply(*prev);
      if (tau_ == 0 && prev->train) {
        grad(*prev, true);
        owner_push(*prev, prep, n_open);
        prepped = true;
      }
    }
    ht.mark(4);
    // staleness tau: the pull of this minibatch sees every push up to tau
    // minibatches back (each push lands tau - 1 calls after its transfer was
    // issued, max_concurrency = tau + 1 minibatches in flight)
    while (tau_ > 0 && (int64_t)pushes_.size() >= tau_) {
      const bool last = (int64_t)pushes_.size() - 1 < tau_;
      if (last) owner_push(*pushes_.front(), prep, n_open);
      else owner_push(*pushes_.front());
      prepped = prepped || last;
      pushes_.pop_front();
    }
    ht.mark(5);
    open(*st, true, prepped ? prep : Tensor());
    pull_ = st;
    ht.mark(6);
    if (early) exchange_deferred();
    ht.mark(7);
    if (tau_ >= 1 && prev && prev->train) {
      grad(*prev, false);  // C3 goes out behind the next call's C2
      pushes_.push_back(prev);
    }
    ht_ = nullptr;
    ++step_;
    return py::make_tuple(true, fwd_mb_, last_u_, last_v_);
  }

  // Complete every minibatch in flight (Psx.flush). Returns the minibatches
  // forwarded here.
  int64_t flush() {
    c10::DeviceGuard g(store_->slots_.device());
    WdCall wc(wd_.get(), "flush", step_);
    set_streams();
    fwd_mb_ = 0;
    if (!pushes_.empty() && pushes_.back()->gvc.defined()) c3(*pushes_.back());
    if (job_ && job_carried_) {  // the begun job carries the last pull's V counts
      std::vector<int64_t> a, b;
      counts(a, b);
    }
    PsxStP st = pull_;
    if (st) {
      if (!st->have_v) vcount_exchange(*st);
      upload_vrecv(*st);
      c2(*st);
      reply(*st);
      if (st->train) grad(*st, true);
    }
    for (auto& p : pushes_) owner_push(*p);  // in minibatch order
    pushes_.clear();
    if (st && st->train) owner_push(*st);
    pull_.reset();
    return fwd_mb_;
  }

  // drop a begun localize (before the Python step runs an evaluation /
  // read-only pull of its own: every rank does it at the same point)
  void drop_job() {
    WdCall wc(wd_.get(), "drop_job", step_);
    if (job_) {
      if (job_deferred_) {
        c10::hip::HIPStreamGuard sg(ls_);
        job_->exchange();
      }
      std::vector<int64_t> a, b;
      counts(a, b);
      finish_job();
    }
  }

  bool busy() const { return (bool)pull_ || !pushes_.empty() || (bool)job_; }
  std::vector<int64_t> wire() const { return {wire_[0], wire_[1], wire_[2], wire_[3]}; }
  void wire_reset() {
    wire_[0] = wire_[1] = wire_[2] = wire_[3] = 0;
    xt_harvest(true);
    for (int c = 0; c < 4; ++c) xt_us_[c] = 0, xt_n_[c] = 0;
  }
  // sampled GPU time per exchange class C0..C3 (RCCL transport; every
  // 16th step, every step with WH_TIMING=comm; events around the grouped send / recv on its stream;
  // it includes the wait for the slowest peer): {mean us x4, samples x4}
  std::vector<double> xtime() {
    xt_harvest(true);
    std::vector<double> o(8, 0.0);
    for (int c = 0; c < 4; ++c) {
      o[c] = xt_n_[c] ? xt_us_[c] / (double)xt_n_[c] : 0.0;
      o[4 + c] = (double)xt_n_[c];
    }
    return o;
  }
  double watchdog_deadline() const { return wd_ ? wd_->deadline() : 0.0; }
  int64_t grows() const { return grows_; }
  int64_t vgrows() const { return vgrows_; }
  int64_t requests() const { return requests_; }
  void set_requests(int64_t r) { requests_ = r; }
  int64_t step() const { return step_; }
  void set_step(int64_t s) { step_ = s; }
  // the guard's last summary {keys, failed inserts, V overflows, V rows}
  std::vector<int64_t> guard_sync() {
    guard_after(true);
    guard_read();
    return {gkeys_, 0, 0, gvused_};
  }

 private:
  // ------------------------------------------------------------ transport
  Tensor a2a(int c, const Tensor& x, const std::vector<int64_t>& send_rows,
             const std::vector<int64_t>& recv_rows, hipEvent_t ready, PsxWork* work) {
    int64_t row = x.element_size();
    for (int64_t d = 1; d < x.dim(); ++d) row *= x.size(d);
    wire_[c] += row * (vsum(send_rows) - send_rows[rank_]);
    work->pending = false;
    work->keep = Tensor();
    if (tx_ == kTxIdentity) return x;
    fault(c);
    Tensor xc = x.contiguous();
    if (tx_ == kTxStaged) {
      mark("staged exchange", c);
      xlog(c, send_rows, recv_rows, "host (staged)", nullptr);
      Tensor r = staged_a2a(xc, send_rows, recv_rows);
      mark("staged exchange returned", c);
      return r;
    }
    std::vector<int64_t> shape(xc.sizes().begin(), xc.sizes().end());
    shape[0] = vsum(recv_rows);
    // issued from xs behind the producer's event only (the compute stream
    // goes on with the work enqueued after the producer: C2 of minibatch
    // i-1 overlaps the backward of i-2), or on S itself when no event is
    // given (C1; the linear step's single stream)
    c10::hip::HIPStream xs = ready ? xs_ : S_stream_;
    if (ready) {
      WH_HIP_CHECK_HOST(hipStreamWaitEvent(xs_.stream(), ready, 0));
      c10::hip::HIPCachingAllocator::recordStream(xc.storage().data_ptr(), xs_);
    }
    c10::hip::HIPStreamGuard sg(xs);
    Tensor out = torch::empty(shape, xc.options());
    if (ready)  // allocated on xs, read on S
      c10::hip::HIPCachingAllocator::recordStream(out.storage().data_ptr(), S_stream_);
    PsxEvP t0 = xt_begin(xs.stream());
    (c == 1 ? rccl_c1_ : rccl_)->a2av(xc.data_ptr(), out.data_ptr(), row, send_rows, recv_rows,
                                      xs.stream());
    xt_end(c, std::move(t0), xs.stream());
    work->keep = xc;
    if (xs.stream() != S_stream_.stream()) {
      if (!work->ev) work->ev = std::make_shared<PsxEv>();
      WH_HIP_CHECK_HOST(hipEventRecord(work->ev->e, xs.stream()));
      work->pending = true;
    }
    mark("exchange issued", c);
    xlog(c, send_rows, recv_rows, xs.stream() == xs_.stream() && !sx_ ? "xs" : "S",
         work->pending ? work->ev : nullptr);
    return out;
  }

  // kTxStaged: the rows through host memory and the gloo group, in order on
  // the current stream (blocking: the correctness rehearsal of the RCCL
  // path with several ranks on one GPU)
  // It executes the same a2a_plan() as RcclComm::a2av (per-peer offsets,
  // the own segment a local copy, zero-byte segments skipped) with one c10d
  // send / recv per peer.
  Tensor staged_a2a(const Tensor& xc, const std::vector<int64_t>& send_rows,
                    const std::vector<int64_t>& recv_rows) {
    Tensor h = xc.to(torch::kCPU).contiguous();  // (waits for the current stream's queue)
    int64_t row = h.element_size();
    for (int64_t d = 1; d < h.dim(); ++d) row *= h.size(d);
    std::vector<int64_t> shape(h.sizes().begin(), h.sizes().end());
    if (shape.empty()) shape.push_back(0);
    shape[0] = vsum(recv_rows);
    Tensor out = torch::empty(shape, h.options());
    const A2aPlan pl = a2a_plan((int)rank_, (int)P_, row, send_rows, recv_rows);
    Tensor hb = h.reshape({-1}).view(torch::kUInt8), ob = out.view({-1}).view(torch::kUInt8);
    std::vector<c10::intrusive_ptr<c10d::Work>> ws;
    for (const auto& g : pl.recvs) {
      std::vector<Tensor> t{ob.narrow(0, g.off, g.bytes)};
      ws.push_back(pg_->recv(t, g.peer, kStagedTag));
    }
    for (const auto& g : pl.sends) {
      std::vector<Tensor> t{hb.narrow(0, g.off, g.bytes)};
      ws.push_back(pg_->send(t, g.peer, kStagedTag));
    }
    if (pl.own_bytes > 0)
      ob.narrow(0, pl.own_dst, pl.own_bytes).copy_(hb.narrow(0, pl.own_src, pl.own_bytes));
    for (auto& w : ws)
      if (w) w->wait();
    return out.to(xc.device());
  }

  // int64 [4P] per peer -> the peers' [4P], on the current stream
  Tensor exchange_counts(const Tensor& send) {
    if (tx_ == kTxIdentity) return send.clone();
    fault(0);
    std::vector<int64_t> four(P_, 4);
    Tensor s = send.contiguous();
    if (tx_ == kTxStaged) {
      mark("staged exchange", 0);
      xlog(0, four, four, "host (staged)", nullptr);
      Tensor r = staged_a2a(s, four, four);
      mark("staged exchange returned", 0);
      return r;
    }
    // one 32-byte send / recv per peer on the current stream (cs): this tiny
    // exchange sits on the path of the step's one host read
    Tensor r = torch::empty_like(s);
    const hipStream_t cur = c10::hip::getCurrentHIPStream(dev_).stream();
    PsxEvP t0 = xt_begin(cur);
    rccl_c0_->a2av(s.data_ptr(), r.data_ptr(), sizeof(int64_t), four, four, cur);
    xt_end(0, std::move(t0), cur);
    PsxEvP ev;
    if (wd_) {
      ev = std::make_shared<PsxEv>();
      WH_HIP_CHECK_HOST(hipEventRecord(ev->e, cur));
    }
    mark("exchange issued", 0);
    xlog(0, four, four, cur == cs_h_ ? "cs" : "S", std::move(ev));
    return r;
  }

  hipEvent_t record(const c10::hip::HIPStream& s) {
    hipEvent_t e = ring_[ring_i_];
    ring_i_ = (ring_i_ + 1) % kRing;
    WH_HIP_CHECK_HOST(hipEventRecord(e, s.stream()));
    return e;
  }
  void wait_on(const c10::hip::HIPStream& waiter, const c10::hip::HIPStream& producer) {
    if (waiter.stream() == producer.stream()) return;
    WH_HIP_CHECK_HOST(hipStreamWaitEvent(waiter.stream(), record(producer), 0));
  }

  // small int64 tables host -> device through a ring of pinned buffers
  Tensor put(const std::vector<int64_t>& a) {
    const int k = pin_i_;
    pin_i_ = (pin_i_ + 1) % kPins;
    if (pin_used_[k]) {
      mark("pinned table ring (host wait)", -1);
      WH_HIP_CHECK_HOST(hipEventSynchronize(pin_ev_[k]));
    }
    if ((int64_t)a.size() > pins_[k].numel())
      pins_[k] = torch::empty({2 * (int64_t)a.size()},
                              torch::TensorOptions().dtype(torch::kInt64).pinned_memory(true));
    std::memcpy(pins_[k].data_ptr(), a.data(), a.size() * sizeof(int64_t));
    Tensor d = torch::empty({(int64_t)a.size()},
                            torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA, dev_));
    if (!a.empty())
      WH_HIP_CHECK_HOST(hipMemcpyAsync(d.data_ptr(), pins_[k].data_ptr(), a.size() * 8,
                                       hipMemcpyHostToDevice, S_stream_.stream()));
    WH_HIP_CHECK_HOST(hipEventRecord(pin_ev_[k], S_stream_.stream()));
    pin_used_[k] = true;
    return d;
  }

  // ------------------------------------------------------------ watchdog
  struct WdCall {  // a call the deadline applies to
    PsxWatchdog* w;
    WdCall(PsxWatchdog* w_, const char* c, int64_t s) : w(w_) {
      if (w) w->enter(c, s);
    }
    ~WdCall() {
      if (w) w->leave();
    }
  };
  void mark(const char* what, int c) {
    if (wd_) wd_->phase(what, c, step_);
  }
  void xlog(int c, const std::vector<int64_t>& s, const std::vector<int64_t>& r, const char* stream,
            PsxEvP ev) {
    if (!wd_) return;
    PsxXLog x;
    x.cls = c;
    x.step = step_;
    x.stream = stream;
    x.send = s;
    x.recv = r;
    x.ev = std::move(ev);
    wd_->log(std::move(x));
  }
  void fault(int c) {
    if (fault_step_ < 0 || step_ != fault_step_) return;
    fault_step_ = -1;
    std::fprintf(stderr, "[psx] WH_FAULT: rank %lld stalls before C%d of step %lld\n",
                 (long long)rank_, c, (long long)step_);
    std::fflush(stderr);
    mark("WH_FAULT stall", c);
    std::this_thread::sleep_for(std::chrono::hours(1));
  }

  // sampled exchange timing (RCCL transport)
  PsxEvP xt_begin(hipStream_t s) {
    if (!xt_on_ || step_ % xt_every_ != 0) return nullptr;
    auto e = std::make_shared<PsxEv>(true);
    WH_HIP_CHECK_HOST(hipEventRecord(e->e, s));
    return e;
  }
  void xt_end(int c, PsxEvP a, hipStream_t s) {
    if (!a) return;
    auto b = std::make_shared<PsxEv>(true);
    WH_HIP_CHECK_HOST(hipEventRecord(b->e, s));
    xt_pend_.push_back({c, std::move(a), std::move(b)});
    if (xt_pend_.size() > 64) xt_harvest(false);
  }
  void xt_harvest(bool sync) {
    std::vector<XtPend> keep;
    for (auto& p : xt_pend_) {
      if (sync) {
        mark("exchange timing read (host wait)", p.cls);
        WH_HIP_CHECK_HOST(hipEventSynchronize(p.b->e));
      } else if (hipEventQuery(p.b->e) != hipSuccess) {
        keep.push_back(std::move(p));
        continue;
      }
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, p.a->e, p.b->e) == hipSuccess) {
        xt_us_[p.cls] += 1000.0 * ms;
        xt_n_[p.cls] += 1;
      }
    }
    xt_pend_.swap(keep);
  }

  // ------------------------------------------------------------ localize
  NativeExchange exchange_fn(PsxStP carried, int64_t flag) {
    return [this, carried, flag](const Tensor& owner_cnt) {
      Tensor vc = carried ? carried->vcnt : Tensor();
      const auto cur = c10::hip::getCurrentHIPStream(dev_);
      wait_on(cs_, S_stream_);
      if (cur.stream() != S_stream_.stream()) wait_on(cs_, cur);  // (called on ls)
      c10::hip::HIPCachingAllocator::recordStream(owner_cnt.storage().data_ptr(), cs_);
      if (vc.defined()) c10::hip::HIPCachingAllocator::recordStream(vc.storage().data_ptr(), cs_);
      c10::hip::HIPStreamGuard sg(cs_);
      // (loopback identity: the kernel fills the receive slot itself)
      auto c0 = ps_c0(owner_cnt, vc.defined() ? c10::optional<Tensor>(vc) : c10::nullopt, P_, flag,
                      tx_ == kTxIdentity);
      if (tx_ != kTxIdentity) c0[1].narrow(0, S_ + 1, 4 * P_).copy_(exchange_counts(c0[0]));
      return std::make_tuple(c0[1], cs_.stream(), (int64_t)4, P_);
    };
  }

  void begin(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
             PsxStP carried, int64_t ready, bool defer) {
    const int64_t flag = offset.numel() > 1 ? 1 : 0;
    wait_on(ls_, S_stream_);
    if (ready) WH_HIP_CHECK_HOST(hipStreamWaitEvent(ls_.stream(), reinterpret_cast<hipEvent_t>(ready), 0));
    for (const Tensor* t : {&keys, &offset}) {
      c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), ls_);
      c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), S_stream_);
    }
    c10::optional<Tensor> v;
    if (val.has_value() && val->defined() && val->numel()) {
      v = *val;
      c10::hip::HIPCachingAllocator::recordStream(val->storage().data_ptr(), ls_);
      c10::hip::HIPCachingAllocator::recordStream(val->storage().data_ptr(), S_stream_);
    }
    c10::hip::HIPStreamGuard sg(ls_);
    job_ = std::make_unique<LocalizeJob>(keys, offset, v, S_, uhint_, exchange_fn(carried, flag),
                                         defer);
    job_keys_ = keys;
    job_carried_ = carried;
    job_deferred_ = defer;
  }

  void exchange_deferred() {
    if (job_ && job_deferred_) {
      c10::hip::HIPStreamGuard sg(ls_);
      job_->exchange();
      job_deferred_ = false;
    }
  }

  void ensure_job(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val) {
    if (job_ && job_keys_.is_same(keys)) return;
    if (job_) {  // a stale job (never expected): finish it in order
      std::vector<int64_t> a, b;
      counts(a, b);
      finish_job();
    }
    begin(keys, offset, val, (pull_ && !pull_->have_v) ? pull_ : PsxStP(), 0, false);
  }

  // the one host read of the step (count exchange C0 of the begun job):
  // send / recv per peer; fills the carried step's V counts; true when no
  // rank has data
  bool counts(std::vector<int64_t>& send, std::vector<int64_t>& recv) {
    exchange_deferred();
    mark("C0 count read (host wait)", 0);
    auto c = job_->counts();
    mark("C0 counts read", 0);
    const int64_t* oc = c[0].data_ptr<int64_t>();
    const Tensor& tail = c[1];
    const int64_t* t = tail.data_ptr<int64_t>();
    TORCH_CHECK(tail.numel() >= 5 * P_, "psx: short count payload");
    if (job_carried_ && !job_carried_->have_v) {
      auto& ca = *job_carried_;
      ca.vrecv.assign(P_, 0);
      ca.vown.assign(P_, 0);
      for (int64_t q = 0; q < P_; ++q) {
        ca.vrecv[q] = t[2 + 4 * q];
        ca.vown[q] = t[4 * P_ + q];
      }
      ca.have_v = true;
    }
    send.assign(P_, 0);
    recv.assign(P_, 0);
    bool any = false;
    for (int64_t p = 0; p < S_; ++p) send[p] = oc[p];
    for (int64_t q = 0; q < P_; ++q) {
      recv[q] = t[4 * q];
      any = any || t[3 + 4 * q] != 0;
    }
    return !any;
  }

  std::vector<Tensor> finish_job() {
    std::vector<Tensor> out = job_->finish();
    job_.reset();
    job_keys_ = Tensor();
    job_carried_.reset();
    job_deferred_ = false;
    return out;
  }

  void vcount_exchange(PsxSt& st) {
    if (linear_) {
      st.vrecv.assign(P_, 0);
      st.vown.assign(P_, 0);
      st.have_v = true;
      return;
    }
    auto zero = torch::zeros({S_ + 1}, st.vcnt.options());
    wait_on(cs_, S_stream_);
    c10::hip::HIPStreamGuard sg(cs_);
    auto c0 = ps_c0(zero, st.vcnt, P_, 1, tx_ == kTxIdentity);
    if (tx_ != kTxIdentity) c0[1].narrow(0, S_ + 1, 4 * P_).copy_(exchange_counts(c0[0]));
    mark("C0 V-count read (host wait)", 0);
    Tensor v = c0[1].cpu();
    mark("C0 V-counts read", 0);
    const int64_t* h = v.data_ptr<int64_t>();
    st.vrecv.assign(P_, 0);
    st.vown.assign(P_, 0);
    for (int64_t q = 0; q < P_; ++q) {
      st.vrecv[q] = h[S_ + 3 + 4 * q];
      st.vown[q] = h[S_ + 1 + 4 * P_ + q];
    }
    st.have_v = true;
  }

  // ------------------------------------------------------------ tables
  PsxStP new_step(const std::vector<int64_t>& send, const std::vector<int64_t>& recv,
                  const Tensor& label, bool train, int64_t data_pass, PsxSt* prev) {
    auto st = std::make_shared<PsxSt>();
    st->send = send;
    st->recv = recv;
    st->label = label;
    st->train = train;
    st->use_cnt = train && data_pass == 0 && !linear_;
    st->seed_step = step_;
    // events of their own per step: at most tau + 2 steps are alive (the
    // pull in flight, the tau pushes in flight and this one), so a pair is
    // reused only kStepEv > kMaxTau + 2 steps later, long after its waits
    // were enqueued
    st->own_open = sev_[sev_i_][0];
    st->own_grad = sev_[sev_i_][1];
    sev_i_ = (sev_i_ + 1) % kStepEv;
    const int64_t vs = std::max<int64_t>(vs_, 1);
    st->Hw.assign(P_, 0);
    st->Ho.assign(P_, 0);
    if (!linear_)
      for (int64_t p = 0; p < P_; ++p) {
        st->Hw[p] = cdiv64(2 * send[p], vs);
        st->Ho[p] = cdiv64(2 * recv[p], vs);
      }
    std::vector<int64_t> a(4 * (P_ + 1) + P_, 0);
    for (int64_t p = 0; p < P_; ++p) {
      a[p + 1] = a[p] + send[p];
      a[P_ + 2 + p] = a[P_ + 1 + p] + st->Hw[p];
      a[2 * P_ + 3 + p] = a[2 * P_ + 2 + p] + recv[p];
      a[3 * P_ + 4 + p] = a[3 * P_ + 3 + p] + st->Ho[p];
    }
    if (prev)
      for (int64_t q = 0; q < P_; ++q) a[4 * P_ + 4 + q] = prev->vrecv[q];
    Tensor t = put(a);
    st->tabs = t;
    st->segS_w = t.narrow(0, 0, P_ + 1);
    st->segHS_w = t.narrow(0, P_ + 1, P_ + 1);
    st->segS_o = t.narrow(0, 2 * P_ + 2, P_ + 1);
    st->segHS_o = t.narrow(0, 3 * P_ + 3, P_ + 1);
    if (prev) prev->vrecv_d = t.narrow(0, 4 * P_ + 4, P_);
    return st;
  }

  void upload_vrecv(PsxSt& st) { st.vrecv_d = put(st.vrecv); }

  void set_loc(PsxSt& st, const std::vector<Tensor>& loc, const Tensor& offset,
               const c10::optional<Tensor>& val) {
    st.uniq = loc[0];
    st.ucnt = loc[1];
    st.lid = loc[3];
    st.csc_off = loc[4];
    st.csc_row = loc[5];
    st.csc_val = loc[6];
    st.U = st.uniq.numel();
    st.offset = offset;
    if (val.has_value() && val->defined() && val->numel()) st.val = *val;
    uhint_ = st.U;
    // the job's outputs (allocated on ls) are read on S from here on
    for (const Tensor* x : {&st.uniq, &st.ucnt, &st.lid, &st.csc_off, &st.csc_row, &st.csc_val})
      if (x->defined() && x->numel())
        c10::hip::HIPCachingAllocator::recordStream(x->storage().data_ptr(), S_stream_);
  }

  // the compute stream of this call; one stream: every phase on it
  void set_streams() {
    S_stream_ = c10::hip::getCurrentHIPStream(dev_);
    if (one_) ls_ = S_stream_;
    if (sx_) cs_ = xs_ = S_stream_;
  }

  // a minibatch's exact AUC into the learner's sum: on the AUC side stream,
  // or in order on the compute stream (one stream)
  void auc(PsxSt& st) {
    if (sx_) auc_acc(st.py, st.label, auc_sum_);
    else auc_acc_side(st.py, st.label, auc_sum_);
  }

  // ------------------------------------------------------------ phases
  void c1(PsxSt& st) {
    c10::optional<Tensor> cnt;
    if (st.use_cnt) cnt = qnb_ ? st.ucnt.clamp_max(255) : st.ucnt;  // TRUNCATE_FLOAT(1)
    Tensor rec = linear_ ? st.uniq : ps_records(st.uniq, cnt);
    // on the exchange stream behind the records (RCCL copies the keys there
    // while the compute stream goes on with the previous minibatch's forward;
    // on the compute stream itself the forward queued behind the transfer)
    hipEvent_t ready = (tx_ == kTxRccl && !sx_) ? record(S_stream_) : nullptr;
    st.keys_o = a2a(1, rec, st.send, st.recv, ready, &st.w_c1);
  }

  void open(PsxSt& st, bool insert, const Tensor& prepped = Tensor()) {
    st.w_c1.wait();
    const int64_t n = vsum(st.recv);
    if (insert) guard_before(n);
    const int64_t rows = linear_ ? 0 : vsum(st.Ho) + n;
    auto o = store_->ps_open(st.keys_o, st.use_cnt, st.segS_o, st.segHS_o, rows, insert, st.train,
                             hp_, threshold_, l1_shrk_, seed_,
                             prepped.defined() ? c10::optional<Tensor>(prepped) : c10::nullopt);
    st.slot = o[0];
    st.vpos = o[1];
    st.chain = o[2];
    st.head = o[3];
    st.rbuf = o[4];
    st.vcnt = o[5];
    st.keys_o = Tensor();
    if (!sx_) WH_HIP_CHECK_HOST(hipEventRecord(st.own_open, S_stream_.stream()));
    st.ev_open = sx_ ? nullptr : st.own_open;
    // the summary every gevery_ opens: in between, guard_before's estimate
    // counts every key inserted since the last one (gsince_), an upper bound
    if (insert && ++gskip_ >= gevery_) guard_after(false);
  }

  void c2(PsxSt& st) {
    std::vector<int64_t> send_rows(P_), recv_rows(P_);
    for (int64_t p = 0; p < P_; ++p) {
      send_rows[p] = linear_ ? st.recv[p] : st.Ho[p] + st.vown[p];
      recv_rows[p] = linear_ ? st.send[p] : st.Hw[p] + st.vrecv[p];
    }
    Tensor x = st.rbuf.narrow(0, 0, vsum(send_rows));
    hipEvent_t ready = st.ev_open;
    if (qnb_ && !linear_) {  // (linear pulls travel exact)
      x = qpack(x, st.recv, st.send, st.vown, st.vrecv, st.Ho, st.Hw, send_rows, recv_rows,
                &st.q2_desc, &st.q2_ext);
      ready = sx_ ? nullptr : record(S_stream_);
    }
    st.rrecv = a2a(2, x, send_rows, recv_rows, ready, &st.w_c2);
    st.ev_open = nullptr;
    st.rbuf = Tensor();
  }

  // fixed_bytes: the float regions x (this side: n keys, v embedding rows, H
  // header rows per peer) -> uint8 wire rows, on S (kv/psx.py Psx._qpack);
  // rows out / in per peer replace send_rows / recv_rows, and the receiving
  // side's table and float extent are kept for qunpack
  struct QLayout {
    std::vector<int64_t> desc, rows;
    int64_t ext = 0;
  };
  QLayout qlayout(const std::vector<int64_t>& n, const std::vector<int64_t>& v,
                  const std::vector<int64_t>& H) const {
    QLayout L;
    L.desc.assign(6 * P_, 0);
    int64_t sf = 0, sq = 0;
    for (int64_t p = 0; p < P_; ++p) {
      int64_t a, vf, nf, ha, nr, ext;
      if (linear_) {
        a = 0, vf = 0, nf = n[p], ha = 0;
        nr = cdiv64(n[p], qW_);
        ext = n[p];
      } else {
        a = 2 * n[p], vf = H[p] * vs_, nf = v[p] * vs_;
        ha = cdiv64(4 * a, qR_);
        nr = v[p];
        ext = (H[p] + v[p]) * vs_;
      }
      const int64_t d[6] = {sf, a, vf, nf, sq, ha};
      for (int k = 0; k < 6; ++k) L.desc[6 * p + k] = d[k];
      L.rows.push_back(ha + nr);
      sf += ext;
      sq += ha + nr;
    }
    L.ext = sf;
    return L;
  }
  Tensor qpack(const Tensor& x, const std::vector<int64_t>& ns, const std::vector<int64_t>& nr,
               const std::vector<int64_t>& vs, const std::vector<int64_t>& vr,
               const std::vector<int64_t>& Hs, const std::vector<int64_t>& Hr,
               std::vector<int64_t>& send_rows, std::vector<int64_t>& recv_rows, Tensor* rdesc,
               int64_t* rext) {
    const QLayout ls = qlayout(ns, vs, Hs), lr = qlayout(nr, vr, Hr);
    TORCH_CHECK(ls.ext == x.numel(), "psx filter: region layout ", ls.ext, " floats vs buffer ",
                x.numel());
    std::vector<int64_t> both(ls.desc);
    both.insert(both.end(), lr.desc.begin(), lr.desc.end());
    Tensor t = put(both);
    ++qcalls_;
    c10::hip::HIPStreamGuard sg(S_stream_);
    Tensor q = ps_qpack(x.contiguous().view({-1}), t.narrow(0, 0, 6 * P_).view({P_, 6}),
                        vsum(ls.rows), qW_, qnb_, qseed_ + (qcalls_ << 20));
    send_rows = ls.rows;
    recv_rows = lr.rows;
    *rdesc = t.narrow(0, 6 * P_, 6 * P_).view({P_, 6});
    *rext = lr.ext;
    return q;
  }
  Tensor qunpack(const Tensor& q, Tensor& desc, int64_t ext) {
    const int64_t vs = linear_ ? 1 : vs_;
    Tensor out = linear_ ? torch::empty({ext}, q.options().dtype(torch::kFloat32))
                         : torch::empty({ext / vs, vs}, q.options().dtype(torch::kFloat32));
    ps_qunpack(q, desc, qW_, qnb_, out);
    desc = Tensor();
    return out;
  }

  void reply(PsxSt& st) {
    st.w_c2.wait();
    if (st.q2_desc.defined()) st.rrecv = qunpack(st.rrecv, st.q2_desc, st.q2_ext);
    const c10::optional<Tensor> val =
        st.val.defined() ? c10::optional<Tensor>(st.val) : c10::nullopt;
    std::vector<Tensor> fw;
    if (linear_) {
      st.hdr = st.rrecv;
      fw = fm_forward(st.offset, st.lid, val, st.rrecv, c10::nullopt, 0, st.label, loss_, met_);
    } else {
      auto u = ps_unpack(st.rrecv, st.U, st.segS_w, st.segHS_w, st.vrecv_d);
      st.hdr = u[0];
      st.rows = u[1];
      fw = fm_forward(st.offset, st.lid, val, st.hdr, st.rrecv, vs_, st.label, loss_, met_);
    }
    st.py = fw[0];
    st.dual = fw[1];
    st.xv = fw[2];
    if (!st.train) auc(st);
    if (st.label.numel()) ++fwd_mb_;
    last_u_ = st.U;
    last_v_ = vsum(st.vrecv);
  }

  void grad(PsxSt& st, bool issue) {
    const c10::optional<Tensor> cv =
        st.csc_val.defined() && st.csc_val.numel() ? c10::optional<Tensor>(st.csc_val)
                                                   : c10::nullopt;
    if (linear_) {
      auto b = fm_backward(st.csc_off, st.csc_row, cv, st.dual, c10::nullopt, st.hdr,
                           c10::nullopt, 0);
      st.gvc = b[0].reshape({-1});
    } else {
      auto b = fm_backward(st.csc_off, st.csc_row, cv, st.dual, st.xv, st.hdr, st.rrecv, vs_);
      if (ht_) ht_->mark(8);
      if (post_on_) grad_post(st, b[1]);
      ps_pack_gw(b[0], b[1], st.segS_w, st.segHS_w, st.vrecv_d);
      st.gvc = b[1];
    }
    if (!sx_) WH_HIP_CHECK_HOST(hipEventRecord(st.own_grad, S_stream_.stream()));
    st.ev_grad = sx_ ? nullptr : st.own_grad;
    if (issue) c3(st);
    auc(st);
    if (ht_) ht_->mark(9);
    st.rrecv = st.hdr = st.rows = st.dual = st.xv = st.lid = Tensor();
    st.csc_off = st.csc_row = st.csc_val = Tensor();
  }

  // clipping / dropout / normalization of the embedding gradient rows
  // (kv/psx.py Psx._grad; learn/difacto/loss.h:145-155); the normalization
  // runs over the V rows only (the header rows zeroed first)
  void grad_post(PsxSt& st, const Tensor& gvc) {
    if (gnorm_) {
      int64_t base = 0;
      for (int64_t q = 0; q < P_; ++q) {
        if (st.Hw[q] > 0) gvc.narrow(0, base, st.Hw[q]).zero_();
        base += st.Hw[q] + st.vrecv[q];
      }
    }
    fm_grad_post(gvc, st.rows, pdim_, clip_, dropout_, seed_ + 7919 * st.seed_step + 1, gnorm_);
  }

  void c3(PsxSt& st) {
    std::vector<int64_t> send_rows(P_), recv_rows(P_);
    for (int64_t p = 0; p < P_; ++p) {
      send_rows[p] = linear_ ? st.send[p] : st.Hw[p] + st.vrecv[p];
      recv_rows[p] = linear_ ? st.recv[p] : st.Ho[p] + st.vown[p];
    }
    Tensor x = st.gvc;
    hipEvent_t ready = st.ev_grad;
    if (qnb_) {
      x = qpack(x, st.send, st.recv, st.vrecv, st.vown, st.Hw, st.Ho, send_rows, recv_rows,
                &st.q3_desc, &st.q3_ext);
      ready = sx_ ? nullptr : record(S_stream_);
    }
    st.gpush = a2a(3, x, send_rows, recv_rows, ready, &st.w_c3);
    st.ev_grad = nullptr;
    st.gvc = Tensor();
  }

  // prep (defined): the next open's chain buffer, zeroed by this push's
  // kernel together with the V-row snapshot (the open's prep launch saved
  // on the compute stream's chain); prep_n its used length
  void owner_push(PsxSt& st, const Tensor& prep = Tensor(), int64_t prep_n = 0) {
    st.w_c3.wait();
    if (st.q3_desc.defined()) st.gpush = qunpack(st.gpush, st.q3_desc, st.q3_ext);
    const c10::optional<Tensor> pc = prep.defined() ? c10::optional<Tensor>(prep) : c10::nullopt;
    if (linear_) {
      store_->ps_push_linear(st.slot, st.chain, st.head, st.segS_o, st.gpush, (int64_t)lin_hp_[0],
                             lin_hp_[1], lin_hp_[2], lin_hp_[3], lin_hp_[4], (double)requests_, pc,
                             prep_n);
      requests_ += P_;  // one request per worker (ps-lite SGD's t)
    } else {
      store_->ps_push(st.slot, st.vpos, st.chain, st.head, st.segS_o, st.segHS_o, st.gpush, hp_,
                      threshold_, l1_shrk_, seed_, pc, prep_n);
    }
    st.gpush = st.slot = st.vpos = st.chain = st.head = Tensor();
  }

  // ------------------------------------------------------------ store guard
  // kv/__init__.py StoreGuard: before an open, the previous summary (one
  // open behind: long complete) is checked -- a lost key or row raises --
  // and the table / V slab grow so the coming open cannot overflow them;
  // after it a summary is enqueued on a side stream.
  // (summary slots 2 / 3 of the store: 0 / 1 belong to the Python guard)
  void guard_read() {
    if (!gpend_) return;
    mark("store summary read (host wait)", -1);
    wait_event(gev_[gk_]);
    gpend_ = false;
    auto h = store_->summary_read(2 + gk_);
    gkeys_ = h[0];
    gvused_ = h[3];
    TORCH_CHECK(h[1] == 0 && h[2] == 0, "parameter store shard lost data: ", h[1],
                " failed inserts, ", h[2], " embedding rows dropped (table ", h[0], "/",
                store_->cap(), " keys, V slab ", h[3], "/", store_->vcap(), " rows)");
  }
  void guard_before(int64_t n) {
    guard_read();
    const int64_t need = gkeys_ + gsince_ + n;
    if ((double)need > max_load_ * (double)store_->cap()) {
      int64_t cap = store_->cap();
      while ((double)need > 0.5 * (double)cap) cap *= 2;
      Tensor remap = store_->grow(cap);
      ++grows_;
      std::vector<PsxSt*> live{pull_.get()};
      for (auto& p : pushes_) live.push_back(p.get());
      for (PsxSt* st : live)
        if (st && st->slot.defined() && st->slot.numel()) {
          auto s64 = st->slot.to(torch::kInt64);
          st->slot = torch::where(s64 >= 0, remap.index_select(0, s64.clamp_min(0)), st->slot);
        }
    }
    if (vs_ > 0) {
      const int64_t vneed = gvused_ + gsince_ + n + grecent_[0] + grecent_[1];
      if (vneed > store_->vcap()) {
        int64_t vcap = std::max<int64_t>(store_->vcap(), 1);
        while (vneed > vcap) vcap *= 2;
        store_->grow_v(vcap);
        ++vgrows_;
      }
    }
    gsince_ += n;
    grecent_[0] = grecent_[1];
    grecent_[1] = n;
  }
  void guard_after(bool sync) {
    gskip_ = 0;
    gk_ ^= 1;
    wait_on(cs_, S_stream_);
    {
      c10::hip::HIPStreamGuard sg(cs_);
      store_->summary_async(2 + gk_);
      WH_HIP_CHECK_HOST(hipEventRecord(gev_[gk_], cs_.stream()));
    }
    gpend_ = true;
    gsince_ = 0;
    if (sync) guard_read();
  }

  static constexpr int kMaxTau = 8;
  static constexpr int kRing = 32, kPins = 8, kStepEv = kMaxTau + 4;
  static constexpr int kStagedTag = 7;
  struct XtPend {
    int cls;
    PsxEvP a, b;
  };
  KVStore* store_;
  int64_t P_, S_, rank_;
  bool linear_;
  std::vector<double> lin_hp_, hp_;
  int64_t threshold_;
  bool l1_shrk_;
  int64_t seed_, loss_;
  Tensor met_, auc_sum_;
  int64_t tau_;
  double max_load_;
  int vs_ = 0;
  PsxTx tx_ = kTxIdentity;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;  // kTxStaged
  std::shared_ptr<RcclComm> rccl_, rccl_c0_, rccl_c1_;  // kTxRccl: C2 / C3, C0, C1
  c10::DeviceIndex dev_ = 0;
  c10::hip::HIPStream S_stream_ = c10::hip::getDefaultHIPStream();
  c10::hip::HIPStream ls_ = c10::hip::getDefaultHIPStream();
  c10::hip::HIPStream cs_ = c10::hip::getDefaultHIPStream();
  c10::hip::HIPStream xs_ = c10::hip::getDefaultHIPStream();
  hipStream_t ls_h_ = nullptr, cs_h_ = nullptr, xs_h_ = nullptr;
  hipEvent_t ring_[kRing] = {};
  hipEvent_t sev_[kStepEv][2] = {};
  int sev_i_ = 0;
  int ring_i_ = 0;
  Tensor pins_[kPins];
  hipEvent_t pin_ev_[kPins] = {};
  bool pin_used_[kPins] = {};
  int pin_i_ = 0;
  std::unique_ptr<LocalizeJob> job_;
  Tensor job_keys_;
  PsxStP job_carried_, pull_;
  std::deque<PsxStP> pushes_;  // backward done, push not yet applied (oldest first)
  bool job_deferred_ = false;
  int64_t uhint_ = 0, step_ = 0, requests_ = 0, fwd_mb_ = 0, last_u_ = 0, last_v_ = 0;
  int64_t wire_[4] = {0, 0, 0, 0};
  std::unique_ptr<HostSplit> timing_{host_split("psx native step")};
  bool one_ = false, sx_ = false;
  HostTimer* ht_ = nullptr;  // (WH_TIMING=step: the running call's marks, for grad's split)
  std::unique_ptr<PsxWatchdog> wd_;  // (transports with peers)
  int64_t fault_step_ = -1;          // WH_FAULT=xstall
  bool xt_on_ = false;
  int64_t xt_every_ = 16;
  std::vector<XtPend> xt_pend_;
  // fixed_bytes filter (qnb_ > 0): bytes per float, seed, floats and bytes
  // per wire record; the seed sequence follows kv/psx.py _QFilter.next_seed
  int qnb_ = 0, qW_ = 0, qR_ = 0;
  int64_t qseed_ = 0, qcalls_ = 0;
  // embedding-gradient post-processing (learn/difacto/loss.h:131-155)
  double clip_ = 0, dropout_ = 0;
  bool gnorm_ = false, post_on_ = false;
  int64_t pdim_ = 0;
  double xt_us_[4] = {0, 0, 0, 0};
  int64_t xt_n_[4] = {0, 0, 0, 0};
  // guard: opens per store summary (the linear step: a launch, an event and
  // a host read less on 3 of 4 steps)
  const int gevery_ = linear_ ? 4 : 1;
  int gskip_ = 0;
  hipEvent_t gev_[2] = {};
  int gk_ = 0;
  bool gpend_ = false;
  int64_t gkeys_ = 0, gvused_ = 0, gsince_ = 0, grecent_[2] = {0, 0}, grows_ = 0, vgrows_ = 0;
};

Tensor c10d_a2a_rows(py::object pg, const Tensor& x, const std::vector<int64_t>& send_rows,
                     const std::vector<int64_t>& recv_rows) {
  return c10d_rows(pg.cast<c10::intrusive_ptr<c10d::ProcessGroup>>(), x, send_rows, recv_rows);
}
