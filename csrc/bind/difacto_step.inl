// The single-shard DiFacto training / evaluation step in ONE native call
// (included by hip_ops.cc after the multi-shard step; the Python twin, kept
// as the CPU path and the test oracle, is models/difacto.py
// DifactoLearner.process with WH_DIFACTO_NATIVE=0).
//
// Reference per-minibatch flow: learn/difacto/async_sgd.h:363-425 on one
// server shard -- push the feature counts (data pass 0) -> pull w and the
// lazily allocated V rows -> FM forward + loss + AUC -> FM backward ->
// gradient clipping / dropout / normalization (learn/difacto/loss.h:145-155)
// -> push (FTRL on w, AdaGrad on V). The Python step spent ~150 us of host
// time per call at the reference tutorial's minibatch of 1000 rows
// (learn/difacto/guide/criteo.conf, doc/tutorial/criteo_kaggle.rst:115-131):
// a dozen op calls, each with its argument parsing, stream bookkeeping and
// allocations, for a GPU step of a few tens of microseconds. Here the same
// kernels are enqueued from C++ with one Python crossing per minibatch.
//
// Streams: the compute stream S (the caller's) and the localize stream ls,
// where the NEXT minibatch's localize runs while this one trains (as in
// LinearStep::step_localize); the AUC runs on the native AUC side stream.
class DifactoStep {
 public:
  // hp: the learner's 8 DiFacto hyper-parameters; post = (grad_clipping,
  // dropout, grad_normalization, dim); direct: the FM kernels read the V
  // rows in place in the store's slab (no post-processing)
  DifactoStep(KVStore* store, std::vector<double> hp, int64_t threshold, bool l1_shrk,
              int64_t seed, int64_t loss, std::vector<double> post, double max_load, bool direct)
      : store_(store), hp_(std::move(hp)), threshold_(threshold), l1_shrk_(l1_shrk), seed_(seed),
        loss_(loss), max_load_(max_load) {
    TORCH_CHECK(hp_.size() == 8 && post.size() == 4, "DifactoStep: hp[8], post[4]");
    vs_ = store->vstride();
    TORCH_CHECK(vs_ > 0, "DifactoStep: an embedding store (vstride > 0)");
    clip_ = post[0];
    dropout_ = post[1];
    gnorm_ = post[2] != 0.0;
    dim_ = (int64_t)post[3];
    post_on_ = clip_ > 0 || dropout_ > 0 || gnorm_;
    direct_ = direct && !post_on_;
    dev_ = store->slots_.device().index();
    c10::DeviceGuard g(store->slots_.device());
    ls_ = c10::hip::getStreamFromExternal(own_stream(dev_, kStreamLinearLs), dev_);
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&ev_s_, hipEventDisableTiming));
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&ev_ls_, hipEventDisableTiming));
    for (auto& e : gev_) WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  DifactoStep(const DifactoStep&) = delete;
  DifactoStep& operator=(const DifactoStep&) = delete;
  ~DifactoStep() {
    if (timing_) timing_->print();
    job_.reset();
    (void)hipDeviceSynchronize();
    (void)hipEventDestroy(ev_s_);
    (void)hipEventDestroy(ev_ls_);
    for (auto& e : gev_) (void)hipEventDestroy(e);
  }

  // One minibatch. train: insert / count / push (else an evaluation pass:
  // find only, AUC on S). step: the learner's step counter (the dropout
  // seed). next_*: the next call's minibatch, whose localize begins now on
  // the localize stream (after `ready`, a hipEvent_t of its producer, or
  // with 0 after everything queued on S). Returns (py, unique keys,
  // embedding rows as a device int64 [1]).
  py::tuple step(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                 const Tensor& label, bool train, int64_t data_pass, const Tensor& met,
                 const Tensor& auc_sum, int64_t step, const c10::optional<Tensor>& nkeys,
                 const c10::optional<Tensor>& noffset, const c10::optional<Tensor>& nval,
                 int64_t ready) {
    c10::DeviceGuard g(keys.device());
    // WH_TIMING=step: s0 localize finish, s1 next localize begin, s2 guard +
    // open/pull, s3 forward, s4 backward + post, s5 push, s6 AUC
    HostTimer ht(timing_.get());
    const hipStream_t S = cur_stream(keys);
    std::vector<Tensor> loc;
    if (job_ && job_keys_.is_same(keys)) {
      loc = job_->finish();
      if (!job_->partitioned()) s_job_ = true;
      for (const Tensor& t : loc)  // allocated on ls, read on S from here on
        if (t.defined() && t.is_cuda() && t.numel())
          c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                                      c10::hip::getCurrentHIPStream(dev_));
    } else {
      if (job_) {  // a stale job: the workspace is the localize stream's until it ends
        WH_HIP_CHECK_HOST(hipEventRecord(ev_ls_, ls_.stream()));
        WH_HIP_CHECK_HOST(hipStreamWaitEvent(S, ev_ls_, 0));
      }
      job_.reset();
      LocalizeJob j(keys, offset, val, 1, hint_, py::none());
      loc = j.finish();
      s_job_ = true;
    }
    job_.reset();
    job_keys_ = Tensor();
    const Tensor &uniq = loc[0], &ucnt = loc[1], &lid = loc[3], &csc_off = loc[4],
                 &csc_row = loc[5], &csc_val = loc[6];
    const int64_t U = uniq.numel();
    hint_ = U;
    ht.mark(0);
    // open + pull (DifactoLearner.process: kv.difacto_open_pull), the
    // feature counts pushed on data pass 0
    const bool push_cnt = train && data_pass == 0;
    if (train) guard_before(U);
    auto o = store_->difacto_open_pull(uniq, train,
                                       push_cnt ? c10::optional<Tensor>(ucnt) : c10::nullopt, hp_,
                                       threshold_, l1_shrk_, seed_, direct_);
    if (train) guard_after();
    const Tensor &slot = o[0], &hdr = o[1], &vc = o[2], &vpos = o[3];
    ht.mark(2);
    // the next minibatch's localize, right after the pull's launch
    if (nkeys.has_value() && nkeys->defined()) begin(*nkeys, *noffset, nval, ready, S);
    ht.mark(1);
    const c10::optional<Tensor> v =
        val.has_value() && val->defined() && val->numel() ? val : c10::nullopt;
    auto fw = fm_forward(offset, lid, v, hdr, vc, vs_, label, loss_, met);
    if (!train) auc_acc(fw[0], label, auc_sum);
    ht.mark(3);
    Tensor m = vpos.narrow(0, vpos.numel() - 1, 1);
    if (train && U > 0) {
      const c10::optional<Tensor> cv =
          csc_val.defined() && csc_val.numel() ? c10::optional<Tensor>(csc_val) : c10::nullopt;
      auto bw = fm_backward(csc_off, csc_row, cv, fw[1], fw[2], hdr, vc, vs_);
      if (post_on_)
        fm_grad_post(bw[1], m, dim_, clip_, dropout_, seed_ + 7919 * step + 1, gnorm_);
      ht.mark(4);
      // (the AUC side stream starts behind the backward: its kernels overlap
      // the push and the next open rather than the backward planning)
      auc_acc_side(fw[0], label, auc_sum);
      ht.mark(6);
      store_->difacto_push(slot, hdr, bw[0], bw[1], hp_, threshold_, l1_shrk_, seed_);
      ht.mark(5);
    } else if (train) {
      auc_acc_side(fw[0], label, auc_sum);
    }
    return py::make_tuple(fw[0], U, m);
  }

  // drop a begun localize (end of a pass, or before a Python-path call)
  void reset() {
    job_.reset();
    job_keys_ = Tensor();
  }
  bool direct() const { return direct_; }
  int64_t grows() const { return grows_; }
  int64_t vgrows() const { return vgrows_; }
  // the guard's last summary {keys, failed inserts, V overflows, V rows}
  std::vector<int64_t> guard_sync() {
    if (!gpend_ && gissued_) guard_after();
    guard_read();
    return {gkeys_, 0, 0, gvused_};
  }

 private:
  void begin(const Tensor& nk, const Tensor& no, const c10::optional<Tensor>& nval, int64_t ready,
             hipStream_t S) {
    // the localize stream waits for S when a localize ran on S (the shared
    // workspace) or when the next minibatch has no producer event (it was
    // made on S, possibly by work queued just now)
    if (s_job_ || !ready) {
      WH_HIP_CHECK_HOST(hipEventRecord(ev_s_, S));
      WH_HIP_CHECK_HOST(hipStreamWaitEvent(ls_.stream(), ev_s_, 0));
      s_job_ = false;
    }
    if (ready) WH_HIP_CHECK_HOST(hipStreamWaitEvent(ls_.stream(), reinterpret_cast<hipEvent_t>(ready), 0));
    for (const Tensor* t : {&nk, &no}) {
      c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), ls_);
      c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(),
                                                  c10::hip::getCurrentHIPStream(dev_));
    }
    c10::optional<Tensor> nv;
    if (nval.has_value() && nval->defined() && nval->numel()) {
      nv = *nval;
      c10::hip::HIPCachingAllocator::recordStream(nval->storage().data_ptr(), ls_);
      c10::hip::HIPCachingAllocator::recordStream(nval->storage().data_ptr(),
                                                  c10::hip::getCurrentHIPStream(dev_));
    }
    c10::hip::HIPStreamGuard sg(ls_);
    job_ = std::make_unique<LocalizeJob>(nk, no, nv, 1, hint_, py::none());
    job_keys_ = nk;
  }

  // ---- store guard (kv/__init__.py StoreGuard; as PsxStep's): before an
  // open the previous summary (one open behind, long complete) is checked --
  // a lost key or row raises -- and the table / V slab grow so the coming
  // open, and the push still in flight, cannot overflow them. Summary slots
  // 2 / 3 of the store (0 / 1 belong to the Python guard).
  void guard_read() {
    if (!gpend_) return;
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
      store_->grow(cap);  // (no slot is held across steps: nothing to remap)
      ++grows_;
    }
    const int64_t vneed = gvused_ + gsince_ + n + grecent_[0] + grecent_[1];
    if (vneed > store_->vcap()) {
      int64_t vcap = std::max<int64_t>(store_->vcap(), 1);
      while (vneed > vcap) vcap *= 2;
      store_->grow_v(vcap);
      ++vgrows_;
    }
    gsince_ += n;
    grecent_[0] = grecent_[1];
    grecent_[1] = n;
  }
  void guard_after() {
    gk_ ^= 1;
    // the summary kernel on the AUC-free side of the compute stream: it is
    // one wave and reads counters only, so it runs in order on S
    store_->summary_async(2 + gk_);
    WH_HIP_CHECK_HOST(hipEventRecord(gev_[gk_], c10::hip::getCurrentHIPStream(dev_).stream()));
    gpend_ = true;
    gsince_ = 0;
    ++gissued_;
  }

  KVStore* store_;
  std::vector<double> hp_;
  int64_t threshold_;
  bool l1_shrk_;
  int64_t seed_, loss_;
  double max_load_;
  int vs_ = 0;
  double clip_ = 0, dropout_ = 0;
  bool gnorm_ = false, post_on_ = false, direct_ = false;
  int64_t dim_ = 0;
  c10::DeviceIndex dev_ = 0;
  c10::hip::HIPStream ls_ = c10::hip::getDefaultHIPStream();
  hipEvent_t ev_s_ = nullptr, ev_ls_ = nullptr;
  std::unique_ptr<LocalizeJob> job_;
  Tensor job_keys_;
  bool s_job_ = false;
  int64_t hint_ = 0;
  hipEvent_t gev_[2] = {};
  int gk_ = 0;
  bool gpend_ = false;
  int64_t gissued_ = 0, gkeys_ = 0, gvused_ = 0, gsince_ = 0, grecent_[2] = {0, 0};
  int64_t grows_ = 0, vgrows_ = 0;
  std::unique_ptr<HostSplit> timing_{host_split("difacto native step")};
};
