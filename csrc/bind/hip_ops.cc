// torch / pybind11 binding layer for the gfx950 HIP kernels (module
// wormhole_amd._hip). Host-only translation unit: validates tensors, sizes
// outputs and launches on the current PyTorch HIP stream.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>

#include <algorithm>
#include <map>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <cmath>
#include <functional>
#include <deque>
#include <map>
#include <mutex>
#include <condition_variable>
#include <thread>
#include <memory>
#include <numeric>
#include <tuple>
#include <string>
#include <vector>

#include "hip/wh_kernels.h"
#include "host/auc_host.h"

namespace {

using torch::Tensor;

inline hipStream_t cur_stream(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONT(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_DT(t, dt) TORCH_CHECK((t).scalar_type() == (dt), #t " has wrong dtype ", (t).scalar_type())
#define CHECK_IN(t, dt) \
  CHECK_DEV(t);         \
  CHECK_CONT(t);        \
  CHECK_DT(t, dt)

template <typename T>
T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

#define WH_HIP_CHECK_HOST(expr)                                                   \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ",  \
                __FILE__, ":", __LINE__);                                       \
  } while (0)

// The host's wait for a step's one device read (the localize counts, the
// store guard's summary): polled for up to 2 ms before a blocking wait. The
// step's next launches go out the moment the read lands instead of after a
// sleeping wait's wake-up (A/B on one box: headline 142.8-143.4 vs
// 140.9-143.5 M, loopback 8 123.8 / 125.7 vs 123.2 / 125.1 M; within noise
// elsewhere: profiles/round6_small_minibatch_host.txt).
inline void wait_event(hipEvent_t e) {
#if !defined(WH_BLOCKING_WAIT)
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return;
    WH_HIP_CHECK_HOST(r == hipErrorNotReady ? hipSuccess : r);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
  }
#endif
  WH_HIP_CHECK_HOST(hipEventSynchronize(e));
}

template <typename T>
const T* optptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined() && t->numel() > 0) ? reinterpret_cast<const T*>(t->data_ptr())
                                                           : nullptr;
}

inline int64_t next_pow2(int64_t x) {
  int64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// Per-device persistent workspaces (allocated once, zero-initialised; the
// kernels that use them leave them in that state). Intentionally leaked: they
// must outlive every stream-ordered use and the process exit order.
struct DevWs {
  Tensor lb;          // look-back scan granules + ticket (wh_lookback.h)
  Tensor auc;         // AUC bucket counters / min-max / area / ticket
  Tensor fwd_ticket;  // arrival counter of the forward's last-block reduction
  // localize hash tables (all ~0 between minibatches) and overflow counters
  // (0 between minibatches), double-buffered so that minibatch i+1's insert
  // can be enqueued before minibatch i's assign has emptied its table
  Tensor loc_tab[2];
  Tensor loc_ovf[2];
  // partitioned localize: its own look-back workspace (a localize may be
  // begun on a side stream, concurrently with other look-back users) and
  // {per-partition publish words, arrival counter}
  Tensor lb_loc, part_ws;
  // heavy-id hints, double-buffered by job parity: keys [2][kPartMaxHeavy]
  // u64, then counts [2][kPartMaxOwners] u32
  Tensor heavy_ws;
  // the backward's scratch (chunk lists, bucket histograms, offsets) per
  // stream, grow-only: reused in stream order by the next backward on the
  // same stream (eight allocations per call were ~20 us of host time, the
  // bound of the small-minibatch multi-shard step)
  std::map<hipStream_t, std::vector<Tensor>> bwd_scratch;
  int heavy_parity = 0;
  int64_t heavy_layout = -1;  // nshard * 65536 + nho of the set the last job elected
  int part_inflight = 0;
  // (non-zeros, unique ids) of the last finished localize: a caller's hint
  // is the previous minibatch's unique count, scaled here by the non-zero
  // ratio when this minibatch is larger (uneven minibatches: CRB records cut
  // parts into short and long blocks; an unscaled hint under-sized the plan,
  // every partition overflowed LDS and the job fell back to the hash path)
  int64_t last_nnz = 0, last_u = -1;
  // pinned count buffers + events of the localize jobs' one host read,
  // reused (a pinned allocation, an event create and destroy per job were
  // host time of the launch-bound small-minibatch step)
  struct PinnedRead {
    int64_t* host = nullptr;
    int64_t cap = 0;
    hipEvent_t ev = nullptr;
    bool busy = false;
  };
  std::vector<std::unique_ptr<PinnedRead>> reads;
  PinnedRead* acquire_read(int64_t n) {
    for (auto& r : reads)
      if (!r->busy && r->cap >= n) {
        r->busy = true;
        return r.get();
      }
    auto r = std::make_unique<PinnedRead>();
    r->cap = std::max<int64_t>(n, 64);
    void* p = nullptr;
    WH_HIP_CHECK_HOST(hipHostMalloc(&p, r->cap * sizeof(int64_t), hipHostMallocDefault));
    r->host = static_cast<int64_t*>(p);
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&r->ev, hipEventDisableTiming));
    r->busy = true;
    reads.push_back(std::move(r));
    return reads.back().get();
  }
  bool loc_dirty[2] = {false, false};
  bool loc_busy[2] = {false, false};
  int loc_next = 0;
};

DevWs& dev_ws(const torch::Device& d) {
  static std::vector<DevWs*> ws(64, nullptr);
  const int i = d.index() < 0 ? 0 : d.index();
  TORCH_CHECK(i < 64, "device index out of range");
  if (!ws[i]) {
    auto o = torch::TensorOptions().device(d);
    auto* w = new DevWs();
    w->lb = torch::zeros({wh::lookback_ws_words()}, o.dtype(torch::kInt64));
    w->auc = torch::zeros({wh::auc_ws_persistent_bytes() / 8}, o.dtype(torch::kInt64));
    w->auc.select(0, wh::auc_ws_lohi_offset() / 8).fill_(-1);
    w->fwd_ticket = torch::zeros({wh::fwd_ticket_words()}, o.dtype(torch::kInt32));
    w->lb_loc = torch::zeros({wh::lookback_ws_words()}, o.dtype(torch::kInt64));
    w->part_ws = torch::zeros({wh::kPartMaxDigits + 2}, o.dtype(torch::kInt64));
    w->heavy_ws = torch::zeros({2 * wh::kPartMaxHeavy + wh::kPartMaxOwners}, o.dtype(torch::kInt64));
    for (int b = 0; b < 2; ++b) {
      w->loc_tab[b] = torch::full({1024}, -1, o.dtype(torch::kInt64));
      w->loc_ovf[b] = torch::zeros({1}, o.dtype(torch::kInt64));
    }
    ws[i] = w;
  }
  return *ws[i];
}

inline wh::Lookback lookback(const torch::Device& d) {
  return wh::lookback_bind(dev_ws(d).lb.data_ptr());
}

// ------------------------------------------------------------------ scan
Tensor scan_excl(const Tensor& in) {
  CHECK_DEV(in); CHECK_CONT(in);
  c10::DeviceGuard g(in.device());
  const int64_t n = in.numel();
  auto o = torch::empty({n + 1}, in.options().dtype(torch::kInt64));
  auto tmp = torch::empty({wh::scan_tmp_elems(n)}, in.options().dtype(torch::kInt64));
  if (in.scalar_type() == torch::kInt32)
    wh::scan_i32(ptr<int32_t>(in), ptr<int64_t>(o), n, ptr<int64_t>(tmp), cur_stream(in));
  else {
    CHECK_DT(in, torch::kInt64);
    wh::scan_i64(ptr<int64_t>(in), ptr<int64_t>(o), n, ptr<int64_t>(tmp), cur_stream(in));
  }
  return o;
}

// -------------------------------------------------------------- localize
// Returns (uniq i64[U], ucnt i32[U], owner_cnt i64[P], lid i32[nnz],
//          csc_off i64[U+1], csc_row i32[nnz], csc_val f32[nnz|0], recv i64[2W|0])
//
// exchange (multi-rank): a callable that takes the device owner counts
// i64[nshard + 1] (last = table-overflow count) and returns the device i64
// [2W] {count from rank q, overflow flag of rank q} of a count all-to-all.
// It runs before the one host read, so the read returns both this rank's
// counts and its peers' (one synchronisation per minibatch instead of two).
// Every rank sees every rank's overflow flag, so all ranks retry together.
//
// Two phases, so that a caller can hide the host read: begin() enqueues the
// hash insert, the owner counts, the count exchange and an ASYNC copy of the
// counts into pinned host memory (+ an event); finish() waits for that event
// only, sizes the outputs and enqueues the rest. A learner begins minibatch
// i+1 right after finishing minibatch i, so the wait overlaps i's training.
// WH_DETERMINISTIC=1: bitwise-repeatable training steps: the
// hash + stable-sort localize and ordered (atomic-free) gradient reductions
bool deterministic() {
  static int on = -1;
  if (on < 0) {
    const char* d = std::getenv("WH_DETERMINISTIC");
    on = d && std::string(d) == "1";
  }
  return on == 1;
}

// WH_TIMING: comma-separated profiling aids (docs/build.md): step, step2,
// loc, ingest, comm. True when `what` is one of the listed items.
bool timing_on(const char* what) {
  const char* e = std::getenv("WH_TIMING");
  if (!e) return false;
  const std::string v = std::string(",") + e + ",";
  return v.find(std::string(",") + what + ",") != std::string::npos;
}

// WH_TIMING=loc: the partitioned dedup stores per-partition phase
// timestamps (100 MHz) into a device buffer (loc_timing_read)
bool loc_timing() {
  static int on = -1;
  if (on < 0) on = timing_on("loc") ? 1 : 0;
  return on == 1;
}
Tensor& loc_timing_buf() {
  static Tensor t;
  if (!t.defined())
    t = torch::zeros({4 * wh::kPartMaxDigits},
                     torch::TensorOptions().dtype(torch::kInt64).device(torch::kCUDA));
  return t;
}

// localize retries after a partition overflowed its LDS table (diagnostics)
int64_t& loc_retries() {
  static int64_t n = 0;
  return n;
}

// The count exchange of a localize job issued from C++ (kv/psx.py's C0,
// ported by PsxStep): returns (payload [owner_cnt (nshard+1) | stride values
// per peer | extra], the stream the payload is ready on, stride, world).
using NativeExchange =
    std::function<std::tuple<Tensor, hipStream_t, int64_t, int64_t>(const Tensor&)>;

class LocalizeJob {
 public:
  // defer_exchange: enqueue the localize kernels now, but call the count
  // exchange (and its async host read) only at exchange(): the multi-shard
  // step begins the next minibatch's localize early on its own stream and
  // issues its count collective later, once the payload it carries (the V
  // row counts of this minibatch's open) exists.
  LocalizeJob(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
              int64_t nshard, int64_t hint, py::object exchange, bool defer_exchange = false)
      : keys_(keys), offset_(offset), nshard_(nshard), exchange_(exchange),
        defer_(defer_exchange) {
    init(val, hint);
  }
  LocalizeJob(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
              int64_t nshard, int64_t hint, NativeExchange nex, bool defer_exchange)
      : keys_(keys), offset_(offset), nshard_(nshard), exchange_(py::none()), nex_(std::move(nex)),
        defer_(defer_exchange) {
    init(val, hint);
  }

  void init(const c10::optional<Tensor>& val, int64_t hint) {
    const Tensor& keys = keys_;
    const Tensor& offset = offset_;
    const int64_t nshard = nshard_;
    CHECK_IN(keys, torch::kInt64);
    CHECK_IN(offset, torch::kInt64);
    TORCH_CHECK(nshard >= 1 && nshard <= 1024, "nshard out of range");
    nnz_ = keys.numel();
    TORCH_CHECK(nnz_ < (int64_t)INT32_MAX, "minibatch too large for int32 local ids");
    if (val.has_value() && val->defined() && val->numel() > 0) {
      CHECK_IN((*val), torch::kFloat32);
      TORCH_CHECK(val->numel() == nnz_);
      val_ = *val;
    }
    {
      DevWs& ws = dev_ws(keys.device());
      if (hint > 0 && hint == ws.last_u && ws.last_nnz > 0 && nnz_ > ws.last_nnz)
        hint = std::min<int64_t>(nnz_, hint * nnz_ / ws.last_nnz + 1);
    }
    // Table size: >= 2*nnz can never overflow; with a hint (the previous
    // minibatch's unique count) use ~2.5x the hint instead, which keeps the
    // scratch table small enough to stay cache resident, and fall back to the
    // safe size if this minibatch overflowed it.
    safe_ = next_pow2(std::max<int64_t>(2 * nnz_, 1024));
    tsize_ = hint > 0 ? std::min(safe_, next_pow2(std::max<int64_t>(hint * 5 / 2, 1024))) : safe_;
    c10::DeviceGuard g(keys.device());
    // the partitioned path unless a deterministic localize is asked for (or
    // the minibatch does not fit its plan); the hash path is the fallback
    const int64_t uest = hint > 0 ? std::min<int64_t>(nnz_, hint * 5 / 4 + 1024) : nnz_;
    plan_ = wh::loc_part_plan(nnz_, offset.numel() - 1, (int)nshard, uest, true);
    part_ = plan_.ok && part_enabled();
    if (!part_) acquire_table();
    enqueue();
  }

  // the hash path is the deterministic one (WH_DETERMINISTIC=1)
  static bool part_enabled() { return !deterministic(); }

  ~LocalizeJob() {
    if (rd_) {  // abandoned before its read: the copy may still be in flight
      (void)hipEventSynchronize(rd_->ev);
      rd_->busy = false;
    }
    if (counted_) dev_ws(keys_.device()).part_inflight--;
    if (tab_ >= 0 && !done_) {
      DevWs& ws = dev_ws(keys_.device());
      ws.loc_busy[tab_] = false;  // abandoned: the table may hold keys
      ws.loc_dirty[tab_] = true;
    }
  }

  // The one host read: waits for the count exchange (retrying the whole
  // begin at the safe table size if any rank overflowed) and returns the
  // host (owner counts [nshard], everything the exchange appended). A
  // caller may enqueue unrelated work between counts() and finish().
  // the deferred count exchange (a no-op unless defer_exchange was given)
  void exchange() {
    TORCH_CHECK(!done_, "localize job already finished");
    if (!defer_ || exchanged_) return;
    c10::DeviceGuard g(keys_.device());
    exchanged_ = true;
    exchange_and_read(owner_cnt_, cur_stream(keys_));
  }

  std::vector<Tensor> counts() {
    TORCH_CHECK(!done_, "localize job already finished");
    if (owner_cnt_h_.defined()) return {owner_cnt_h_, recv_h_};
    TORCH_CHECK(!defer_ || exchanged_, "localize: counts() before the deferred exchange()");
    c10::DeviceGuard g(keys_.device());
    DevWs& ws = dev_ws(keys_.device());
    while (true) {
      wait_event(rd_->ev);
      const int64_t* h = rd_->host;
      const bool own = h[nshard_] != 0;
      bool over = own;
      for (int64_t q = 1; q < nrecv_; q += stride_) over |= h[nshard_ + 1 + q] != 0;
      if (!over) break;
      if (part_) {  // a partition overflowed its LDS table (here or on a peer)
        ++loc_retries();
        part_ = false;
        if (counted_) {
          ws.part_inflight--;
          counted_ = false;
        }
        acquire_table();
        tsize_ = safe_;
        enqueue();
        continue;
      }
      TORCH_CHECK(!(own && tsize_ >= safe_), "localize: table overflow");
      // every rank saw the same flags: all retry at the safe size together
      ws.loc_dirty[tab_] = true;
      tsize_ = safe_;
      enqueue();
    }
    const int64_t* h = rd_->host;
    owner_cnt_h_ = torch::empty({nshard_}, torch::kInt64);
    for (int64_t p = 0; p < nshard_; ++p) owner_cnt_h_.data_ptr<int64_t>()[p] = h[p];
    // everything after the owner counts (the peers' values and any extra)
    const int64_t ntail = dev_counts_.numel() - nshard_ - 1;
    recv_h_ = torch::empty({nrecv_ ? ntail : 0}, torch::kInt64);
    for (int64_t q = 0; q < recv_h_.numel(); ++q)
      recv_h_.data_ptr<int64_t>()[q] = h[nshard_ + 1 + q];
    rd_->busy = false;  // read and copied out: back to the pool
    rd_ = nullptr;
    return {owner_cnt_h_, recv_h_};
  }

  // the partitioned path: every output is produced on the job's stream
  // before the count read. (The hash path finishes on the caller's stream
  // and returns its scratch table to the device pool from there: a job
  // begun later on another stream must be ordered after that finish.)
  bool partitioned() const { return part_; }

  std::vector<Tensor> finish() {
    counts();
    c10::DeviceGuard g(keys_.device());
    auto s = cur_stream(keys_);
    DevWs& ws = dev_ws(keys_.device());
    auto i32 = keys_.options().dtype(torch::kInt32);
    auto i64 = keys_.options().dtype(torch::kInt64);
    Tensor owner_cnt_h = owner_cnt_h_, recv_h = recv_h_;
    int64_t U = 0;
    for (int64_t p = 0; p < nshard_; ++p) U += owner_cnt_h.data_ptr<int64_t>()[p];
    ws.last_nnz = nnz_;
    ws.last_u = U;
    if (part_) {  // everything was computed before the host read
      done_ = true;
      if (counted_) {
        ws.part_inflight--;
        counted_ = false;
      }
      return {uniq_.narrow(0, 0, U), ucnt_.narrow(0, 0, U), owner_cnt_h, lid_,
              csc_off_.narrow(0, 0, U + 1), csc_row_, csc_val_, recv_h};
    }
    const int64_t nnz = nnz_, nrows = offset_.numel() - 1;
    const float* vp = val_.defined() ? ptr<float>(val_) : nullptr;
    auto tlid = torch::empty({tsize_}, i32);
    auto uniq = torch::empty({U}, i64);
    wh::loc_assign(reinterpret_cast<uint64_t*>(tkeys_.data_ptr()), tsize_, (int)nshard_,
                   ptr<int64_t>(blkoff_), ptr<int32_t>(tlid),
                   reinterpret_cast<uint64_t*>(uniq.data_ptr()), s);
    ws.loc_dirty[tab_] = false;  // loc_assign empties the table again
    ws.loc_busy[tab_] = false;
    done_ = true;
    auto row_of = torch::empty({std::max<int64_t>(nnz, 1)}, i32);
    const int64_t n1 = std::max<int64_t>(nnz, 1);
    auto lid = torch::empty({nnz}, i32);
    auto work = torch::empty({3 * n1}, i32);  // pos | sorted lid | sorted pos
    wh::loc_rows_lid(ptr<int64_t>(offset_), nrows, ptr<int32_t>(slot_of_), ptr<int32_t>(tlid),
                     ptr<int32_t>(row_of), ptr<int32_t>(lid), vp ? ptr<int32_t>(work) : nullptr,
                     s);
    const size_t sbytes = wh::loc_sort_tmp_bytes(nnz, U);
    auto stmp = torch::empty({(int64_t)sbytes + 16}, keys_.options().dtype(torch::kUInt8));
    auto csc_off = torch::empty({U + 1}, i64);
    auto ucnt = torch::empty({U}, i32);
    auto csc_row = torch::empty({nnz}, i32);
    auto csc_val = vp ? torch::empty({nnz}, keys_.options().dtype(torch::kFloat32))
                      : torch::empty({0}, keys_.options().dtype(torch::kFloat32));
    int32_t* wp = ptr<int32_t>(work);
    wh::loc_csc(ptr<int32_t>(row_of), vp, nnz, U, ptr<int32_t>(lid), wp, wp + n1, wp + 2 * n1,
                stmp.data_ptr(), sbytes, ptr<int64_t>(csc_off), ptr<int32_t>(ucnt),
                ptr<int32_t>(csc_row), vp ? ptr<float>(csc_val) : nullptr, s);
    return {uniq, ucnt, owner_cnt_h, lid, csc_off, csc_row, csc_val, recv_h};
  }

 private:
  void acquire_table() {
    DevWs& ws = dev_ws(keys_.device());
    tab_ = ws.loc_next;
    if (ws.loc_busy[tab_]) tab_ ^= 1;
    TORCH_CHECK(!ws.loc_busy[tab_], "localize: at most two minibatches in flight per device");
    ws.loc_busy[tab_] = true;
    ws.loc_next = tab_ ^ 1;
  }

  // partitioned path: every output is produced before the count read
  Tensor enqueue_part() {
    auto s = cur_stream(keys_);
    DevWs& ws = dev_ws(keys_.device());
    auto i32 = keys_.options().dtype(torch::kInt32);
    auto i64 = keys_.options().dtype(torch::kInt64);
    const int64_t nnz = nnz_, nrows = offset_.numel() - 1;
    const int nsh = (int)nshard_;
    const float* vp = val_.defined() ? ptr<float>(val_) : nullptr;
    auto owner_cnt = torch::empty({nshard_ + 1}, i64);
    {
      // the job's outputs carved from ONE allocation (six separate tensors
      // were six trips through the allocator per minibatch; the views keep
      // the block alive as long as any of them is in use)
      int64_t at = 0;
      auto carve = [&](int64_t bytes) {
        const int64_t o = at;
        at += (bytes + 255) / 256 * 256;
        return o;
      };
      const int64_t o_u = carve(nnz * 8), o_c = carve(nnz * 4), o_o = carve((nnz + 1) * 8),
                    o_r = carve(nnz * 4), o_v = carve(vp ? nnz * 4 : 0), o_l = carve(nnz * 4);
      auto blk = torch::empty({std::max<int64_t>(at, 256)}, keys_.options().dtype(torch::kUInt8));
      auto view = [&](int64_t o, int64_t n, torch::ScalarType dt, int64_t esz) {
        return blk.narrow(0, o, n * esz).view(dt);
      };
      uniq_ = view(o_u, nnz, torch::kInt64, 8);
      ucnt_ = view(o_c, nnz, torch::kInt32, 4);
      csc_off_ = view(o_o, nnz + 1, torch::kInt64, 8);
      csc_row_ = view(o_r, nnz, torch::kInt32, 4);
      csc_val_ = view(o_v, vp ? nnz : 0, torch::kFloat32, 4);
      lid_ = view(o_l, nnz, torch::kInt32, 4);
    }
    // heavy-id hints: read the set the previous job elected, elect into the
    // other buffer; a job begun while another is in flight uses none
    wh::PartHeavy hv{};
    if (plan_.nho > 0) {
      auto* hk = reinterpret_cast<uint64_t*>(ws.heavy_ws.data_ptr());
      auto* hc = reinterpret_cast<uint32_t*>(hk + 2 * wh::kPartMaxHeavy);
      const int cur = ws.heavy_parity, nxt = cur ^ 1;
      if (ws.part_inflight == 0) {
        const int64_t layout = nshard_ * 65536 + plan_.nho;
        hv.keys = hk + cur * wh::kPartMaxHeavy;
        hv.cnt = hc + cur * wh::kPartMaxOwners;
        hv.nho = ws.heavy_layout == layout ? plan_.nho : 0;  // else: elected for another layout
        ws.heavy_layout = layout;
        hv.next_keys = hk + nxt * wh::kPartMaxHeavy;
        hv.next_cnt = hc + nxt * wh::kPartMaxOwners;
        hv.nho_next = plan_.nho;
        hv.thr = (uint32_t)std::max<int64_t>(1024, nnz / 1024);
        ws.heavy_parity = nxt;
      }
    }
    ws.part_inflight++;
    counted_ = true;
    // the job's temporaries in ONE allocation (eight separate tensors were
    // eight trips through the allocator and dispatcher per minibatch: host
    // time is the bound of the multi-shard step at 10k rows); the stream-
    // ordered allocator keeps it safe to drop at the end of this call
    const int64_t nh = (int64_t)plan_.ndig * plan_.ntiles;
    const int64_t ng = wh::loc_part_groups(plan_) * plan_.ndig;
    int64_t at = 0;
    auto carve = [&](int64_t bytes) {
      const int64_t o = at;
      at += (bytes + 255) / 256 * 256;
      return o;
    };
    const int64_t o_hist = carve(nh * 4), o_gsum = carve(ng * 4),
                  o_base = carve((plan_.ndig + 1) * 8), o_pk = carve(nnz * 8), o_pr = carve(nnz * 4),
                  o_pv = carve(vp ? nnz * 4 : 0), o_pos = carve(nnz * 4), o_plid = carve(nnz * 4);
    auto tmp = torch::empty({std::max<int64_t>(at, 256)}, keys_.options().dtype(torch::kUInt8));
    char* tb = static_cast<char*>(tmp.data_ptr());
    auto* hist = reinterpret_cast<uint32_t*>(tb + o_hist);
    auto* gsum = reinterpret_cast<uint32_t*>(tb + o_gsum);
    auto* base = reinterpret_cast<int64_t*>(tb + o_base);
    auto* pk = reinterpret_cast<uint64_t*>(tb + o_pk);
    auto* pr = reinterpret_cast<int32_t*>(tb + o_pr);
    auto* pv = vp ? reinterpret_cast<float*>(tb + o_pv) : nullptr;
    auto* pos_of = reinterpret_cast<int32_t*>(tb + o_pos);
    auto* plid = reinterpret_cast<int32_t*>(tb + o_plid);
    const auto* kp = reinterpret_cast<const uint64_t*>(keys_.data_ptr());
    wh::loc_part_hist(kp, ptr<int64_t>(offset_), nrows, nsh, plan_, hv, hist, s);
    wh::loc_part_offsets(plan_, hist, gsum, base, s);
    wh::loc_part_scatter(kp, vp, ptr<int64_t>(offset_), nrows, nsh, plan_, hv, base, gsum, hist, pk,
                         pr, pv, pos_of, s);
    auto* pw = reinterpret_cast<unsigned long long*>(ws.part_ws.data_ptr());
    wh::loc_part_dedup(pk, pr, pv, nnz, nsh, plan_, hv, base,
                       wh::lookback_bind(ws.lb_loc.data_ptr()),
                       reinterpret_cast<uint64_t*>(uniq_.data_ptr()), ptr<int32_t>(ucnt_),
                       ptr<int64_t>(csc_off_), ptr<int32_t>(csc_row_),
                       vp ? ptr<float>(csc_val_) : nullptr, plid, pw,
                       reinterpret_cast<unsigned int*>(pw + wh::kPartMaxDigits),
                       ptr<int64_t>(owner_cnt), s, loc_timing() ? ptr<int64_t>(loc_timing_buf()) : nullptr);
    wh::loc_part_lid(pos_of, plid, nnz, ptr<int32_t>(lid_), s);
    return owner_cnt;
  }

  void enqueue() {
    auto s = cur_stream(keys_);
    DevWs& ws = dev_ws(keys_.device());
    auto i32 = keys_.options().dtype(torch::kInt32);
    auto i64 = keys_.options().dtype(torch::kInt64);
    Tensor owner_cnt;
    if (part_) {
      owner_cnt = enqueue_part();
    } else {
      owner_cnt = enqueue_hash(ws, s, i32, i64);
    }
    owner_cnt_ = owner_cnt;
    // (an overflow retry from counts() exchanges at once: every rank retries
    // there together)
    if (!defer_ || exchanged_) exchange_and_read(owner_cnt, s);
  }

  Tensor enqueue_hash(DevWs& ws, hipStream_t s, const torch::TensorOptions& i32,
                      const torch::TensorOptions& i64) {
    // The table is a persistent per-device slab that loc_assign leaves
    // empty, so a minibatch costs no clearing pass; it is re-filled only
    // after an overflow retry or an abandoned job (loc_dirty).
    if (ws.loc_tab[tab_].numel() < tsize_) {
      ws.loc_tab[tab_] = torch::full({safe_}, -1, i64);
      ws.loc_ovf[tab_].zero_();
      ws.loc_dirty[tab_] = false;
    } else if (ws.loc_dirty[tab_]) {
      ws.loc_tab[tab_].fill_(-1);
      ws.loc_ovf[tab_].zero_();
      ws.loc_dirty[tab_] = false;
    }
    tkeys_ = ws.loc_tab[tab_].narrow(0, 0, tsize_);
    ws.loc_dirty[tab_] = true;  // until loc_assign has run
    slot_of_ = torch::empty({std::max<int64_t>(nnz_, 1)}, i32);
    auto owner_cnt = torch::empty({nshard_ + 1}, i64);  // [nshard] = overflow count
    wh::loc_insert(reinterpret_cast<const uint64_t*>(keys_.data_ptr()), nnz_,
                   reinterpret_cast<uint64_t*>(tkeys_.data_ptr()), tsize_,
                   ptr<int32_t>(slot_of_), ptr<int64_t>(ws.loc_ovf[tab_]), s);
    blkoff_ = torch::empty({nshard_ * wh::loc_owner_blocks(tsize_)}, i64);
    wh::loc_owner_count(reinterpret_cast<const uint64_t*>(tkeys_.data_ptr()), tsize_,
                        (int)nshard_, ptr<int64_t>(blkoff_), ptr<int64_t>(owner_cnt),
                        ptr<int64_t>(ws.loc_ovf[tab_]), s);
    return owner_cnt;
  }

  void exchange_and_read(const Tensor& owner_cnt, hipStream_t s) {
    Tensor both = owner_cnt;
    nrecv_ = 0;
    hipStream_t cs = s;  // stream of the count read
    if (nex_) {
      auto r = nex_(owner_cnt);
      both = std::get<0>(r);
      cs = std::get<1>(r);
      stride_ = std::get<2>(r);
      const int64_t world = std::get<3>(r);
      TORCH_CHECK(both.scalar_type() == torch::kInt64 && stride_ >= 2 &&
                      both.numel() >= nshard_ + 1 + stride_ * world,
                  "localize: bad native exchange payload");
      nrecv_ = stride_ * world;
    } else if (!exchange_.is_none()) {
      py::object r = exchange_(owner_cnt);
      if (py::isinstance<py::tuple>(r)) {
        // extended protocol (kv/psx.py): (payload, stream handle, stride,
        // world). payload = [owner_cnt (nshard+1) | stride values per peer,
        // {count, overflow flag, ...} | extra], already on that stream;
        // the read goes on that stream so the compute stream never waits
        // for the exchange.
        auto t = r.cast<py::tuple>();
        TORCH_CHECK(t.size() == 4, "localize: extended exchange returns 4 items");
        both = t[0].cast<Tensor>();
        cs = reinterpret_cast<hipStream_t>(t[1].cast<intptr_t>());
        stride_ = t[2].cast<int64_t>();
        const int64_t world = t[3].cast<int64_t>();
        TORCH_CHECK(both.scalar_type() == torch::kInt64 && stride_ >= 2 &&
                        both.numel() >= nshard_ + 1 + stride_ * world,
                    "localize: bad extended exchange payload");
        nrecv_ = stride_ * world;
      } else {
        Tensor recv = r.cast<Tensor>();
        TORCH_CHECK(recv.scalar_type() == torch::kInt64 && recv.numel() % 2 == 0,
                    "localize: exchange must return int64 [2 * world]");
        stride_ = 2;
        nrecv_ = recv.numel();
        both = torch::cat({owner_cnt, recv.reshape({-1}).to(owner_cnt.device())});
      }
    }
    dev_counts_ = both.contiguous();
    DevWs& ws = dev_ws(keys_.device());
    if (rd_ && rd_->cap < dev_counts_.numel()) {  // (a retry: the last copy was waited for)
      rd_->busy = false;
      rd_ = nullptr;
    }
    if (!rd_) rd_ = ws.acquire_read(dev_counts_.numel());
    // an async copy into pinned memory + an event: nothing blocks here
    WH_HIP_CHECK_HOST(hipMemcpyAsync(rd_->host, dev_counts_.data_ptr(),
                                     dev_counts_.numel() * sizeof(int64_t),
                                     hipMemcpyDeviceToHost, cs));
    WH_HIP_CHECK_HOST(hipEventRecord(rd_->ev, cs));
  }

  Tensor keys_, offset_, val_;
  int64_t nshard_, nnz_ = 0, safe_ = 0, tsize_ = 0, nrecv_ = 0, stride_ = 2;
  py::object exchange_;
  NativeExchange nex_;
  bool defer_ = false, exchanged_ = false;
  Tensor owner_cnt_;
  int tab_ = -1;
  bool done_ = false;
  Tensor tkeys_, slot_of_, blkoff_, dev_counts_, owner_cnt_h_, recv_h_;
  Tensor uniq_, ucnt_, csc_off_, csc_row_, csc_val_, lid_;  // partitioned path outputs
  wh::PartPlan plan_{};
  bool part_ = false;
  bool counted_ = false;  // in DevWs::part_inflight
  DevWs::PinnedRead* rd_ = nullptr;  // the count read's pinned buffer + event
};

std::vector<Tensor> localize(const Tensor& keys, const Tensor& offset,
                             const c10::optional<Tensor>& val, int64_t nshard, int64_t hint,
                             py::object exchange) {
  LocalizeJob job(keys, offset, val, nshard, hint, exchange);
  return job.finish();
}

// --------------------------------------------------------------- KVStore
class KVStore {
 public:
  KVStore(int64_t cap, int64_t vcap, int64_t dim, int64_t device) {
    TORCH_CHECK(cap > 0 && (cap & (cap - 1)) == 0, "cap must be a power of two");
    TORCH_CHECK(dim >= 0 && dim <= 256, "embedding dim must be in [0, 256]");
    dim_ = dim;
    vstride_ = dim == 0 ? 0 : (int)(4 * next_pow2((dim + 3) / 4));
    auto dev = torch::Device(torch::kCUDA, device);
    c10::DeviceGuard g(dev);
    auto f32 = torch::TensorOptions().dtype(torch::kFloat32).device(dev);
    // AoS slot table [cap, 8] x 4 bytes = wh::KVSlot; the per-field tensors
    // below are strided views into it (shared storage, writable)
    auto sl = torch::zeros({cap, 8}, f32.dtype(torch::kInt32));
    sl.view(torch::kInt64).select(1, 0).fill_(-1);  // key: empty
    sl.select(1, 5).fill_(-1);                      // vrow: none
    set_slots(sl);
    if (dim > 0) {
      V_ = torch::zeros({std::max<int64_t>(vcap, 1), vstride_}, f32);
      VG_ = torch::zeros({std::max<int64_t>(vcap, 1), vstride_}, f32);
    }
    vnext_ = torch::zeros({1}, f32.dtype(torch::kInt32));
    stats_ = torch::zeros({wh::kStatShards, wh::kStatStride}, f32.dtype(torch::kInt64));
    cap_ = cap;
    vcap_ = dim > 0 ? vcap : 0;
  }

  wh::KVTable table() const {
    wh::KVTable t;
    t.sl = reinterpret_cast<wh::KVSlot*>(slots_.data_ptr());
    t.V = dim_ > 0 ? ptr<float>(V_) : nullptr;
    t.VG = dim_ > 0 ? ptr<float>(VG_) : nullptr;
    t.vnext = ptr<int32_t>(vnext_);
    t.stats = ptr<int64_t>(stats_);
    t.cap = cap_;
    t.vcap = vcap_;
    t.vstride = vstride_;
    t.dim = (int)dim_;
    return t;
  }

  Tensor find(const Tensor& keys, bool insert) {
    CHECK_IN(keys, torch::kInt64);
    c10::DeviceGuard g(keys.device());
    auto slot = torch::empty({keys.numel()}, keys.options().dtype(torch::kInt32));
    wh::kv_find(table(), reinterpret_cast<const uint64_t*>(keys.data_ptr()), keys.numel(),
                insert ? 1 : 0, ptr<int32_t>(slot), cur_stream(keys));
    return slot;
  }

  Tensor occupied() {
    c10::DeviceGuard g(keys_.device());
    auto out = torch::empty({cap_}, keys_.options().dtype(torch::kInt32));
    auto n = torch::zeros({1}, keys_.options());
    wh::kv_occupied(table(), ptr<int32_t>(out), ptr<int64_t>(n), cur_stream(keys_));
    return out.narrow(0, 0, n.item<int64_t>());
  }

  Tensor linear_pull(const Tensor& slot) {
    CHECK_IN(slot, torch::kInt32);
    c10::DeviceGuard g(slot.device());
    auto out = torch::empty({slot.numel()}, slot.options().dtype(torch::kFloat32));
    wh::linear_pull(table(), ptr<int32_t>(slot), slot.numel(), ptr<float>(out), cur_stream(slot));
    return out;
  }

  void linear_push(const Tensor& slot, const Tensor& grad, int64_t algo, double alpha, double beta,
                   double l1, double l2, double sgd_eta) {
    CHECK_IN(slot, torch::kInt32);
    CHECK_IN(grad, torch::kFloat32);
    TORCH_CHECK(grad.numel() >= slot.numel());
    c10::DeviceGuard g(slot.device());
    wh::LinearHP hp{(int)algo, (float)alpha, (float)beta, (float)l1, (float)l2, (float)sgd_eta};
    wh::linear_push(table(), ptr<int32_t>(slot), ptr<float>(grad), slot.numel(), hp,
                    cur_stream(slot));
  }

  static wh::DifactoHP dhp(const std::vector<double>& h, int64_t threshold, bool l1_shrk,
                           int64_t seed) {
    TORCH_CHECK(h.size() == 8, "difacto hyper-parameter vector must have 8 entries");
    wh::DifactoHP hp;
    hp.alpha = (float)h[0]; hp.beta = (float)h[1]; hp.l1 = (float)h[2]; hp.l2 = (float)h[3];
    hp.v_alpha = (float)h[4]; hp.v_beta = (float)h[5]; hp.v_l2 = (float)h[6];
    hp.v_init = (float)h[7];
    hp.threshold = (uint32_t)threshold;
    hp.l1_shrk = l1_shrk ? 1 : 0;
    hp.seed = (uint64_t)seed;
    return hp;
  }

  void difacto_push_cnt(const Tensor& slot, const Tensor& cnt, const std::vector<double>& h,
                        int64_t threshold, bool l1_shrk, int64_t seed) {
    CHECK_IN(slot, torch::kInt32);
    CHECK_DEV(cnt); CHECK_CONT(cnt);
    TORCH_CHECK(cnt.scalar_type() == torch::kFloat32 || cnt.scalar_type() == torch::kInt32,
                "counts must be float32 or int32");
    TORCH_CHECK(cnt.numel() >= slot.numel());
    c10::DeviceGuard g(slot.device());
    const bool f = cnt.scalar_type() == torch::kFloat32;
    wh::difacto_push_cnt(table(), ptr<int32_t>(slot), f ? ptr<float>(cnt) : nullptr,
                         f ? nullptr : ptr<int32_t>(cnt), slot.numel(),
                         dhp(h, threshold, l1_shrk, seed), cur_stream(slot));
  }

  // Variable-length pull. Returns (hdr [n,2] f32 {w, vidx bits}, vc [mcap, vstride],
  // vpos i64 [n+1]); m = vpos[n] stays on the device (vc is sized by the
  // host-side bound mcap = n so the step needs no host synchronisation).
  std::vector<Tensor> difacto_pull(const Tensor& slot, bool l1_shrk) {
    CHECK_IN(slot, torch::kInt32);
    c10::DeviceGuard g(slot.device());
    auto s = cur_stream(slot);
    const int64_t n = slot.numel();
    auto f32 = slot.options().dtype(torch::kFloat32);
    auto hdr = torch::empty({n, 2}, f32);
    const int64_t mcap = vstride_ > 0 ? n : 0;
    auto vc = torch::empty({mcap, (int64_t)std::max(vstride_, 1)}, f32);
    if (n > 0) {
      auto vpos = torch::empty({n + 1}, slot.options().dtype(torch::kInt64));
      if (wh::difacto_pull_fused(table(), ptr<int32_t>(slot), n, l1_shrk ? 1 : 0,
                                 lookback(slot.device()), ptr<float>(hdr), ptr<int64_t>(vpos),
                                 ptr<float>(vc), s))
        return {hdr, vc, vpos};
    }
    auto vflag = torch::empty({std::max<int64_t>(n, 1)}, slot.options());
    auto vpos = torch::zeros({n + 1}, slot.options().dtype(torch::kInt64));
    wh::difacto_pull_hdr(table(), ptr<int32_t>(slot), n, l1_shrk ? 1 : 0, ptr<float>(hdr),
                         ptr<int32_t>(vflag), s);
    if (vstride_ > 0 && n > 0) {
      auto stmp = torch::empty({wh::scan_tmp_elems(n)}, vpos.options());
      wh::scan_i32(ptr<int32_t>(vflag), ptr<int64_t>(vpos), n, ptr<int64_t>(stmp), s);
      wh::difacto_pull_rows(table(), ptr<int32_t>(slot), n, ptr<int32_t>(vflag),
                            ptr<int64_t>(vpos), ptr<float>(hdr), ptr<float>(vc), s);
    }
    return {hdr, vc, vpos};
  }

  // Single-shard open + pull in one launch. Returns (slot i32 [n], hdr, vc,
  // vpos) like find() followed by difacto_push_cnt() (when cnt is given) and
  // difacto_pull(). Keys must be distinct.
  std::vector<Tensor> difacto_open_pull(const Tensor& keys, bool insert,
                                        const c10::optional<Tensor>& cnt,
                                        const std::vector<double>& h, int64_t threshold,
                                        bool l1_shrk, int64_t seed, bool direct) {
    CHECK_IN(keys, torch::kInt64);
    const int32_t* cp = nullptr;
    if (cnt.has_value() && cnt->defined()) {
      CHECK_IN((*cnt), torch::kInt32);
      TORCH_CHECK(cnt->numel() >= keys.numel(), "open_pull: count size mismatch");
      cp = ptr<int32_t>(*cnt);
    }
    c10::DeviceGuard g(keys.device());
    auto s = cur_stream(keys);
    const int64_t n = keys.numel();
    auto f32 = keys.options().dtype(torch::kFloat32);
    auto slot = torch::empty({n}, keys.options().dtype(torch::kInt32));
    auto hdr = torch::empty({n, 2}, f32);
    auto vpos = torch::empty({n + 1}, keys.options());
    // direct: no pulled copy -- hdr's vidx column holds the table's V row and
    // the "pulled rows" are the V slab itself (one shard: the forward and
    // backward read the rows in place; the push writes them after both)
    direct = direct && vstride_ > 0;
    auto vc = direct ? V_ : torch::empty({vstride_ > 0 ? n : 0, (int64_t)std::max(vstride_, 1)}, f32);
    if (n == 0) {
      vpos.zero_();
      return {slot, hdr, vc, vpos};
    }
    if (!wh::difacto_open_pull(table(), reinterpret_cast<const uint64_t*>(keys.data_ptr()), n,
                               cp, dhp(h, threshold, l1_shrk, seed), insert ? 1 : 0,
                               lookback(keys.device()), ptr<int32_t>(slot), ptr<float>(hdr),
                               ptr<int64_t>(vpos), direct ? nullptr : ptr<float>(vc), s)) {
      // (too many keys for the one-launch path: the compact pull below)
      slot = find(keys, insert);
      if (cp) difacto_push_cnt(slot, *cnt, h, threshold, l1_shrk, seed);
      auto r = difacto_pull(slot, l1_shrk);
      return {slot, r[0], r[1], r[2]};
    }
    return {slot, hdr, vc, vpos};
  }

  // hdr: this shard's pull header for the same keys (owner vidx numbering)
  void difacto_push(const Tensor& slot, const Tensor& hdr, const Tensor& gw, const Tensor& gvc,
                    const std::vector<double>& h, int64_t threshold, bool l1_shrk,
                    int64_t seed) {
    CHECK_IN(slot, torch::kInt32);
    CHECK_IN(hdr, torch::kFloat32);
    CHECK_IN(gw, torch::kFloat32);
    CHECK_DEV(gvc); CHECK_CONT(gvc); CHECK_DT(gvc, torch::kFloat32);
    const int64_t n = slot.numel();
    TORCH_CHECK(hdr.numel() == 2 * n && gw.numel() == n, "push: hdr/gw size mismatch");
    TORCH_CHECK(vstride_ == 0 || (gvc.dim() == 2 && gvc.size(1) == vstride_),
                "push: gvc must be [m, vstride]");
    c10::DeviceGuard g(slot.device());
    wh::difacto_push(table(), ptr<int32_t>(slot), ptr<float>(hdr), ptr<float>(gw),
                     gvc.numel() ? ptr<float>(gvc) : nullptr, n, dhp(h, threshold, l1_shrk, seed),
                     cur_stream(slot));
  }

  // ---------------------------------------------------- multi-shard (psx.hip)
  // Owner side of a P-shard minibatch. keys: int64 [n] or int32 records
  // [n, 3] {key lo, key hi, count}; segS / segHS: device int64 [P+1]; rows_cap:
  // rows of the reply buffer to allocate (>= segHS[P] + n). Returns (slot,
  // vpos [n+1], chain [n] (int32 view of the chain links), head uint8 [n],
  // rbuf [rows_cap, vstride], vcnt [P]).
  // chain_in: a chain buffer [>= n] the preceding push on this stream
  // zeroed (ps_push prep_chain), with vbase snapshotted there too: the open
  // then skips its own prep launch
  std::vector<Tensor> ps_open(const Tensor& keys, bool use_cnt, const Tensor& segS,
                              const Tensor& segHS, int64_t rows_cap, bool insert, bool chains,
                              const std::vector<double>& h, int64_t threshold, bool l1_shrk,
                              int64_t seed, const c10::optional<Tensor>& chain_in = c10::nullopt) {
    CHECK_DEV(keys); CHECK_CONT(keys);
    CHECK_IN(segS, torch::kInt64);
    CHECK_IN(segHS, torch::kInt64);
    const bool rec = keys.scalar_type() == torch::kInt32;
    TORCH_CHECK(rec ? (keys.dim() == 2 && keys.size(1) == 3) : keys.scalar_type() == torch::kInt64,
                "ps_open: keys must be int64 [n] or int32 records [n, 3]");
    TORCH_CHECK(!use_cnt || rec, "ps_open: counts travel in the records");
    const int64_t n = keys.size(0);
    const int P = (int)segS.numel() - 1;
    TORCH_CHECK(P >= 1 && segHS.numel() == P + 1, "ps_open: bad segment tables");
    TORCH_CHECK(n < (1 << 24), "ps_open: at most 2^24 - 1 keys per minibatch and shard");
    epoch_ = epoch_ % 255 + 1;  // 1..255; a wrap to 1 sweeps the table's tags
    ++opens_;
    TORCH_CHECK(vstride_ == 0 || rows_cap >= n, "ps_open: reply buffer too small");
    c10::DeviceGuard g(keys.device());
    auto s = cur_stream(keys);
    auto i32 = keys.options().dtype(torch::kInt32);
    auto f32 = keys.options().dtype(torch::kFloat32);
    // the open's outputs from ONE allocation (see LocalizeJob::enqueue_part)
    const int64_t n1 = std::max<int64_t>(n, 1);
    int64_t at = 0;
    auto carve = [&](int64_t bytes) {
      const int64_t o = at;
      at += (bytes + 255) / 256 * 256;
      return o;
    };
    const int64_t o_s = carve(n1 * 4), o_w = carve(n1 * 4), o_p = carve((n + 1) * 8),
                  o_h = carve(n1);
    auto blk = torch::empty({at}, keys.options().dtype(torch::kUInt8));
    auto slot = blk.narrow(0, o_s, n1 * 4).view(torch::kInt32);
    auto wout = blk.narrow(0, o_w, n1 * 4).view(torch::kFloat32);
    auto vpos = blk.narrow(0, o_p, (n + 1) * 8).view(torch::kInt64);
    const bool prepped = chain_in.has_value() && chain_in->defined() && chain_in->numel() > 0;
    if (prepped) {
      CHECK_IN((*chain_in), torch::kInt32);
      TORCH_CHECK(chain_in->numel() >= std::max<int64_t>(n, 1), "ps_open: prepped chain too small");
      TORCH_CHECK(vbase_.defined(), "ps_open: prepped without a push prep");
    }
    auto chain = prepped ? *chain_in : torch::empty({n1}, i32);
    auto head = blk.narrow(0, o_h, n1);
    // linear (vstride 0): the reply is w_out itself (returned in rbuf's place)
    auto rbuf = torch::empty({vstride_ > 0 ? rows_cap : 0, (int64_t)std::max(vstride_, 1)}, f32);
    // linear: no V rows, a cached all-zero vcnt (read only; no fill launch per open)
    Tensor vcnt;
    if (vstride_ == 0) {
      if (!vcnt0_.defined() || vcnt0_.numel() != P || vcnt0_.device() != keys.device())
        vcnt0_ = torch::zeros({P}, keys.options().dtype(torch::kInt64));
      vcnt = vcnt0_;
    } else {
      vcnt = torch::empty({P}, keys.options().dtype(torch::kInt64));
    }
    if (!vbase_.defined()) vbase_ = torch::empty({1}, vnext_.options());
    const bool ok = wh::ps_open(
        table(), rec ? nullptr : reinterpret_cast<const uint64_t*>(keys.data_ptr()),
        rec ? ptr<int32_t>(keys) : nullptr, n, use_cnt ? 1 : 0, dhp(h, threshold, l1_shrk, seed),
        insert ? 1 : 0, chains ? 1 : 0, (uint32_t)epoch_, ptr<int32_t>(vbase_),
        ptr<int64_t>(segS), ptr<int64_t>(segHS), P, lookback(keys.device()), ptr<int32_t>(slot),
        ptr<float>(wout), ptr<int64_t>(vpos), reinterpret_cast<uint32_t*>(chain.data_ptr()),
        reinterpret_cast<uint8_t*>(head.data_ptr()), ptr<float>(rbuf), ptr<int64_t>(vcnt), s,
        prepped ? 1 : 0);
    TORCH_CHECK(ok, "ps_open: limits exceeded (P <= 256, n < 2^24)");
    return {slot.narrow(0, 0, n), vpos, chain.narrow(0, 0, n), head.narrow(0, 0, n),
            vstride_ > 0 ? rbuf : wout.narrow(0, 0, n), vcnt};
  }

  // the next open's prep folded into a push (see ps_open chain_in): zero
  // prep_chain's first prep_n entries and snapshot vnext into vbase
  wh::PsPrep push_prep(const c10::optional<Tensor>& prep_chain, int64_t prep_n) {
    wh::PsPrep pr;
    if (!(prep_chain.has_value() && prep_chain->defined() && prep_chain->numel() > 0)) return pr;
    CHECK_IN((*prep_chain), torch::kInt32);
    TORCH_CHECK(prep_n >= 0 && prep_n <= prep_chain->numel(), "push prep: chain too small");
    if (!vbase_.defined()) vbase_ = torch::empty({1}, vnext_.options());
    pr.chain = reinterpret_cast<uint32_t*>(prep_chain->data_ptr());
    pr.n = prep_n;
    pr.vbase = ptr<int32_t>(vbase_);
    return pr;
  }

  // Linear owner push of a P-shard minibatch: g [n] = the gradients pushed
  // for this owner's received keys (segment order); t0 = SGD requests so far.
  void ps_push_linear(const Tensor& slot, const c10::optional<Tensor>& chain,
                      const c10::optional<Tensor>& head, const Tensor& segS, const Tensor& g,
                      int64_t algo, double alpha, double beta, double l1, double l2, double t0,
                      const c10::optional<Tensor>& prep_chain = c10::nullopt,
                      int64_t prep_n = 0) {
    CHECK_IN(slot, torch::kInt32);
    CHECK_IN(segS, torch::kInt64);
    CHECK_IN(g, torch::kFloat32);
    const int64_t n = slot.numel();
    TORCH_CHECK(g.numel() == n, "ps_push_linear: gradient size mismatch");
    TORCH_CHECK(vstride_ == 0, "ps_push_linear needs a linear store");
    const uint32_t* cp = nullptr;
    const uint8_t* hp = nullptr;
    if (chain.has_value() && chain->defined()) {
      CHECK_IN((*chain), torch::kInt32);
      TORCH_CHECK(head.has_value() && head->defined() && chain->numel() == n &&
                      head->numel() == n, "ps_push_linear: chain / head size mismatch");
      cp = reinterpret_cast<const uint32_t*>(chain->data_ptr());
      hp = reinterpret_cast<const uint8_t*>(head->data_ptr());
    }
    c10::DeviceGuard dg(slot.device());
    wh::LinearHP h{(int)algo, (float)alpha, (float)beta, (float)l1, (float)l2, 0.f};
    TORCH_CHECK(wh::ps_push_linear(table(), ptr<int32_t>(slot), cp, hp, n, ptr<int64_t>(segS),
                                   (int)segS.numel() - 1, ptr<float>(g), h, t0, cur_stream(slot),
                                   push_prep(prep_chain, prep_n)),
                "ps_push_linear: limits exceeded (P <= 256)");
  }

  // Owner side push of a P-shard minibatch: gbuf = the received push buffer
  // (rows in the reply layout of the matching ps_open).
  void ps_push(const Tensor& slot, const Tensor& vpos, const c10::optional<Tensor>& chain,
               const c10::optional<Tensor>& head, const Tensor& segS, const Tensor& segHS,
               const Tensor& gbuf, const std::vector<double>& h, int64_t threshold, bool l1_shrk,
               int64_t seed, const c10::optional<Tensor>& prep_chain = c10::nullopt,
               int64_t prep_n = 0) {
    CHECK_IN(slot, torch::kInt32);
    CHECK_IN(vpos, torch::kInt64);
    CHECK_IN(segS, torch::kInt64);
    CHECK_IN(segHS, torch::kInt64);
    CHECK_IN(gbuf, torch::kFloat32);
    const int64_t n = slot.numel();
    TORCH_CHECK(vpos.numel() == n + 1, "ps_push: vpos size mismatch");
    const uint32_t* cp = nullptr;
    const uint8_t* hp = nullptr;
    if (chain.has_value() && chain->defined()) {
      CHECK_IN((*chain), torch::kInt32);
      TORCH_CHECK(head.has_value() && head->defined(), "ps_push: chain without head flags");
      CHECK_IN((*head), torch::kUInt8);
      TORCH_CHECK(chain->numel() == n && head->numel() == n, "ps_push: chain size mismatch");
      cp = reinterpret_cast<const uint32_t*>(chain->data_ptr());
      hp = reinterpret_cast<const uint8_t*>(head->data_ptr());
    }
    const int P = (int)segS.numel() - 1;
    c10::DeviceGuard g(slot.device());
    TORCH_CHECK(wh::ps_push(table(), ptr<int32_t>(slot), ptr<int64_t>(vpos), cp, hp, n,
                            ptr<int64_t>(segS), ptr<int64_t>(segHS), P, ptr<float>(gbuf),
                            dhp(h, threshold, l1_shrk, seed), cur_stream(slot),
                            push_prep(prep_chain, prep_n)),
                "ps_push: limits exceeded");
  }

  // ------------------------------------------------------- growth / health
  // Re-hash into a table of newcap (power of two) slots; returns the old ->
  // new slot map (int32 [old cap]) for the slot ids of in-flight sessions.
  Tensor grow(int64_t newcap) {
    TORCH_CHECK(newcap > cap_ && (newcap & (newcap - 1)) == 0,
                "grow: new capacity must be a larger power of two");
    c10::DeviceGuard g(slots_.device());
    auto s = cur_stream(slots_);
    auto ns = torch::zeros({newcap, 8}, slots_.options());
    ns.view(torch::kInt64).select(1, 0).fill_(-1);
    ns.select(1, 5).fill_(-1);
    auto remap = torch::empty({cap_}, slots_.options());
    wh::kv_rehash(reinterpret_cast<const wh::KVSlot*>(slots_.data_ptr()), cap_,
                  reinterpret_cast<wh::KVSlot*>(ns.data_ptr()), newcap, ptr<int32_t>(remap),
                  ptr<int64_t>(stats_), s);
    set_slots(ns);
    cap_ = newcap;
    return remap;
  }

  // enlarge the V slab to newvcap rows (rows keep their ids)
  void grow_v(int64_t newvcap) {
    TORCH_CHECK(dim_ > 0 && newvcap > vcap_, "grow_v: new capacity must be larger");
    c10::DeviceGuard g(slots_.device());
    auto f32 = V_.options();
    auto nv = torch::empty({newvcap, vstride_}, f32);
    auto ng = torch::empty({newvcap, vstride_}, f32);
    nv.narrow(0, 0, V_.size(0)).copy_(V_);
    ng.narrow(0, 0, VG_.size(0)).copy_(VG_);
    nv.narrow(0, V_.size(0), newvcap - V_.size(0)).zero_();
    ng.narrow(0, VG_.size(0), newvcap - VG_.size(0)).zero_();
    V_ = nv;
    VG_ = ng;
    vcap_ = newvcap;
  }

  // device int64 [4] {keys, failed inserts, V-slab overflows, V rows used}
  Tensor summary() {
    c10::DeviceGuard g(slots_.device());
    auto out = torch::empty({4}, stats_.options());
    wh::kv_summary(table(), ptr<int64_t>(out), cur_stream(slots_));
    return out;
  }

  // The summary written by its kernel straight into coherent host memory
  // (slot 0..3; the store guard alternates two), on the current stream; read
  // with summary_read once an event recorded after it has completed. A
  // 32-byte copy into pinned memory instead cost ~40 us of host time.
  void summary_async(int64_t slot) {
    TORCH_CHECK(slot >= 0 && slot < 4, "summary slot out of range");
    c10::DeviceGuard g(slots_.device());
    if (!sum_host_) {
      void* p = nullptr;
      WH_HIP_CHECK_HOST(hipHostMalloc(&p, 4 * 64, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(p, 0, 4 * 64);
      sum_host_.reset(static_cast<int64_t*>(p));
    }
    wh::kv_summary(table(), sum_host_.get() + 8 * slot, cur_stream(slots_));
  }
  std::vector<int64_t> summary_read(int64_t slot) const {
    TORCH_CHECK(sum_host_ && slot >= 0 && slot < 4, "no summary in that slot");
    const volatile int64_t* h = sum_host_.get() + 8 * slot;
    return {h[0], h[1], h[2], h[3]};
  }
  struct HostFree {
    void operator()(int64_t* p) const { (void)hipHostFree(p); }
  };
  std::unique_ptr<int64_t, HostFree> sum_host_;

  int64_t dim() const { return dim_; }
  int64_t vstride() const { return vstride_; }
  int64_t cap() const { return cap_; }
  int64_t vcap() const { return vcap_; }

  Tensor slots_, keys_, w_, z_, sq_, cnt_, vrow_, V_, VG_, vnext_, stats_, vbase_, vcnt0_;
  int64_t epoch_ = 0;  // ps_open chain-tag epoch (1..255)
  int64_t opens_ = 0;  // ps_open calls so far (tests: the epoch wrapped)

 private:
  void set_slots(const Tensor& sl) {
    slots_ = sl;
    auto as_i64 = slots_.view(torch::kInt64);   // [cap, 4]
    auto as_f32 = slots_.view(torch::kFloat32); // [cap, 8]
    keys_ = as_i64.select(1, 0);
    w_ = as_f32.select(1, 2);
    z_ = as_f32.select(1, 3);
    sq_ = as_f32.select(1, 4);
    vrow_ = slots_.select(1, 5);
    cnt_ = slots_.select(1, 6);
  }

  int64_t cap_ = 0, vcap_ = 0, dim_ = 0;
  int vstride_ = 0;
};

// --------------------------------------------------------------------- FM
// difacto: w_or_hdr = hdr [U,2], vc = [m, vstride]; linear: w_or_hdr = w [U]
std::vector<Tensor> fm_forward(const Tensor& offset, const Tensor& lid,
                               const c10::optional<Tensor>& val, const Tensor& w_or_hdr,
                               const c10::optional<Tensor>& vc, int64_t vstride,
                               const Tensor& label, int64_t loss, const Tensor& met) {
  CHECK_IN(offset, torch::kInt64);
  CHECK_IN(lid, torch::kInt32);
  CHECK_IN(w_or_hdr, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  CHECK_IN(met, torch::kFloat64);
  TORCH_CHECK(vstride >= 0 && vstride <= 256 && vstride % 4 == 0, "bad vstride");
  TORCH_CHECK(met.numel() >= 4, "met needs 4 doubles");
  const int64_t nrows = offset.numel() - 1;
  TORCH_CHECK(label.numel() == nrows, "label size mismatch");
  const float* vcp = nullptr;
  if (vstride > 0) {
    TORCH_CHECK(w_or_hdr.dim() == 2 && w_or_hdr.size(1) == 2, "hdr must be [U, 2]");
    TORCH_CHECK(vc.has_value() && vc->defined(), "vc required");
    CHECK_IN((*vc), torch::kFloat32);
    TORCH_CHECK(vc->numel() == 0 || (vc->dim() == 2 && vc->size(1) == vstride), "vc must be [m, vstride]");
    vcp = vc->numel() ? ptr<float>(*vc) : nullptr;
  }
  const float* vp = optptr<float>(val);
  c10::DeviceGuard g(offset.device());
  // py, dual, xv and the metric partials from ONE allocation (the views keep
  // it alive; four allocations were host time of the small-minibatch step)
  int64_t at = 0;
  auto carve = [&](int64_t bytes) {
    const int64_t o = at;
    at += (bytes + 255) / 256 * 256;
    return o;
  };
  const int64_t nxv = vstride > 0 ? nrows * vstride : 0;
  const int64_t o_py = carve(nrows * 4), o_du = carve(nrows * 4), o_xv = carve(nxv * 4),
                o_pt = carve(wh::fm_fwd_partials() * 8);
  auto blk = torch::empty({std::max<int64_t>(at, 256)}, offset.options().dtype(torch::kUInt8));
  auto py = blk.narrow(0, o_py, nrows * 4).view(torch::kFloat32);
  auto dual = blk.narrow(0, o_du, nrows * 4).view(torch::kFloat32);
  auto xv = blk.narrow(0, o_xv, nxv * 4).view(torch::kFloat32);
  auto part = blk.narrow(0, o_pt, wh::fm_fwd_partials() * 8).view(torch::kFloat64);
  // a 5th metric slot asks for the per-minibatch flipped accuracy (linear)
  const int lossf = (int)loss | (met.numel() >= 5 ? 256 : 0);
  wh::fm_forward(nrows, ptr<int64_t>(offset), ptr<int32_t>(lid), vp, ptr<float>(w_or_hdr), vcp,
                 (int)vstride, ptr<float>(label), lossf, ptr<float>(py), ptr<float>(dual),
                 vstride > 0 ? ptr<float>(xv) : nullptr, ptr<double>(met), ptr<double>(part),
                 ptr<unsigned int>(dev_ws(offset.device()).fwd_ticket), cur_stream(offset));
  return {py, dual, xv};
}

// Backward scratch + outputs, allocated by phase 1 (the plan):
// {gw, gvc, chunk_key, chunk_beg, meta_v, bucket_hist, chunk_cnt, chunk_off,
//  scan_tmp, det (empty unless deterministic)}
static std::vector<Tensor> fm_bwd_alloc(const Tensor& csc_off, int64_t nnz, int64_t U,
                                        int64_t vc_rows, int64_t vstride) {
  auto f32 = csc_off.options().dtype(torch::kFloat32);
  auto i32 = csc_off.options().dtype(torch::kInt32);
  auto i64 = csc_off.options().dtype(torch::kInt64);
  auto gw = torch::empty({U}, f32);
  Tensor gvc = vstride > 0 ? torch::empty({vc_rows, vstride}, f32) : torch::empty({0}, f32);
  const int64_t cap = wh::fm_bwd_chunks_bound(U, nnz);
  const int64_t mb = vstride > 0 ? wh::fm_bwd_meta_bound(U, nnz) : 1;
  Tensor det = deterministic() ? torch::empty({wh::fm_bwd_det_floats(U, nnz, (int)vstride)}, f32)
                               : torch::empty({0}, f32);
  return {gw, gvc, torch::empty({cap}, i32), torch::empty({cap}, i32),
          torch::empty({2 * 4 * mb}, i32), torch::empty({wh::fm_bwd_bucket_scratch()}, i32),
          torch::empty({std::max<int64_t>(2 * U, 1)}, i64), torch::empty({2 * (U + 1)}, i64),
          torch::empty({wh::scan_tmp_elems(U)}, i64), det};
}

// fm_bwd_alloc's layout with the scratch entries (2..9) taken from the
// stream's grow-only workspace (only gw / gvc are fresh: they are outputs)
static std::vector<Tensor> fm_bwd_alloc_ws(const Tensor& csc_off, int64_t nnz, int64_t U,
                                           int64_t vc_rows, int64_t vstride) {
  auto f32 = csc_off.options().dtype(torch::kFloat32);
  auto i32 = csc_off.options().dtype(torch::kInt32);
  auto i64 = csc_off.options().dtype(torch::kInt64);
  const int64_t cap = wh::fm_bwd_chunks_bound(U, nnz);
  const int64_t mb = vstride > 0 ? wh::fm_bwd_meta_bound(U, nnz) : 1;
  const int64_t need[8] = {cap, cap, 2 * 4 * mb, wh::fm_bwd_bucket_scratch(),
                           std::max<int64_t>(2 * U, 1), 2 * (U + 1), wh::scan_tmp_elems(U),
                           deterministic() ? wh::fm_bwd_det_floats(U, nnz, (int)vstride) : 0};
  const c10::TensorOptions opt[8] = {i32, i32, i32, i32, i64, i64, i64, f32};
  auto& ws = dev_ws(csc_off.device()).bwd_scratch[cur_stream(csc_off)];
  if (ws.size() != 8) ws.assign(8, Tensor());
  std::vector<Tensor> pl(10);
  pl[0] = torch::empty({U}, f32);
  pl[1] = vstride > 0 ? torch::empty({vc_rows, vstride}, f32) : torch::empty({0}, f32);
  for (int i = 0; i < 8; ++i) {
    if (!ws[i].defined() || ws[i].numel() < need[i])
      ws[i] = torch::empty({std::max<int64_t>(need[i] + need[i] / 4, 1)}, opt[i]);
    pl[2 + i] = need[i] == 0 ? ws[i].narrow(0, 0, 0) : ws[i];
  }
  return pl;
}

static void fm_bwd_launch(const std::vector<Tensor>& pl, const Tensor& csc_off,
                          const Tensor& csc_row, const float* csc_val, const float* dual,
                          const float* xv, const Tensor& w_or_hdr, const float* vcp,
                          int64_t vstride, int64_t nrows, int phase) {
  const int64_t U = csc_off.numel() - 1;
  const wh::Lookback lb = lookback(csc_off.device());
  const Tensor& gvc = pl[1];
  wh::fm_backward(U, csc_row.numel(), nrows, ptr<int64_t>(csc_off), ptr<int32_t>(csc_row),
                  csc_val, dual, xv, ptr<float>(w_or_hdr), vcp, (int)vstride, ptr<float>(pl[0]),
                  gvc.numel() ? ptr<float>(gvc) : nullptr, ptr<int32_t>(pl[2]),
                  ptr<int32_t>(pl[3]), ptr<int32_t>(pl[4]), ptr<int32_t>(pl[5]),
                  ptr<int64_t>(pl[6]), ptr<int64_t>(pl[7]), ptr<int64_t>(pl[8]), &lb,
                  cur_stream(csc_off), pl[9].numel() ? ptr<float>(pl[9]) : nullptr, phase);
}

static void fm_bwd_check(const Tensor& csc_off, const Tensor& csc_row, const Tensor& w_or_hdr,
                         int64_t vstride) {
  CHECK_IN(csc_off, torch::kInt64);
  CHECK_IN(csc_row, torch::kInt32);
  CHECK_IN(w_or_hdr, torch::kFloat32);
  TORCH_CHECK(vstride >= 0 && vstride <= 256 && vstride % 4 == 0, "bad vstride");
  TORCH_CHECK(w_or_hdr.numel() == (csc_off.numel() - 1) * (vstride > 0 ? 2 : 1),
              "w/hdr must have U rows");
}

// returns (gw [U], gvc [like vc]) (linear: gvc is empty)
std::vector<Tensor> fm_backward(const Tensor& csc_off, const Tensor& csc_row,
                                const c10::optional<Tensor>& csc_val, const Tensor& dual,
                                const c10::optional<Tensor>& xv, const Tensor& w_or_hdr,
                                const c10::optional<Tensor>& vc, int64_t vstride) {
  fm_bwd_check(csc_off, csc_row, w_or_hdr, vstride);
  CHECK_IN(dual, torch::kFloat32);
  c10::DeviceGuard g(csc_off.device());
  const float* vcp = nullptr;
  int64_t vrows = 0;
  if (vstride > 0) {
    TORCH_CHECK(vc.has_value() && vc->defined() && xv.has_value() && xv->defined(), "vc/xv required");
    CHECK_IN((*vc), torch::kFloat32);
    CHECK_IN((*xv), torch::kFloat32);
    vrows = vc->numel() ? vc->size(0) : 0;
    vcp = vc->numel() ? ptr<float>(*vc) : nullptr;
  }
  auto pl = fm_bwd_alloc_ws(csc_off, csc_row.numel(), csc_off.numel() - 1, vrows, vstride);
  fm_bwd_launch(pl, csc_off, csc_row, optptr<float>(csc_val), ptr<float>(dual),
                vstride > 0 ? optptr<float>(xv) : nullptr, w_or_hdr, vcp, vstride, dual.numel(), 0);
  return {pl[0], pl[1]};
}

// Phase 1 of the backward on the CURRENT stream (the planning that needs no
// dual: chunk lists, zeroed multi-chunk gradients, V-chunk bucketing); the
// returned plan is finished by fm_backward_run (same CSC / header / vc).
std::vector<Tensor> fm_backward_plan(const Tensor& csc_off, const Tensor& csc_row,
                                     const Tensor& w_or_hdr, int64_t vc_rows, int64_t nrows,
                                     int64_t vstride) {
  fm_bwd_check(csc_off, csc_row, w_or_hdr, vstride);
  TORCH_CHECK(vc_rows >= 0 && nrows >= 0, "bad sizes");
  c10::DeviceGuard g(csc_off.device());
  auto pl = fm_bwd_alloc(csc_off, csc_row.numel(), csc_off.numel() - 1, vc_rows, vstride);
  fm_bwd_launch(pl, csc_off, csc_row, nullptr, nullptr, nullptr, w_or_hdr, nullptr, vstride,
                nrows, 1);
  return pl;
}

std::vector<Tensor> fm_backward_run(const std::vector<Tensor>& plan, const Tensor& csc_off,
                                    const Tensor& csc_row, const c10::optional<Tensor>& csc_val,
                                    const Tensor& dual, const c10::optional<Tensor>& xv,
                                    const Tensor& w_or_hdr, const c10::optional<Tensor>& vc,
                                    int64_t vstride) {
  fm_bwd_check(csc_off, csc_row, w_or_hdr, vstride);
  CHECK_IN(dual, torch::kFloat32);
  TORCH_CHECK(plan.size() == 10, "fm_backward_run: not a backward plan");
  c10::DeviceGuard g(csc_off.device());
  const float* vcp = nullptr;
  if (vstride > 0) {
    TORCH_CHECK(vc.has_value() && vc->defined() && xv.has_value() && xv->defined(), "vc/xv required");
    CHECK_IN((*vc), torch::kFloat32);
    CHECK_IN((*xv), torch::kFloat32);
    TORCH_CHECK(plan[1].dim() == 2 && plan[1].size(0) == (vc->numel() ? vc->size(0) : 0),
                "fm_backward_run: vc rows differ from the plan's");
    vcp = vc->numel() ? ptr<float>(*vc) : nullptr;
  }
  TORCH_CHECK(plan[0].numel() == csc_off.numel() - 1, "fm_backward_run: U differs from the plan's");
  fm_bwd_launch(plan, csc_off, csc_row, optptr<float>(csc_val), ptr<float>(dual),
                vstride > 0 ? optptr<float>(xv) : nullptr, w_or_hdr, vcp, vstride, dual.numel(), 2);
  return {plan[0], plan[1]};
}

// gvc [mcap, vstride]; m: device int64 tensor holding the live row count
void fm_grad_post(const Tensor& gvc, const Tensor& m, int64_t dim, double clip, double dropout,
                  int64_t seed, bool normalize) {
  CHECK_IN(gvc, torch::kFloat32);
  CHECK_IN(m, torch::kInt64);
  if (gvc.numel() == 0) return;
  TORCH_CHECK(gvc.dim() == 2, "gvc must be [m, vstride]");
  const int64_t vstride = gvc.size(1);
  c10::DeviceGuard g(gvc.device());
  auto s = cur_stream(gvc);
  Tensor sumsq;
  if (normalize) sumsq = torch::zeros({1}, gvc.options().dtype(torch::kFloat64));
  wh::fm_grad_post(ptr<int64_t>(m), gvc.size(0), ptr<float>(gvc), (int)vstride, (int)dim,
                   (float)clip, (float)dropout, (uint64_t)seed,
                   normalize ? ptr<double>(sumsq) : nullptr, s);
  if (normalize)
    wh::fm_grad_scale(ptr<int64_t>(m), gvc.size(0), ptr<float>(gvc), (int)vstride, (int)dim,
                      ptr<double>(sumsq), s);
}

// worker side of the multi-shard exchange (psx.hip). rbuf: the received pull
// reply [R, vstride]; segS/segHS: int64 [P+1] over the keys sent per owner;
// vrecv: int64 [P] V rows received per owner. Returns (hdr [U, 2], rows
// int64 [1] = R actually used).
std::vector<Tensor> ps_unpack(const Tensor& rbuf, int64_t U, const Tensor& segS,
                              const Tensor& segHS, const Tensor& vrecv) {
  CHECK_IN(rbuf, torch::kFloat32);
  CHECK_IN(segS, torch::kInt64);
  CHECK_IN(segHS, torch::kInt64);
  CHECK_IN(vrecv, torch::kInt64);
  TORCH_CHECK(rbuf.dim() == 2, "ps_unpack: rbuf must be [R, vstride]");
  const int P = (int)segS.numel() - 1;
  TORCH_CHECK(segHS.numel() == P + 1 && vrecv.numel() == P, "ps_unpack: bad segment tables");
  c10::DeviceGuard g(rbuf.device());
  auto hdr = torch::empty({U, 2}, rbuf.options());
  auto rows = torch::empty({1}, segS.options());
  TORCH_CHECK(wh::ps_unpack(ptr<float>(rbuf), U, (int)rbuf.size(1), ptr<int64_t>(segS),
                            ptr<int64_t>(segHS), ptr<int64_t>(vrecv), P, ptr<float>(hdr),
                            ptr<int64_t>(rows), cur_stream(rbuf)),
              "ps_unpack: limits exceeded");
  return {hdr, rows};
}

// 12-byte key records {lo, hi, count} int32 [U, 3] (ucnt optional)
Tensor ps_records(const Tensor& uniq, const c10::optional<Tensor>& ucnt) {
  CHECK_IN(uniq, torch::kInt64);
  const int32_t* cp = nullptr;
  if (ucnt.has_value() && ucnt->defined()) {
    CHECK_IN((*ucnt), torch::kInt32);
    TORCH_CHECK(ucnt->numel() == uniq.numel(), "ps_records: count size mismatch");
    cp = ptr<int32_t>(*ucnt);
  }
  c10::DeviceGuard g(uniq.device());
  auto rec = torch::empty({uniq.numel(), 3}, uniq.options().dtype(torch::kInt32));
  wh::ps_records(reinterpret_cast<const uint64_t*>(uniq.data_ptr()), cp, uniq.numel(),
                 ptr<int32_t>(rec), cur_stream(uniq));
  return rec;
}

// C0 buffers from the owner counts [S+1] (S shards + the overflow flag), the
// V row counts [P] (optional) and this rank's has-data flag: (send int64
// [4P], payload int64 [S+1+5P]; payload[S+1 : S+1+4P] is the exchange's
// receive slot)
std::vector<Tensor> ps_c0(const Tensor& owner_cnt, const c10::optional<Tensor>& vcnt, int64_t P,
                          int64_t flag, bool loopback = false) {
  CHECK_IN(owner_cnt, torch::kInt64);
  const int S = (int)owner_cnt.numel() - 1;
  TORCH_CHECK(S >= 1 && S <= P, "ps_c0: owner counts must cover 1..P shards");
  const int64_t* vp = nullptr;
  if (vcnt.has_value() && vcnt->defined()) {
    CHECK_IN((*vcnt), torch::kInt64);
    TORCH_CHECK(vcnt->numel() == P, "ps_c0: vcnt size mismatch");
    vp = ptr<int64_t>(*vcnt);
  }
  c10::DeviceGuard g(owner_cnt.device());
  auto send = torch::empty({4 * P}, owner_cnt.options());
  auto payload = torch::empty({S + 1 + 5 * P}, owner_cnt.options());
  TORCH_CHECK(wh::ps_c0(ptr<int64_t>(owner_cnt), vp, S, (int)P, flag, ptr<int64_t>(send),
                        ptr<int64_t>(payload), cur_stream(owner_cnt), loopback ? 1 : 0),
              "ps_c0: too many peers");
  return {send, payload};
}

// gw [U] into the header rows of the push buffer gbuf [R, vstride] (in place)
void ps_pack_gw(const Tensor& gw, const Tensor& gbuf, const Tensor& segS, const Tensor& segHS,
                const Tensor& vrecv) {
  CHECK_IN(gw, torch::kFloat32);
  CHECK_IN(gbuf, torch::kFloat32);
  CHECK_IN(segS, torch::kInt64);
  CHECK_IN(segHS, torch::kInt64);
  CHECK_IN(vrecv, torch::kInt64);
  TORCH_CHECK(gbuf.dim() == 2, "ps_pack_gw: gbuf must be [R, vstride]");
  const int P = (int)segS.numel() - 1;
  c10::DeviceGuard g(gw.device());
  TORCH_CHECK(wh::ps_pack_gw(ptr<float>(gw), gw.numel(), (int)gbuf.size(1), ptr<int64_t>(segS),
                             ptr<int64_t>(segHS), ptr<int64_t>(vrecv), P, ptr<float>(gbuf),
                             cur_stream(gw)),
              "ps_pack_gw: limits exceeded");
}

// worker side of a multi-shard pull: renumber hdr vidx into local compact
// order; returns m as a device int64 [1] tensor
Tensor vidx_renumber(const Tensor& hdr) {
  CHECK_IN(hdr, torch::kFloat32);
  c10::DeviceGuard g(hdr.device());
  const int64_t n = hdr.numel() / 2;
  if (n > 0) {
    auto cnt = torch::empty({1}, hdr.options().dtype(torch::kInt64));
    if (wh::vidx_renumber_fused(ptr<float>(hdr), n, lookback(hdr.device()), ptr<int64_t>(cnt),
                                cur_stream(hdr)))
      return cnt;
  }
  auto flag = torch::empty({std::max<int64_t>(n, 1)}, hdr.options().dtype(torch::kInt32));
  auto pos = torch::zeros({n + 1}, hdr.options().dtype(torch::kInt64));
  auto stmp = torch::empty({wh::scan_tmp_elems(n)}, pos.options());
  wh::vidx_renumber(ptr<float>(hdr), n, ptr<int32_t>(flag), ptr<int64_t>(pos), ptr<int64_t>(stmp),
                    cur_stream(hdr));
  return pos.narrow(0, n, 1);
}

// WH_TIMING=step: host time per section of a native step, summed and
// printed (mean us per call) every 1000 calls and at exit -- the launch-
// bound small-minibatch path. WH_TIMING=step2: also the absolute
// steady-clock ns of every mark of calls 200..219 (to line up with a
// rocprofv3 kernel trace)
// every live split, so that a process leaving through os._exit (the bin/
// launchers) can still print them: timing_flush()
struct HostSplit;
std::mutex& split_mu() {
  static std::mutex m;
  return m;
}
std::vector<HostSplit*>& live_splits() {
  static auto* v = new std::vector<HostSplit*>();
  return *v;
}
struct HostSplit {
  const char* name;
  double us[10] = {};
  int64_t calls = 0;
  bool abs = false;
  std::vector<std::array<int64_t, 11>> marks;
  explicit HostSplit(const char* n) : name(n) {
    std::lock_guard<std::mutex> lk(split_mu());
    live_splits().push_back(this);
  }
  ~HostSplit() {
    std::lock_guard<std::mutex> lk(split_mu());
    auto& v = live_splits();
    v.erase(std::remove(v.begin(), v.end(), this), v.end());
  }
  HostSplit(const HostSplit&) = delete;
  HostSplit& operator=(const HostSplit&) = delete;
  void print() const {
    std::fprintf(stderr, "[%s host us/call over %lld]", name, (long long)calls);
    for (int i = 0; i < 10; ++i)
      if (us[i] > 0) std::fprintf(stderr, " s%d %.2f", i, us[i] / calls);
    std::fprintf(stderr, "\n");
    for (const auto& m : marks) {
      std::fprintf(stderr, "[%s marks ns]", name);
      for (int64_t v : m) std::fprintf(stderr, " %lld", (long long)v);
      std::fprintf(stderr, "\n");
    }
  }
};
class HostTimer {
 public:
  explicit HostTimer(HostSplit* h) : h_(h) {
    if (h_) {
      t_ = std::chrono::steady_clock::now();
      rec_ = h_->abs && h_->calls >= 200 && h_->calls < 220;
      if (rec_) m_.fill(0), m_[0] = ns(t_);
    }
  }
  void mark(int i) {
    if (!h_) return;
    const auto n = std::chrono::steady_clock::now();
    h_->us[i] += std::chrono::duration<double, std::micro>(n - t_).count();
    if (rec_ && i + 1 < 11) m_[i + 1] = ns(n);
    t_ = n;
  }
  ~HostTimer() {
    if (!h_) return;
    if (rec_) h_->marks.push_back(m_);
    if (++h_->calls % 1000 == 0) h_->print();
  }

 private:
  static int64_t ns(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(t.time_since_epoch()).count();
  }
  HostSplit* h_;
  std::chrono::steady_clock::time_point t_;
  bool rec_ = false;
  std::array<int64_t, 11> m_{};
};
// print every live split now (a short run's summary: the splits print every
// 1000 calls and at their step's destruction, which os._exit skips)
void timing_flush() {
  std::lock_guard<std::mutex> lk(split_mu());
  for (const HostSplit* h : live_splits())
    if (h->calls > 0) h->print();
  std::fflush(stderr);
}

static HostSplit* host_split(const char* name) {
  const bool abs = timing_on("step2");
  if (!abs && !timing_on("step")) return nullptr;
  auto* h = new HostSplit(name);
  h->abs = abs;
  return h;
}

// -------------------------------------------------------------- metrics
void auc_after_side(c10::DeviceIndex d, hipStream_t s);
// auc_sum[0] += exact AUC of (py, label) (sort-free bucketed rank sum)
void auc_acc(const Tensor& py, const Tensor& label, const Tensor& auc_sum) {
  CHECK_IN(py, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  CHECK_IN(auc_sum, torch::kFloat64);
  TORCH_CHECK(py.numel() == label.numel(), "auc: py/label size mismatch");
  TORCH_CHECK(py.numel() < (int64_t)1 << 30, "auc: at most 2^30 examples per call");
  c10::DeviceGuard g(py.device());
  auc_after_side(py.device().index(), cur_stream(py));  // (the workspace is shared)
  const int64_t n = py.numel();
  const int64_t wsb = wh::auc_ws_bytes(n);
  Tensor scratch;
  if (wsb) scratch = torch::empty({wsb}, py.options().dtype(torch::kUInt8));
  wh::auc_accumulate(ptr<float>(py), ptr<float>(label), n, dev_ws(py.device()).auc.data_ptr(),
                     wsb ? scratch.data_ptr() : nullptr, ptr<double>(auc_sum), cur_stream(py));
}

// The same on a per-device side stream owned here (it waits for the current
// stream first; auc_join makes the current stream wait for it): the Python
// form of this (stream objects, wait_stream, a stream context) cost ~30 us
// of host time per minibatch, which bounds small-minibatch training.
// Streams of the native layer's own (not the c10 pool's round-robin streams,
// one of which RCCL also takes for its internal stream): created once per
// device and role and never destroyed -- the caching allocator records
// events on every stream a block was used on when the block is freed, which
// can be after the step object that used the stream is gone.
enum OwnStream { kStreamLinearLs, kStreamPsxLs, kStreamPsxCs, kStreamPsxXs, kStreamAuc, kOwnStreams };
hipStream_t own_stream(int dev, int role) {
  static std::mutex mu;
  static std::map<std::pair<int, int>, hipStream_t> m;
  std::lock_guard<std::mutex> lk(mu);
  auto& h = m[{dev, role}];
  if (!h) WH_HIP_CHECK_HOST(hipStreamCreateWithFlags(&h, hipStreamNonBlocking));
  return h;
}

struct AucSide {
  c10::hip::HIPStream s;
  hipEvent_t in, out;
  bool dirty = false;  // AUC work queued on the side stream since the last join
};

AucSide* auc_side(c10::DeviceIndex d, bool create) {
  static std::map<int, AucSide*> m;
  auto it = m.find(d);
  if (it != m.end()) return it->second;
  if (!create) return nullptr;
  // a stream of its own: the pool's round-robin streams are shared (RCCL's
  // internal stream comes from the same pool), and AUC kernels queued on a
  // collective's stream would wait for it
  auto st = c10::hip::getStreamFromExternal(own_stream(d, kStreamAuc), d);
  auto* a = new AucSide{st, nullptr, nullptr};
  WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&a->in, hipEventDisableTiming));
  WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&a->out, hipEventDisableTiming));
  m[d] = a;
  return a;
}

// the stream s waits for the side stream's queued AUC work, if any
void auc_after_side(c10::DeviceIndex d, hipStream_t s) {
  AucSide* a = auc_side(d, false);
  if (!a || !a->dirty) return;
  WH_HIP_CHECK_HOST(hipEventRecord(a->out, a->s.stream()));
  WH_HIP_CHECK_HOST(hipStreamWaitEvent(s, a->out, 0));
  a->dirty = false;
}

// Optionally (WH_AUC_HOST_THREADS=N > 0), a large training minibatch's AUC
// on N host threads: the side stream copies (py, label) into pinned memory
// and a worker computes the exact AUC (csrc/host/auc_host.h: the device
// chain's definition) once the copy's event completes, so the GPU runs no
// AUC kernels. Each job remembers the auc_sum it belongs to; auc_join
// (auc_sum) waits for that tensor's jobs and adds their AUCs, folded in
// submission order (a deterministic sum). Off by default: on the headline
// step (100k rows) it measured level with the device chain (140.0 / 141.9 M
// vs 140.7 / 139.5 M, profiles/round6_p1_isolated.txt), although dropping
// the AUC altogether gains 3-5 % -- the side stream's event pair, the two
// copies and the join remain.
class HostAuc {
 public:
  // the pool new jobs go to (nullptr: the device chain)
  static HostAuc* get() {
    init();
    return on() ? pool() : nullptr;
  }
  // the pool pending jobs are in (also after enable(0))
  static HostAuc* any() {
    init();
    return pool();
  }
  static void enable(int nt) {
    init();
    if (nt > 0 && !pool()) pool() = new HostAuc(nt);
    on() = nt > 0;
  }

  void submit(const float* py, const float* lab, int64_t n, hipStream_t s, const void* target) {
    Job* j = nullptr;
    {
      std::unique_lock<std::mutex> lk(mu_);
      // back-pressure: the host falls this far behind only if its threads are starved
      space_cv_.wait(lk, [&] { return outstanding_ < kMaxOutstanding; });
      ++outstanding_;
      for (size_t k = 0; k < free_.size(); ++k)
        if (free_[k]->cap >= n) {
          j = free_[k];
          free_.erase(free_.begin() + k);
          break;
        }
    }
    if (!j) {
      j = new Job();
      WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&j->ev, hipEventDisableTiming));
    }
    if (j->cap < n) {
      if (j->buf) WH_HIP_CHECK_HOST(hipHostFree(j->buf));
      j->cap = std::max<int64_t>(n, 1 << 17);
      WH_HIP_CHECK_HOST(hipHostMalloc(reinterpret_cast<void**>(&j->buf), 2 * j->cap * sizeof(float),
                                      hipHostMallocDefault));
    }
    j->n = n;
    j->target = target;
    j->done = false;
    WH_HIP_CHECK_HOST(hipMemcpyAsync(j->buf, py, n * sizeof(float), hipMemcpyDeviceToHost, s));
    WH_HIP_CHECK_HOST(hipMemcpyAsync(j->buf + j->cap, lab, n * sizeof(float), hipMemcpyDeviceToHost, s));
    WH_HIP_CHECK_HOST(hipEventRecord(j->ev, s));
    std::lock_guard<std::mutex> lk(mu_);
    j->seq = next_seq_++;
    pending_.push_back(j);
    queue_.push_back(j);
    work_cv_.notify_one();
  }

  bool has(const void* target) {
    std::lock_guard<std::mutex> lk(mu_);
    if (acc_.count(target)) return true;
    for (Job* j : pending_)
      if (j->target == target) return true;
    return false;
  }

  // wait for target's jobs; their AUCs summed in submission order
  double join(const void* target) {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] {
      for (Job* j : pending_)
        if (j->target == target) return false;
      return true;
    });
    auto it = acc_.find(target);
    if (it == acc_.end()) return 0;
    const double sum = it->second;
    acc_.erase(it);
    return sum;
  }

 private:
  struct Job {
    hipEvent_t ev = nullptr;
    float* buf = nullptr;  // [cap] scores, then [cap] labels
    int64_t cap = 0, n = 0;
    const void* target = nullptr;
    uint64_t seq = 0;
    double result = 0;
    bool done = false;
  };
  static constexpr int kMaxOutstanding = 64;
  static HostAuc*& pool() {
    static HostAuc* p = nullptr;  // never destroyed: os._exit ends the process
    return p;
  }
  static bool& on() {
    static bool b = false;
    return b;
  }
  static void init() {
    static const bool once = [] {
      const char* e = std::getenv("WH_AUC_HOST_THREADS");
      const int nt = e ? std::atoi(e) : 0;
      if (nt > 0) pool() = new HostAuc(nt);
      on() = nt > 0;
      return true;
    }();
    (void)once;
  }

  explicit HostAuc(int nt) {
    for (int t = 0; t < nt; ++t) std::thread([this] { run(); }).detach();
  }

  void run() {
    std::vector<uint64_t> ws;
    for (;;) {
      Job* j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        work_cv_.wait(lk, [&] { return !queue_.empty(); });
        j = queue_.front();
        queue_.pop_front();
      }
      WH_HIP_CHECK_HOST(hipEventSynchronize(j->ev));
      const double r = wh::auc_exact_host(j->buf, j->buf + j->cap, j->n, ws);
      std::lock_guard<std::mutex> lk(mu_);
      j->result = r;
      j->done = true;
      // fold finished jobs into their target's sum in submission order (a
      // deterministic sum) and recycle them, so jobs never wait for a join
      while (!pending_.empty() && pending_.front()->done) {
        Job* f = pending_.front();
        pending_.pop_front();
        acc_[f->target] += f->result;
        free_.push_back(f);
        --outstanding_;
      }
      done_cv_.notify_all();
      space_cv_.notify_all();
    }
  }

  std::mutex mu_;
  std::condition_variable work_cv_, done_cv_, space_cv_;
  std::deque<Job*> queue_;
  std::deque<Job*> pending_;  // submitted, not yet folded (submission order)
  std::map<const void*, double> acc_;  // folded AUC sums per target
  std::vector<Job*> free_;
  uint64_t next_seq_ = 0;
  int outstanding_ = 0;
};

void auc_acc_side(const Tensor& py, const Tensor& label, const Tensor& auc_sum) {
  CHECK_IN(py, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  CHECK_IN(auc_sum, torch::kFloat64);
  TORCH_CHECK(py.numel() == label.numel(), "auc: py/label size mismatch");
  TORCH_CHECK(py.numel() < (int64_t)1 << 30, "auc: at most 2^30 examples per call");
  // a small minibatch's AUC is ONE launch of a few microseconds (the
  // pairwise k_auc_small): it runs in order on the current stream, without
  // the side stream's event pair (~4 us of host time in a launch-bound
  // 1000-row step)
  if (py.numel() <= 4096) return auc_acc(py, label, auc_sum);
  c10::DeviceGuard g(py.device());
  AucSide* a = auc_side(py.device().index(), true);
  WH_HIP_CHECK_HOST(hipEventRecord(a->in, cur_stream(py)));
  WH_HIP_CHECK_HOST(hipStreamWaitEvent(a->s.stream(), a->in, 0));
  c10::hip::HIPCachingAllocator::recordStream(py.storage().data_ptr(), a->s);
  c10::hip::HIPCachingAllocator::recordStream(label.storage().data_ptr(), a->s);
  if (HostAuc* h = HostAuc::get()) {  // (the copies touch no shared workspace: not dirty)
    h->submit(ptr<float>(py), ptr<float>(label), py.numel(), a->s.stream(), auc_sum.data_ptr());
    return;
  }
  a->dirty = true;
  c10::hip::HIPStreamGuard sg(a->s);  // the scratch is the side stream's
  const int64_t n = py.numel();
  const int64_t wsb = wh::auc_ws_bytes(n);
  Tensor scratch;
  if (wsb) scratch = torch::empty({wsb}, py.options().dtype(torch::kUInt8));
  wh::auc_accumulate(ptr<float>(py), ptr<float>(label), n, dev_ws(py.device()).auc.data_ptr(),
                     wsb ? scratch.data_ptr() : nullptr, ptr<double>(auc_sum), a->s.stream());
}

void auc_join(const Tensor& auc_sum) {
  if (!auc_sum.is_cuda()) return;
  c10::DeviceGuard g(auc_sum.device());
  auc_after_side(auc_sum.device().index(), cur_stream(auc_sum));
  HostAuc* h = HostAuc::any();
  if (h && h->has(auc_sum.data_ptr())) {
    const double s = h->join(auc_sum.data_ptr());
    auc_sum.add_(s);
  }
}

Tensor auc(const Tensor& py, const Tensor& label) {
  auto out = torch::zeros({1}, py.options().dtype(torch::kFloat64));
  auc_acc(py, label, out);
  return out;
}

// reference path: rocPRIM radix sort + rank-sum (kept as a cross-check)
Tensor auc_sorted(const Tensor& py, const Tensor& label) {
  CHECK_IN(py, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  c10::DeviceGuard g(py.device());
  const int64_t n = py.numel();
  auto pys = torch::empty_like(py);
  auto lab = torch::empty_like(label);
  const size_t sbytes = wh::auc_sort_tmp_bytes(n);
  auto stmp = torch::empty({(int64_t)sbytes + 16}, py.options().dtype(torch::kUInt8));
  wh::sort_by_score(ptr<float>(py), ptr<float>(label), n, ptr<float>(pys), ptr<float>(lab),
                    stmp.data_ptr(), sbytes, cur_stream(py));
  auto tmp = torch::empty({n / 2 + 1 + n + 1 + wh::scan_tmp_elems(n)},
                          py.options().dtype(torch::kInt64));
  auto out = torch::empty({2}, py.options().dtype(torch::kFloat64));
  wh::auc_from_sorted(ptr<float>(lab), n, ptr<double>(out), ptr<int64_t>(tmp), cur_stream(py));
  return out.narrow(0, 0, 1);
}

// keys % m (uint64 semantics), returned as a new tensor
Tensor key_mod(const Tensor& keys, int64_t m) {
  CHECK_IN(keys, torch::kInt64);
  TORCH_CHECK(m > 0, "max_key must be positive");
  c10::DeviceGuard g(keys.device());
  auto out = keys.clone();
  wh::key_mod(reinterpret_cast<uint64_t*>(out.data_ptr()), out.numel(), (uint64_t)m,
              cur_stream(keys));
  return out;
}

// ------------------------------------------------------- payload filter
// x [rows, w] f32 -> uint8 [rows, record_bytes]
Tensor quant_rows(const Tensor& x, int64_t nb, int64_t seed) {
  CHECK_IN(x, torch::kFloat32);
  TORCH_CHECK(nb >= 1 && nb <= 3, "fixed_bytes must be 1, 2 or 3");
  TORCH_CHECK(x.dim() == 2, "quant_rows: x must be [rows, w]");
  c10::DeviceGuard g(x.device());
  const int w = (int)x.size(1);
  auto out = torch::empty({x.size(0), wh::quant_record_bytes(w, (int)nb)},
                          x.options().dtype(torch::kUInt8));
  wh::quant_rows(ptr<float>(x), x.size(0), w, (int)nb, (uint64_t)seed, ptr<uint8_t>(out),
                 cur_stream(x));
  return out;
}

Tensor dequant_rows(const Tensor& q, int64_t w, int64_t nb) {
  CHECK_IN(q, torch::kUInt8);
  TORCH_CHECK(nb >= 1 && nb <= 3, "fixed_bytes must be 1, 2 or 3");
  TORCH_CHECK(q.dim() == 2 && q.size(1) == wh::quant_record_bytes((int)w, (int)nb),
              "dequant_rows: bad record size");
  c10::DeviceGuard g(q.device());
  auto x = torch::empty({q.size(0), w}, q.options().dtype(torch::kFloat32));
  wh::dequant_rows(ptr<uint8_t>(q), q.size(0), (int)w, (int)nb, ptr<float>(x), cur_stream(q));
  return x;
}

// region filter of the multi-shard exchange (quant.hip qregion_*): x the
// float layout (flat view), desc int64 [P, 6] on the device, built and
// bounds-checked on the host (kv/psx.py _QFilter) against x / out sizes.
Tensor ps_qpack(const Tensor& x, const Tensor& desc, int64_t rows, int64_t W, int64_t nb,
                int64_t seed) {
  CHECK_IN(x, torch::kFloat32);
  CHECK_IN(desc, torch::kInt64);
  TORCH_CHECK(nb >= 1 && nb <= 3 && W >= 1 && W <= 1024, "ps_qpack: bad record shape");
  TORCH_CHECK(desc.dim() == 2 && desc.size(1) == 6 && desc.size(0) >= 1, "ps_qpack: desc [P, 6]");
  c10::DeviceGuard g(x.device());
  auto out = torch::empty({rows, wh::quant_record_bytes((int)W, (int)nb)},
                          x.options().dtype(torch::kUInt8));
  wh::qregion_pack(ptr<float>(x), ptr<int64_t>(desc), (int)desc.size(0), rows, (int)W, (int)nb,
                   (uint64_t)seed, ptr<uint8_t>(out), cur_stream(x));
  return out;
}

void ps_qunpack(const Tensor& q, const Tensor& desc, int64_t W, int64_t nb, const Tensor& out) {
  CHECK_IN(q, torch::kUInt8);
  CHECK_IN(desc, torch::kInt64);
  CHECK_IN(out, torch::kFloat32);
  TORCH_CHECK(nb >= 1 && nb <= 3 && q.dim() == 2 &&
                  q.size(1) == wh::quant_record_bytes((int)W, (int)nb),
              "ps_qunpack: bad record size");
  TORCH_CHECK(desc.dim() == 2 && desc.size(1) == 6 && desc.size(0) >= 1, "ps_qunpack: desc [P, 6]");
  c10::DeviceGuard g(q.device());
  wh::qregion_unpack(ptr<uint8_t>(q), ptr<int64_t>(desc), (int)desc.size(0), q.size(0), (int)W,
                     (int)nb, ptr<float>(out), cur_stream(q));
}

Tensor trunc_u8(const Tensor& c) {
  CHECK_IN(c, torch::kInt32);
  c10::DeviceGuard g(c.device());
  auto out = torch::empty({c.numel()}, c.options().dtype(torch::kUInt8));
  wh::trunc_u8(ptr<int32_t>(c), c.numel(), ptr<uint8_t>(out), cur_stream(c));
  return out;
}

// ---------------------------------------------------------------- synth
std::vector<Tensor> synth_criteo(int64_t nrows, int64_t seed, int64_t step, const Tensor& card) {
  CHECK_IN(card, torch::kInt64);
  c10::DeviceGuard g(card.device());
  const int nfield = (int)card.numel();
  auto keys = torch::empty({nrows * nfield}, card.options());
  auto label = torch::empty({nrows}, card.options().dtype(torch::kFloat32));
  auto offset = torch::empty({nrows + 1}, card.options());
  wh::synth_criteo(nrows, (uint64_t)seed, (uint64_t)step, ptr<int64_t>(card), nfield,
                   reinterpret_cast<uint64_t*>(keys.data_ptr()), ptr<float>(label),
                   ptr<int64_t>(offset), cur_stream(card));
  return {keys, label, offset};
}

Tensor gather_rows(const Tensor& in, const Tensor& idx) {
  CHECK_IN(in, torch::kFloat32);
  CHECK_IN(idx, torch::kInt32);
  c10::DeviceGuard g(in.device());
  const int64_t width = in.dim() > 1 ? in.numel() / in.size(0) : 1;
  auto out = torch::empty({idx.numel(), width}, in.options());
  wh::gather_rows(ptr<float>(in), ptr<int32_t>(idx), idx.numel(), (int)width, ptr<float>(out),
                  cur_stream(in));
  return in.dim() > 1 ? out : out.view({idx.numel()});
}

int64_t vstride_for(int64_t dim) { return dim == 0 ? 0 : 4 * next_pow2((dim + 3) / 4); }

// ------------------------------------------------------------------ gbdt
Tensor gbdt_bin(const Tensor& X, const Tensor& cuts, const Tensor& cut_off) {
  CHECK_IN(X, torch::kFloat32);
  CHECK_IN(cuts, torch::kFloat32);
  CHECK_IN(cut_off, torch::kInt32);
  TORCH_CHECK(X.dim() == 2 && cut_off.numel() == X.size(1) + 1);
  c10::DeviceGuard g(X.device());
  auto B = torch::empty({X.size(0), X.size(1)}, X.options().dtype(torch::kUInt8));
  wh::gbdt_bin(ptr<float>(X), X.size(0), (int)X.size(1), ptr<float>(cuts), ptr<int32_t>(cut_off),
               ptr<uint8_t>(B), cur_stream(X));
  return B;
}

// tasks [T, 5] (slot, fbeg, fcnt, rbeg, rend); red [R, 6] (slot, fbeg, fcnt,
// t0, nt, tstride) sums the fp32 partials of tasks t0 + k * tstride into hist
// qscale [2] float32 = {2^eg, 2^eh}: fixed-point scales of g and h (see gbdt.hip);
// [3] = {2^eg, 2^eh, R}: int32 LDS sums over <= R rows (k_hist W32)
void gbdt_hist(const Tensor& B, int64_t nbin, const Tensor& ridx, const Tensor& gpair,
               const Tensor& qscale, const Tensor& tasks, const Tensor& red, int64_t max_fcnt,
               const Tensor& hist) {
  CHECK_IN(B, torch::kUInt8);
  CHECK_IN(ridx, torch::kInt32);
  CHECK_IN(gpair, torch::kFloat32);
  CHECK_IN(tasks, torch::kInt32);
  CHECK_IN(red, torch::kInt32);
  CHECK_IN(hist, torch::kFloat64);
  TORCH_CHECK(nbin >= 1 && nbin <= 255, "nbin must be in [1, 255]");
  CHECK_IN(qscale, torch::kFloat32);
  TORCH_CHECK(qscale.numel() == 2 || qscale.numel() == 3,
              "qscale must hold {scale_g, scale_h} or {scale_g, scale_h, int32 rows}");
  TORCH_CHECK(wh::gbdt_hist_lds((int)max_fcnt, (int)nbin) <= 160 * 1024, "feature group too wide");
  TORCH_CHECK(tasks.dim() == 2 && tasks.size(1) == 5);
  TORCH_CHECK(red.dim() == 2 && red.size(1) == 6);
  const int f = (int)B.size(1);
  TORCH_CHECK(hist.numel() % ((int64_t)f * nbin * 2) == 0, "hist must be [S, F, nbin, 2]");
  // dword row loads need every group 4-aligned; the caller guarantees equal
  // multiple-of-4 groups when f % 4 == 0 (checked again here on the host copy)
  bool dw = f % 4 == 0 && max_fcnt % 4 == 0;
  c10::DeviceGuard g(B.device());
  auto part = torch::empty({tasks.size(0) * wh::gbdt_hist_pstride((int)max_fcnt, (int)nbin)},
                           gpair.options().dtype(torch::kInt64));
  wh::gbdt_hist(ptr<uint8_t>(B), f, (int)nbin, ptr<int32_t>(ridx), ptr<float>(gpair),
                ptr<float>(qscale), ptr<int32_t>(tasks), (int)tasks.size(0), ptr<int32_t>(red),
                (int)red.size(0), (int)max_fcnt, dw, ptr<int64_t>(part), ptr<double>(hist),
                cur_stream(B), nullptr, 0, nullptr, qscale.numel() == 3);
}

// ------------------------------------------------------------------ lbfgs
Tensor owlqn_dir(const Tensor& g, const Tensor& w, double l1, const c10::optional<Tensor>& out) {
  CHECK_IN(g, torch::kFloat32);
  CHECK_IN(w, torch::kFloat32);
  TORCH_CHECK(g.numel() == w.numel());
  c10::DeviceGuard dg(g.device());
  Tensor d = out.has_value() ? *out : torch::empty_like(g);
  if (out.has_value()) {
    CHECK_IN(d, torch::kFloat32);
    TORCH_CHECK(d.numel() == g.numel(), "owlqn_dir: out size");
  }
  wh::owlqn_dir(ptr<float>(g), ptr<float>(w), g.numel(), (float)l1, ptr<float>(d), cur_stream(g));
  return d;
}

Tensor owlqn_fix_dot(const Tensor& d, const Tensor& steep, bool fix) {
  CHECK_IN(d, torch::kFloat32);
  CHECK_IN(steep, torch::kFloat32);
  TORCH_CHECK(d.numel() == steep.numel());
  c10::DeviceGuard dg(d.device());
  auto part = torch::empty({wh::owlqn_part_doubles()}, d.options().dtype(torch::kFloat64));
  auto v = torch::empty({1}, d.options().dtype(torch::kFloat64));
  wh::owlqn_fix_dot(ptr<float>(d), ptr<float>(steep), d.numel(), fix ? 1 : 0, ptr<double>(part),
                    ptr<double>(v), cur_stream(d));
  return v;
}

std::vector<Tensor> owlqn_step(const Tensor& w, const Tensor& d, double alpha, bool fix) {
  CHECK_IN(w, torch::kFloat32);
  CHECK_IN(d, torch::kFloat32);
  TORCH_CHECK(w.numel() == d.numel());
  c10::DeviceGuard dg(w.device());
  auto nw = torch::empty_like(w);
  auto part = torch::empty({wh::owlqn_part_doubles()}, w.options().dtype(torch::kFloat64));
  auto l1 = torch::empty({1}, w.options().dtype(torch::kFloat64));
  wh::owlqn_step(ptr<float>(w), ptr<float>(d), w.numel(), (float)alpha, fix ? 1 : 0,
                 ptr<float>(nw), ptr<double>(part), ptr<double>(l1), cur_stream(w));
  return {nw, l1};
}

// <H[r], H[probe k]> for every row r of the history [R, n]: [R, K] fp64
Tensor hist_dots(const Tensor& H, const std::vector<int64_t>& probes) {
  CHECK_IN(H, torch::kFloat32);
  TORCH_CHECK(H.dim() == 2, "hist_dots: H must be [R, n]");
  const int R = (int)H.size(0), K = (int)probes.size();
  std::vector<int32_t> pr(K);
  for (int k = 0; k < K; ++k) {
    TORCH_CHECK(probes[k] >= 0 && probes[k] < R, "hist_dots: probe row out of range");
    pr[k] = (int32_t)probes[k];
  }
  c10::DeviceGuard dg(H.device());
  auto part = torch::empty({wh::owlqn_part_doubles() * 4}, H.options().dtype(torch::kFloat64));
  auto out = torch::empty({R, K}, H.options().dtype(torch::kFloat64));
  TORCH_CHECK(wh::hist_dots(ptr<float>(H), R, H.size(1), H.size(1), pr.data(), K,
                            ptr<double>(part), ptr<double>(out), cur_stream(H)),
              "hist_dots: 1..4 probes, row length a multiple of 4");
  return out;
}

// the direction slice d = sum coef[r] H[rows[r]] (fp32, list order), sign
// fixed against H[steep_row]; returns (d, sum d * steep as fp64 [1])
std::vector<Tensor> dir_fix_dot(const Tensor& H, const std::vector<int64_t>& rows,
                                const std::vector<double>& coef, int64_t steep_row, bool fix,
                                int64_t n) {
  CHECK_IN(H, torch::kFloat32);
  TORCH_CHECK(H.dim() == 2 && rows.size() == coef.size() && rows.size() <= 64,
              "dir_fix_dot: <= 64 rows of H [R, n]");
  const int R = (int)H.size(0);
  std::vector<int32_t> r32(rows.size());
  std::vector<float> c32(rows.size());
  for (size_t i = 0; i < rows.size(); ++i) {
    TORCH_CHECK(rows[i] >= 0 && rows[i] < R, "dir_fix_dot: row out of range");
    r32[i] = (int32_t)rows[i];
    c32[i] = (float)coef[i];
  }
  TORCH_CHECK(steep_row >= 0 && steep_row < R, "dir_fix_dot: steep row out of range");
  if (n < 0) n = H.size(1);
  TORCH_CHECK(n <= H.size(1), "dir_fix_dot: n exceeds the row length");
  c10::DeviceGuard dg(H.device());
  auto d = torch::empty({n}, H.options());
  auto part = torch::empty({wh::owlqn_part_doubles()}, H.options().dtype(torch::kFloat64));
  auto v = torch::empty({1}, H.options().dtype(torch::kFloat64));
  wh::dir_fix_dot(ptr<float>(H), n, H.size(1), r32.data(), c32.data(), (int)rows.size(),
                  (int)steep_row, fix ? 1 : 0, ptr<float>(d), ptr<double>(part), ptr<double>(v),
                  cur_stream(H));
  return {d, v};
}

Tensor multi_dot(const Tensor& H, const Tensor& ia, const Tensor& ib) {
  CHECK_IN(H, torch::kFloat32);
  CHECK_IN(ia, torch::kInt32);
  CHECK_IN(ib, torch::kInt32);
  TORCH_CHECK(H.dim() == 2 && ia.numel() == ib.numel());
  c10::DeviceGuard dg(H.device());
  const int R = (int)H.size(0), np = (int)ia.numel();
  auto out = torch::zeros({np}, H.options().dtype(torch::kFloat64));
  TORCH_CHECK(wh::multi_dot(ptr<float>(H), R, H.size(1), ptr<int32_t>(ia), ptr<int32_t>(ib), np,
                            ptr<double>(out), cur_stream(H)),
              "multi_dot: at most 64 rows and 64 pairs");
  return out;
}

Tensor gbdt_split(const Tensor& hist, const Tensor& totals, const Tensor& valid, double alpha,
                  double lambda, double min_child_weight) {
  CHECK_IN(hist, torch::kFloat64);
  CHECK_IN(totals, torch::kFloat64);
  CHECK_IN(valid, torch::kBool);
  c10::DeviceGuard g(hist.device());
  TORCH_CHECK(hist.dim() == 4 && hist.size(3) == 2, "hist must be [S, F, nbin, 2]");
  const int S = (int)hist.size(0), F = (int)hist.size(1), nbin = (int)hist.size(2);
  TORCH_CHECK(totals.numel() == 2 * (int64_t)S, "totals must be [S, 2]");
  TORCH_CHECK(valid.numel() == (int64_t)F * nbin, "valid must be [F, nbin]");
  auto out = torch::empty({S, 6}, hist.options());
  auto cand = torch::empty({std::max<int64_t>((int64_t)S * F * 4, 1)}, hist.options());
  TORCH_CHECK(wh::gbdt_split(ptr<double>(hist), ptr<double>(totals),
                             reinterpret_cast<const uint8_t*>(valid.data_ptr()), S, F, nbin,
                             alpha, lambda, min_child_weight, ptr<double>(cand), ptr<double>(out),
                             cur_stream(hist)),
              "gbdt_split: nbin > 1024 or empty input");
  return out;
}

Tensor gbdt_seg_fill(const Tensor& beg, const Tensor& node, int64_t n) {
  CHECK_IN(beg, torch::kInt32);
  CHECK_IN(node, torch::kInt32);
  TORCH_CHECK(beg.numel() == node.numel() && beg.numel() > 0, "segment arrays mismatch");
  c10::DeviceGuard g(beg.device());
  auto out = torch::empty({n}, beg.options());
  wh::gbdt_seg_fill(ptr<int32_t>(beg), ptr<int32_t>(node), (int)beg.numel(), n, ptr<int32_t>(out),
                    cur_stream(beg));
  return out;
}

// partition the positions of the split nodes; returns the new ridx
Tensor gbdt_partition(const Tensor& B, const Tensor& ridx, const Tensor& pos_node,
                      const Tensor& node_feat, const Tensor& node_bin, const Tensor& node_defl,
                      const Tensor& seg_beg, const Tensor& seg_end, Tensor nleft_out,
                      const c10::optional<Tensor>& Bc) {
  CHECK_IN(B, torch::kUInt8);
  const uint8_t* bc = nullptr;
  if (Bc.has_value() && Bc->defined()) {
    CHECK_IN((*Bc), torch::kUInt8);
    TORCH_CHECK(Bc->dim() == 2 && Bc->size(0) == B.size(1) && Bc->size(1) == B.size(0),
                "Bc must be B transposed ([f, nrows])");
    bc = ptr<uint8_t>(*Bc);
  }
  CHECK_IN(ridx, torch::kInt32);
  CHECK_IN(pos_node, torch::kInt32);
  c10::DeviceGuard g(B.device());
  auto s = cur_stream(B);
  const int64_t n = ridx.numel();
  auto left = torch::empty({n}, ridx.options());
  wh::gbdt_goleft(ptr<uint8_t>(B), bc, B.size(0), (int)B.size(1), ptr<int32_t>(ridx), n,
                  ptr<int32_t>(pos_node), ptr<int32_t>(node_feat), ptr<int32_t>(node_bin),
                  ptr<uint8_t>(node_defl), ptr<int32_t>(left), s);
  auto lscan = torch::empty({n + 1}, ridx.options().dtype(torch::kInt64));
  auto tmp = torch::empty({wh::scan_tmp_elems(n)}, lscan.options());
  wh::scan_i32(ptr<int32_t>(left), ptr<int64_t>(lscan), n, ptr<int64_t>(tmp), s);
  // nleft[node] = lscan[end] - lscan[beg]
  auto nl = (lscan.index_select(0, seg_end.to(torch::kInt64)) -
             lscan.index_select(0, seg_beg.to(torch::kInt64))).to(torch::kInt32);
  nleft_out.copy_(nl);
  auto out = torch::empty_like(ridx);
  wh::gbdt_scatter(ptr<int32_t>(ridx), n, ptr<int32_t>(pos_node), ptr<int32_t>(node_feat),
                   ptr<int32_t>(seg_beg), ptr<int32_t>(nleft_out), ptr<int32_t>(left),
                   ptr<int64_t>(lscan), ptr<int32_t>(out), s);
  return out;
}

void gbdt_leaf_add(const Tensor& ridx, const Tensor& pos_node, const Tensor& leaf,
                   const Tensor& margin) {
  CHECK_IN(ridx, torch::kInt32);
  CHECK_IN(leaf, torch::kFloat32);
  CHECK_IN(margin, torch::kFloat32);
  c10::DeviceGuard g(ridx.device());
  wh::gbdt_leaf_add(ptr<int32_t>(ridx), ridx.numel(), ptr<int32_t>(pos_node), ptr<float>(leaf),
                    ptr<float>(margin), cur_stream(ridx));
}

// tree arrays: int32 feat / bin / left / right, uint8 defl, float val [nodes]
// (gpair f32 [n, 2], stats f64 [4] = {sum g, sum h, max|g|, max|h|})
std::vector<Tensor> gbdt_gpair(const Tensor& margin, const Tensor& label,
                               const c10::optional<Tensor>& weight, bool logistic) {
  CHECK_IN(margin, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  const int64_t n = margin.numel();
  TORCH_CHECK(label.numel() == n, "gbdt_gpair: label size mismatch");
  const float* wp = nullptr;
  if (weight.has_value() && weight->defined()) {
    CHECK_IN((*weight), torch::kFloat32);
    TORCH_CHECK(weight->numel() == n, "gbdt_gpair: weight size mismatch");
    wp = ptr<float>(*weight);
  }
  c10::DeviceGuard g(margin.device());
  static std::vector<Tensor> scratch(64);  // per device, the ticket tail stays zeroed
  const int dev = margin.device().index();
  if (!scratch[dev].defined())
    scratch[dev] = torch::zeros({wh::gbdt_gpair_scratch()}, margin.options().dtype(torch::kFloat64));
  auto gp = torch::empty({n, 2}, margin.options());
  auto st = n > 0 ? torch::empty({4}, margin.options().dtype(torch::kFloat64))  // k_gpair writes all 4
                  : torch::zeros({4}, margin.options().dtype(torch::kFloat64));
  if (n > 0)
    wh::gbdt_gpair(n, ptr<float>(margin), ptr<float>(label), wp, logistic, ptr<float>(gp),
                   ptr<double>(scratch[dev]), ptr<double>(st), cur_stream(margin));
  return {gp, st};
}

// {2^eg, 2^eh[, R]} (f32) from m = {max|g|, max|h|} (f32 [2], on the device)
Tensor gbdt_qscale(const Tensor& m, double nglobal, int64_t R) {
  CHECK_IN(m, torch::kFloat32);
  TORCH_CHECK(m.numel() == 2 && nglobal >= 1 && R >= 0, "gbdt_qscale: bad arguments");
  c10::DeviceGuard g(m.device());
  auto out = torch::empty({R > 0 ? 3 : 2}, m.options());
  wh::gbdt_qscale(ptr<float>(m), nglobal, (int)R, ptr<float>(out), cur_stream(m));
  return out;
}

void gbdt_leaf_walk(const Tensor& B, const Tensor& feat, const Tensor& bin, const Tensor& defl,
                    const Tensor& left, const Tensor& right, const Tensor& val,
                    const Tensor& margin, bool lds) {
  CHECK_IN(B, torch::kUInt8);
  CHECK_IN(feat, torch::kInt32);
  CHECK_IN(bin, torch::kInt32);
  CHECK_IN(defl, torch::kUInt8);
  CHECK_IN(left, torch::kInt32);
  CHECK_IN(right, torch::kInt32);
  CHECK_IN(val, torch::kFloat32);
  CHECK_IN(margin, torch::kFloat32);
  TORCH_CHECK(B.dim() == 2 && margin.numel() == B.size(0), "leaf_walk: B must be [n, f]");
  const int64_t nn = feat.numel();
  TORCH_CHECK(bin.numel() == nn && defl.numel() == nn && left.numel() == nn &&
                  right.numel() == nn && val.numel() == nn && nn > 0,
              "leaf_walk: tree array sizes differ");
  c10::DeviceGuard g(B.device());
  TORCH_CHECK(nn <= INT32_MAX, "leaf_walk: too many nodes");
  wh::gbdt_leaf_walk(ptr<uint8_t>(B), B.size(0), (int)B.size(1), (int)nn, ptr<int32_t>(feat),
                     ptr<int32_t>(bin), ptr<uint8_t>(defl), ptr<int32_t>(left),
                     ptr<int32_t>(right), ptr<float>(val), ptr<float>(margin), cur_stream(B), lds);
}

void gbdt_predict(const Tensor& X, const Tensor& feat, const Tensor& thr, const Tensor& left,
                  const Tensor& right, const Tensor& defl, const Tensor& leaf, const Tensor& margin) {
  CHECK_IN(X, torch::kFloat32);
  CHECK_IN(margin, torch::kFloat32);
  c10::DeviceGuard g(X.device());
  wh::gbdt_predict(ptr<float>(X), X.size(0), (int)X.size(1), ptr<int32_t>(feat), ptr<float>(thr),
                   ptr<int32_t>(left), ptr<int32_t>(right), ptr<uint8_t>(defl), ptr<float>(leaf),
                   ptr<float>(margin), cur_stream(X));
}

// ---------------------------------------------------------------- kmeans
Tensor kmeans_pack_x(const Tensor& X) {
  CHECK_IN(X, torch::kFloat32);
  TORCH_CHECK(X.dim() == 2, "X must be [n, f]");
  c10::DeviceGuard g(X.device());
  const int64_t n = X.size(0);
  const int f = (int)X.size(1);
  const int ks = wh::kmeans_ks(f);
  auto Xp = torch::empty({(n + 31) / 32 * ks * 64}, X.options());
  wh::kmeans_pack_x(ptr<float>(X), n, f, ptr<float>(Xp), cur_stream(X));
  return Xp;
}

Tensor kmeans_pack_c(const Tensor& C) {
  CHECK_IN(C, torch::kFloat32);
  TORCH_CHECK(C.dim() == 2, "C must be [k, f]");
  c10::DeviceGuard g(C.device());
  const int k = (int)C.size(0), f = (int)C.size(1);
  auto Cp = torch::empty({wh::kmeans_cp_elems(k, f)}, C.options());
  wh::kmeans_pack_c(ptr<float>(C), k, f, ptr<float>(Cp), cur_stream(C));
  return Cp;
}

std::vector<Tensor> kmeans_assign(const Tensor& Xp, int64_t n, int64_t f, const Tensor& Cp,
                                  int64_t k) {
  CHECK_IN(Xp, torch::kFloat32);
  CHECK_IN(Cp, torch::kFloat32);
  const int ks = wh::kmeans_ks((int)f);
  TORCH_CHECK(Xp.numel() == (n + 31) / 32 * ks * 64, "packed X size mismatch");
  TORCH_CHECK(Cp.numel() == wh::kmeans_cp_elems((int)k, (int)f), "packed C size mismatch");
  c10::DeviceGuard g(Xp.device());
  auto assign = torch::empty({n}, Xp.options().dtype(torch::kInt32));
  auto score = torch::empty({n}, Xp.options());
  wh::kmeans_assign(ptr<float>(Xp), n, (int)f, ptr<float>(Cp), (int)k, ptr<int32_t>(assign),
                    ptr<float>(score), cur_stream(Xp));
  return {assign, score};
}

// split precision: X [n, f] -> (packed bf16 hi/lo fragments (uint8), row norms)
std::vector<Tensor> kmeans_pack_x3(const Tensor& X) {
  CHECK_IN(X, torch::kFloat32);
  TORCH_CHECK(X.dim() == 2, "X must be [n, f]");
  c10::DeviceGuard g(X.device());
  const int64_t n = X.size(0);
  const int f = (int)X.size(1);
  TORCH_CHECK(wh::kmeans_x3_supported(f), "split-precision assign needs 1 <= f <= 128");
  auto Xp = torch::empty({wh::kmeans_x3_xp_bytes(n, f)}, X.options().dtype(torch::kUInt8));
  wh::kmeans_pack_x3(ptr<float>(X), n, f, Xp.data_ptr(), cur_stream(X));
  auto xn = X.norm(2, {1}).contiguous();
  return {Xp, xn};
}

Tensor kmeans_pack_c3(const Tensor& C) {
  CHECK_IN(C, torch::kFloat32);
  c10::DeviceGuard g(C.device());
  const int k = (int)C.size(0), f = (int)C.size(1);
  TORCH_CHECK(wh::kmeans_x3_supported(f), "split-precision assign needs 1 <= f <= 128");
  auto Cp = torch::empty({wh::kmeans_x3_cp_bytes(k, f)}, C.options().dtype(torch::kUInt8));
  wh::kmeans_pack_c3(ptr<float>(C), k, f, Cp.data_ptr(), cur_stream(C));
  return Cp;
}

// returns (assign i32 [n], score f32 [n], near-tie count (device i32 [1]))
std::vector<Tensor> kmeans_assign_x3(const Tensor& Xp, const Tensor& xnorm, const Tensor& X,
                                     const Tensor& Cp, const Tensor& C) {
  CHECK_IN(X, torch::kFloat32);
  CHECK_IN(C, torch::kFloat32);
  CHECK_IN(xnorm, torch::kFloat32);
  CHECK_DEV(Xp);
  CHECK_DEV(Cp);
  c10::DeviceGuard g(X.device());
  const int64_t n = X.size(0);
  const int f = (int)X.size(1), k = (int)C.size(0);
  TORCH_CHECK(C.size(1) == f && xnorm.numel() == n, "shape mismatch");
  TORCH_CHECK(Xp.numel() == wh::kmeans_x3_xp_bytes(n, f), "packed X size mismatch");
  TORCH_CHECK(Cp.numel() == wh::kmeans_x3_cp_bytes(k, f), "packed C size mismatch");
  auto assign = torch::empty({n}, X.options().dtype(torch::kInt32));
  auto score = torch::empty({n}, X.options());
  auto amb = torch::empty({n + 1}, X.options().dtype(torch::kInt32));
  auto ct = torch::empty({(int64_t)k * f}, X.options());
  wh::kmeans_assign_x3(Xp.data_ptr(), ptr<float>(xnorm), ptr<float>(X), n, f, Cp.data_ptr(),
                       ptr<float>(C), k, ptr<int32_t>(assign), ptr<float>(score),
                       ptr<int32_t>(amb), ptr<float>(ct), cur_stream(X));
  return {assign, score, amb.narrow(0, 0, 1)};
}

Tensor kmeans_accum(const Tensor& X, const Tensor& assign, int64_t k) {
  CHECK_IN(X, torch::kFloat32);
  CHECK_IN(assign, torch::kInt32);
  c10::DeviceGuard g(X.device());
  const int64_t n = X.size(0);
  const int f = (int)X.size(1);
  TORCH_CHECK(assign.numel() == n);
  auto sums = torch::zeros({k, f + 1}, X.options());
  // counting-sort path unless k / f are too large for it (then atomics)
  if (n > 0) {
    auto scratch = torch::empty({wh::kmeans_accum_scratch(n, (int)k)},
                                X.options().dtype(torch::kUInt8));
    if (wh::kmeans_accum_sorted(ptr<float>(X), n, f, (int)k, ptr<int32_t>(assign),
                                ptr<float>(sums), scratch.data_ptr(), cur_stream(X)))
      return sums;
  }
  wh::kmeans_accum(ptr<float>(X), n, f, ptr<int32_t>(assign), ptr<float>(sums), cur_stream(X));
  return sums;
}

// sparse k-means (CSR rows): offset int64 [n + 1] (offset[0] == 0), col int32
// [nnz] (all < F = Ct.size(0), checked by the caller once per dataset), val
// float [nnz] or None (all ones), Ct [F, Kp] float (transposed centroids)
Tensor kmeans_assign_csr(const Tensor& offset, const Tensor& col, const c10::optional<Tensor>& val,
                         const Tensor& Ct, int64_t K) {
  CHECK_IN(offset, torch::kInt64);
  CHECK_IN(col, torch::kInt32);
  CHECK_IN(Ct, torch::kFloat32);
  const int64_t n = offset.numel() - 1;
  TORCH_CHECK(n >= 0 && Ct.dim() == 2 && K >= 1 && Ct.size(1) >= K && Ct.size(1) % 4 == 0,
              "kmeans_assign_csr: Ct must be [F, Kp >= K], Kp % 4 == 0");
  const float* vp = nullptr;
  if (val.has_value() && val->defined()) {
    CHECK_IN((*val), torch::kFloat32);
    TORCH_CHECK(val->numel() == col.numel(), "kmeans_assign_csr: val / col size");
    vp = ptr<float>(*val);
  }
  c10::DeviceGuard g(Ct.device());
  auto assign = torch::empty({std::max<int64_t>(n, 0)}, Ct.options().dtype(torch::kInt32));
  wh::kmeans_assign_csr(ptr<int64_t>(offset), ptr<int32_t>(col), vp, n, ptr<float>(Ct), (int)K,
                        (int)Ct.size(1), ptr<int32_t>(assign), cur_stream(Ct));
  return assign;
}

Tensor kmeans_accum_csr(const Tensor& offset, const Tensor& col, const c10::optional<Tensor>& val,
                        const Tensor& assign, int64_t K, int64_t F) {
  CHECK_IN(offset, torch::kInt64);
  CHECK_IN(col, torch::kInt32);
  CHECK_IN(assign, torch::kInt32);
  const int64_t n = offset.numel() - 1;
  TORCH_CHECK(assign.numel() == n && K >= 1 && F >= 1, "kmeans_accum_csr: sizes");
  const float* vp = nullptr;
  if (val.has_value() && val->defined()) {
    CHECK_IN((*val), torch::kFloat32);
    vp = ptr<float>(*val);
  }
  c10::DeviceGuard g(col.device());
  auto sums = torch::zeros({K, F + 1}, col.options().dtype(torch::kFloat32));
  wh::kmeans_accum_csr(ptr<int64_t>(offset), ptr<int32_t>(col), vp, n, ptr<int32_t>(assign),
                       (int)F, ptr<float>(sums), cur_stream(col));
  return sums;
}

// (new C [k, f], empty-cluster count int64 [1]) from sums [k, f + 1] and C
std::vector<Tensor> kmeans_update(const Tensor& sums, const Tensor& C) {
  CHECK_IN(sums, torch::kFloat32);
  CHECK_IN(C, torch::kFloat32);
  TORCH_CHECK(C.dim() == 2 && sums.dim() == 2 && sums.size(0) == C.size(0) &&
                  sums.size(1) == C.size(1) + 1,
              "kmeans_update: sums must be [k, f + 1] for C [k, f]");
  c10::DeviceGuard g(C.device());
  auto out = torch::empty_like(C);
  auto nempty = torch::zeros({1}, C.options().dtype(torch::kInt64));
  wh::kmeans_update(ptr<float>(sums), ptr<float>(C), (int)C.size(0), (int)C.size(1),
                    ptr<float>(out), reinterpret_cast<unsigned long long*>(nempty.data_ptr()),
                    cur_stream(C));
  return {out, nempty};
}

Tensor spmv(const Tensor& offset, const Tensor& col, const c10::optional<Tensor>& val,
            const Tensor& x) {
  CHECK_IN(offset, torch::kInt64);
  CHECK_IN(col, torch::kInt32);
  CHECK_IN(x, torch::kFloat32);
  c10::DeviceGuard g(offset.device());
  const int64_t nrows = offset.numel() - 1;
  auto y = torch::empty({nrows}, x.options());
  wh::spmv(nrows, ptr<int64_t>(offset), ptr<int32_t>(col), optptr<float>(val), ptr<float>(x),
           ptr<float>(y), cur_stream(x));
  return y;
}

Tensor spmv_t(const Tensor& csc_off, const Tensor& csc_row, const c10::optional<Tensor>& csc_val,
              const Tensor& p) {
  CHECK_IN(csc_off, torch::kInt64);
  CHECK_IN(csc_row, torch::kInt32);
  CHECK_IN(p, torch::kFloat32);
  c10::DeviceGuard g(p.device());
  // the linear backward's chunked segmented sums (fm.hip k_chunk_plan /
  // k_bwd_scalar): a column is cut into chunks of at most a wave's width
  // and multi-chunk columns are summed across chunks, so a power-law head
  // (one Criteo value in a third of all rows) costs what its chunk count
  // costs -- one lane per column serialised such a column (298 ms per
  // L-BFGS gradient pass at 4M Criteo rows)
  const int64_t ncol = csc_off.numel() - 1;
  auto wdummy = torch::empty({ncol}, p.options());  // (vstride 0: never read)
  auto pl = fm_bwd_alloc(csc_off, csc_row.numel(), ncol, 0, 0);
  fm_bwd_launch(pl, csc_off, csc_row, optptr<float>(csc_val), ptr<float>(p), nullptr, wdummy,
                nullptr, 0, p.numel(), 0);
  return pl[0];
}


// ------------------------------------------------------------------ glm
// column-start bits of a CSC with nnz entries (glm.hip), as int64 words
Tensor glm_heads(const Tensor& csc_off, int64_t nnz) {
  CHECK_IN(csc_off, torch::kInt64);
  c10::DeviceGuard g(csc_off.device());
  const int64_t words = wh::glm_heads_words(nnz);
  auto hb = torch::empty({words}, csc_off.options());
  wh::glm_heads(ptr<int64_t>(csc_off), csc_off.numel() - 1,
                reinterpret_cast<uint64_t*>(hb.data_ptr<int64_t>()), words, cur_stream(csc_off));
  return hb;
}

// rows of a linear model: mode 0 -> (None, [loss, 0]); 1 -> (pred - label,
// [loss, sum]); 2 -> (margin, None). bias: index of the bias weight in w (or -1)
std::vector<c10::optional<Tensor>> glm_fwd(int64_t mode, const Tensor& offset, const Tensor& gcol,
                                           const c10::optional<Tensor>& val, const Tensor& w,
                                           int64_t bias, double base,
                                           const c10::optional<Tensor>& label, int64_t loss) {
  CHECK_IN(offset, torch::kInt64);
  CHECK_IN(gcol, torch::kInt32);
  CHECK_IN(w, torch::kFloat32);
  TORCH_CHECK(mode >= 0 && mode <= 3, "glm_fwd: mode 0 / 1 / 2 / 3");
  TORCH_CHECK(bias < w.numel(), "glm_fwd: bias index out of range");
  const int64_t nrows = offset.numel() - 1;
  if (mode != 2) {
    TORCH_CHECK(label.has_value() && label->defined() && label->numel() == nrows,
                "glm_fwd: label [nrows] needed");
    CHECK_IN((*label), torch::kFloat32);
  }
  if (val.has_value() && val->defined() && val->numel())
    TORCH_CHECK(val->numel() == gcol.numel(), "glm_fwd: val must match gcol");
  c10::DeviceGuard g(w.device());
  c10::optional<Tensor> out, sums;
  if (mode != 0) out = torch::empty({nrows}, w.options());
  Tensor part;
  if (mode != 2) {
    sums = torch::empty({2}, w.options().dtype(torch::kFloat64));
    part = torch::empty({std::max<int64_t>(2 * wh::glm_fwd_blocks(nrows), 2)},
                        w.options().dtype(torch::kFloat64));
  }
  const float* vp = (val.has_value() && val->defined() && val->numel()) ? ptr<float>(*val) : nullptr;
  wh::glm_fwd((int)mode, nrows, ptr<int64_t>(offset), ptr<int32_t>(gcol), vp, ptr<float>(w),
              bias >= 0 ? ptr<float>(w) + bias : nullptr, (float)base,
              mode != 2 ? ptr<float>(*label) : nullptr, (int)loss,
              out.has_value() ? ptr<float>(*out) : nullptr,
              mode != 2 ? ptr<double>(part) : nullptr,
              sums.has_value() ? ptr<double>(*sums) : nullptr, cur_stream(w));
  return {out, sums};
}

// (pred - label, [loss, sum]) from the margins glm_fwd mode 3 stored
std::vector<Tensor> glm_grad_from_margin(const Tensor& margin, const Tensor& label, int64_t loss) {
  CHECK_IN(margin, torch::kFloat32);
  CHECK_IN(label, torch::kFloat32);
  TORCH_CHECK(margin.numel() == label.numel(), "glm_grad_from_margin: sizes differ");
  c10::DeviceGuard g(margin.device());
  const int64_t n = margin.numel();
  auto out = torch::empty({n}, margin.options());
  auto sums = torch::empty({2}, margin.options().dtype(torch::kFloat64));
  auto part = torch::empty({std::max<int64_t>(2 * wh::glm_fwd_blocks(n), 2)},
                           margin.options().dtype(torch::kFloat64));
  wh::glm_grad_from_margin(n, ptr<float>(margin), ptr<float>(label), (int)loss, ptr<float>(out),
                           ptr<double>(part), ptr<double>(sums), cur_stream(margin));
  return {out, sums};
}

// grad[ucol[c]] (+)= sum over column c's CSC entries of g[row] (* val);
// grad must be zero where the columns land
// ucol: the runs' output indices, or an EMPTY tensor for the run index itself
void glm_xtg(const Tensor& crow, const c10::optional<Tensor>& cval, const Tensor& hb,
             const Tensor& col0, const Tensor& ucol, const Tensor& g, Tensor& grad,
             bool all_atomic) {
  CHECK_IN(crow, torch::kInt32);
  CHECK_IN(hb, torch::kInt64);
  CHECK_IN(col0, torch::kInt32);
  const bool has_u = ucol.numel() > 0;
  if (has_u) CHECK_IN(ucol, torch::kInt32);
  CHECK_IN(g, torch::kFloat32);
  CHECK_IN(grad, torch::kFloat32);
  const int64_t nnz = crow.numel();
  TORCH_CHECK((reinterpret_cast<uintptr_t>(crow.data_ptr()) & 15) == 0,
              "glm_xtg: CSC rows must be 16-byte aligned");
  TORCH_CHECK(hb.numel() >= wh::glm_heads_words(nnz), "glm_xtg: short column-start bits");
  TORCH_CHECK(col0.numel() >= wh::glm_xtg_waves(nnz), "glm_xtg: short per-wave columns");
  const float* vp = (cval.has_value() && cval->defined() && cval->numel()) ? ptr<float>(*cval) : nullptr;
  if (vp) TORCH_CHECK(cval->numel() == nnz, "glm_xtg: val must match rows");
  c10::DeviceGuard dg(g.device());
  wh::glm_xtg(nnz, ptr<int32_t>(crow), vp, reinterpret_cast<const uint64_t*>(ptr<int64_t>(hb)),
              ptr<int32_t>(col0), has_u ? ptr<int32_t>(ucol) : nullptr, ptr<float>(g),
              ptr<float>(grad), all_atomic ? 1 : 0, cur_stream(g));
}

void glm_runs_reduce(const Tensor& coff, const Tensor& rlist, const Tensor& S, const Tensor& cgid,
                     Tensor& grad) {
  CHECK_IN(coff, torch::kInt64);
  CHECK_IN(rlist, torch::kInt32);
  CHECK_IN(S, torch::kFloat32);
  CHECK_IN(cgid, torch::kInt32);
  CHECK_IN(grad, torch::kFloat32);
  TORCH_CHECK(cgid.numel() == coff.numel() - 1, "glm_runs_reduce: cgid / coff sizes");
  c10::DeviceGuard dg(S.device());
  wh::glm_runs_reduce(cgid.numel(), ptr<int64_t>(coff), ptr<int32_t>(rlist), ptr<float>(S),
                      ptr<int32_t>(cgid), ptr<float>(grad), cur_stream(S));
}

// ------------------------------------------------------------- gbdt (CSR)
Tensor gbdt_bin_csr(const Tensor& fid, const c10::optional<Tensor>& val, int64_t ncol,
                    const Tensor& cuts, const Tensor& cut_off) {
  CHECK_IN(fid, torch::kInt32);
  CHECK_IN(cuts, torch::kFloat32);
  CHECK_IN(cut_off, torch::kInt32);
  TORCH_CHECK(cut_off.numel() == ncol + 1, "cut_off must be [ncol + 1]");
  c10::DeviceGuard g(fid.device());
  auto gbin = torch::empty_like(fid);
  wh::gbdt_bin_csr(ptr<int32_t>(fid), optptr<float>(val), fid.numel(), (int)ncol, ptr<float>(cuts),
                   ptr<int32_t>(cut_off), ptr<int32_t>(gbin), cur_stream(fid));
  return gbin;
}

// tasks [T, 3] {slot, rbeg, rend} (device int32) -> hist double [nslot, tb, 2]
Tensor gbdt_hist_csr(const Tensor& row_off, const Tensor& gbin, const Tensor& ridx,
                     const Tensor& gpair, const Tensor& qscale, const Tensor& tasks,
                     int64_t max_rows, int64_t tb, int64_t nslot) {
  CHECK_IN(row_off, torch::kInt64);
  CHECK_IN(gbin, torch::kInt32);
  CHECK_IN(ridx, torch::kInt32);
  CHECK_IN(gpair, torch::kFloat32);
  CHECK_IN(qscale, torch::kFloat32);
  CHECK_IN(tasks, torch::kInt32);
  c10::DeviceGuard g(gbin.device());
  auto hist = torch::empty({nslot, tb, 2}, gpair.options().dtype(torch::kFloat64));
  auto hq = torch::empty({std::max<int64_t>(nslot * tb * 2, 1)}, gpair.options().dtype(torch::kInt64));
  wh::gbdt_hist_csr(ptr<int64_t>(row_off), ptr<int32_t>(gbin), ptr<int32_t>(ridx),
                    ptr<float>(gpair), ptr<float>(qscale), ptr<int32_t>(tasks),
                    (int)(tasks.numel() / 3), (int)max_rows, tb, (int)nslot, ptr<int64_t>(hq),
                    ptr<double>(hist), cur_stream(gbin));
  return hist;
}

Tensor gbdt_split_csr(const Tensor& hist, const Tensor& totals, const Tensor& cut_off,
                      const c10::optional<Tensor>& fvalid, double alpha, double lambda, double mcw) {
  CHECK_IN(hist, torch::kFloat64);
  CHECK_IN(totals, torch::kFloat64);
  CHECK_IN(cut_off, torch::kInt32);
  c10::DeviceGuard g(hist.device());
  const int S = (int)hist.size(0);
  const int F = (int)cut_off.numel() - 1;
  auto out = torch::empty({S, 6}, hist.options());
  auto cand = torch::empty({std::max<int64_t>((int64_t)S * F * 5, 1)}, hist.options());
  wh::gbdt_split_csr(ptr<double>(hist), hist.size(1), ptr<double>(totals), ptr<int32_t>(cut_off),
                     optptr<uint8_t>(fvalid), S, F, alpha, lambda, mcw, ptr<double>(cand),
                     ptr<double>(out), cur_stream(hist));
  return out;
}

Tensor gbdt_partition_csr(const Tensor& row_off, const Tensor& fid, const Tensor& gbin,
                          const Tensor& cut_off, const Tensor& ridx, const Tensor& pos_node,
                          const Tensor& node_feat, const Tensor& node_bin, const Tensor& node_defl,
                          const Tensor& seg_beg, const Tensor& seg_end, Tensor nleft_out) {
  CHECK_IN(row_off, torch::kInt64);
  CHECK_IN(fid, torch::kInt32);
  CHECK_IN(gbin, torch::kInt32);
  CHECK_IN(ridx, torch::kInt32);
  CHECK_IN(pos_node, torch::kInt32);
  c10::DeviceGuard g(ridx.device());
  auto s = cur_stream(ridx);
  const int64_t n = ridx.numel();
  auto left = torch::empty({n}, ridx.options());
  wh::gbdt_goleft_csr(ptr<int64_t>(row_off), ptr<int32_t>(fid), ptr<int32_t>(gbin),
                      ptr<int32_t>(cut_off), ptr<int32_t>(ridx), n, ptr<int32_t>(pos_node),
                      ptr<int32_t>(node_feat), ptr<int32_t>(node_bin), ptr<uint8_t>(node_defl),
                      ptr<int32_t>(left), s);
  auto lscan = torch::empty({n + 1}, ridx.options().dtype(torch::kInt64));
  auto tmp = torch::empty({wh::scan_tmp_elems(n)}, lscan.options());
  wh::scan_i32(ptr<int32_t>(left), ptr<int64_t>(lscan), n, ptr<int64_t>(tmp), s);
  auto nl = (lscan.index_select(0, seg_end.to(torch::kInt64)) -
             lscan.index_select(0, seg_beg.to(torch::kInt64))).to(torch::kInt32);
  nleft_out.copy_(nl);
  auto out = torch::empty_like(ridx);
  wh::gbdt_scatter(ptr<int32_t>(ridx), n, ptr<int32_t>(pos_node), ptr<int32_t>(node_feat),
                   ptr<int32_t>(seg_beg), ptr<int32_t>(nleft_out), ptr<int32_t>(left),
                   ptr<int64_t>(lscan), ptr<int32_t>(out), s);
  return out;
}

void gbdt_predict_csr(const Tensor& row_off, const Tensor& fid, const c10::optional<Tensor>& val,
                      const Tensor& feat, const Tensor& thr, const Tensor& left,
                      const Tensor& right, const Tensor& defl, const Tensor& leaf,
                      const Tensor& margin) {
  CHECK_IN(row_off, torch::kInt64);
  CHECK_IN(fid, torch::kInt32);
  CHECK_IN(margin, torch::kFloat32);
  c10::DeviceGuard g(fid.device());
  wh::gbdt_predict_csr(ptr<int64_t>(row_off), ptr<int32_t>(fid), optptr<float>(val),
                       row_off.numel() - 1, ptr<int32_t>(feat), ptr<float>(thr),
                       ptr<int32_t>(left), ptr<int32_t>(right), ptr<uint8_t>(defl),
                       ptr<float>(leaf), ptr<float>(margin), cur_stream(fid));
}

// ------------------------------------------------------------ text ingest
// text: uint8 [nbytes] of nlines whole lines (device) -> (keys i64 [nnz],
// label f32 [nlines], offset i64 [nlines + 1]); one host read (the key
// count) sizes the compacted keys
std::vector<Tensor> parse_criteo(const Tensor& text, int64_t nlines, bool train) {
  CHECK_IN(text, torch::kUInt8);
  c10::DeviceGuard g(text.device());
  auto s = cur_stream(text);
  auto o = text.options();
  const int64_t nb = text.numel();
  const int64_t nt = wh::text_tiles(nb);
  auto tile_cnt = torch::empty({std::max<int64_t>(nt, 1)}, o.dtype(torch::kInt32));
  auto tile_off = torch::empty({nt + 1}, o.dtype(torch::kInt64));
  auto stmp = torch::empty({wh::scan_tmp_elems(std::max<int64_t>(nt, 1))}, o.dtype(torch::kInt64));
  auto start = torch::empty({nlines + 1}, o.dtype(torch::kInt64));
  wh::text_lines(ptr<uint8_t>(text), nb, ptr<int32_t>(tile_cnt), ptr<int64_t>(tile_off),
                   ptr<int64_t>(stmp), ptr<int64_t>(start), s);
  auto padded = torch::empty({std::max<int64_t>(nlines * 39, 1)}, o.dtype(torch::kInt64));
  auto cnt = torch::empty({std::max<int64_t>(nlines, 1)}, o.dtype(torch::kInt32));
  auto label = torch::empty({nlines}, o.dtype(torch::kFloat32));
  wh::criteo_fields(ptr<uint8_t>(text), nb, ptr<int64_t>(start), nlines, train,
                    reinterpret_cast<uint64_t*>(padded.data_ptr()), ptr<int32_t>(cnt),
                    ptr<float>(label), s);
  auto off = torch::empty({nlines + 1}, o.dtype(torch::kInt64));
  auto stmp2 = torch::empty({wh::scan_tmp_elems(std::max<int64_t>(nlines, 1))}, o.dtype(torch::kInt64));
  if (nlines > 0) wh::scan_i32(ptr<int32_t>(cnt), ptr<int64_t>(off), nlines, ptr<int64_t>(stmp2), s);
  else off.zero_();
  const int64_t nnz = off[nlines].item<int64_t>();
  auto keys = torch::empty({nnz}, o.dtype(torch::kInt64));
  wh::criteo_compact(reinterpret_cast<const uint64_t*>(padded.data_ptr()), ptr<int64_t>(off),
                     nlines, reinterpret_cast<uint64_t*>(keys.data_ptr()), s);
  return {keys, label, off};
}

// text: uint8 [nbytes] of nlines whole libsvm lines (device) -> (keys i64,
// label f32, offset i64, value f32 or None when every value is 1, weight f32
// or None when no line has one), as the host parser returns them
std::vector<Tensor> parse_libsvm(const Tensor& text, int64_t nlines) {
  CHECK_IN(text, torch::kUInt8);
  c10::DeviceGuard g(text.device());
  auto s = cur_stream(text);
  auto o = text.options();
  const int64_t nb = text.numel();
  const int64_t nt = wh::text_tiles(nb);
  auto tile_cnt = torch::empty({std::max<int64_t>(nt, 1)}, o.dtype(torch::kInt32));
  auto tile_off = torch::empty({nt + 1}, o.dtype(torch::kInt64));
  auto stmp = torch::empty({wh::scan_tmp_elems(std::max<int64_t>(std::max(nt, nlines), 1))},
                           o.dtype(torch::kInt64));
  auto start = torch::empty({nlines + 1}, o.dtype(torch::kInt64));
  wh::text_lines(ptr<uint8_t>(text), nb, ptr<int32_t>(tile_cnt), ptr<int64_t>(tile_off),
                 ptr<int64_t>(stmp), ptr<int64_t>(start), s);
  auto cnt = torch::empty({std::max<int64_t>(nlines, 1)}, o.dtype(torch::kInt32));
  auto off = torch::zeros({nlines + 1}, o.dtype(torch::kInt64));
  wh::libsvm_count(ptr<uint8_t>(text), nb, ptr<int64_t>(start), nlines, ptr<int32_t>(cnt), s);
  if (nlines > 0) wh::scan_i32(ptr<int32_t>(cnt), ptr<int64_t>(off), nlines, ptr<int64_t>(stmp), s);
  const int64_t nnz = off[nlines].item<int64_t>();
  auto keys = torch::empty({nnz}, o.dtype(torch::kInt64));
  auto val = torch::empty({nnz}, o.dtype(torch::kFloat32));
  auto label = torch::empty({nlines}, o.dtype(torch::kFloat32));
  auto weight = torch::empty({nlines}, o.dtype(torch::kFloat32));
  auto flags = torch::zeros({2}, o.dtype(torch::kInt32));
  wh::libsvm_fill(ptr<uint8_t>(text), nb, ptr<int64_t>(start), nlines, ptr<int64_t>(off),
                  reinterpret_cast<uint64_t*>(keys.data_ptr()), ptr<float>(val), ptr<float>(label),
                  ptr<float>(weight), ptr<int32_t>(flags), s);
  auto f = flags.cpu();
  const int32_t* fp = f.data_ptr<int32_t>();
  // (an undefined tensor reaches Python as None)
  return {keys, label, off, fp[0] ? val : Tensor(), fp[1] ? weight : Tensor()};
}

// rows `sel` of a CSR block (keys, off, val?, label) -> (keys, val?, label)
// of the gathered block whose offsets `noff` [nsel + 1] hold nnz at the end
std::vector<Tensor> csr_gather(const Tensor& keys, const Tensor& off, const c10::optional<Tensor>& val,
                     const Tensor& label, const Tensor& sel, const Tensor& noff, int64_t nnz) {
  CHECK_IN(keys, torch::kInt64);
  CHECK_IN(off, torch::kInt64);
  CHECK_IN(label, torch::kFloat32);
  CHECK_IN(sel, torch::kInt64);
  CHECK_IN(noff, torch::kInt64);
  TORCH_CHECK(noff.numel() == sel.numel() + 1 && label.numel() + 1 == off.numel());
  if (val) {
    CHECK_IN((*val), torch::kFloat32);
    TORCH_CHECK(val->numel() == keys.numel());
  }
  c10::DeviceGuard g(keys.device());
  auto s = cur_stream(keys);
  auto okeys = torch::empty({nnz}, keys.options());
  auto olabel = torch::empty({sel.numel()}, label.options());
  Tensor oval;
  if (val) oval = torch::empty({nnz}, val->options());
  wh::csr_gather(ptr<int64_t>(off), reinterpret_cast<const uint64_t*>(keys.data_ptr()),
                 val ? ptr<float>(*val) : nullptr, ptr<float>(label), ptr<int64_t>(sel),
                 sel.numel(), ptr<int64_t>(noff), reinterpret_cast<uint64_t*>(okeys.data_ptr()),
                 val ? ptr<float>(oval) : nullptr, ptr<float>(olabel), s);
  return {okeys, val ? oval : Tensor(), olabel};
}

// ------------------------------------------------------------ gbdt grower
// Depth-wise histogram tree growth with the level loop in C++ (reference:
// xgboost hist updater driven by bin/xgboost.dmlc). Per level
// ONE host synchronisation: the split results of this level and the
// partition counts of the previous one come back in a single pinned copy;
// the child row segments the histograms need are derived on the device
// (k_child_segs), histogram tasks address them by chunk index, and the
// sibling histograms are parent - built child in one kernel. Host tables go
// down as one pinned upload per level. (The Python level loop it replaces
// left the GPU idle ~60% of each tree on per-node Python work and two syncs
// per level.)
struct GrowParams {
  double eta, alpha, lambda, mcw, rt_eps;
  int max_depth;
};

class PinnedBuf {
 public:
  template <typename T>
  T* get(int64_t n) {
    const int64_t bytes = std::max<int64_t>(n * (int64_t)sizeof(T), 8);
    if (!t_.defined() || t_.numel() < bytes)
      t_ = torch::empty({bytes * 2}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(true));
    return reinterpret_cast<T*>(t_.data_ptr());
  }
  Tensor tensor() const { return t_; }

 private:
  Tensor t_;
};

// A ring of pinned staging buffers for stream-ordered uploads: a slot is
// rewritten only after the copy that last read it has run (its event), so
// the host never has to drain the stream to reuse staging memory.
class PinnedRing {
 public:
  static constexpr int N = 4;
  ~PinnedRing() {
    for (auto& e : ev_)
      if (e) (void)hipEventDestroy(e);
  }
  template <typename T>
  T* get(int64_t n) {
    cur_ = (cur_ + 1) % N;
    if (ev_[cur_]) WH_HIP_CHECK_HOST(hipEventSynchronize(ev_[cur_]));
    return buf_[cur_].get<T>(n);
  }
  Tensor tensor() const { return buf_[cur_].tensor(); }
  // after enqueuing the copy that reads the current slot
  void mark(hipStream_t s) {
    if (!ev_[cur_]) WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&ev_[cur_], hipEventDisableTiming));
    WH_HIP_CHECK_HOST(hipEventRecord(ev_[cur_], s));
  }

 private:
  PinnedBuf buf_[N];
  hipEvent_t ev_[N] = {nullptr, nullptr, nullptr, nullptr};
  int cur_ = N - 1;
};

static double l1_threshold(double g, double alpha) {
  if (alpha <= 0) return g;
  return g > alpha ? g - alpha : (g < -alpha ? g + alpha : 0.0);
}

py::tuple gbdt_grow(const Tensor& B, const Tensor& Bc, const Tensor& ridx0, const Tensor& gpair,
                    const Tensor& qscale, const Tensor& valid, int64_t nbin,
                    std::vector<std::pair<int64_t, int64_t>> fgroups, int64_t max_fcnt,
                    std::vector<double> root_tot, std::vector<float> cut_vals,
                    std::vector<int64_t> cut_off, double eta, double alpha, double lambda,
                    double mcw, int64_t max_depth, double rt_eps, py::object allreduce) {
  CHECK_IN(B, torch::kUInt8);
  CHECK_IN(Bc, torch::kUInt8);
  CHECK_IN(ridx0, torch::kInt32);
  CHECK_IN(gpair, torch::kFloat32);
  CHECK_IN(qscale, torch::kFloat32);
  CHECK_DEV(valid);
  c10::DeviceGuard g(B.device());
  auto s = cur_stream(B);
  const int64_t n = ridx0.numel();
  const int F = (int)B.size(1);
  TORCH_CHECK(n < (int64_t)INT32_MAX, "rows must fit int32");
  const int G = (int)fgroups.size();
  const bool dw = F % 4 == 0 && max_fcnt % 4 == 0;
  const int64_t per = (int64_t)F * nbin * 2;
  auto f64 = B.options().dtype(torch::kFloat64);
  auto i32 = B.options().dtype(torch::kInt32);
  const int chunk = (int)std::max<int64_t>(8192, (n + 1023) / 1024);
  const bool reduce = !allreduce.is_none();
  // host tree
  std::vector<int> feat, bin, defl, left, right, parent;
  std::vector<double> gain, cover, bw, leaf;
  std::vector<std::array<double, 2>> tot;
  auto add = [&](int par) {
    feat.push_back(-1), bin.push_back(0), defl.push_back(0), left.push_back(-1),
        right.push_back(-1), parent.push_back(par), gain.push_back(0), cover.push_back(0),
        bw.push_back(0), leaf.push_back(0), tot.push_back({0, 0});
    return (int)feat.size() - 1;
  };
  auto weight = [&](double G_, double H_) {
    if (H_ < mcw) return 0.0;
    return -l1_threshold(G_, alpha) / (H_ + lambda);
  };
  const int root = add(-1);
  tot[root] = {root_tot[0], root_tot[1]};
  std::map<int, std::pair<int, int>> seg;  // live frontier segments (node -> [b, e))
  seg[root] = {0, (int)n};
  std::vector<std::array<int, 3>> done;    // finished leaves: node, b, e
  // staging rings for the uploads (node tables, task lists), a plain buffer
  // for the one download per level (read right after its synchronisation)
  PinnedRing up, up_tasks;
  PinnedBuf down;
  Tensor ridx = ridx0;
  // histogram of the given (slot -> [b, e) device segments); tasks by chunk
  // histogram of the given (slot -> [b, e) device segments); tasks by chunk.
  // Prepared (task lists built and uploaded, outputs allocated) before the
  // level's partition is enqueued, so the histogram launch follows the
  // child segments without host work in between.
  struct HistPlan {
    Tensor d, hist, part;
    int64_t nt = 0, nr = 0;
  };
  auto plan_hist = [&](const std::vector<int64_t>& seglen) -> HistPlan {
    const int S = (int)seglen.size();
    std::vector<int32_t> tasks, red;
    for (int k = 0; k < S; ++k) {
      const int64_t nch = std::max<int64_t>(1, (seglen[k] + chunk - 1) / chunk);
      const int t0 = (int)(tasks.size() / 5);
      for (int64_t c = 0; c < nch; ++c)
        for (auto& fg : fgroups) {
          tasks.insert(tasks.end(), {k, (int)fg.first, (int)fg.second, (int)c, chunk});
        }
      for (int gi = 0; gi < G; ++gi)
        red.insert(red.end(), {k, (int)fgroups[gi].first, (int)fgroups[gi].second, t0 + gi,
                               (int)nch, G});
    }
    HistPlan hp;
    hp.nt = (int64_t)tasks.size() / 5;
    hp.nr = (int64_t)red.size() / 6;
    int32_t* h = up_tasks.get<int32_t>(tasks.size() + red.size());
    std::memcpy(h, tasks.data(), tasks.size() * 4);
    std::memcpy(h + tasks.size(), red.data(), red.size() * 4);
    hp.d = up_tasks.tensor().narrow(0, 0, (int64_t)(tasks.size() + red.size()) * 4)
               .to(B.device(), /*non_blocking=*/true).view(torch::kInt32);
    up_tasks.mark(s);
    hp.hist = torch::empty({S, F, nbin, 2}, f64);
    hp.part = torch::empty({hp.nt * wh::gbdt_hist_pstride((int)max_fcnt, (int)nbin)},
                           gpair.options().dtype(torch::kInt64));
    return hp;
  };
  auto run_hist = [&](const HistPlan& hp, const Tensor& dseg) -> Tensor {
    wh::gbdt_hist(ptr<uint8_t>(B), F, (int)nbin, ptr<int32_t>(ridx), ptr<float>(gpair),
                  ptr<float>(qscale), ptr<int32_t>(hp.d), (int)hp.nt,
                  ptr<int32_t>(hp.d) + hp.nt * 5, (int)hp.nr, (int)max_fcnt, dw,
                  ptr<int64_t>(hp.part), ptr<double>(hp.hist), s, ptr<int32_t>(dseg), chunk,
                  nullptr, qscale.numel() == 3);
    // (no drain here: the staging ring waits for this copy only when its slot
    // comes round again; the histogram allreduce is stream-ordered)
    if (reduce) allreduce(hp.hist);
    return hp.hist;
  };
  Tensor dseg_root = torch::tensor({0, (int)n}, torch::TensorOptions().dtype(torch::kInt32))
                         .to(B.device());
  Tensor H_front = run_hist(plan_hist({n}), dseg_root);
  std::vector<int> frontier{root};
  // splits whose children's segments wait for the partition counts
  std::vector<std::array<int, 5>> pending;  // nd, l, r, b, e
  Tensor nleft_dev;
  for (int depth = 0; depth <= max_depth && !frontier.empty(); ++depth) {
    const int S = (int)frontier.size();
    const bool last = depth == max_depth;
    Tensor split_out;
    if (!last) {
      double* th = up.get<double>(2 * S);
      for (int k = 0; k < S; ++k) th[2 * k] = tot[frontier[k]][0], th[2 * k + 1] = tot[frontier[k]][1];
      auto T = up.tensor().narrow(0, 0, 16 * S).to(B.device(), true).view(torch::kFloat64);
      up.mark(s);
      split_out = torch::empty({S, 6}, f64);
      auto cand = torch::empty({std::max<int64_t>((int64_t)S * F * 4, 1)}, f64);
      TORCH_CHECK(wh::gbdt_split(ptr<double>(H_front), ptr<double>(T),
                                 reinterpret_cast<const uint8_t*>(valid.data_ptr()), S, F,
                                 (int)nbin, alpha, lambda, mcw, ptr<double>(cand),
                                 ptr<double>(split_out), s),
                  "gbdt_split failed");
    }
    // the level's one synchronisation: split results + previous partition counts
    const int64_t nl_n = nleft_dev.defined() ? nleft_dev.numel() : 0;
    double* hdown = down.get<double>(6 * (last ? 0 : S) + nl_n / 2 + 2);
    if (!last)
      WH_HIP_CHECK_HOST(hipMemcpyAsync(hdown, split_out.data_ptr(), 48 * S, hipMemcpyDeviceToHost, s));
    int32_t* nl_h = reinterpret_cast<int32_t*>(hdown + 6 * (last ? 0 : S));
    if (nl_n)
      WH_HIP_CHECK_HOST(hipMemcpyAsync(nl_h, nleft_dev.data_ptr(), 4 * nl_n, hipMemcpyDeviceToHost, s));
    WH_HIP_CHECK_HOST(hipStreamSynchronize(s));
    for (auto& pd : pending) {
      const int m = pd[3] + nl_h[pd[0]];
      seg[pd[1]] = {pd[3], m};
      seg[pd[2]] = {m, pd[4]};
    }
    pending.clear();
    for (int nd : frontier) {
      cover[nd] = tot[nd][1];
      bw[nd] = weight(tot[nd][0], tot[nd][1]);
      leaf[nd] = eta * bw[nd];
    }
    if (last) break;
    std::vector<int> split_k;
    for (int k = 0; k < S; ++k) {
      const double* o = hdown + 6 * k;
      if (!(o[0] > rt_eps)) continue;
      const int nd = frontier[k];
      const int f = (int)o[1], b = (int)o[2];
      feat[nd] = f, bin[nd] = b, defl[nd] = (int)o[3], gain[nd] = o[0];
      const int l = add(nd), r = add(nd);
      left[nd] = l, right[nd] = r;
      tot[l] = {o[4], o[5]};
      tot[r] = {tot[nd][0] - o[4], tot[nd][1] - o[5]};
      split_k.push_back(k);
    }
    if (split_k.empty()) break;
    const int nnode = (int)feat.size();
    const int nsplit = (int)split_k.size();
    // segment tiling of [0, n) for the position -> node map (gaps: -1)
    std::vector<std::pair<int, int>> tiles;  // (begin, node)
    {
      std::vector<std::array<int, 3>> all;
      for (auto& kv : seg) all.push_back({kv.second.first, kv.second.second, kv.first});
      std::sort(all.begin(), all.end());
      int cur = 0;
      for (auto& a : all) {
        if (a[0] > cur) tiles.push_back({cur, -1});
        tiles.push_back({a[0], a[2]});
        cur = a[1];
      }
      if (cur < n) tiles.push_back({cur, -1});
    }
    const int nt = (int)tiles.size();
    // one pinned upload: node feat / bin / seg_beg / seg_end [nnode], defl
    // (bytes) [nnode], tiles beg / node [nt], split table [nsplit x 4], parent slots
    const int64_t nwords = 6LL * nnode + (nnode + 3) / 4 + 2LL * nt + 5LL * nsplit;
    int32_t* hw = up.get<int32_t>(nwords);
    std::memset(hw, 0, nwords * 4);
    int32_t *h_feat = hw, *h_bin = hw + nnode, *h_sb = hw + 2 * nnode, *h_se = hw + 3 * nnode;
    uint8_t* h_defl = reinterpret_cast<uint8_t*>(hw + 4 * nnode);
    int32_t* h_tb = hw + 4 * nnode + (nnode + 3) / 4;
    int32_t* h_tn = h_tb + nt;
    int32_t* h_sp = h_tn + nt;
    int32_t* h_par = h_sp + 4 * nsplit;
    int32_t* h_lc = h_par + nsplit;      // partition cursors (device-updated)
    int32_t* h_rc = h_lc + nnode;
    for (int i = 0; i < nnode; ++i) h_feat[i] = -1;
    std::vector<int64_t> small_len(nsplit);
    for (int q = 0; q < nsplit; ++q) {
      const int k = split_k[q], nd = frontier[k];
      h_feat[nd] = feat[nd], h_bin[nd] = bin[nd], h_defl[nd] = (uint8_t)defl[nd];
      const auto sg = seg[nd];
      h_sb[nd] = sg.first, h_se[nd] = sg.second;
      h_lc[nd] = sg.first, h_rc[nd] = sg.second;
      // build the child with the smaller GLOBAL hessian, derive the other
      const int l = left[nd], r = right[nd];
      const int build_left = tot[l][1] <= tot[r][1] ? 1 : 0;
      h_sp[4 * q] = nd, h_sp[4 * q + 1] = sg.first, h_sp[4 * q + 2] = sg.second,
      h_sp[4 * q + 3] = build_left;
      h_par[q] = k;
      small_len[q] = sg.second - sg.first;  // upper bound of the built child's rows
    }
    for (int i = 0; i < nt; ++i) h_tb[i] = tiles[i].first, h_tn[i] = tiles[i].second;
    auto dw32 = up.tensor().narrow(0, 0, nwords * 4).to(B.device(), true).view(torch::kInt32);
    up.mark(s);
    const int32_t* d = ptr<int32_t>(dw32);
    const int32_t *d_feat = d, *d_bin = d + nnode, *d_sb = d + 2 * nnode;
    const uint8_t* d_defl = reinterpret_cast<const uint8_t*>(d + 4 * nnode);
    const int32_t* d_tb = d + 4 * nnode + (nnode + 3) / 4;
    const int32_t* d_tn = d_tb + nt;
    const int32_t* d_sp = d_tn + nt;
    const int32_t* d_par = d_sp + 4 * nsplit;
    int32_t* d_lc = const_cast<int32_t*>(d_par + nsplit);
    int32_t* d_rc = d_lc + nnode;
    // the built children's histogram tasks, sized by the host-side bounds
    const HistPlan hplan = plan_hist(small_len);
    auto ridx_new = torch::empty_like(ridx);
    nleft_dev = torch::empty({nnode}, i32);
    if (!wh::gbdt_partition_cursor(ptr<uint8_t>(B), ptr<uint8_t>(Bc), B.size(0), F,
                                   ptr<int32_t>(ridx), n, d_tb, 1, d_tn, nt, d_feat, d_bin, d_defl,
                                   d_lc, d_rc, d_sb, nnode, ptr<int32_t>(nleft_dev),
                                   ptr<int32_t>(ridx_new), s)) {
      // position -> node map, flags, scan, per-node left counts, stable scatter
      auto pos_node = torch::empty({n}, i32);
      wh::gbdt_seg_fill(d_tb, d_tn, nt, n, ptr<int32_t>(pos_node), s);
      auto sb64 = dw32.narrow(0, 2 * nnode, nnode).to(torch::kInt64);
      auto se64 = dw32.narrow(0, 3 * nnode, nnode).to(torch::kInt64);
      auto leftf = torch::empty({n}, i32);
      wh::gbdt_goleft(ptr<uint8_t>(B), ptr<uint8_t>(Bc), B.size(0), F, ptr<int32_t>(ridx), n,
                      ptr<int32_t>(pos_node), d_feat, d_bin, d_defl, ptr<int32_t>(leftf), s);
      auto lscan = torch::empty({n + 1}, B.options().dtype(torch::kInt64));
      auto stmp = torch::empty({wh::scan_tmp_elems(n)}, lscan.options());
      wh::scan_i32(ptr<int32_t>(leftf), ptr<int64_t>(lscan), n, ptr<int64_t>(stmp), s);
      nleft_dev = (lscan.index_select(0, se64) - lscan.index_select(0, sb64)).to(torch::kInt32);
      wh::gbdt_scatter(ptr<int32_t>(ridx), n, ptr<int32_t>(pos_node), d_feat, d_sb,
                       ptr<int32_t>(nleft_dev), ptr<int32_t>(leftf), ptr<int64_t>(lscan),
                       ptr<int32_t>(ridx_new), s);
    }
    ridx = ridx_new;
    // built children's rows, from the device counts
    auto dseg = torch::empty({2 * nsplit}, i32);
    wh::gbdt_child_segs(d_sp, nsplit, ptr<int32_t>(nleft_dev), ptr<int32_t>(dseg), s);
    Tensor hs = run_hist(hplan, dseg);
    auto H_next = torch::empty({2 * nsplit, F, nbin, 2}, f64);
    wh::gbdt_sibling(ptr<double>(H_front), ptr<double>(hs), d_sp, d_par, nsplit, per,
                     ptr<double>(H_next), s);
    // next frontier [l, r] per split; unsplit frontier nodes are final leaves
    std::vector<int> nf;
    std::vector<bool> was_split(S, false);
    for (int q = 0; q < nsplit; ++q) {
      const int k = split_k[q], nd = frontier[k];
      was_split[k] = true;
      const auto sg = seg[nd];
      pending.push_back({nd, left[nd], right[nd], sg.first, sg.second});
      seg.erase(nd);
      nf.push_back(left[nd]), nf.push_back(right[nd]);
    }
    for (int k = 0; k < S; ++k)
      if (!was_split[k]) {
        const int nd = frontier[k];
        auto it = seg.find(nd);
        if (it != seg.end()) {
          done.push_back({nd, it->second.first, it->second.second});
          seg.erase(it);
        }
      }
    frontier = nf;
    H_front = H_next;
  }
  if (!pending.empty()) {  // (a loop that ended right after a partition)
    std::vector<int32_t> nl(nleft_dev.numel());
    auto hn = nleft_dev.cpu();
    for (auto& pd : pending) {
      const int m = pd[3] + hn.data_ptr<int32_t>()[pd[0]];
      seg[pd[1]] = {pd[3], m};
      seg[pd[2]] = {m, pd[4]};
    }
  }
  for (auto& kv : seg) done.push_back({kv.first, kv.second.first, kv.second.second});
  std::vector<float> cond(feat.size(), 0.f);
  for (size_t i = 0; i < feat.size(); ++i)
    if (feat[i] >= 0) cond[i] = cut_vals[cut_off[feat[i]] + bin[i]];
  py::list segs;
  for (auto& dn : done) segs.append(py::make_tuple(dn[0], dn[1], dn[2]));
  return py::make_tuple(feat, bin, cond, defl, left, right, parent, gain, cover, bw, leaf, segs,
                        ridx);
}

// The same tree as gbdt_grow with the level loop on the device: heap-numbered
// nodes, the split decisions, partition set-up, child segments and the
// histogram task lists are written by kernels (gbdt.hip k_gd_apply /
// k_gd_children), so the host enqueues every level without waiting and reads
// the finished tree ONCE (gbdt_grow syncs once per level: ~1.5 ms of idle
// GPU per depth-8 tree of 11M rows). Every max_depth level is enqueued; the
// levels below a tree's last split find no live node and do no row work but
// the partition's pass.
// A device grower's heap node table (host copy, float64 [2^(D+1) - 1, REC])
// -> the tree lists, renumbered breadth-first: (feat, bin, cond, defl, left,
// right, parent, gain, cover, base weight, leaf, [(leaf id, begin, end)])
py::tuple gbdt_tree_from_nodes(const Tensor& hn, const std::vector<float>& cut_vals,
                               const std::vector<int64_t>& cut_off) {
  const int REC = wh::gbdt_node_rec();
  TORCH_CHECK(!hn.is_cuda() && hn.scalar_type() == torch::kFloat64 && hn.is_contiguous() &&
                  hn.dim() == 2 && hn.size(1) == REC,
              "gbdt_tree_from_nodes: a host float64 node table");
  const int NN = (int)hn.size(0);
  const double* r = hn.data_ptr<double>();
  std::vector<int> id_of(NN, -1), order;
  for (int h = 0; h < NN; ++h)
    if (r[(int64_t)h * REC] != 0.0) {
      id_of[h] = (int)order.size();
      order.push_back(h);
    }
  const size_t M = order.size();
  std::vector<int> feat(M), bin(M), defl(M), left(M, -1), right(M, -1), parent(M, -1);
  std::vector<double> gain(M), cover(M), bw(M), leaf(M);
  std::vector<float> cond(M, 0.f);
  py::list segs;
  for (size_t i = 0; i < M; ++i) {
    const int h = order[i];
    const double* q = r + (int64_t)h * REC;
    feat[i] = (int)q[1], bin[i] = (int)q[2], defl[i] = (int)q[3];
    gain[i] = q[4], cover[i] = q[5], bw[i] = q[6], leaf[i] = q[7];
    if (feat[i] >= 0) {
      TORCH_CHECK(2 * h + 2 < NN, "gbdt_tree_from_nodes: a split at the last depth");
      left[i] = id_of[2 * h + 1], right[i] = id_of[2 * h + 2];
      TORCH_CHECK(left[i] >= 0 && right[i] >= 0, "gbdt_tree_from_nodes: a split node lost a child");
      parent[left[i]] = (int)i, parent[right[i]] = (int)i;
      cond[i] = cut_vals[cut_off[feat[i]] + bin[i]];
    } else {
      segs.append(py::make_tuple((int)i, (int)q[8], (int)q[9]));
    }
  }
  return py::make_tuple(feat, bin, cond, defl, left, right, parent, gain, cover, bw, leaf, segs);
}

// margin += the leaf value each row reaches in a device grower's heap node
// table (device float64 [NN, REC]): the table becomes the walk's compact
// arrays on the device (one small kernel), then the usual row walk
void gbdt_walk_heap(const Tensor& B, const Tensor& nodes, const Tensor& margin, bool lds) {
  CHECK_IN(B, torch::kUInt8);
  CHECK_IN(nodes, torch::kFloat64);
  CHECK_IN(margin, torch::kFloat32);
  const int REC = wh::gbdt_node_rec();
  TORCH_CHECK(nodes.dim() == 2 && nodes.size(1) == REC && nodes.size(0) > 0 &&
                  nodes.size(0) <= 65535,
              "gbdt_walk_heap: a heap node table");
  TORCH_CHECK(B.dim() == 2 && margin.numel() == B.size(0), "gbdt_walk_heap: B must be [n, f]");
  c10::DeviceGuard g(B.device());
  const int64_t NN = nodes.size(0);
  auto buf = torch::empty({6 * NN}, B.options().dtype(torch::kInt32));
  int32_t* b = ptr<int32_t>(buf);
  int32_t *feat = b, *bin = b + NN, *left = b + 2 * NN, *right = b + 3 * NN;
  float* leaf = reinterpret_cast<float*>(b + 4 * NN);
  uint8_t* defl = reinterpret_cast<uint8_t*>(b + 5 * NN);
  auto s = cur_stream(B);
  wh::gbdt_heap_tree(ptr<double>(nodes), (int)NN, feat, bin, defl, left, right, leaf, s);
  wh::gbdt_leaf_walk(ptr<uint8_t>(B), B.size(0), (int)B.size(1), (int)NN, feat, bin, defl, left,
                     right, leaf, ptr<float>(margin), s, lds);
}

py::tuple gbdt_grow_dev(const Tensor& B, const Tensor& Bc, const Tensor& ridx0, const Tensor& gpair,
                        const Tensor& qscale, const Tensor& valid, int64_t nbin,
                        std::vector<std::pair<int64_t, int64_t>> fgroups, int64_t max_fcnt,
                        const Tensor& root_tot, std::vector<float> cut_vals,
                        std::vector<int64_t> cut_off, double eta, double alpha, double lambda,
                        double mcw, int64_t max_depth, double rt_eps, py::object allreduce,
                        py::object reduce_scatter, py::object pick, int64_t f_lo, bool walk,
                        bool defer) {
  // Multi-rank: either every level's built histograms are allreduced (all
  // features on every rank), or -- reduce_scatter / pick given
  // (models/gbdt.py HistExchange) -- each rank receives the global sums of
  // its feature slice [f_lo, f_lo + Fl) only, keeps the node histograms of
  // that slice, searches its features, and the per-slot best candidates are
  // reduced over the ranks by `pick`.
  CHECK_IN(root_tot, torch::kFloat64);  // {sum g, sum h} stays on the device: no host wait
  TORCH_CHECK(root_tot.numel() == 2, "gbdt_grow_dev: root totals are {sum g, sum h}");
  CHECK_IN(B, torch::kUInt8);
  CHECK_IN(Bc, torch::kUInt8);
  CHECK_IN(ridx0, torch::kInt32);
  CHECK_IN(gpair, torch::kFloat32);
  CHECK_IN(qscale, torch::kFloat32);
  CHECK_DEV(valid);
  TORCH_CHECK(max_depth >= 0 && max_depth <= 10, "gbdt_grow_dev: max_depth in [0, 10]");
  c10::DeviceGuard g(B.device());
  auto s = cur_stream(B);
  const int64_t n = ridx0.numel();
  const int F = (int)B.size(1);
  TORCH_CHECK(n < (int64_t)INT32_MAX, "rows must fit int32");
  const int G = (int)fgroups.size();
  const bool dw = F % 4 == 0 && max_fcnt % 4 == 0;
  auto f64 = B.options().dtype(torch::kFloat64);
  auto i32 = B.options().dtype(torch::kInt32);
  auto u8 = B.options().dtype(torch::kUInt8);
  const int chunk = (int)std::max<int64_t>(8192, (n + 1023) / 1024);
  const bool shard = !reduce_scatter.is_none();
  TORCH_CHECK(!shard || !pick.is_none(), "gbdt_grow_dev: reduce_scatter needs pick");
  const bool reduce = shard || !allreduce.is_none();
  // rank partials -> global sums: all features, or this rank's slice
  auto reduce_hist = [&](Tensor h) -> Tensor {
    if (!reduce) return h;
    if (!shard) {
      allreduce(h);
      return h;
    }
    Tensor r = reduce_scatter(h).cast<Tensor>();
    TORCH_CHECK(r.scalar_type() == torch::kFloat64 && r.is_contiguous() &&
                    r.device() == h.device() && r.dim() == 4 && r.size(0) == h.size(0) &&
                    r.size(1) <= F && f_lo + r.size(1) <= F,
                "gbdt_grow_dev: reduce_scatter returned a bad slice");
    return r;
  };
  const int D = (int)max_depth, NN = (2 << D) - 1, Smax = 1 << D, REC = wh::gbdt_node_rec();
  const int64_t pstride = wh::gbdt_hist_pstride((int)max_fcnt, (int)nbin);
  // one small upload: root segment, feature groups, slot iota, then the root
  // histogram's task list -- the same for every tree of a model, so kept
  // per (device, rows, depth, groups) instead of uploaded per tree
  std::vector<int32_t> hw;
  hw.reserve(3 + 2 * G + Smax);
  hw.push_back(0), hw.push_back((int32_t)n), hw.push_back(1);
  for (auto& fg : fgroups) hw.push_back((int32_t)fg.first), hw.push_back((int32_t)fg.second);
  for (int i = 0; i < Smax; ++i) hw.push_back(i);
  const int64_t nch_root = std::max<int64_t>(1, (n + chunk - 1) / chunk);
  std::vector<int32_t> root_tasks;
  {
    std::vector<int32_t> red;
    for (int64_t c = 0; c < nch_root; ++c)
      for (auto& fg : fgroups)
        root_tasks.insert(root_tasks.end(), {0, (int)fg.first, (int)fg.second, (int)c, chunk});
    for (int gi = 0; gi < G; ++gi)
      red.insert(red.end(), {0, (int)fgroups[gi].first, (int)fgroups[gi].second, gi, (int)nch_root, G});
    root_tasks.insert(root_tasks.end(), red.begin(), red.end());
  }
  // (never destroyed: device tensors must not be freed by static teardown)
  static auto& upload_cache = *new std::map<std::vector<int32_t>, std::pair<Tensor, Tensor>>();
  std::vector<int32_t> ukey = hw;
  ukey.push_back((int32_t)B.device().index());
  ukey.push_back(D);
  auto uit = upload_cache.find(ukey);
  if (uit == upload_cache.end()) {
    if (upload_cache.size() > 16) upload_cache.clear();
    auto a = torch::from_blob(hw.data(), {(int64_t)hw.size()}, torch::kInt32).to(B.device());
    auto b = torch::from_blob(root_tasks.data(), {(int64_t)root_tasks.size()}, torch::kInt32)
                 .to(B.device());
    uit = upload_cache.emplace(ukey, std::make_pair(a, b)).first;
  }
  auto hdev = uit->second.first;
  const int32_t* d_root_seg = ptr<int32_t>(hdev);
  const int32_t* d_fg = d_root_seg + 3;
  const int32_t* d_iota = d_fg + 2 * G;
  Tensor tot_cur = root_tot;
  Tensor seg_cur = hdev.narrow(0, 0, 2);
  Tensor alive_cur = hdev.narrow(0, 2, 1).view(torch::kUInt8).narrow(0, 0, 1);  // (= 1: the root)
  auto nodes = torch::empty({NN, REC}, f64);  // every depth's apply writes all its slots' records
  const uint8_t* vp = reinterpret_cast<const uint8_t*>(valid.data_ptr());
  Tensor ridx = ridx0;
  // root histogram: the host's task list over [0, n)
  Tensor H_front;
  {
    const Tensor& d = uit->second.second;
    const int64_t nt = nch_root * G;
    H_front = torch::empty({1, F, nbin, 2}, f64);
    auto part = torch::empty({nt * pstride}, gpair.options().dtype(torch::kInt64));
    wh::gbdt_hist(ptr<uint8_t>(B), F, (int)nbin, ptr<int32_t>(ridx), ptr<float>(gpair),
                  ptr<float>(qscale), ptr<int32_t>(d), (int)nt, ptr<int32_t>(d) + nt * 5, G,
                  (int)max_fcnt, dw, ptr<int64_t>(part), ptr<double>(H_front), s,
                  ptr<int32_t>(seg_cur), chunk, nullptr, qscale.numel() == 3);
    H_front = reduce_hist(H_front);
  }
  const int Fl = (int)H_front.size(1);  // features of the node histograms kept here
  const int64_t per = (int64_t)Fl * nbin * 2;
  for (int d = 0; d <= D; ++d) {
    const int S = 1 << d;
    const bool last = d == D;
    Tensor so;
    if (!last) {
      so = torch::empty({S, 6}, f64);
      if (Fl > 0) {
        auto cand = torch::empty({(int64_t)S * Fl * 4}, f64);
        TORCH_CHECK(wh::gbdt_split(ptr<double>(H_front), ptr<double>(tot_cur),
                                   vp + (int64_t)f_lo * nbin, S, Fl, (int)nbin, alpha, lambda, mcw,
                                   ptr<double>(cand), ptr<double>(so), s),
                    "gbdt_split failed");
      } else {  // (more ranks than features: this rank owns none)
        so.zero_();
        so.select(1, 0).fill_(-std::numeric_limits<double>::infinity());
      }
      if (shard) {
        so.select(1, 1).add_((double)f_lo);  // global feature ids
        so = pick(so).cast<Tensor>().contiguous();
        TORCH_CHECK(so.scalar_type() == torch::kFloat64 && so.size(0) == S && so.size(1) == 6,
                    "gbdt_grow_dev: pick returned a bad candidate table");
      }
    }
    auto pi = torch::empty({4 * S}, i32);  // pfeat | pbin | lcur | rcur
    auto pb = torch::empty({3 * S}, u8);   // pdefl | split | build_left
    Tensor tot_next = last ? Tensor() : torch::empty({2 * S, 2}, f64);
    int32_t* pfeat = ptr<int32_t>(pi);
    uint8_t* pdefl = ptr<uint8_t>(pb);
    wh::gbdt_dev_apply(S, S - 1, last, last ? nullptr : ptr<double>(so), ptr<double>(tot_cur),
                       ptr<int32_t>(seg_cur), ptr<uint8_t>(alive_cur), eta, alpha, lambda, mcw,
                       rt_eps, ptr<double>(nodes), pfeat, pfeat + S, pdefl, pfeat + 2 * S,
                       pfeat + 3 * S, pdefl + S, pdefl + 2 * S,
                       last ? nullptr : ptr<double>(tot_next), nullptr, s);
    if (last) break;
    // walk: the caller adds the leaf values by walking the tree over each
    // row's bins (models/gbdt.py _finish), so the level whose children are
    // the max-depth leaves needs neither their rows partitioned nor their
    // histograms (never split): only the children's totals (from the split
    // search, above) and the node table (~9 % of a depth-8 tree)
    const bool leaves_next = walk && d + 1 == D;
    // partition of the split slots' rows on the device segment table (the
    // segment begins read in place from seg_cur's {begin, end} pairs; the
    // children read the left cursors: no copy, no count kernel)
    auto ridx_new = leaves_next ? ridx : torch::empty_like(ridx);
    if (n > 0 && !leaves_next)
      TORCH_CHECK(wh::gbdt_partition_cursor(ptr<uint8_t>(B), ptr<uint8_t>(Bc), B.size(0), F,
                                            ptr<int32_t>(ridx), n, ptr<int32_t>(seg_cur), 2, d_iota,
                                            S, pfeat, pfeat + S, pdefl, pfeat + 2 * S, pfeat + 3 * S,
                                            nullptr, S, nullptr, ptr<int32_t>(ridx_new), s),
                  "gbdt_grow_dev: partition refused the segment table");
    ridx = ridx_new;
    // next level's segments, the built children, their histogram tasks
    const int64_t ub = ((n + chunk - 1) / chunk + S) * G;  // >= the tasks of the built children
    auto seg_next = torch::empty({4 * S}, i32);
    auto alive_next = torch::empty({2 * S}, u8);
    auto dseg = torch::empty({2 * S}, i32);
    auto sp = torch::empty({5 * S + 1}, i32);  // sp [S x 4] | par [S] | ntask
    auto tasks = torch::empty({std::max<int64_t>(ub, 1) * 5}, i32);
    auto red = torch::empty({(int64_t)S * G * 6}, i32);
    TORCH_CHECK(wh::gbdt_dev_children(S, ptr<int32_t>(seg_cur), pdefl + S, pdefl + 2 * S,
                                      pfeat + 2 * S, d_fg, G, chunk, ptr<int32_t>(seg_next),
                                      ptr<uint8_t>(alive_next), ptr<int32_t>(dseg),
                                      ptr<int32_t>(sp), ptr<int32_t>(sp) + 4 * S, ptr<int32_t>(tasks),
                                      ptr<int32_t>(sp) + 5 * S, ptr<int32_t>(red), s),
                "gbdt_grow_dev: too many slots");
    if (leaves_next) {  // (leaf segments: left child empty -- unused by the walk)
      tot_cur = tot_next;
      seg_cur = seg_next;
      alive_cur = alive_next;
      continue;
    }
    auto part = torch::empty({std::max<int64_t>(ub, 1) * pstride}, gpair.options().dtype(torch::kInt64));
    auto H_next = torch::empty({2 * S, Fl, nbin, 2}, f64);
    if (!reduce) {  // one rank: the reduce writes both children (no hs, no sibling launch)
      wh::gbdt_hist(ptr<uint8_t>(B), F, (int)nbin, ptr<int32_t>(ridx), ptr<float>(gpair),
                    ptr<float>(qscale), ptr<int32_t>(tasks), (int)std::max<int64_t>(ub, 1),
                    ptr<int32_t>(red), S * G, (int)max_fcnt, dw, ptr<int64_t>(part),
                    ptr<double>(H_next), s, ptr<int32_t>(dseg), chunk, ptr<int32_t>(sp) + 5 * S,
                    qscale.numel() == 3, ptr<double>(H_front), ptr<int32_t>(sp),
                    ptr<int32_t>(sp) + 4 * S);
    } else {
      auto hs = torch::empty({S, F, nbin, 2}, f64);
      wh::gbdt_hist(ptr<uint8_t>(B), F, (int)nbin, ptr<int32_t>(ridx), ptr<float>(gpair),
                    ptr<float>(qscale), ptr<int32_t>(tasks), (int)std::max<int64_t>(ub, 1),
                    ptr<int32_t>(red), S * G, (int)max_fcnt, dw, ptr<int64_t>(part),
                    ptr<double>(hs), s, ptr<int32_t>(dseg), chunk, ptr<int32_t>(sp) + 5 * S,
                    qscale.numel() == 3);
      hs = reduce_hist(hs);
      wh::gbdt_sibling(ptr<double>(H_front), ptr<double>(hs), ptr<int32_t>(sp),
                       ptr<int32_t>(sp) + 4 * S, S, per, ptr<double>(H_next), s);
    }
    H_front = H_next;
    tot_cur = tot_next;
    seg_cur = seg_next;
    alive_cur = alive_next;
  }
  // the finished tree: ONE host read, renumbered breadth-first (the host
  // grower's creation order) -- or, defer: the device node table itself, for
  // a heap walk on the device (gbdt_walk_heap) and a host read one tree later
  // (gbdt_tree_from_nodes), so the host's tree bookkeeping overlaps the next
  // tree instead of idling the GPU between trees
  if (defer) return py::make_tuple(nodes, ridx);
  py::tuple t = gbdt_tree_from_nodes(nodes.cpu(), cut_vals, cut_off);
  return py::make_tuple(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8], t[9], t[10], t[11],
                        ridx);
}

}  // namespace

// ------------------------------------------------------ native P=1 step
// The single-shard linear training step in ONE native call (reference
// AsgdWorker::ProcessMinibatch, learn/linear/async_sgd.h:240-288, on one
// server shard): finish this minibatch's localize (begun by the previous
// call) -> begin the next one on the localize stream -> store guard (summary
// of the previous open; device rehash past the load bound) -> find/insert ->
// pull -> forward + loss + metrics -> AUC on its side stream -> backward ->
// push (SGD / AdaGrad / FTRL). At the reference's minibatch of 10000 rows
// the GPU work is ~80 us of kernels per step while the same sequence driven
// from Python cost ~250 us of host time per step; here the host only pays
// the launches.
class LinearStep {
 public:
  // h: 4 words of coherent host memory the summary kernel writes directly
  // (a 32-byte hipMemcpyAsync to pinned memory cost ~40 us of host time)
  struct Summ {
    int64_t* h = nullptr;
    hipEvent_t ev = nullptr;
    int64_t issued = 0;
    bool pending = false;
  };
  static constexpr int kSumm = 4;
  LinearStep(KVStore* store, int64_t algo, double alpha, double beta, double l1, double l2,
             int64_t loss, double max_load, bool direct)
      : store_(store), algo_(algo), alpha_(alpha), beta_(beta), l1_(l1), l2_(l2), loss_(loss),
        max_load_(max_load) {
    TORCH_CHECK(store->vstride() == 0, "LinearStep needs a linear store");
    // the localize-free step unless a bitwise-repeatable one is asked for
    // (its per-slot gradient sums are float atomics)
    direct_ = direct && !deterministic();
    dev_ = store->slots_.device().index();
    c10::DeviceGuard g(store->slots_.device());
    ls_ = c10::hip::getStreamFromExternal(own_stream(dev_, kStreamLinearLs), dev_);
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&ev_s_, hipEventDisableTiming));
    WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&ev_ls_, hipEventDisableTiming));
  }
  ~LinearStep() {
    job_.reset();
    (void)hipEventDestroy(ev_s_);
    (void)hipEventDestroy(ev_ls_);
    for (Summ& m : sum_) {
      if (m.ev) (void)hipEventSynchronize(m.ev);
      if (m.ev) (void)hipEventDestroy(m.ev);
      if (m.h) (void)hipHostFree(m.h);
    }
  }

  // one minibatch; returns the predictions py [rows]. next_*: the next
  // call's minibatch, whose localize begins now (on the localize stream,
  // after `ready` -- a hipEvent_t handle of its producer -- or, with 0, after
  // everything queued on the current stream).
  Tensor step(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
              const Tensor& label, bool train, const Tensor& met, const Tensor& auc_sum,
              const c10::optional<Tensor>& nkeys, const c10::optional<Tensor>& noffset,
              const c10::optional<Tensor>& nval, int64_t ready) {
    if (use_direct(keys.numel())) {
      if (job_) reset();  // (a localize begun for this minibatch by a larger one before)
      return step_direct(keys, offset, val, label, train, met, auc_sum, ready);
    }
    // begin the next minibatch's localize only if it will take this path
    const bool nl = nkeys.has_value() && nkeys->defined() && !use_direct(nkeys->numel());
    Tensor py = step_localize(keys, offset, val, label, train, met, auc_sum,
                              nl ? nkeys : c10::nullopt, nl ? noffset : c10::nullopt,
                              nl ? nval : c10::nullopt, nl ? ready : 0);
    if (!nl && ready)  // the next (direct-path) minibatch is read on S after this step
      WH_HIP_CHECK_HOST(hipStreamWaitEvent(cur_stream(keys), reinterpret_cast<hipEvent_t>(ready), 0));
    return py;
  }

  // The localize-free step (csrc/hip/linear_direct.hip): touch (dedup per
  // row tile in LDS, find-or-insert, slot list) -> forward on the slots ->
  // AUC -> per-slot gradient sums -> push over the slot list. No host read;
  // the next minibatch's producer event is waited for at the END of this
  // step's work on S.
  Tensor step_direct(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                     const Tensor& label, bool train, const Tensor& met, const Tensor& auc_sum,
                     int64_t ready) {
    CHECK_IN(keys, torch::kInt64);
    CHECK_IN(offset, torch::kInt64);
    CHECK_IN(label, torch::kFloat32);
    CHECK_IN(met, torch::kFloat64);
    const int64_t nrows = offset.numel() - 1, nnz = keys.numel();
    TORCH_CHECK(label.numel() == nrows, "label size mismatch");
    const float* vp = nullptr;
    if (val.has_value() && val->defined() && val->numel()) {
      CHECK_IN((*val), torch::kFloat32);
      TORCH_CHECK(val->numel() == nnz, "val size mismatch");
      vp = ptr<float>(*val);
    }
    HostTimer ht(timing_.get());
    c10::DeviceGuard g(keys.device());
    const hipStream_t S = cur_stream(keys);
    auto i32 = keys.options().dtype(torch::kInt32);
    // inputs produced on another stream (a data generator / copy stream)
    // are read on S: their blocks are not reused before S is done with them
    {
      auto cs = c10::hip::getCurrentHIPStream(dev_);
      for (const Tensor* x : {&keys, &offset, &label})
        c10::hip::HIPCachingAllocator::recordStream(x->storage().data_ptr(), cs);
      if (vp) c10::hip::HIPCachingAllocator::recordStream(val->storage().data_ptr(), cs);
    }
    ht.mark(0);
    // store guard: the previous step's summary (long complete), then room
    // for every id of this minibatch to be new
    if (train) guard_before(nnz);
    if (!grad_.defined() || grad_.numel() < store_->cap())
      grad_ = torch::zeros({store_->cap()}, keys.options().dtype(torch::kFloat32));
    // the overflow list's counter: zero between steps (the push re-zeroes it)
    if (!ovf_cnt_.defined()) ovf_cnt_ = torch::zeros({1}, i32);
    ht.mark(1);
    // one int32 block (slot per non-zero | per-tile slot lists | overflow
    // list | per-tile counts) and one float block (py | dual)
    const int R = wh::ld_rows_per_tile(nnz, nrows);
    const int T = wh::ld_tile_table(nnz);
    const int64_t nz1 = std::max<int64_t>(nnz, 1);
    const int64_t ntiles = nrows > 0 ? (nrows + R - 1) / R : 0;
    auto iws = torch::empty({2 * nz1 + ntiles * (T + 1)}, i32);
    int32_t* lid = ptr<int32_t>(iws);
    int32_t* ovf = lid + nz1;
    int32_t* tlist = ovf + nz1;
    unsigned int* tcnt = reinterpret_cast<unsigned int*>(tlist + ntiles * T);
    unsigned int* ovf_cnt = reinterpret_cast<unsigned int*>(ovf_cnt_.data_ptr());
    auto fws = torch::empty({2 * std::max<int64_t>(nrows, 1)}, keys.options().dtype(torch::kFloat32));
    auto py = fws.narrow(0, 0, nrows);
    float* dual = ptr<float>(fws) + std::max<int64_t>(nrows, 1);
    auto part = torch::empty({wh::fm_fwd_partials()}, met.options());
    ht.mark(2);
    ++stamp_;
    if (stamp_ == 0) stamp_ = 1;
    wh::KVTable t = store_->table();
    wh::ld_touch(t, reinterpret_cast<const uint64_t*>(keys.data_ptr()), ptr<int64_t>(offset),
                 nrows, nnz, R, stamp_, train ? 1 : 0, lid, tlist, tcnt, ovf, ovf_cnt, S);
    ht.mark(3);
    if (train) guard_after(S, nnz);
    ht.mark(4);
    const int lossf = (int)loss_ | (met.numel() >= 5 ? 256 : 0);
    wh::lin_forward_strided(nrows, ptr<int64_t>(offset), lid, vp,
                            reinterpret_cast<const float*>(t.sl) + 2, 8, ptr<float>(label), lossf,
                            ptr<float>(fws), dual, ptr<double>(met), ptr<double>(part),
                            ptr<unsigned int>(dev_ws(keys.device()).fwd_ticket), S);
    ht.mark(5);
    if (train && nnz > 0) {
      wh::ld_backward(lid, vp, ptr<int64_t>(offset), nrows, nnz, R, dual, ptr<float>(grad_), S);
      ++pushes_;
      wh::LinearHP hp{(int)algo_, (float)alpha_, (float)beta_, (float)l1_, (float)l2_,
                      (float)((beta_ + std::sqrt((double)pushes_)) / alpha_)};
      wh::ld_push(t, ntiles, T, tlist, tcnt, ovf, ovf_cnt, ptr<float>(grad_), hp, S);
    }
    ht.mark(6);
    // the AUC side stream is enqueued last: its host work (event, stream
    // switch) no longer sits between the forward and backward launches
    auc_acc_side(py, label, auc_sum);
    ht.mark(7);
    // the next minibatch (produced on another stream) is read by S after
    // this step's work: order S after its producer now
    if (ready) WH_HIP_CHECK_HOST(hipStreamWaitEvent(S, reinterpret_cast<hipEvent_t>(ready), 0));
    ht.mark(8);
    return py;
  }

  Tensor step_localize(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                       const Tensor& label, bool train, const Tensor& met, const Tensor& auc_sum,
                       const c10::optional<Tensor>& nkeys, const c10::optional<Tensor>& noffset,
                       const c10::optional<Tensor>& nval, int64_t ready) {
    c10::DeviceGuard g(keys.device());
    const hipStream_t S = cur_stream(keys);
    // this minibatch's localize
    std::vector<Tensor> loc;
    if (job_ && job_keys_.is_same(keys)) {
      loc = job_->finish();
      // a hash-path job emptied its scratch table on S: the next job on the
      // localize stream (which may reuse that table) waits for S
      if (!job_->partitioned()) s_job_ = true;
      // the job's outputs were allocated on the localize stream and are read
      // on S from here on: their blocks go back to the localize stream's
      // pool only once S's queued work is done (so the localize stream
      // never has to wait for S before the next job)
      for (const Tensor& t : loc)
        if (t.defined() && t.is_cuda() && t.numel())
          c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(),
                                                      c10::hip::getCurrentHIPStream(dev_));
    } else {
      // (no job begun for this minibatch) localize on S, after any job still
      // running on the localize stream: both use the device's localize
      // workspace
      if (job_) {
        WH_HIP_CHECK_HOST(hipEventRecord(ev_ls_, ls_.stream()));
        WH_HIP_CHECK_HOST(hipStreamWaitEvent(S, ev_ls_, 0));
      }
      job_.reset();
      LocalizeJob j(keys, offset, val, 1, hint_, py::none());
      loc = j.finish();
      s_job_ = true;
    }
    job_.reset();
    const Tensor &uniq = loc[0], &lid = loc[3], &csc_off = loc[4], &csc_row = loc[5],
                 &csc_val = loc[6];
    const int64_t U = uniq.numel();
    hint_ = U;
    // the next minibatch's localize, on its own stream behind everything
    // queued on S so far (its outputs may reuse blocks S still reads)
    if (nkeys.has_value() && nkeys->defined()) {
      // the localize stream waits for S when a localize ran on S (the
      // workspace is S's until then) or when the next minibatch has no
      // producer event: it was then made on S (slices, offset rebasing, the
      // handover from a parse stream), possibly by work queued just now
      if (s_job_ || !ready) {
        WH_HIP_CHECK_HOST(hipEventRecord(ev_s_, S));
        WH_HIP_CHECK_HOST(hipStreamWaitEvent(ls_.stream(), ev_s_, 0));
        s_job_ = false;
      }
      if (ready) WH_HIP_CHECK_HOST(hipStreamWaitEvent(ls_.stream(), reinterpret_cast<hipEvent_t>(ready), 0));
      for (const Tensor* t : {&*nkeys, &*noffset}) {
        c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(), ls_);
        c10::hip::HIPCachingAllocator::recordStream(t->storage().data_ptr(),
                                                    c10::hip::getCurrentHIPStream(dev_));
      }
      c10::optional<Tensor> nv;
      if (nval.has_value() && nval->defined() && nval->numel()) {
        nv = *nval;
        c10::hip::HIPCachingAllocator::recordStream(nval->storage().data_ptr(), ls_);
      }
      c10::hip::HIPStreamGuard sg(ls_);
      job_ = std::make_unique<LocalizeJob>(*nkeys, *noffset, nv, 1, hint_, py::none());
      job_keys_ = *nkeys;
    }
    // store guard: the previous open's summary (long complete), then room
    // for this open's inserts
    if (train) guard_before(U);
    Tensor slot = store_->find(uniq, train);
    if (train) guard_after(S, U);
    Tensor w = store_->linear_pull(slot);
    auto fw = fm_forward(offset, lid, val, w, c10::nullopt, 0, label, loss_, met);
    auc_acc_side(fw[0], label, auc_sum);
    if (train && U > 0) {
      auto bw = fm_backward(csc_off, csc_row,
                            csc_val.numel() ? c10::optional<Tensor>(csc_val) : c10::nullopt,
                            fw[1], c10::nullopt, w, c10::nullopt, 0);
      ++pushes_;
      const double eta = (beta_ + std::sqrt((double)pushes_)) / alpha_;
      store_->linear_push(slot, bw[0], algo_, alpha_, beta_, l1_, l2_, eta);
    }
    return fw[0];
  }

  // drop a begun localize (end of a pass)
  void reset() { job_.reset(); job_keys_ = Tensor(); }

  // ---- store guard without a per-step host wait: table summaries (keys,
  // failed inserts) are read when their event has completed (polled), the
  // key count in between is bounded by the inserts issued since; only a
  // table close to its load bound waits for the newest summary before
  // deciding to grow (nothing in flight references old slots: a grow is
  // stream-ordered before this step's inserts)
  void guard_read(Summ& m) {
    const volatile int64_t* h = m.h;
    m.pending = false;
    TORCH_CHECK(h[1] == 0, "parameter store shard lost data: ", h[1], " failed inserts (table ",
                h[0], "/", store_->cap(), " keys)");
    if (m.issued >= base_issued_) {
      base_keys_ = h[0];
      base_issued_ = m.issued;
    }
  }
  void guard_poll(bool block) {
    for (Summ& m : sum_) {
      if (!m.pending) continue;
      if (block) WH_HIP_CHECK_HOST(hipEventSynchronize(m.ev));
      else if (hipEventQuery(m.ev) != hipSuccess) continue;
      guard_read(m);
    }
  }
  int64_t keys_bound() const { return base_keys_ + (issued_ - base_issued_); }
  void guard_before(int64_t n_new) {
    guard_poll(false);
    const double lim = max_load_ * (double)store_->cap();
    if (keys_bound() + n_new > lim) {
      guard_poll(true);  // the exact count before growing
      if (keys_bound() + n_new > lim) {
        int64_t cap = store_->cap();
        while (keys_bound() + n_new > 0.5 * cap) cap *= 2;
        store_->grow(cap);
        ++grows_;
      }
    }
  }
  // A summary (a kernel and a 32-byte read-back on the compute stream) every
  // kGuardEvery steps, or every step once the bound nears the load limit:
  // between summaries the bound grows by the inserts issued, so a late
  // summary only makes the grow decision more conservative, and a failed
  // insert still stops training within kGuardEvery steps (and at the flush).
  static constexpr int kGuardEvery = 8;
  void guard_after(hipStream_t S, int64_t n_new, bool force = false) {
    issued_ += n_new;
    const double lim = max_load_ * (double)store_->cap();
    if (!force && ++guard_step_ % kGuardEvery != 0 &&
        keys_bound() + (double)n_new * kGuardEvery < 0.9 * lim)
      return;
    Summ& m = sum_[sum_i_];
    sum_i_ = (sum_i_ + 1) % kSumm;
    if (m.pending) {  // (the GPU is kSumm steps behind: wait for the oldest)
      WH_HIP_CHECK_HOST(hipEventSynchronize(m.ev));
      guard_read(m);
    }
    if (!m.h) {
      void* p = nullptr;
      WH_HIP_CHECK_HOST(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
      m.h = static_cast<int64_t*>(p);
      std::memset(p, 0, 64);
      WH_HIP_CHECK_HOST(hipEventCreateWithFlags(&m.ev, hipEventDisableTiming));
    }
    wh::kv_summary(store_->table(), m.h, S);
    WH_HIP_CHECK_HOST(hipEventRecord(m.ev, S));
    m.issued = issued_;
    m.pending = true;
  }

  // a summary now, waited for: raises on a failed insert (end of a pass,
  // before the model is read)
  void guard_sync() {
    c10::DeviceGuard g(store_->slots_.device());
    guard_after(c10::hip::getCurrentHIPStream(dev_).stream(), 0, true);
    guard_poll(true);
  }

  int64_t grows() const { return grows_; }
  bool direct() const { return direct_; }
  // the localize-free step pays off while a minibatch is small (launch- and
  // latency-bound: the reference's 10000 rows: 71.0 vs 55.1 M ex/s); above
  // 600k non-zeros (~15k Criteo rows; at 25k rows the localize path is
  // ahead, 129 vs 109 M ex/s) the localize's global dedup does fewer table
  // probes and atomics than per-tile dedup
  bool use_direct(int64_t nnz) const { return direct_ && nnz <= 600000; }
  int64_t pushes() const { return pushes_; }
  void set_pushes(int64_t p) { pushes_ = p; }

 private:
  KVStore* store_;
  int64_t algo_;
  double alpha_, beta_, l1_, l2_;
  int64_t loss_;
  double max_load_;
  int dev_ = 0;
  c10::hip::HIPStream ls_ = c10::hip::getDefaultHIPStream();
  hipEvent_t ev_s_ = nullptr, ev_ls_ = nullptr;
  bool s_job_ = false;
  bool direct_ = true;
  // direct step: per-slot gradient sums (all zero between steps), the
  // overflow slot list's counter (zero between steps)
  Tensor grad_, ovf_cnt_;
  uint32_t stamp_ = 0;
  std::unique_ptr<HostSplit> timing_{host_split("linear direct step")};
  int64_t guard_step_ = 0;
  std::unique_ptr<LocalizeJob> job_;
  Tensor job_keys_;
  Summ sum_[kSumm];
  int sum_i_ = 0;
  int64_t issued_ = 0, base_keys_ = 0, base_issued_ = 0;
  int64_t hint_ = 0, grows_ = 0, pushes_ = 0;
};

#include "rccl_comm.h"
#include "psx_native.inl"
#include "difacto_step.inl"

PYBIND11_MODULE(_hip, m) {
  m.doc() = "wormhole_amd gfx950 HIP kernels";
  m.def("scan_excl", &scan_excl);
  py::class_<LocalizeJob>(m, "LocalizeJob")
      .def(py::init<const Tensor&, const Tensor&, const c10::optional<Tensor>&, int64_t, int64_t,
                    py::object, bool>(),
           py::arg("keys"), py::arg("offset"), py::arg("val") = py::none(), py::arg("nshard") = 1,
           py::arg("hint") = 0, py::arg("exchange") = py::none(),
           py::arg("defer_exchange") = false)
      .def("exchange", &LocalizeJob::exchange)
      .def("counts", &LocalizeJob::counts)
      .def("finish", &LocalizeJob::finish);
  m.def("loc_timing_read", []() { return loc_timing_buf().clone(); });
  m.def("loc_retries", []() { return loc_retries(); },
        "localize jobs redone on the hash path after a partition overflow (count)");
  py::class_<LinearStep>(m, "LinearStep")
      .def(py::init<KVStore*, int64_t, double, double, double, double, int64_t, double, bool>(),
           py::arg("store"), py::arg("algo"), py::arg("alpha"), py::arg("beta"), py::arg("l1"),
           py::arg("l2"), py::arg("loss"), py::arg("max_load") = 0.7, py::arg("direct") = true,
           py::keep_alive<1, 2>())
      .def("step", &LinearStep::step, py::arg("keys"), py::arg("offset"), py::arg("val"),
           py::arg("label"), py::arg("train"), py::arg("met"), py::arg("auc_sum"),
           py::arg("next_keys") = py::none(), py::arg("next_offset") = py::none(),
           py::arg("next_val") = py::none(), py::arg("ready") = 0)
      .def("reset", &LinearStep::reset)
      .def("guard_sync", &LinearStep::guard_sync)
      .def_property_readonly("grows", &LinearStep::grows)
      .def_property_readonly("direct", [](const LinearStep& l) { return l.direct(); })
      .def_property("pushes", &LinearStep::pushes, &LinearStep::set_pushes);
  py::class_<RcclComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<const std::string&, int64_t, int64_t, int64_t>(), py::arg("uid"),
           py::arg("nranks"), py::arg("rank"), py::arg("device"))
      .def_static("unique_id", &RcclComm::unique_id)
      .def("close", &RcclComm::close)
      .def("a2av", &RcclComm::a2av_t, py::arg("x"), py::arg("send_rows"), py::arg("recv_rows"))
      .def("allreduce_sum", [](RcclComm& c, Tensor t) { c.allreduce_sum(t); })
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("device", &RcclComm::device);
  m.attr("PSX_TX_IDENTITY") = (int)kTxIdentity;
  m.attr("PSX_TX_RCCL") = (int)kTxRccl;
  m.attr("PSX_TX_STAGED") = (int)kTxStaged;
  py::class_<PsxStep>(m, "PsxStep")
      .def(py::init<KVStore*, int64_t, int64_t, int64_t, int64_t, py::object, py::object, bool,
                    std::vector<double>, std::vector<double>, int64_t, bool, int64_t, int64_t,
                    Tensor, Tensor, int64_t, double, int64_t, std::vector<int64_t>,
                    std::vector<double>>(),
           py::arg("store"), py::arg("P"), py::arg("S"), py::arg("rank"), py::arg("tx"),
           py::arg("pg"), py::arg("rccl"), py::arg("linear"), py::arg("lin_hp"), py::arg("hp"), py::arg("threshold"),
           py::arg("l1_shrk"), py::arg("seed"), py::arg("loss"), py::arg("met"),
           py::arg("auc_sum"), py::arg("tau"), py::arg("max_load"), py::arg("cu_reserve"),
           py::arg("filt") = std::vector<int64_t>{0, 0},
           py::arg("post") = std::vector<double>{0.0, 0.0, 0.0, 0.0},
           py::keep_alive<1, 2>())
      .def("train", &PsxStep::train, py::arg("keys"), py::arg("offset"), py::arg("val"),
           py::arg("label"), py::arg("data_pass"), py::arg("next_keys") = py::none(),
           py::arg("next_offset") = py::none(), py::arg("next_val") = py::none(),
           py::arg("ready") = 0)
      .def("flush", &PsxStep::flush)
      .def("drop_job", &PsxStep::drop_job)
      .def("guard_sync", &PsxStep::guard_sync)
      .def("wire", &PsxStep::wire)
      .def("wire_reset", &PsxStep::wire_reset)
      .def("xtime", &PsxStep::xtime,
           "sampled GPU us per exchange C0..C3 and the sample counts (RCCL transport)")
      .def_property_readonly("watchdog_deadline", &PsxStep::watchdog_deadline)
      .def_property_readonly("busy", &PsxStep::busy)
      .def_property_readonly("grows", &PsxStep::grows)
      .def_property_readonly("vgrows", &PsxStep::vgrows)
      .def_property("requests", &PsxStep::requests, &PsxStep::set_requests)
      .def_property("step", &PsxStep::step, &PsxStep::set_step);
  m.def("a2a_plan", &a2a_plan_py, py::arg("rank"), py::arg("world"), py::arg("row_bytes"),
        py::arg("send_rows"), py::arg("recv_rows"),
        "one rank's per-peer all-to-all-v plan: (esz, (own_src, own_dst, own_bytes), sends, recvs)");
  py::class_<DifactoStep>(m, "DifactoStep")
      .def(py::init<KVStore*, std::vector<double>, int64_t, bool, int64_t, int64_t,
                    std::vector<double>, double, bool>(),
           py::arg("store"), py::arg("hp"), py::arg("threshold"), py::arg("l1_shrk"),
           py::arg("seed"), py::arg("loss"), py::arg("post"), py::arg("max_load"),
           py::arg("direct"), py::keep_alive<1, 2>())
      .def("step", &DifactoStep::step, py::arg("keys"), py::arg("offset"), py::arg("val"),
           py::arg("label"), py::arg("train"), py::arg("data_pass"), py::arg("met"),
           py::arg("auc_sum"), py::arg("step"), py::arg("next_keys") = py::none(),
           py::arg("next_offset") = py::none(), py::arg("next_val") = py::none(),
           py::arg("ready") = 0)
      .def("reset", &DifactoStep::reset)
      .def("guard_sync", &DifactoStep::guard_sync)
      .def_property_readonly("direct", &DifactoStep::direct)
      .def_property_readonly("grows", &DifactoStep::grows)
      .def_property_readonly("vgrows", &DifactoStep::vgrows);
  m.def("c10d_a2a_rows", &c10d_a2a_rows, py::arg("pg"), py::arg("x"), py::arg("send_rows"),
        py::arg("recv_rows"));
  m.def("localize", &localize, py::arg("keys"), py::arg("offset"), py::arg("val") = py::none(),
        py::arg("nshard") = 1, py::arg("hint") = 0, py::arg("exchange") = py::none());
  m.def("fm_forward", &fm_forward);
  m.def("set_cu_reserve", [](int64_t n) { wh::fm_set_cu_reserve((int)n); },
        "CUs the persistent FM kernels leave free for concurrent collectives");
  m.def("cu_reserve", []() { return (int64_t)wh::fm_cu_reserve(); });
  m.def("fm_backward", &fm_backward);
  m.def("fm_backward_plan", &fm_backward_plan);
  m.def("fm_backward_run", &fm_backward_run);
  m.def("fm_grad_post", &fm_grad_post);
  m.def("vidx_renumber", &vidx_renumber);
  m.def("ps_unpack", &ps_unpack);
  m.def("ps_pack_gw", &ps_pack_gw);
  m.def("ps_records", &ps_records);
  m.def("ps_c0", &ps_c0, py::arg("owner_cnt"), py::arg("vcnt"), py::arg("P"), py::arg("flag"),
        py::arg("loopback") = false);
  m.def("auc", &auc);
  m.def("quant_rows", &quant_rows);
  m.def("key_mod", &key_mod);
  m.def("dequant_rows", &dequant_rows);
  m.def("trunc_u8", &trunc_u8);
  m.def("ps_qpack", &ps_qpack, py::arg("x"), py::arg("desc"), py::arg("rows"), py::arg("W"),
        py::arg("nb"), py::arg("seed"));
  m.def("ps_qunpack", &ps_qunpack, py::arg("q"), py::arg("desc"), py::arg("W"), py::arg("nb"),
        py::arg("out"));
  m.def("auc_acc", &auc_acc);
  m.def("auc_acc_side", &auc_acc_side);
  m.def("auc_join", &auc_join);
  m.def("auc_host_threads", [](int n) { HostAuc::enable(n); },
        "large training minibatches' AUC on n host threads (0: the device chain)");
  m.def("timing_flush", &timing_flush);
  m.def("auc_sorted", &auc_sorted);
  m.def("synth_criteo", &synth_criteo);
  m.def("gather_rows", &gather_rows);
  m.def("vstride_for", &vstride_for);
  m.def("spmv", &spmv, py::arg("offset"), py::arg("col"), py::arg("val"), py::arg("x"));
  m.def("gbdt_bin", &gbdt_bin);
  m.def("gbdt_hist", &gbdt_hist, py::arg("B"), py::arg("nbin"), py::arg("ridx"), py::arg("gpair"),
        py::arg("qscale"), py::arg("tasks"), py::arg("red"), py::arg("max_fcnt"), py::arg("hist"));
  m.def("gbdt_partition", &gbdt_partition, py::arg("B"), py::arg("ridx"), py::arg("pos_node"),
        py::arg("node_feat"), py::arg("node_bin"), py::arg("node_defl"), py::arg("seg_beg"),
        py::arg("seg_end"), py::arg("nleft"), py::arg("Bc") = py::none());
  m.def("gbdt_seg_fill", &gbdt_seg_fill);
  m.def("gbdt_split", &gbdt_split);
  m.def("owlqn_dir", &owlqn_dir, py::arg("g"), py::arg("w"), py::arg("l1"),
        py::arg("out") = py::none());
  m.def("owlqn_fix_dot", &owlqn_fix_dot);
  m.def("owlqn_step", &owlqn_step);
  m.def("multi_dot", &multi_dot);
  m.def("hist_dots", &hist_dots, py::arg("H"), py::arg("probes"));
  m.def("dir_fix_dot", &dir_fix_dot, py::arg("H"), py::arg("rows"), py::arg("coef"),
        py::arg("steep_row"), py::arg("fix"), py::arg("n") = -1);
  m.def("glm_heads", &glm_heads, py::arg("csc_off"), py::arg("nnz"));
  m.def("glm_fwd", &glm_fwd, py::arg("mode"), py::arg("offset"), py::arg("gcol"), py::arg("val"),
        py::arg("w"), py::arg("bias"), py::arg("base"), py::arg("label"), py::arg("loss"));
  m.def("glm_xtg", &glm_xtg, py::arg("crow"), py::arg("cval"), py::arg("hb"), py::arg("col0"),
        py::arg("ucol"), py::arg("g"), py::arg("grad"), py::arg("all_atomic") = false);
  m.def("glm_grad_from_margin", &glm_grad_from_margin, py::arg("margin"), py::arg("label"),
        py::arg("loss"));
  m.def("glm_runs_reduce", &glm_runs_reduce, py::arg("coff"), py::arg("rlist"), py::arg("S"),
        py::arg("cgid"), py::arg("grad"));
  m.def("gbdt_leaf_add", &gbdt_leaf_add);
  m.def("gbdt_leaf_walk", &gbdt_leaf_walk, py::arg("B"), py::arg("feat"), py::arg("bin"),
        py::arg("defl"), py::arg("left"), py::arg("right"), py::arg("val"), py::arg("margin"),
        py::arg("lds") = true, "margins += the tree's leaf per row (lds: the LDS-resident walk "
        "when the tree and row tile fit; else the global-memory walk)");
  m.def("gbdt_predict", &gbdt_predict);
  m.def("kmeans_pack_x", &kmeans_pack_x);
  m.def("kmeans_pack_c", &kmeans_pack_c);
  m.def("kmeans_assign", &kmeans_assign);
  m.def("kmeans_accum", &kmeans_accum);
  m.def("kmeans_update", &kmeans_update);
  m.def("kmeans_assign_csr", &kmeans_assign_csr, py::arg("offset"), py::arg("col"),
        py::arg("val"), py::arg("Ct"), py::arg("K"));
  m.def("kmeans_accum_csr", &kmeans_accum_csr, py::arg("offset"), py::arg("col"), py::arg("val"),
        py::arg("assign"), py::arg("K"), py::arg("F"));
  m.def("kmeans_pack_x3", &kmeans_pack_x3);
  // every argument named: the Python side calls these by keyword (a dropped
  // argument fails on the CPU signature test, tests/test_native_signatures.py)
  m.def("gbdt_grow", &gbdt_grow, py::arg("B"), py::arg("Bc"), py::arg("ridx0"), py::arg("gpair"),
        py::arg("qscale"), py::arg("valid"), py::arg("nbin"), py::arg("fgroups"), py::arg("max_fcnt"),
        py::arg("root_tot"), py::arg("cut_vals"), py::arg("cut_off"), py::arg("eta"), py::arg("alpha"),
        py::arg("reg_lambda"), py::arg("min_child_weight"), py::arg("max_depth"), py::arg("rt_eps"),
        py::arg("allreduce"));
  m.def("gbdt_grow_dev", &gbdt_grow_dev, py::arg("B"), py::arg("Bc"), py::arg("ridx0"), py::arg("gpair"),
        py::arg("qscale"), py::arg("valid"), py::arg("nbin"), py::arg("fgroups"), py::arg("max_fcnt"),
        py::arg("root_tot"), py::arg("cut_vals"), py::arg("cut_off"), py::arg("eta"), py::arg("alpha"),
        py::arg("reg_lambda"), py::arg("min_child_weight"), py::arg("max_depth"), py::arg("rt_eps"),
        py::arg("allreduce"), py::arg("reduce_scatter") = py::none(), py::arg("pick") = py::none(),
        py::arg("f_lo") = 0, py::arg("walk") = false, py::arg("defer") = false);
  m.def("gbdt_tree_from_nodes", &gbdt_tree_from_nodes);
  m.def("gbdt_walk_heap", &gbdt_walk_heap, py::arg("B"), py::arg("nodes"), py::arg("margin"),
        py::arg("lds") = true);
  m.def("gbdt_gpair", &gbdt_gpair);
  m.def("gbdt_qscale", &gbdt_qscale);
  // the ingest ops block on one small device read each: the GIL is released
  // so a producer thread's parsing overlaps the training loop
  m.def("parse_criteo", &parse_criteo, py::call_guard<py::gil_scoped_release>());
  m.def("parse_libsvm", &parse_libsvm, py::call_guard<py::gil_scoped_release>());
  m.def("csr_gather", &csr_gather, py::call_guard<py::gil_scoped_release>());
  m.def("gbdt_bin_csr", &gbdt_bin_csr);
  m.def("gbdt_hist_csr", &gbdt_hist_csr);
  m.def("gbdt_split_csr", &gbdt_split_csr);
  m.def("gbdt_partition_csr", &gbdt_partition_csr);
  m.def("gbdt_predict_csr", &gbdt_predict_csr);
  m.def("kmeans_pack_c3", &kmeans_pack_c3);
  m.def("kmeans_assign_x3", &kmeans_assign_x3);
  m.def("spmv_t", &spmv_t, py::arg("csc_off"), py::arg("csc_row"), py::arg("csc_val"),
        py::arg("p"));
  py::class_<KVStore>(m, "KVStore")
      .def(py::init<int64_t, int64_t, int64_t, int64_t>(), py::arg("cap"), py::arg("vcap"),
           py::arg("dim"), py::arg("device"))
      .def("find", &KVStore::find)
      .def("occupied", &KVStore::occupied)
      .def("linear_pull", &KVStore::linear_pull)
      .def("linear_push", &KVStore::linear_push)
      .def("difacto_push_cnt", &KVStore::difacto_push_cnt)
      .def("difacto_pull", &KVStore::difacto_pull)
      .def("difacto_open_pull", &KVStore::difacto_open_pull, py::arg("keys"), py::arg("insert"),
           py::arg("cnt"), py::arg("h"), py::arg("threshold"), py::arg("l1_shrk"), py::arg("seed"),
           py::arg("direct") = false)
      .def("difacto_push", &KVStore::difacto_push)
      .def("ps_open", &KVStore::ps_open, py::arg("keys"), py::arg("use_cnt"), py::arg("segS"),
           py::arg("segHS"), py::arg("rows_cap"), py::arg("insert"), py::arg("chains"), py::arg("h"),
           py::arg("threshold"), py::arg("l1_shrk"), py::arg("seed"),
           py::arg("chain_in") = py::none())
      .def("ps_push", &KVStore::ps_push, py::arg("slot"), py::arg("vpos"), py::arg("chain"),
           py::arg("head"), py::arg("segS"), py::arg("segHS"), py::arg("gbuf"), py::arg("h"),
           py::arg("threshold"), py::arg("l1_shrk"), py::arg("seed"),
           py::arg("prep_chain") = py::none(), py::arg("prep_n") = 0)
      .def("ps_push_linear", &KVStore::ps_push_linear, py::arg("slot"), py::arg("chain"),
           py::arg("head"), py::arg("segS"), py::arg("g"), py::arg("algo"), py::arg("alpha"),
           py::arg("beta"), py::arg("l1"), py::arg("l2"), py::arg("t0"),
           py::arg("prep_chain") = py::none(), py::arg("prep_n") = 0)
      .def("grow", &KVStore::grow)
      .def("grow_v", &KVStore::grow_v)
      .def("summary", &KVStore::summary)
      .def("summary_async", &KVStore::summary_async)
      .def("summary_read", &KVStore::summary_read)
      .def_property_readonly("dim", &KVStore::dim)
      .def_property_readonly("vstride", &KVStore::vstride)
      .def_property_readonly("cap", &KVStore::cap)
      .def_property_readonly("vcap", &KVStore::vcap)
      .def_readonly("ps_opens", &KVStore::opens_)
      .def_readonly("slots", &KVStore::slots_)
      .def_readonly("keys", &KVStore::keys_)
      .def_readonly("w", &KVStore::w_)
      .def_readonly("z", &KVStore::z_)
      .def_readonly("sq", &KVStore::sq_)
      .def_readonly("cnt", &KVStore::cnt_)
      .def_readonly("vrow", &KVStore::vrow_)
      .def_readonly("V", &KVStore::V_)
      .def_readonly("VG", &KVStore::VG_)
      .def_readonly("vnext", &KVStore::vnext_)
      .def_property_readonly("stats", [](const KVStore& k) {
        // counters summed over their shards: [8] int64 (a copy)
        return k.stats_.narrow(1, 0, wh::kStatCount).sum(0);
      })
      .def("reset_stats", [](KVStore& k, int64_t i0, int64_t i1) {
        k.stats_.narrow(1, i0, i1 - i0).zero_();
      })
      .def("add_stat", [](KVStore& k, int64_t i, int64_t v) {
        k.stats_.select(1, i).narrow(0, 0, 1).add_(v);
      });
}
