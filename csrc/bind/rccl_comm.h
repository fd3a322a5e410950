// A communicator of our own on RCCL's C API: the data plane of the
// multi-shard parameter-server step (csrc/bind/psx_native.inl) over xGMI.
//
// Replaces ps-lite's per-minibatch ZPull / ZPush / ZVPull / ZVPush messages
// (learn/linear/async_sgd.h:252-287, learn/difacto/async_sgd.h:373-424) with
// one grouped point-to-point all-to-all-v per exchange: every peer segment
// goes out as its own ncclSend / ncclRecv pair on the issuing HIP stream, so
// the 7 xGMI links of an MI355X carry the 7 peer slices at once, and the
// host pays one ncclGroupStart / ncclGroupEnd per exchange instead of a
// c10d ProcessGroup call (argument checks, work objects, RCCL's internal
// stream hand-off: 20-70 us of host time each, profiles/r5k_*).
//
// The per-peer work of one rank is computed once, by a2a_plan(), and the
// transports only execute it: RcclComm::a2av below (ncclSend / ncclRecv per
// peer) and the gloo-staged rehearsal of psx_native.inl (c10d send / recv per
// peer on host copies), so the multi-process CPU / shared-GPU tests run the
// very offsets, own-segment copy and zero-row skips an 8-GPU run takes.
//
// The communicator is built with ncclCommInitRank from an id that rank 0
// makes (unique_id()) and the Python side passes around through the c10d
// store (wormhole_amd/parallel/comm.py Comm.rccl). A 1-rank communicator
// stands in for P virtual peers in the one-GPU loopback rehearsal (the own
// segment a device copy, the other P-1 one send / recv pair to self).
#pragma once

#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <string>
#include <vector>

#define WH_NCCL_CHECK(x)                                                              \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error in ", #x, ": ", ncclGetErrorString(r_)); \
  } while (0)

// One rank's share of a row-wise all-to-all-v, in bytes.
struct A2aPlan {
  struct Seg {
    int peer;
    int64_t off, bytes;  // offset into this rank's send (or recv) buffer
  };
  // the rows' natural element size, a function of row_bytes alone (reported
  // to the tests); a2av itself moves ncclUint8, so its datatype never
  // depends on this rank's buffer alignment
  int esz = 1;
  int64_t own_src = 0, own_dst = 0, own_bytes = 0;  // the own segment: a local copy
  std::vector<Seg> sends, recvs;                     // peer order, zero-byte segments left out
};

// rank of world (world == 1 with P > 1 segments: virtual rank 0 of P, the
// loopback rehearsal: segment 0 is the own copy and segments 1..P-1 --
// contiguous on both sides -- ONE send / recv pair to self, since RCCL
// serialises several operations to one peer over separate launches (21
// pairs to self per step took 9 launches of ~29 us), which a real rank's one
// operation per peer does not pay; the segments must then be symmetric).
// Zero-byte segments are skipped on both sides: this rank's send_rows[q] is
// q's recv_rows[rank] (the count exchange C0 makes them so), so a skipped
// send is always matched by a skipped receive.
inline A2aPlan a2a_plan(int rank, int world, int64_t row_bytes,
                        const std::vector<int64_t>& send_rows,
                        const std::vector<int64_t>& recv_rows) {
  const int P = (int)send_rows.size();
  TORCH_CHECK((int)recv_rows.size() == P, "a2a_plan: row vectors differ in length");
  TORCH_CHECK(row_bytes >= 0, "a2a_plan: negative row size");
  const bool virt = world == 1 && P > 1;
  TORCH_CHECK(virt || P == world, "a2a_plan: ", P, " segments for ", world, " ranks");
  TORCH_CHECK(rank >= 0 && rank < world, "a2a_plan: bad rank");
  A2aPlan pl;
  pl.esz = (row_bytes & 7) == 0 ? 8 : (row_bytes & 3) == 0 ? 4 : 1;
  if (virt) {
    int64_t rest = 0;
    for (int q = 0; q < P; ++q) {
      TORCH_CHECK(send_rows[q] >= 0 && send_rows[q] == recv_rows[q],
                  "a2a_plan: loopback segments must be symmetric");
      if (q > 0) rest += send_rows[q] * row_bytes;
    }
    pl.own_bytes = send_rows[0] * row_bytes;
    if (rest > 0) {
      pl.sends.push_back({0, pl.own_bytes, rest});
      pl.recvs.push_back({0, pl.own_bytes, rest});
    }
    return pl;
  }
  int64_t so = 0, ro = 0;
  for (int q = 0; q < P; ++q) {
    TORCH_CHECK(send_rows[q] >= 0 && recv_rows[q] >= 0, "a2a_plan: negative row count");
    const int64_t sb = send_rows[q] * row_bytes, rb = recv_rows[q] * row_bytes;
    if (q == rank) {
      TORCH_CHECK(sb == rb, "a2a_plan: own segment sizes differ (", sb, " vs ", rb, ")");
      pl.own_src = so;
      pl.own_dst = ro;
      pl.own_bytes = sb;
    } else {
      if (sb > 0) pl.sends.push_back({q, so, sb});
      if (rb > 0) pl.recvs.push_back({q, ro, rb});
    }
    so += sb;
    ro += rb;
  }
  return pl;
}

class RcclComm {
 public:
  static py::bytes unique_id() {
    ncclUniqueId id;
    WH_NCCL_CHECK(ncclGetUniqueId(&id));
    return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
  }

  // Collective over the `nranks` processes that pass the same id (blocks
  // until all have joined; the GIL is released meanwhile).
  RcclComm(const std::string& id, int64_t nranks, int64_t rank, int64_t device)
      : world_((int)nranks), rank_((int)rank), dev_((int)device) {
    TORCH_CHECK(id.size() == NCCL_UNIQUE_ID_BYTES, "RcclComm: id must be ",
                NCCL_UNIQUE_ID_BYTES, " bytes");
    TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "RcclComm: bad rank / size");
    ncclUniqueId u;
    std::memcpy(u.internal, id.data(), NCCL_UNIQUE_ID_BYTES);
    c10::DeviceGuard g(c10::Device(c10::kCUDA, (c10::DeviceIndex)dev_));
    py::gil_scoped_release nogil;
    ncclComm_t c = nullptr;
    WH_NCCL_CHECK(ncclCommInitRank(&c, world_, u, rank_));
    comm_ = c;
  }
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;
  // (no destroy at exit: ncclCommDestroy after the HIP runtime began its
  // own teardown can hang; close() is the orderly end)
  ~RcclComm() = default;

  void close() {
    ncclComm_t c = comm_.exchange(nullptr);
    if (c) {
      c10::DeviceGuard g(c10::Device(c10::kCUDA, (c10::DeviceIndex)dev_));
      (void)hipDeviceSynchronize();
      WH_NCCL_CHECK(ncclCommDestroy(c));
    }
  }

  int size() const { return world_; }
  int rank() const { return rank_; }
  int device() const { return dev_; }

  // An asynchronous error of the communicator (a peer gone, a transport
  // failure): ncclSuccess while healthy. Safe from any thread (the step's
  // watchdog polls it).
  ncclResult_t async_error() const {
    ncclComm_t c = comm_;
    if (!c) return ncclSuccess;
    ncclResult_t e = ncclSuccess;
    if (ncclCommGetAsyncError(c, &e) != ncclSuccess) return ncclSystemError;
    return e;
  }
  std::string async_error_str() const {
    const ncclResult_t e = async_error();
    return e == ncclSuccess ? std::string() : std::string(ncclGetErrorString(e));
  }
  // Abandon the communicator (its kernels in flight are told to stop): the
  // watchdog's last act before the process exits, so a stuck peer exchange
  // does not outlive it. Callable from another thread while the owner waits.
  void abort() {
    ncclComm_t c = comm_.exchange(nullptr);
    if (c) (void)ncclCommAbort(c);
  }

  // Row-wise all-to-all-v of bytes on stream s: peer q's segment of `send`
  // (send_rows[q] rows of row_bytes, segments in peer order) goes to q, and
  // q's segment for this rank lands at recv's q-th offset, per a2a_plan().
  void a2av(const void* send, void* recv, int64_t row_bytes, const std::vector<int64_t>& send_rows,
            const std::vector<int64_t>& recv_rows, hipStream_t s) {
    TORCH_CHECK(comm_ != nullptr, "RcclComm: closed");
    const A2aPlan pl = a2a_plan(rank_, world_, row_bytes, send_rows, recv_rows);
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    // bytes on the wire (ncclUint8): the element type of a send must match
    // its receive on the peer, and a type picked from this rank's own buffer
    // alignment is not something the peer can know -- point-to-point RCCL
    // moves bytes either way, so nothing is lost
    if (pl.own_bytes > 0)
      WH_HIP_CHECK_HOST(hipMemcpyAsync(rp + pl.own_dst, sp + pl.own_src, (size_t)pl.own_bytes,
                                       hipMemcpyDeviceToDevice, s));
    if (pl.sends.empty() && pl.recvs.empty()) return;
    WH_NCCL_CHECK(ncclGroupStart());
    // (one peer's send and receive adjacent, in peer order: the grouped
    // operations of every rank then form the same pairwise schedule)
    size_t i = 0, j = 0;
    while (i < pl.sends.size() || j < pl.recvs.size()) {
      const int ps = i < pl.sends.size() ? pl.sends[i].peer : 1 << 30;
      const int pr = j < pl.recvs.size() ? pl.recvs[j].peer : 1 << 30;
      if (ps <= pr) {
        const auto& g = pl.sends[i++];
        WH_NCCL_CHECK(ncclSend(sp + g.off, (size_t)g.bytes, ncclUint8, g.peer, comm_, s));
      } else {
        const auto& g = pl.recvs[j++];
        WH_NCCL_CHECK(ncclRecv(rp + g.off, (size_t)g.bytes, ncclUint8, g.peer, comm_, s));
      }
    }
    WH_NCCL_CHECK(ncclGroupEnd());
  }

  // tensor front end of a2av (rows = dim 0), on the current stream
  Tensor a2av_t(const Tensor& x, const std::vector<int64_t>& send_rows,
                const std::vector<int64_t>& recv_rows) {
    TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "RcclComm.a2av: contiguous device tensor");
    int64_t row = x.element_size();
    for (int64_t d = 1; d < x.dim(); ++d) row *= x.size(d);
    std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
    int64_t n = 0;
    for (int64_t r : recv_rows) n += r;
    if (shape.empty()) shape.push_back(0);
    shape[0] = n;
    Tensor out = torch::empty(shape, x.options());
    c10::DeviceGuard g(x.device());
    a2av(x.data_ptr(), out.data_ptr(), row, send_rows, recv_rows,
         c10::hip::getCurrentHIPStream(x.device().index()).stream());
    return out;
  }

  // sum all-reduce in place (f32 / f64 / i64), on the current stream
  void allreduce_sum(Tensor& t) {
    TORCH_CHECK(comm_ != nullptr && t.is_cuda() && t.is_contiguous(), "RcclComm.allreduce");
    ncclDataType_t dt = t.scalar_type() == torch::kFloat32   ? ncclFloat32
                        : t.scalar_type() == torch::kFloat64 ? ncclFloat64
                        : t.scalar_type() == torch::kInt64   ? ncclInt64
                                                             : ncclNumTypes;
    TORCH_CHECK(dt != ncclNumTypes, "RcclComm.allreduce: f32 / f64 / i64 only");
    c10::DeviceGuard g(t.device());
    WH_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), (size_t)t.numel(), dt, ncclSum, comm_,
                                c10::hip::getCurrentHIPStream(t.device().index()).stream()));
  }

 private:
  std::atomic<ncclComm_t> comm_{nullptr};
  int world_ = 1, rank_ = 0, dev_ = 0;
};

// a2a_plan for Python (tests): (esz, (own_src, own_dst, own_bytes),
// [(peer, off, bytes)] sends, [(peer, off, bytes)] recvs)
inline py::tuple a2a_plan_py(int64_t rank, int64_t world, int64_t row_bytes,
                             const std::vector<int64_t>& send_rows,
                             const std::vector<int64_t>& recv_rows) {
  const A2aPlan pl = a2a_plan((int)rank, (int)world, row_bytes, send_rows, recv_rows);
  py::list s, r;
  for (const auto& g : pl.sends) s.append(py::make_tuple(g.peer, g.off, g.bytes));
  for (const auto& g : pl.recvs) r.append(py::make_tuple(g.peer, g.off, g.bytes));
  return py::make_tuple(pl.esz, py::make_tuple(pl.own_src, pl.own_dst, pl.own_bytes), s, r);
}
