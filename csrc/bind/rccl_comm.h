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
// The communicator is built with ncclCommInitRank from an id that rank 0
// makes (unique_id()) and the Python side passes around through the c10d
// store (wormhole_amd/parallel/comm.py Comm.rccl). A 1-rank communicator
// stands in for P virtual peers in the one-GPU loopback rehearsal (the own
// segment a device copy, the other P-1 one send / recv pair to self).
#pragma once

#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#define WH_NCCL_CHECK(x)                                                              \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error in ", #x, ": ", ncclGetErrorString(r_)); \
  } while (0)

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
    WH_NCCL_CHECK(ncclCommInitRank(&comm_, world_, u, rank_));
  }
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;
  // (no destroy at exit: ncclCommDestroy after the HIP runtime began its
  // own teardown can hang; close() is the orderly end)
  ~RcclComm() = default;

  void close() {
    if (comm_) {
      c10::DeviceGuard g(c10::Device(c10::kCUDA, (c10::DeviceIndex)dev_));
      (void)hipDeviceSynchronize();
      WH_NCCL_CHECK(ncclCommDestroy(comm_));
      comm_ = nullptr;
    }
  }

  int size() const { return world_; }
  int rank() const { return rank_; }
  int device() const { return dev_; }

  // Row-wise all-to-all-v of bytes on stream s: peer q's segment of `send`
  // (send_rows[q] rows of row_bytes, segments in peer order) goes to q, and
  // q's segment for this rank lands at recv's q-th offset. The own segment
  // is a device copy. With a 1-rank communicator and P > 1 row counts (the
  // loopback rehearsal: virtual rank 0 of P) segment 0 is the own copy and
  // segments 1..P-1 -- contiguous on both sides -- ONE send / recv pair to
  // self: RCCL serialises several operations to one peer over separate
  // launches (21 pairs to self per step took 9 launches of ~29 us), which a
  // real rank's one operation per peer does not pay; send_rows must equal
  // recv_rows. Zero-row segments are skipped on both sides (the row counts
  // are symmetric by construction).
  void a2av(const void* send, void* recv, int64_t row_bytes, const std::vector<int64_t>& send_rows,
            const std::vector<int64_t>& recv_rows, hipStream_t s) {
    TORCH_CHECK(comm_ != nullptr, "RcclComm: closed");
    // the widest element the rows and both buffers allow: RCCL's copy loop
    // moves elements of the given type (8-byte rows and 256-byte embedding
    // rows as int64, 12-byte key records as int32)
    const uintptr_t al = reinterpret_cast<uintptr_t>(send) | reinterpret_cast<uintptr_t>(recv) |
                         (uintptr_t)row_bytes;
    const int esz = (al & 7) == 0 ? 8 : (al & 3) == 0 ? 4 : 1;
    const ncclDataType_t dt = esz == 8 ? ncclInt64 : esz == 4 ? ncclInt32 : ncclUint8;
    const int P = (int)send_rows.size();
    TORCH_CHECK((int)recv_rows.size() == P, "RcclComm.a2av: row vectors differ in length");
    const bool virt = world_ == 1 && P > 1;
    TORCH_CHECK(virt || P == world_, "RcclComm.a2av: ", P, " segments for ", world_, " ranks");
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    int64_t so = 0, ro = 0;
    bool open = false;
    if (virt) {
      int64_t own = send_rows[0] * row_bytes, rest = 0;
      for (int q = 0; q < P; ++q) {
        TORCH_CHECK(send_rows[q] == recv_rows[q],
                    "RcclComm.a2av: loopback segments must be symmetric");
        if (q > 0) rest += send_rows[q] * row_bytes;
      }
      if (own > 0) WH_HIP_CHECK_HOST(hipMemcpyAsync(rp, sp, (size_t)own, hipMemcpyDeviceToDevice, s));
      if (rest > 0) {
        WH_NCCL_CHECK(ncclGroupStart());
        WH_NCCL_CHECK(ncclSend(sp + own, (size_t)(rest / esz), dt, 0, comm_, s));
        WH_NCCL_CHECK(ncclRecv(rp + own, (size_t)(rest / esz), dt, 0, comm_, s));
        WH_NCCL_CHECK(ncclGroupEnd());
      }
      return;
    }
    for (int q = 0; q < P; ++q) {
      const int64_t sb = send_rows[q] * row_bytes, rb = recv_rows[q] * row_bytes;
      if (q == rank_) {
        TORCH_CHECK(sb == rb, "RcclComm.a2av: own segment sizes differ");
        if (sb > 0) WH_HIP_CHECK_HOST(hipMemcpyAsync(rp + ro, sp + so, (size_t)sb,
                                                     hipMemcpyDeviceToDevice, s));
      } else {
        if (sb > 0 || rb > 0) {
          if (!open) WH_NCCL_CHECK(ncclGroupStart());
          open = true;
        }
        if (sb > 0) WH_NCCL_CHECK(ncclSend(sp + so, (size_t)(sb / esz), dt, q, comm_, s));
        if (rb > 0) WH_NCCL_CHECK(ncclRecv(rp + ro, (size_t)(rb / esz), dt, q, comm_, s));
      }
      so += sb;
      ro += rb;
    }
    if (open) WH_NCCL_CHECK(ncclGroupEnd());
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
  ncclComm_t comm_ = nullptr;
  int world_ = 1, rank_ = 0, dev_ = 0;
};
