// pybind11 registration of the native host runtime (wormhole_amd._host).
#include <torch/extension.h>

#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <memory>
#include <mutex>
#include <thread>

#include "auc_host.h"
#include "common.h"
#include "io.h"
#include "remote_fs.h"
#include "localizer.h"
#include "parsers.h"
#include "scheduler.h"
#include "van.h"
#include "workload_pool.h"

namespace wh {
namespace host {


namespace {

using torch::Tensor;

py::list conf_to_py(const std::vector<ConfItem>& items) {
  py::list out;
  for (const auto& it : items) {
    if (it.kind == 'm')
      out.append(py::make_tuple(it.key, std::string("m"), conf_to_py(it.children)));
    else
      out.append(py::make_tuple(it.key, std::string(1, it.kind), it.value));
  }
  return out;
}

// pinned = page-locked host memory (torch's caching host allocator), so the
// learner's .to(device, non_blocking=True) is a real asynchronous DMA
template <class T, class A>
Tensor vec_to_tensor(const std::vector<T, A>& v, torch::ScalarType dt, bool pinned = false) {
  auto t = torch::empty({(int64_t)v.size()}, torch::TensorOptions().dtype(dt).pinned_memory(pinned));
  if (!v.empty()) std::memcpy(t.data_ptr(), v.data(), v.size() * sizeof(T));
  return t;
}

py::tuple block_to_py(const RowBlock& b, bool pinned = false) {
  py::object val = py::none(), wt = py::none();
  if (!b.value.empty()) val = py::cast(vec_to_tensor(b.value, torch::kFloat32, pinned));
  if (!b.weight.empty()) wt = py::cast(vec_to_tensor(b.weight, torch::kFloat32, pinned));
  return py::make_tuple(vec_to_tensor(b.index, torch::kInt64, pinned),
                        vec_to_tensor(b.offset, torch::kInt64, pinned), val,
                        vec_to_tensor(b.label, torch::kFloat32, pinned), wt);
}

RowBlock py_to_block(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                     const Tensor& label, const c10::optional<Tensor>& weight) {
  RowBlock b;
  auto k = keys.contiguous().to(torch::kInt64);
  auto o = offset.contiguous().to(torch::kInt64);
  auto l = label.contiguous().to(torch::kFloat32);
  b.index.assign((const uint64_t*)k.data_ptr(), (const uint64_t*)k.data_ptr() + k.numel());
  b.offset.assign(o.data_ptr<int64_t>(), o.data_ptr<int64_t>() + o.numel());
  b.label.assign(l.data_ptr<float>(), l.data_ptr<float>() + l.numel());
  if (val && val->defined() && val->numel()) {
    auto v = val->contiguous().to(torch::kFloat32);
    b.value.assign(v.data_ptr<float>(), v.data_ptr<float>() + v.numel());
  }
  if (weight && weight->defined() && weight->numel()) {
    auto w = weight->contiguous().to(torch::kFloat32);
    b.weight.assign(w.data_ptr<float>(), w.data_ptr<float>() + w.numel());
  }
  return b;
}

// whole split of a file as one block (for the BSP apps that keep their split resident)
py::tuple load_split(const std::string& path, int part, int nparts, const std::string& fmt) {
  py::gil_scoped_release nogil;
  ThreadedReader r(path, part, nparts, fmt);
  RowBlock all, b;
  bool any_val = false;
  while (r.Next(&b)) {
    if (!b.value.empty() && !any_val) {
      any_val = true;
      all.value.assign(all.index.size(), 1.f);
    }
    const int64_t base = (int64_t)all.index.size();
    all.label.insert(all.label.end(), b.label.begin(), b.label.end());
    if (!b.weight.empty()) all.weight.insert(all.weight.end(), b.weight.begin(), b.weight.end());
    for (size_t i = 1; i < b.offset.size(); ++i) all.offset.push_back(base + b.offset[i]);
    all.index.insert(all.index.end(), b.index.begin(), b.index.end());
    if (any_val) {
      if (b.value.empty()) all.value.resize(all.index.size(), 1.f);
      else all.value.insert(all.value.end(), b.value.begin(), b.value.end());
    }
  }
  py::gil_scoped_acquire g;
  return block_to_py(all);
}

// Whole-line text batches for device-side parsing (csrc/hip/ingest.hip):
// the part's byte range [begin, end) (line-aligned by InputSplit) is read in
// large blocks by a background thread, cut after every mb-th newline with
// memchr (empty lines do not count), each batch a (pinned) tensor (a final
// line without a newline gets one). next() -> (uint8 tensor, lines) or None.
class PyTextBatches {
 public:
  PyTextBatches(const std::string& path, int part, int nparts, int64_t mb, bool pinned,
                int64_t depth)
      : mb_(std::max<int64_t>(mb, 1)), pinned_(pinned), depth_(std::max<int64_t>(depth, 1)) {
    InputSplit split(path, part, nparts, false);
    begin_ = split.begin();
    end_ = split.end();
    path_ = IsRemote(path) ? path : ResolvePath(path);
    th_ = std::thread([this] { Run(); });
  }
  ~PyTextBatches() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  py::object next() {
    std::pair<Tensor, int64_t> item;
    bool got = false;
    std::string err;
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !q_.empty() || done_ || !err_.empty(); });
      if (!err_.empty()) {
        err = err_;
      } else if (!q_.empty()) {
        item = std::move(q_.front());
        q_.pop_front();
        got = true;
      }
    }
    cv_.notify_all();
    if (!err.empty()) throw std::runtime_error(err);
    if (!got) return py::none();
    return py::make_tuple(item.first, item.second);
  }

 private:
  Tensor Alloc(int64_t n) {
    return torch::empty({n}, torch::TensorOptions().dtype(torch::kUInt8).pinned_memory(pinned_));
  }
  void Push(Tensor t, int64_t lines) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return (int64_t)q_.size() < depth_ || stop_; });
    q_.emplace_back(std::move(t), lines);
    cv_.notify_all();
  }
  // file bytes are read straight into the (pinned) batch buffer; only the
  // partial line after a cut is copied into the next buffer
  void Run() {
    try {
      // a local file through stdio, a remote one (WebHDFS / S3) through
      // ranged reads with a read-ahead window
      std::unique_ptr<RemoteReader> rr;
      std::FILE* fp = nullptr;
      if (IsRemote(path_)) {
        rr = std::make_unique<RemoteReader>(path_, 16 << 20);
        rr->Seek(begin_);
      } else {
        fp = std::fopen(path_.c_str(), "rb");
        if (!fp) throw std::runtime_error("cannot open " + path_);
        std::fseek(fp, begin_, SEEK_SET);
      }
      int64_t left = end_ - begin_;
      int64_t cap = 4 << 20;
      Tensor cur = Alloc(cap);
      int64_t have = 0, scan = 0, lines = 0;
      bool eof = left <= 0;
      while (true) {
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (stop_) break;
        }
        char* b = static_cast<char*>(cur.data_ptr());
        int64_t cut = 0;
        while (scan < have) {
          const char* q = static_cast<const char*>(std::memchr(b + scan, '\n', have - scan));
          if (!q) {
            scan = have;
            break;
          }
          scan = (int64_t)(q - b) + 1;
          // empty lines are not lines (parsers skip them; ingest.hip is_end)
          if (q == b || q[-1] == '\n') continue;
          if (++lines == mb_) {
            cut = scan;
            break;
          }
        }
        if (cut) {
          // the next buffer is sized from this batch (+1/8 headroom)
          cap = std::max<int64_t>(cap, cut + cut / 8 + (have - cut) + 1);
          Tensor nxt = Alloc(cap);
          std::memcpy(nxt.data_ptr(), b + cut, have - cut);
          Push(cur.narrow(0, 0, cut), mb_);
          cur = nxt;
          have -= cut;
          scan = lines = 0;
          continue;
        }
        if (eof) {
          if (have) {
            const bool add = b[have - 1] != '\n';
            if (add) b[have++] = '\n';  // room: have < cap always holds here
            Push(cur.narrow(0, 0, have), lines + (add ? 1 : 0));
          }
          break;
        }
        if (have + 1 >= cap) {  // a batch longer than the buffer: grow
          cap *= 2;
          Tensor g = Alloc(cap);
          std::memcpy(g.data_ptr(), b, have);
          cur = g;
          b = static_cast<char*>(cur.data_ptr());
        }
        const int64_t want = std::min<int64_t>(left, cap - 1 - have);
        const int64_t got = rr ? (int64_t)rr->Read(b + have, (size_t)want)
                               : (int64_t)std::fread(b + have, 1, (size_t)want, fp);
        have += got;
        left -= got;
        if (got == 0 || left <= 0) eof = true;
      }
      if (fp) std::fclose(fp);
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> lk(mu_);
      err_ = e.what();
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      done_ = true;
    }
    cv_.notify_all();
  }

  int64_t mb_;
  bool pinned_;
  int64_t depth_;
  int64_t begin_ = 0, end_ = 0;
  std::string path_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::pair<Tensor, int64_t>> q_;
  bool stop_ = false, done_ = false;
  std::string err_;
};

class PyMinibatchIter {
 public:
  PyMinibatchIter(const std::string& path, int part, int nparts, const std::string& fmt,
                  int64_t mb, int64_t shuf, double neg, int64_t seed, bool pinned)
      : it_(path, part, nparts, fmt, (size_t)mb, (size_t)shuf, (float)neg, (uint64_t)seed),
        pinned_(pinned) {}
  py::object next() {
    bool ok;
    Tensor k, o, l, v, w;
    {
      // the assembly AND the copies into (pinned) tensors run without the
      // GIL: a shuffle-buffer block is hundreds of MB of keys, and the
      // training loop keeps running meanwhile
      py::gil_scoped_release nogil;
      ok = it_.Next();
      if (ok) {
        const RowBlock& b = it_.Value();
        k = vec_to_tensor(b.index, torch::kInt64, pinned_);
        o = vec_to_tensor(b.offset, torch::kInt64, pinned_);
        l = vec_to_tensor(b.label, torch::kFloat32, pinned_);
        if (!b.value.empty()) v = vec_to_tensor(b.value, torch::kFloat32, pinned_);
        if (!b.weight.empty()) w = vec_to_tensor(b.weight, torch::kFloat32, pinned_);
      }
    }
    if (!ok) return py::none();
    py::object val = v.defined() ? py::cast(v) : py::none();
    py::object wt = w.defined() ? py::cast(w) : py::none();
    return py::make_tuple(k, o, val, l, wt);
  }

 private:
  MinibatchIter it_;
  bool pinned_;
};

// CSR blocks of `rows` rows (file order) in (pinned) tensors, for the device
// shuffle buffer (wormhole_amd/data/device_text.py): CRB records decoded
// straight into the block (next_crb), other formats' parsed chunks copied
// into it by a thread pool (next_blocks). MinibatchIter assembled a RowBlock
// first and then copied it into tensors, both on one thread -- the round-2
// bound of CRB input (two copies of ~330 MB per million Criteo rows).
class PyBlockIter {
 public:
  PyBlockIter(const std::string& path, int part, int nparts, const std::string& fmt,
              int64_t rows, bool pinned, int nthreads)
      : rows_(std::max<int64_t>(rows, 1)), pinned_(pinned),
        ncopy_(std::max(1, std::min(8, (int)std::thread::hardware_concurrency()))) {
    if (fmt == "crb") {
      split_.reset(new InputSplit(path, part, nparts, true));
      ndec_ = nthreads > 0 ? nthreads : ThreadedReader::DefaultThreads();
    } else {
      reader_.reset(new ThreadedReader(path, part, nparts, fmt, nthreads));
    }
  }

  py::object next() { return split_ ? next_crb() : next_blocks(); }

 private:
  // pinned output tensors of a block (values / weights only when present)
  struct Out {
    Tensor k, o, l, v, w;
  };
  Out alloc(int64_t rows, int64_t nnz, bool any_v, bool any_w) {
    auto opt = [&](torch::ScalarType dt) {
      return torch::TensorOptions().dtype(dt).pinned_memory(pinned_);
    };
    Out out;
    out.k = torch::empty({nnz}, opt(torch::kInt64));
    out.o = torch::empty({rows + 1}, opt(torch::kInt64));
    out.l = torch::empty({rows}, opt(torch::kFloat32));
    if (any_v) out.v = torch::empty({nnz}, opt(torch::kFloat32));
    if (any_w) out.w = torch::empty({rows}, opt(torch::kFloat32));
    return out;
  }
  static py::object to_py(Out& out, bool binary) {
    // every value 1: binary data (reference minibatch_iter.h:114-116)
    if (binary) out.v = Tensor();
    py::object val = out.v.defined() ? py::cast(out.v) : py::none();
    py::object wt = out.w.defined() ? py::cast(out.w) : py::none();
    return py::make_tuple(out.k, out.o, val, out.l, wt);
  }
  // f(i, w): item i on worker w (0 <= w < nthreads; worker 0 is the
  // calling thread)
  template <class F>
  static void parallel(size_t n, int nthreads, F&& f) {
    std::atomic<size_t> next{0};
    auto work = [&](int w) {
      for (size_t i = next++; i < n; i = next++) f(i, w);
    };
    const int nt = (int)std::min<size_t>((size_t)nthreads, n);
    std::vector<std::thread> th;
    std::exception_ptr err;
    std::mutex em;
    auto guarded = [&](int w) {
      try {
        work(w);
      } catch (...) {
        std::lock_guard<std::mutex> lk(em);
        if (!err) err = std::current_exception();
        next = n;
      }
    };
    for (int t = 1; t < nt; ++t) th.emplace_back(guarded, t);
    guarded(0);
    for (auto& t : th) t.join();
    if (err) std::rethrow_exception(err);
  }

  // CRB: records are located in the part's mapping, their row offsets
  // decoded, and every section LZ4-decoded by a thread pool STRAIGHT into
  // its slice of the (pinned) output block -- no RowBlock in between and no
  // second copy (host memory traffic was the bound: ~1 GB per million
  // Criteo rows through decode + copy, ~0.45 GB now). A record straddling
  // two blocks is carried over (its sections decoded once per block, into
  // scratch, for the rows each needs).
  py::object next_crb() {
    struct Piece {
      std::shared_ptr<CRBRecord> r;
      int64_t r0, r1, row_base, nnz_base;
    };
    std::vector<Piece> pieces;
    Out out;
    bool binary = false;
    {
      py::gil_scoped_release nogil;
      int64_t have = 0;
      std::vector<std::shared_ptr<CRBRecord>> fresh;
      while (have < rows_) {
        if (!carry_) {
          auto r = std::make_shared<CRBRecord>();
          const char* p;
          size_t n;
          if (!split_->NextRecordView(&p, &n, &r->spill)) break;
          CRBLocate(p, n, r.get());
          if (r->nrows == 0) continue;
          carry_ = r;
          carry_pos_ = 0;
          fresh.push_back(r);
        }
        const int64_t take = std::min<int64_t>(rows_ - have, carry_->nrows - carry_pos_);
        pieces.push_back({carry_, carry_pos_, carry_pos_ + take, have, 0});
        carry_pos_ += take;
        have += take;
        if (carry_pos_ == carry_->nrows) carry_.reset();
      }
      if (pieces.empty()) {
        py::gil_scoped_acquire g;
        return py::none();
      }
      parallel(fresh.size(), ndec_, [&](size_t i, int) { CRBDecodeOffsets(fresh[i].get()); });
      int64_t nnz = 0;
      bool any_v = false, any_w = false;
      for (auto& pc : pieces) {
        pc.nnz_base = nnz;
        nnz += pc.r->off[pc.r1] - pc.r->off[pc.r0];
        any_v = any_v || pc.r->csz[3] > 0;
        any_w = any_w || pc.r->csz[4] > 0;
      }
      out = alloc(have, nnz, any_v, any_w);
      uint64_t* kp = reinterpret_cast<uint64_t*>(out.k.data_ptr());
      int64_t* op = out.o.data_ptr<int64_t>();
      float* lp = out.l.data_ptr<float>();
      float* vp = any_v ? out.v.data_ptr<float>() : nullptr;
      float* wp = any_w ? out.w.data_ptr<float>() : nullptr;
      op[0] = 0;
      std::atomic<bool> non_one{false};
      // per-worker LZ4 scratch kept across calls (the workers are new
      // threads each call: a thread_local buffer was re-allocated per block)
      if (scratch_.size() < (size_t)std::max(ndec_, 1)) scratch_.resize(std::max(ndec_, 1));
      parallel(pieces.size(), ndec_, [&](size_t i, int w) {
        std::vector<char>& tmp = scratch_[w];
        const Piece& pc = pieces[i];
        const CRBRecord& r = *pc.r;
        const int64_t n = pc.r1 - pc.r0, s = r.off[pc.r0], e = r.off[pc.r1];
        // rows with non-zeros need the index section (a record without one
        // is corrupt: the keys would be left as whatever the block held)
        if (!CRBDecodeRows(r, 2, pc.r0, pc.r1, kp + pc.nnz_base, &tmp))
          WH_CHECK(e == s, "crb record has non-zeros but no index section");
        if (!CRBDecodeRows(r, 0, pc.r0, pc.r1, lp + pc.row_base, &tmp))
          std::fill(lp + pc.row_base, lp + pc.row_base + n, 0.f);
        for (int64_t q = 0; q < n; ++q) op[pc.row_base + q + 1] = pc.nnz_base + (r.off[pc.r0 + q + 1] - s);
        if (vp) {
          float* v = vp + pc.nnz_base;
          if (!CRBDecodeRows(r, 3, pc.r0, pc.r1, v, &tmp)) {
            std::fill(v, v + (e - s), 1.f);
          } else {
            for (int64_t j = 0; j < e - s && !non_one.load(std::memory_order_relaxed); ++j)
              if (v[j] != 1.f) non_one = true;
          }
        }
        if (wp && !CRBDecodeRows(r, 4, pc.r0, pc.r1, wp + pc.row_base, &tmp))
          std::fill(wp + pc.row_base, wp + pc.row_base + n, 1.f);
      });
      binary = vp && !non_one;
    }
    return to_py(out, binary);
  }

  // other formats: chunks parsed by a ThreadedReader into RowBlocks, whose
  // row ranges a thread pool copies into their slices of the output
  py::object next_blocks() {
    struct Piece {
      std::shared_ptr<RowBlock> b;
      int64_t r0, r1, row_base, nnz_base;
    };
    std::vector<Piece> pieces;
    Out out;
    bool binary = false;
    {
      py::gil_scoped_release nogil;
      int64_t have = 0, nnz = 0;
      bool any_v = false, any_w = false;
      while (have < rows_) {
        if (!cur_ || cur_pos_ == (int64_t)cur_->size()) {
          // a block no piece holds any more goes back to the reader (its
          // buffers are recycled by the parsers)
          std::shared_ptr<RowBlock> b;
          for (auto& q : pool_)
            if (q.use_count() == 1) {
              b = q;
              break;
            }
          if (!b) {
            b = std::make_shared<RowBlock>();
            if (pool_.size() < 8) pool_.push_back(b);
          }
          if (!reader_->Next(b.get())) {
            cur_.reset();
            break;
          }
          cur_ = std::move(b);
          cur_pos_ = 0;
          continue;
        }
        const int64_t take = std::min(rows_ - have, (int64_t)cur_->size() - cur_pos_);
        const int64_t pn = cur_->offset[cur_pos_ + take] - cur_->offset[cur_pos_];
        pieces.push_back({cur_, cur_pos_, cur_pos_ + take, have, nnz});
        any_v = any_v || !cur_->value.empty();
        any_w = any_w || !cur_->weight.empty();
        cur_pos_ += take;
        have += take;
        nnz += pn;
      }
      if (pieces.empty()) {
        py::gil_scoped_acquire g;
        return py::none();
      }
      out = alloc(have, nnz, any_v, any_w);
      uint64_t* kp = reinterpret_cast<uint64_t*>(out.k.data_ptr());
      int64_t* op = out.o.data_ptr<int64_t>();
      float* lp = out.l.data_ptr<float>();
      float* vp = any_v ? out.v.data_ptr<float>() : nullptr;
      float* wp = any_w ? out.w.data_ptr<float>() : nullptr;
      op[0] = 0;
      std::atomic<bool> non_one{false};
      parallel(pieces.size(), ncopy_, [&](size_t i, int) {
        const Piece& pc = pieces[i];
        const RowBlock& b = *pc.b;
        const int64_t s = b.offset[pc.r0], e = b.offset[pc.r1], n = pc.r1 - pc.r0;
        std::memcpy(kp + pc.nnz_base, b.index.data() + s, (e - s) * sizeof(uint64_t));
        std::memcpy(lp + pc.row_base, b.label.data() + pc.r0, n * sizeof(float));
        for (int64_t r = 0; r < n; ++r)
          op[pc.row_base + r + 1] = pc.nnz_base + (b.offset[pc.r0 + r + 1] - s);
        if (vp) {
          if (b.value.empty()) {
            std::fill(vp + pc.nnz_base, vp + pc.nnz_base + (e - s), 1.f);
          } else {
            std::memcpy(vp + pc.nnz_base, b.value.data() + s, (e - s) * sizeof(float));
            for (int64_t j = s; j < e && !non_one.load(std::memory_order_relaxed); ++j)
              if (b.value[j] != 1.f) non_one = true;
          }
        }
        if (wp) {
          if (b.weight.empty()) std::fill(wp + pc.row_base, wp + pc.row_base + n, 1.f);
          else std::memcpy(wp + pc.row_base, b.weight.data() + pc.r0, n * sizeof(float));
        }
      });
      binary = vp && !non_one;
    }
    return to_py(out, binary);
  }

  int64_t rows_;
  bool pinned_;
  int ncopy_, ndec_ = 1;
  std::vector<std::vector<char>> scratch_;  // next_crb's LZ4 scratch, one per decode worker
  // CRB
  std::unique_ptr<InputSplit> split_;
  std::shared_ptr<CRBRecord> carry_;
  int64_t carry_pos_ = 0;
  // other formats
  std::unique_ptr<ThreadedReader> reader_;
  std::shared_ptr<RowBlock> cur_;
  int64_t cur_pos_ = 0;
  std::vector<std::shared_ptr<RowBlock>> pool_;
};

py::tuple localize_cpu(const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                       int64_t nshard, int64_t nthreads) {
  auto k = keys.contiguous();
  auto o = offset.contiguous();
  Tensor v;
  const float* vp = nullptr;
  if (val && val->defined() && val->numel()) {
    v = val->contiguous();
    vp = v.data_ptr<float>();
  }
  LocalizeResult r;
  {
    py::gil_scoped_release nogil;
    LocalizeCPU((const uint64_t*)k.data_ptr(), (size_t)k.numel(), o.data_ptr<int64_t>(),
                (size_t)o.numel() - 1, vp, (int)nshard, (int)nthreads, &r);
  }
  return py::make_tuple(vec_to_tensor(r.uniq, torch::kInt64), vec_to_tensor(r.ucnt, torch::kInt32),
                        vec_to_tensor(r.owner_cnt, torch::kInt64), vec_to_tensor(r.lid, torch::kInt32),
                        vec_to_tensor(r.csc_off, torch::kInt64), vec_to_tensor(r.csc_row, torch::kInt32),
                        vec_to_tensor(r.csc_val, torch::kFloat32));
}

}  // namespace

void register_all(py::module& m) {
  m.def("parse_conf", [](const std::string& text) { return conf_to_py(ParseConf(text)); });
  m.def("arg2proto", &Arg2Proto, "dmlc::Config-format text -> protobuf text format");
  m.def("debug_str", [](const Tensor& t, int m) {
    auto c = t.detach().cpu().contiguous().reshape({-1});
    const int64_t n = c.numel();
    switch (c.scalar_type()) {
      case torch::kFloat32: return DebugStr(c.data_ptr<float>(), n, m);
      case torch::kFloat64: return DebugStr(c.data_ptr<double>(), n, m);
      case torch::kInt32: return DebugStr(c.data_ptr<int32_t>(), n, m);
      case torch::kInt64: return DebugStr(c.data_ptr<int64_t>(), n, m);
      default: return DebugStr(c.to(torch::kFloat64).data_ptr<double>(), n, m);
    }
  }, py::arg("t"), py::arg("m") = 5);
  m.def("debug_str_block", [](const Tensor& keys, const Tensor& offset,
                              const c10::optional<Tensor>& val, const Tensor& label) {
    return DebugStr(py_to_block(keys.cpu(), offset.cpu(),
                                val ? c10::optional<Tensor>(val->cpu()) : c10::nullopt,
                                label.cpu(), c10::nullopt));
  }, py::arg("keys"), py::arg("offset"), py::arg("val") = py::none(), py::arg("label"));
  // the host AUC of csrc/host/auc_host.h (the device layer can run it on
  // worker threads for large training minibatches: WH_AUC_HOST_THREADS)
  m.def("auc_exact", [](torch::Tensor py, torch::Tensor label) {
    TORCH_CHECK(!py.is_cuda() && py.scalar_type() == torch::kFloat32 &&
                    label.scalar_type() == torch::kFloat32 && py.numel() == label.numel(),
                "auc_exact: float32 CPU tensors of one size");
    auto p = py.contiguous();
    auto l = label.contiguous();
    std::vector<uint64_t> ws;
    return wh::auc_exact_host(p.data_ptr<float>(), l.data_ptr<float>(), p.numel(), ws);
  });
  m.def("cityhash64", [](py::bytes b) {
    std::string s = b;
    return CityHash64(s.data(), s.size());
  });
  m.def("lz4_compress", [](py::bytes b) {
    std::string s = b;
    std::string out(LZ4CompressBound((int)s.size()), '\0');
    int n = LZ4Compress(s.data(), &out[0], (int)s.size(), (int)out.size());
    out.resize(n);
    return py::bytes(out);
  });
  m.def("lz4_decompress", [](py::bytes b, int64_t size) {
    std::string s = b;
    std::string out(size, '\0');
    int n = LZ4Decompress(s.data(), &out[0], (int)s.size(), (int)size);
    if (n != size) throw std::runtime_error("lz4: corrupt input");
    return py::bytes(out);
  });
  // ps-lite COMPRESSING filter for host (gloo) transfers: each peer's chunk
  // of an all-to-all-v LZ4-compressed on its own; a chunk LZ4 cannot shrink
  // travels raw (its size negated). Returns (packed bytes, signed sizes).
  m.def("lz4_pack", [](const Tensor& src, const std::vector<int64_t>& nbytes) {
    TORCH_CHECK(src.device().is_cpu() && src.is_contiguous() && src.scalar_type() == torch::kUInt8,
                "lz4_pack: contiguous uint8 CPU tensor");
    int64_t bound = 0, total = 0;
    for (int64_t n : nbytes) {
      TORCH_CHECK(n >= 0 && n < (int64_t)INT32_MAX / 2, "lz4_pack: chunk size out of range");
      bound += LZ4CompressBound((int)n);
      total += n;
    }
    TORCH_CHECK(total == src.numel(), "lz4_pack: chunk sizes do not cover the input");
    Tensor out = torch::empty({std::max<int64_t>(bound, 1)}, torch::kUInt8);
    std::vector<int64_t> csz(nbytes.size());
    int64_t used = 0;
    {
      py::gil_scoped_release nogil;
      const char* in = reinterpret_cast<const char*>(src.data_ptr());
      char* o = reinterpret_cast<char*>(out.data_ptr());
      for (size_t i = 0; i < nbytes.size(); ++i) {
        const int n = (int)nbytes[i];
        int c = n > 0 ? LZ4Compress(in, o + used, n, LZ4CompressBound(n)) : 0;
        if (n > 0 && (c <= 0 || c >= n)) {  // incompressible: stored
          std::memcpy(o + used, in, n);
          csz[i] = -(int64_t)n;
          c = n;
        } else {
          csz[i] = c;
        }
        in += n;
        used += c;
      }
    }
    return py::make_tuple(out.narrow(0, 0, used), csz);
  });
  m.def("lz4_unpack", [](const Tensor& packed, const std::vector<int64_t>& csz,
                         const std::vector<int64_t>& nbytes, Tensor dst) {
    TORCH_CHECK(packed.device().is_cpu() && packed.is_contiguous() &&
                    dst.device().is_cpu() && dst.is_contiguous() &&
                    packed.scalar_type() == torch::kUInt8 && dst.scalar_type() == torch::kUInt8,
                "lz4_unpack: contiguous uint8 CPU tensors");
    TORCH_CHECK(csz.size() == nbytes.size(), "lz4_unpack: size lists differ");
    int64_t need = 0, have = 0;
    for (size_t i = 0; i < csz.size(); ++i) {
      need += std::llabs(csz[i]);
      have += nbytes[i];
    }
    TORCH_CHECK(need == packed.numel() && have == dst.numel(), "lz4_unpack: sizes do not match");
    py::gil_scoped_release nogil;
    const char* in = reinterpret_cast<const char*>(packed.data_ptr());
    char* o = reinterpret_cast<char*>(dst.data_ptr());
    for (size_t i = 0; i < csz.size(); ++i) {
      const int64_t n = nbytes[i], c = csz[i];
      if (c < 0) {
        if (-c != n) throw std::runtime_error("lz4_unpack: stored chunk size mismatch");
        std::memcpy(o, in, n);
      } else if (n > 0) {
        if (LZ4Decompress(in, o, (int)c, (int)n) != n) throw std::runtime_error("lz4: corrupt chunk");
      }
      in += std::llabs(c);
      o += n;
    }
  });
  // (the file-system calls release the GIL: a remote URI is network I/O)
  m.def("match_file", &MatchFile, py::call_guard<py::gil_scoped_release>());
  m.def("resolve_path", &ResolvePath);
  m.def("list_directory", &ListDirectory, py::call_guard<py::gil_scoped_release>());
  m.def("file_size", &FileSize, py::call_guard<py::gil_scoped_release>());
  // native WebHDFS / S3 (remote_fs.h): the Python side's model and
  // prediction files go through these (wormhole_amd/utils/fs.py)
  m.def("is_remote", &IsRemote);
  m.def("remote_list", [](const std::string& uri) {
    py::list out;
    std::vector<RemoteEntry> es;
    {
      py::gil_scoped_release nogil;
      es = RemoteList(uri);
    }
    for (const auto& e : es) out.append(py::make_tuple(e.uri, e.size));
    return out;
  });
  m.def("remote_size", [](const std::string& uri) {
    py::gil_scoped_release nogil;
    return RemoteSize(uri);
  });
  m.def("remote_read", [](const std::string& uri, int64_t off, int64_t len) {
    std::string d;
    {
      py::gil_scoped_release nogil;
      d = RemoteRead(uri, off, len);
    }
    return py::bytes(d);
  }, py::arg("uri"), py::arg("off") = 0, py::arg("len") = (int64_t)1 << 62);
  m.def("remote_write", [](const std::string& uri, const std::string& data) {
    py::gil_scoped_release nogil;
    RemoteWrite(uri, data);
  });
  // (tests) a whole object read sequentially through a RemoteReader of the
  // given window in `chunk`-byte reads: (bytes, windows from the read-ahead)
  m.def("remote_read_stream", [](const std::string& uri, int64_t window, int64_t chunk) {
    std::string out;
    int64_t pre = 0;
    {
      py::gil_scoped_release nogil;
      RemoteReader r(uri, window);
      std::string buf((size_t)std::max<int64_t>(chunk, 1), '\0');
      while (true) {
        const size_t n = r.Read(&buf[0], buf.size());
        if (n == 0) break;
        out.append(buf.data(), n);
      }
      pre = r.prefetched();
    }
    return py::make_tuple(py::bytes(out), pre);
  });
  // streaming remote writes (S3 multipart / WebHDFS append), one part held;
  // dropped unclosed, its destructor aborts the upload over the network:
  // without the GIL (a Python thread -- a test's in-process server -- may be
  // the one that has to answer)
  struct NoGilDelete {
    void operator()(RemoteWriter* w) const {
      py::gil_scoped_release nogil;
      delete w;
    }
  };
  py::class_<RemoteWriter, std::unique_ptr<RemoteWriter, NoGilDelete>>(m, "RemoteWriter")
      .def(py::init<const std::string&, int64_t>(), py::arg("uri"), py::arg("part_bytes") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("write", [](RemoteWriter& w, py::bytes b) {
        std::string d = b;
        py::gil_scoped_release nogil;
        w.Write(d.data(), d.size());
      })
      .def("close", &RemoteWriter::Close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("parts", &RemoteWriter::parts);
  m.def("sigv4_authorization", &SigV4Authorization, py::arg("method"), py::arg("host"),
        py::arg("path"), py::arg("query"), py::arg("amz_date"), py::arg("payload_sha256"),
        py::arg("region"), py::arg("key_id"), py::arg("secret"), py::arg("token") = "");
  m.def("load_split", &load_split, py::arg("path"), py::arg("part") = 0, py::arg("nparts") = 1,
        py::arg("fmt") = "libsvm");
  m.def("read_text_split", [](const std::string& path, int part, int nparts) {
    std::string chunk, all;
    {
      py::gil_scoped_release nogil;
      InputSplit s(path, part, nparts, false);
      while (s.NextChunk(&chunk)) all += chunk;
    }
    return py::bytes(all);
  });
  m.def("read_recordio", [](const std::string& path, int part, int nparts) {
    std::vector<std::string> recs;
    {
      py::gil_scoped_release nogil;
      InputSplit s(path, part, nparts, true);
      std::string rec;
      while (s.NextRecord(&rec)) recs.push_back(rec);
    }
    py::list out;
    for (const auto& r : recs) out.append(py::bytes(r));
    return out;
  });
  m.def("crb_encode", [](const Tensor& keys, const Tensor& offset, const c10::optional<Tensor>& val,
                         const Tensor& label, const c10::optional<Tensor>& weight) {
    return py::bytes(CRBEncode(py_to_block(keys, offset, val, label, weight)));
  }, py::arg("keys"), py::arg("offset"), py::arg("val") = py::none(), py::arg("label"),
     py::arg("weight") = py::none());
  m.def("crb_decode", [](py::bytes b) {
    std::string s = b;
    RowBlock blk;
    CRBDecode(s.data(), s.size(), &blk);
    return block_to_py(blk);
  });
  m.def("parse_text", [](py::bytes b, const std::string& fmt) {
    std::string s = b;
    RowBlock blk;
    const char* p = s.data();
    const char* e = p + s.size();
    if (fmt == "libsvm") ParseLibSVM(p, e, &blk);
    else if (fmt == "criteo") ParseCriteo(p, e, true, &blk);
    else if (fmt == "criteo_test") ParseCriteo(p, e, false, &blk);
    else if (fmt == "adfea") ParseAdfea(p, e, &blk);
    else throw std::runtime_error("unknown text format " + fmt);
    return block_to_py(blk);
  });
  m.def("localize_cpu", &localize_cpu, py::arg("keys"), py::arg("offset"),
        py::arg("val") = py::none(), py::arg("nshard") = 1, py::arg("nthreads") = 4);

  py::class_<RecordIOWriter>(m, "RecordIOWriter")
      .def(py::init<const std::string&>())
      .def("write", [](RecordIOWriter& w, py::bytes b) {
        std::string s = b;
        w.WriteRecord(s);
      })
      .def("close", &RecordIOWriter::Close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("bytes_written", &RecordIOWriter::bytes_written);

  py::class_<PyTextBatches>(m, "TextBatches")
      .def(py::init<const std::string&, int, int, int64_t, bool, int64_t>(),
           py::call_guard<py::gil_scoped_release>(), py::arg("path"),
           py::arg("part"), py::arg("nparts"), py::arg("minibatch"), py::arg("pinned") = true,
           py::arg("depth") = 3)
      .def("next", &PyTextBatches::next);
  py::class_<PyMinibatchIter>(m, "MinibatchIter")
      .def(py::init<const std::string&, int, int, const std::string&, int64_t, int64_t, double,
                    int64_t, bool>(),
           py::call_guard<py::gil_scoped_release>(),
           py::arg("path"), py::arg("part"), py::arg("nparts"), py::arg("fmt"),
           py::arg("minibatch"), py::arg("shuffle_buf") = 0, py::arg("neg_sampling") = 1.0,
           py::arg("seed") = 0, py::arg("pinned") = false)
      .def("next", &PyMinibatchIter::next);
  py::class_<PyBlockIter>(m, "BlockIter")
      .def(py::init<const std::string&, int, int, const std::string&, int64_t, bool, int>(),
           py::call_guard<py::gil_scoped_release>(),
           py::arg("path"), py::arg("part"), py::arg("nparts"), py::arg("fmt"), py::arg("rows"),
           py::arg("pinned") = true, py::arg("nthreads") = 0)
      .def("next", &PyBlockIter::next);

  py::class_<WorkloadPool>(m, "WorkloadPool")
      .def(py::init<bool, uint64_t, double, double, int, double>(), py::arg("shuffle") = false,
           py::arg("seed") = 0, py::arg("straggler_factor") = 2.0,
           py::arg("straggler_min_sec") = 5.0, py::arg("straggler_min_done") = 10,
           py::arg("period") = 2.0)
      .def("add", &WorkloadPool::Add, py::arg("files"), py::arg("npart"), py::arg("node") = "")
      .def("clear", &WorkloadPool::Clear)
      .def("get", [](WorkloadPool& p, const std::string& node) -> py::object {
        Assignment a;
        if (!p.Get(node, &a)) return py::none();
        return py::make_tuple(a.filename, a.k, a.n);
      })
      .def("finish", &WorkloadPool::Finish)
      .def("finish_one", &WorkloadPool::FinishOne)
      .def("reset", &WorkloadPool::Reset)
      .def("remove_straggler", &WorkloadPool::RemoveStraggler)
      .def("is_finished", &WorkloadPool::IsFinished)
      .def("set_verbose", &WorkloadPool::set_verbose)
      .def_property_readonly("num_finished", &WorkloadPool::num_finished)
      .def_property_readonly("num_assigned", &WorkloadPool::num_assigned)
      .def_property_readonly("num_requeued", &WorkloadPool::num_requeued);

  m.def("run_scheduler", [](py::dict conf, int num_workers, int num_servers, Van& van) {
    SchedulerConf c;
    auto str = [&](const char* k, std::string* v) {
      if (conf.contains(k) && !conf[k].is_none()) *v = py::cast<std::string>(conf[k]);
    };
    auto i32 = [&](const char* k, int* v) {
      if (conf.contains(k) && !conf[k].is_none()) *v = py::cast<int>(conf[k]);
    };
    auto f64 = [&](const char* k, double* v) {
      if (conf.contains(k) && !conf[k].is_none()) *v = py::cast<double>(conf[k]);
    };
    auto bol = [&](const char* k, bool* v) {
      if (conf.contains(k) && !conf[k].is_none()) *v = py::cast<bool>(conf[k]);
    };
    str("app", &c.app); str("train_data", &c.train_data); str("val_data", &c.val_data);
    str("data_format", &c.data_format); str("model_in", &c.model_in);
    str("model_out", &c.model_out); str("predict_out", &c.predict_out);
    i32("max_data_pass", &c.max_data_pass); i32("save_iter", &c.save_iter);
    i32("load_iter", &c.load_iter); i32("num_parts_per_file", &c.num_parts_per_file);
    f64("print_sec", &c.print_sec); bol("local_data", &c.local_data);
    bol("early_stop", &c.early_stop); f64("min_objv_decr", &c.min_objv_decr);
    bol("resume", &c.resume);
    if (conf.contains("max_objv") && !conf["max_objv"].is_none()) {
      c.has_max_objv = true;
      c.max_objv = py::cast<double>(conf["max_objv"]);
    }
    py::gil_scoped_release nogil;
    Scheduler(c, num_workers, num_servers, &van).Run();
  }, py::arg("conf"), py::arg("num_workers"), py::arg("num_servers"), py::arg("van"),
     "Run the native parameter-server scheduler (epoch loop, workload dispatch, progress "
     "table, load/save fan-out) until the job ends");
  py::class_<Van>(m, "Van")
      .def(py::init<>())
      .def("listen", &Van::Listen)
      .def("connect", &Van::Connect, py::arg("host"), py::arg("port"), py::arg("my_id"),
           py::arg("timeout") = 60.0)
      .def("send", [](Van& v, const std::string& to, py::bytes b) {
        std::string s = b;
        py::gil_scoped_release nogil;
        return v.Send(to, s);
      })
      .def("recv", [](Van& v, double timeout) -> py::object {
        std::string from, msg;
        bool ok;
        {
          py::gil_scoped_release nogil;
          ok = v.Recv(timeout, &from, &msg);
        }
        if (!ok) return py::none();
        return py::make_tuple(from, py::bytes(msg));
      })
      .def("peers", &Van::Peers)
      .def("close", [](Van& v) {
        py::gil_scoped_release nogil;
        v.Close();
      })
      .def_property_readonly("port", &Van::port);
}

}  // namespace host
}  // namespace wh
