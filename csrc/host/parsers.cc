// Text / binary row-block parsers (reference: dmlc LibSVMParser [ext],
// learn/base/criteo_parser.h, learn/base/adfea_parser.h,
// learn/base/compressed_row_block.h) and the threaded minibatch iterator
// (learn/base/minibatch_iter.h: fixed-size minibatches of part k/n of a
// file, optional shuffle buffer, negative down-sampling).
#include "parsers.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <numeric>

namespace wh {
namespace host {

namespace {

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n'; }
inline bool is_eol(char c) { return c == '\n' || c == '\r'; }

}  // namespace

// libsvm:  label[:weight] idx[:value] idx[:value] ...
void ParseLibSVM(const char* p, const char* end, RowBlock* blk) {
  blk->clear();
  bool any_val = false;
  while (p < end) {
    while (p < end && is_space(*p)) ++p;
    if (p >= end) break;
    // label
    char* q;
    float label = std::strtof(p, &q);
    if (q == p) throw std::runtime_error("libsvm: bad label");
    p = q;
    if (p < end && *p == ':') {
      ++p;
      float w = std::strtof(p, &q);
      p = q;
      blk->weight.resize(blk->label.size(), 1.f);
      blk->weight.push_back(w);
    } else if (!blk->weight.empty()) {
      blk->weight.push_back(1.f);
    }
    blk->label.push_back(label);
    while (p < end && !is_eol(*p)) {
      while (p < end && (*p == ' ' || *p == '\t')) ++p;
      if (p >= end || is_eol(*p)) break;
      uint64_t idx = std::strtoull(p, &q, 10);
      if (q == p) throw std::runtime_error("libsvm: bad feature index");
      p = q;
      float v = 1.f;
      if (p < end && *p == ':') {
        ++p;
        v = std::strtof(p, &q);
        p = q;
      }
      if (v != 1.f && !any_val) {
        any_val = true;
        blk->value.assign(blk->index.size(), 1.f);
      }
      blk->index.push_back(idx);
      if (any_val) blk->value.push_back(v);
    }
    blk->offset.push_back((int64_t)blk->index.size());
  }
}

// criteo TSV: [label] 13 integer fields, 26 categorical (8-char hex) fields
void ParseCriteo(const char* p, const char* end, bool is_train, RowBlock* blk) {
  blk->clear();
  // a Criteo line is ~200-250 bytes with up to 39 ids: reserve once
  const size_t rows_est = (size_t)(end - p) / 180 + 16;
  blk->label.reserve(rows_est);
  blk->offset.reserve(rows_est + 1);
  blk->index.reserve(rows_est * 39);
  auto find = [&](const char* s, char c) {
    while (s != end && *s != c && !is_eol(*s)) ++s;
    return s;
  };
  while (p < end) {
    while (p < end && is_eol(*p)) ++p;
    if (p >= end) break;
    const char* pp;
    if (is_train) {
      pp = find(p, '\t');
      if (pp == p) throw std::runtime_error("criteo: no label, try criteo_test");
      blk->label.push_back(std::strtof(p, nullptr));  // stops at the tab
      p = (pp < end && *pp == '\t') ? pp + 1 : pp;  // a label-only line stays one row
    } else {
      blk->label.push_back(0.f);
    }
    for (uint64_t i = 0; i < 13; ++i) {
      pp = find(p, '\t');
      if (pp > p)
        blk->index.push_back((CityHash64(p, pp - p) >> 10) | (i << 54));
      p = pp;
      if (p < end && *p == '\t') ++p;
    }
    for (uint64_t i = 0; i < 26; ++i) {
      if (p >= end || is_eol(*p)) break;
      pp = find(p, '\t');
      if (pp > p)
        blk->index.push_back((CityHash64(p, pp - p) >> 10) | ((i + 13) << 54));
      p = pp;
      if (p < end && *p == '\t') ++p;
    }
    while (p < end && !is_eol(*p)) ++p;
    blk->offset.push_back((int64_t)blk->index.size());
  }
}

// adfea: "<lineid> <count> <label> idx:gid idx:gid ..." (learn/base/adfea_parser.h:43-79)
void ParseAdfea(const char* p, const char* end, RowBlock* blk) {
  blk->clear();
  int i = 0;
  while (p != end && std::isspace((unsigned char)*p)) ++p;
  while (p != end) {
    const char* head = p;
    while (p != end && std::isdigit((unsigned char)*p)) ++p;
    if (head == p) throw std::runtime_error("adfea: unexpected character");
    if (p != end && *p == ':') {
      ++p;
      uint64_t idx = std::strtoull(head, nullptr, 10);
      uint64_t gid = std::strtoull(p, nullptr, 10);
      idx = (idx >> 10) | (gid << 54);
      while (p != end && std::isdigit((unsigned char)*p)) ++p;
      blk->index.push_back(idx);
    } else {
      if (i == 2) {
        i = 0;
        if (!blk->label.empty()) blk->offset.push_back((int64_t)blk->index.size());
        blk->label.push_back(*head == '1' ? 1.f : 0.f);
      } else {
        ++i;
      }
    }
    while (p != end && std::isspace((unsigned char)*p)) ++p;
  }
  if (!blk->label.empty()) blk->offset.push_back((int64_t)blk->index.size());
}

// ------------------------------------------------------------------- CRB
namespace {
constexpr int kCRBMagic = 1196140743;
void put_int(std::string* s, int v) { s->append(reinterpret_cast<const char*>(&v), 4); }
void put_section(std::string* s, const void* data, size_t bytes) {
  if (!data || bytes == 0) {
    put_int(s, 0);
    return;
  }
  std::vector<char> dst(LZ4CompressBound((int)bytes));
  const int n = LZ4Compress((const char*)data, dst.data(), (int)bytes, (int)dst.size());
  WH_CHECK(n > 0, "lz4 compression failed");
  put_int(s, n);
  s->append(dst.data(), n);
}
}  // namespace

std::string CRBEncode(const RowBlock& in) {
  RowBlock b = in;
  b.compact_binary();
  const int nrows = (int)b.size();
  const int nnz = (int)(b.offset.back() - b.offset.front());
  std::string s;
  put_int(&s, kCRBMagic);
  put_int(&s, (int)sizeof(uint64_t));
  put_int(&s, nrows);
  std::vector<size_t> off(b.offset.begin(), b.offset.end());
  put_section(&s, b.label.data(), nrows * sizeof(float));
  put_section(&s, off.data(), (nrows + 1) * sizeof(size_t));
  put_section(&s, b.index.data(), nnz * sizeof(uint64_t));
  put_section(&s, b.value.empty() ? nullptr : b.value.data(), nnz * sizeof(float));
  put_section(&s, b.weight.empty() ? nullptr : b.weight.data(), nrows * sizeof(float));
  return s;
}

void CRBDecode(const char* data, size_t size, RowBlock* blk) {
  blk->clear();
  size_t cur = 0;
  auto get_int = [&]() {
    WH_CHECK(cur + 4 <= size, "truncated crb record");
    int v;
    std::memcpy(&v, data + cur, 4);
    cur += 4;
    return v;
  };
  auto section = [&](void* dst, size_t bytes) -> bool {
    const int cp = get_int();
    if (cp <= 0) return false;
    WH_CHECK(cur + cp <= size, "truncated crb section");
    const int got = LZ4Decompress(data + cur, (char*)dst, cp, (int)bytes);
    WH_CHECK(got == (int)bytes, "crb section size mismatch");
    cur += cp;
    return true;
  };
  WH_CHECK(get_int() == kCRBMagic, "wrong data format (not a CRB record)");
  const int isz = get_int();
  WH_CHECK(isz == 8 || isz == 4, "unsupported crb index width");
  const int nrows = get_int();
  blk->label.resize(nrows);
  if (!section(blk->label.data(), nrows * sizeof(float))) blk->label.assign(nrows, 0.f);
  std::vector<size_t> off(nrows + 1, 0);
  section(off.data(), (nrows + 1) * sizeof(size_t));
  blk->offset.assign(off.begin(), off.end());
  const int64_t base = blk->offset[0];
  for (auto& o : blk->offset) o -= base;
  const int nnz = (int)blk->offset.back();
  // (a record whose rows hold non-zeros must carry the index section)
  if (isz == 8) {
    blk->index.resize(nnz);
    WH_CHECK(section(blk->index.data(), nnz * sizeof(uint64_t)) || nnz == 0,
             "crb record has non-zeros but no index section");
  } else {
    std::vector<uint32_t> tmp(nnz);
    WH_CHECK(section(tmp.data(), nnz * sizeof(uint32_t)) || nnz == 0,
             "crb record has non-zeros but no index section");
    blk->index.assign(tmp.begin(), tmp.end());
  }
  blk->value.resize(nnz);
  if (!section(blk->value.data(), nnz * sizeof(float))) blk->value.clear();
  blk->weight.resize(nrows);
  if (!section(blk->weight.data(), nrows * sizeof(float))) blk->weight.clear();
}

void CRBLocate(const char* data, size_t size, CRBRecord* r) {
  if (data != r->spill.data()) {
    r->view = data;
  }
  size_t cur = 0;
  auto get_int = [&]() {
    WH_CHECK(cur + 4 <= size, "truncated crb record");
    int v;
    std::memcpy(&v, data + cur, 4);
    cur += 4;
    return v;
  };
  WH_CHECK(get_int() == kCRBMagic, "wrong data format (not a CRB record)");
  r->isz = get_int();
  WH_CHECK(r->isz == 8 || r->isz == 4, "unsupported crb index width");
  r->nrows = get_int();
  WH_CHECK(r->nrows >= 0, "bad crb row count");
  for (int s = 0; s < 5; ++s) {
    r->csz[s] = get_int();
    r->at[s] = cur;
    if (r->csz[s] > 0) {
      WH_CHECK(cur + r->csz[s] <= size, "truncated crb section");
      cur += r->csz[s];
    }
  }
  r->off.clear();
}

void CRBDecodeOffsets(CRBRecord* r) {
  const int n = r->nrows;
  std::vector<size_t> o(n + 1, 0);
  if (r->csz[1] > 0) {
    const int got = LZ4Decompress(r->base() + r->at[1], (char*)o.data(), r->csz[1],
                                  (int)((n + 1) * sizeof(size_t)));
    WH_CHECK(got == (int)((n + 1) * sizeof(size_t)), "crb section size mismatch");
  }
  r->off.resize(n + 1);
  for (int i = 0; i <= n; ++i) r->off[i] = (int64_t)(o[i] - o[0]);
}

bool CRBDecodeRows(const CRBRecord& r, int sec, int64_t r0, int64_t r1, void* dst,
                   std::vector<char>* tmp) {
  if (r.csz[sec] <= 0) return false;
  const bool per_nnz = sec == 2 || sec == 3;
  const int64_t total = per_nnz ? r.nnz() : r.nrows;
  const int64_t a = per_nnz ? r.off[r0] : r0, b = per_nnz ? r.off[r1] : r1;
  const int esz = sec == 2 ? r.isz : 4;
  const int bytes = (int)(total * esz);
  const char* src = r.base() + r.at[sec];
  if (a == 0 && b == total && !(sec == 2 && esz == 4)) {  // whole section, in place
    WH_CHECK(LZ4Decompress(src, (char*)dst, r.csz[sec], bytes) == bytes,
             "crb section size mismatch");
    return true;
  }
  if (tmp->size() < (size_t)bytes + 64) tmp->resize((size_t)bytes + 64);
  WH_CHECK(LZ4Decompress(src, tmp->data(), r.csz[sec], bytes) == bytes,
           "crb section size mismatch");
  if (sec == 2 && esz == 4) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(tmp->data());
    uint64_t* d = static_cast<uint64_t*>(dst);
    for (int64_t j = a; j < b; ++j) d[j - a] = s32[j];
  } else {
    std::memcpy(dst, tmp->data() + a * esz, (size_t)(b - a) * esz);
  }
  return true;
}

// --------------------------------------------------------------- parsing
BlockReader::BlockReader(const std::string& path, int part, int nparts, const std::string& fmt)
    : fmt_(fmt) {
  if (fmt != "libsvm" && fmt != "criteo" && fmt != "criteo_test" && fmt != "adfea" &&
      fmt != "crb")
    throw std::runtime_error("unknown datatype " + fmt);
  split_.reset(new InputSplit(path, part, nparts, fmt == "crb"));
}

bool BlockReader::NextRaw(std::string* buf) {
  if (fmt_ == "crb") return split_->NextRecord(buf);
  // 1 MB text chunks: a 10 MB virtual part still feeds ~10 parser threads
  return split_->NextChunk(buf, 1 << 20);
}

void BlockReader::ParseRaw(const std::string& fmt, const std::string& buf, RowBlock* blk) {
  if (fmt == "crb") {
    CRBDecode(buf.data(), buf.size(), blk);
    return;
  }
  const char* p = buf.data();
  const char* e = p + buf.size();
  if (fmt == "libsvm") ParseLibSVM(p, e, blk);
  else if (fmt == "criteo") ParseCriteo(p, e, true, blk);
  else if (fmt == "criteo_test") ParseCriteo(p, e, false, blk);
  else ParseAdfea(p, e, blk);
}

bool BlockReader::Next(RowBlock* blk) {
  std::string buf;
  while (true) {
    if (!NextRaw(&buf)) return false;
    ParseRaw(fmt_, buf, blk);
    if (fmt_ == "crb" || blk->size() > 0) return true;
  }
}

// ------------------------------------------------------ threaded parser
int ThreadedReader::DefaultThreads() {
  if (const char* e = std::getenv("WH_PARSE_THREADS")) {
    const int n = std::atoi(e);
    if (n > 0) return n;
  }
  const int hw = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(16, hw));
}

ThreadedReader::ThreadedReader(const std::string& path, int part, int nparts,
                               const std::string& fmt, int nthreads, size_t depth)
    : reader_(path, part, nparts, fmt) {
  const int n = nthreads > 0 ? nthreads : DefaultThreads();
  window_ = depth * (size_t)n;
  for (int t = 0; t < n; ++t) th_.emplace_back([this] { Work(); });
}

ThreadedReader::~ThreadedReader() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_)
    if (t.joinable()) t.join();
}

void ThreadedReader::Work() {
  try {
    while (true) {
      {  // bounded look-ahead: at most window_ chunks parsed ahead of the consumer
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          return stop_ || total_ >= 0 || next_read_ - next_out_ < (int64_t)window_;
        });
        if (stop_ || total_ >= 0) return;
      }
      std::string buf;
      int64_t seq;
      bool ok;
      const bool crb = reader_.fmt() == "crb";
      const char* rec = nullptr;
      size_t rec_n = 0;
      {
        std::lock_guard<std::mutex> io(io_mu_);
        // crb: only the record's header is read under the lock; the body
        // is decoded from the mapping by this thread, in parallel
        ok = crb ? reader_.NextRecordView(&rec, &rec_n, &buf) : reader_.NextRaw(&buf);
        std::lock_guard<std::mutex> lk(mu_);
        seq = next_read_;
        if (ok) {
          ++next_read_;
        } else if (total_ < 0) {
          total_ = next_read_;
        }
      }
      if (!ok) {
        cv_.notify_all();
        return;
      }
      RowBlock b;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!spare_.empty()) {
          b = std::move(spare_.back());
          spare_.pop_back();
        }
      }
      b.clear();  // (keeps the recycled capacity)
      if (crb) CRBDecode(rec, rec_n, &b);
      else BlockReader::ParseRaw(reader_.fmt(), buf, &b);
      {
        std::lock_guard<std::mutex> lk(mu_);
        ready_.emplace(seq, std::move(b));
      }
      cv_.notify_all();
    }
  } catch (const std::exception& e) {
    std::lock_guard<std::mutex> lk(mu_);
    if (err_.empty()) err_ = e.what();
    if (total_ < 0) total_ = next_read_;
    cv_.notify_all();
  }
}

bool ThreadedReader::Next(RowBlock* out) {
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [&] {
      return !err_.empty() || ready_.count(next_out_) ||
             (total_ >= 0 && next_out_ >= total_);
    });
    if (!err_.empty()) throw std::runtime_error(err_);
    auto it = ready_.find(next_out_);
    if (it == ready_.end()) return false;  // all chunks consumed
    std::swap(*out, it->second);
    if (it->second.index.capacity() && spare_.size() < window_) spare_.push_back(std::move(it->second));
    ready_.erase(it);
    ++next_out_;
    cv_.notify_all();
    if (out->size() > 0 || reader_.fmt() == "crb") return true;
  }
}

// ------------------------------------------------------- minibatch iter
MinibatchIter::MinibatchIter(const std::string& path, int part, int nparts,
                             const std::string& fmt, size_t mb_size, size_t shuf_buf,
                             float neg_sampling, uint64_t seed, int nthreads)
    : mb_size_(mb_size), shuf_buf_(shuf_buf), neg_(neg_sampling), rng_(seed) {
  WH_CHECK(mb_size > 0, "minibatch size must be positive");
  if (shuf_buf) {
    WH_CHECK(shuf_buf > mb_size, "shuffle buffer must exceed the minibatch size");
    inner_.reset(new MinibatchIter(path, part, nparts, fmt, shuf_buf, 0, 1.f, seed + 1, nthreads));
  } else {
    reader_.reset(new ThreadedReader(path, part, nparts, fmt, nthreads));
  }
}

bool MinibatchIter::Next() {
  mb_.clear();
  if (mb_.index.capacity() == 0) {  // first minibatch: reserve for ~40 ids per row
    mb_.label.reserve(mb_size_);
    mb_.offset.reserve(mb_size_ + 1);
    mb_.index.reserve(mb_size_ * 40);
  }
  while (mb_.size() < mb_size_) {
    if (start_ == end_) {
      if (!inner_) {
        if (!reader_->Next(&in_)) break;
      } else {
        if (!inner_->Next()) break;
        in_ = inner_->Value();
        perm_.resize(in_.size());
        std::iota(perm_.begin(), perm_.end(), 0);
        std::shuffle(perm_.begin(), perm_.end(), rng_);
      }
      start_ = 0;
      end_ = in_.size();
    }
    const size_t len = std::min(end_ - start_, mb_size_ - mb_.size());
    if (!inner_) {  // in order: one bulk copy
      mb_.append_rows(in_, start_, start_ + len);
    } else {
      std::uniform_real_distribution<float> U(0.f, 1.f);
      sel_.clear();
      for (size_t i = start_; i < start_ + len; ++i) {
        const size_t r = perm_[i];
        // negative down-sampling keeps a negative with probability neg_sampling
        // (the reference drops with that probability, §2.9 item 7: fixed here
        // to the documented "down sampling ratio" meaning)
        if (neg_ < 1.f && in_.label[r] <= 0.f && U(rng_) > neg_) continue;
        sel_.push_back(r);
      }
      mb_.append_gather(in_, sel_.data(), sel_.size());
    }
    start_ += len;
  }
  mb_.compact_binary();
  return mb_.size() > 0;
}

}  // namespace host
}  // namespace wh
