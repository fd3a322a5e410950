// Shared host-side types of the native runtime.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <sstream>
#include <string>
#include <cstring>
#include <vector>

namespace wh {
namespace host {

#define WH_CHECK(cond, msg)                                                   \
  do {                                                                        \
    if (!(cond)) throw std::runtime_error(std::string("check failed: ") +    \
                                          #cond + ": " + (msg));             \
  } while (0)

// CSR minibatch / parse block (reference dmlc::RowBlockContainer<uint64_t>):
// offsets are absolute into index/value, value empty == all ones.
// std::vector storage that resize() leaves uninitialised: a decoded block
// (CRB sections, parsed chunks) overwrites every element anyway, and
// value-initialising first cost a whole extra pass over ~330 MB per million
// Criteo rows
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = DefaultInitAlloc<U>;
  };
  DefaultInitAlloc() = default;
  template <class U>
  DefaultInitAlloc(const DefaultInitAlloc<U>&) noexcept {}
  template <class U>
  void construct(U* p) noexcept {
    ::new (static_cast<void*>(p)) U;
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
template <class T>
using hvec = std::vector<T, DefaultInitAlloc<T>>;

struct RowBlock {
  hvec<float> label;
  hvec<int64_t> offset{0};
  hvec<uint64_t> index;
  hvec<float> value;
  hvec<float> weight;

  size_t size() const { return offset.size() - 1; }
  size_t nnz() const { return index.size(); }
  void clear() {
    label.clear();
    offset.assign(1, 0);
    index.clear();
    value.clear();
    weight.clear();
  }
  // append row r of another block
  void push_row(const RowBlock& b, size_t r) {
    label.push_back(b.label[r]);
    if (!b.weight.empty()) weight.push_back(b.weight[r]);
    const int64_t s = b.offset[r], e = b.offset[r + 1];
    const bool bval = !b.value.empty();
    if (bval && value.size() < index.size()) value.resize(index.size(), 1.f);
    for (int64_t j = s; j < e; ++j) {
      index.push_back(b.index[j]);
      if (bval) value.push_back(b.value[j]);
      else if (!value.empty()) value.push_back(1.f);
    }
    offset.push_back((int64_t)index.size());
  }
  // rows [r0, r1) of b appended in bulk (memcpy of the id / value ranges)
  void append_rows(const RowBlock& b, size_t r0, size_t r1) {
    if (r1 <= r0) return;
    const int64_t s = b.offset[r0], e = b.offset[r1];
    const int64_t base = (int64_t)index.size();
    const bool bval = !b.value.empty();
    if (bval && value.size() < index.size()) value.resize(index.size(), 1.f);
    label.insert(label.end(), b.label.begin() + r0, b.label.begin() + r1);
    if (!b.weight.empty()) weight.insert(weight.end(), b.weight.begin() + r0, b.weight.begin() + r1);
    index.insert(index.end(), b.index.begin() + s, b.index.begin() + e);
    if (bval) value.insert(value.end(), b.value.begin() + s, b.value.begin() + e);
    else if (!value.empty()) value.resize(index.size(), 1.f);
    const size_t o0 = offset.size();
    offset.resize(o0 + (r1 - r0));
    for (size_t r = r0; r < r1; ++r) offset[o0 + (r - r0)] = base + (b.offset[r + 1] - s);
  }
  // rows[0..n) of b appended in that order (the shuffle buffer's gather):
  // one resize per array, then a memcpy per row
  void append_gather(const RowBlock& b, const size_t* rows, size_t n) {
    if (n == 0) return;
    const bool bval = !b.value.empty(), bw = !b.weight.empty();
    if (bval && value.size() < index.size()) value.resize(index.size(), 1.f);
    size_t add = 0;
    for (size_t i = 0; i < n; ++i) add += (size_t)(b.offset[rows[i] + 1] - b.offset[rows[i]]);
    size_t pos = index.size();
    const size_t l0 = label.size(), o0 = offset.size(), w0 = weight.size();
    index.resize(pos + add);
    if (bval || !value.empty()) value.resize(pos + add, 1.f);
    label.resize(l0 + n);
    offset.resize(o0 + n);
    if (bw) weight.resize(w0 + n);
    for (size_t i = 0; i < n; ++i) {
      const size_t r = rows[i];
      const int64_t s = b.offset[r], e = b.offset[r + 1];
      const size_t len = (size_t)(e - s);
      std::memcpy(&index[pos], &b.index[s], len * sizeof(uint64_t));
      if (bval) std::memcpy(&value[pos], &b.value[s], len * sizeof(float));
      pos += len;
      label[l0 + i] = b.label[r];
      if (bw) weight[w0 + i] = b.weight[r];
      offset[o0 + i] = (int64_t)pos;
    }
  }
  // drop the value array when every value is 1 (reference minibatch_iter.h:114-116)
  void compact_binary() {
    for (float v : value)
      if (v != 1.f) return;
    value.clear();
  }
};

// ---- config ---------------------------------------------------------------
struct ConfItem {
  std::string key;
  char kind;  // 's' quoted string, 't' bare token (number/enum/bool), 'm' message
  std::string value;
  std::vector<ConfItem> children;
};
std::vector<ConfItem> ParseConf(const std::string& text);
std::string Arg2Proto(const std::string& text);

// ---- debug strings (reference learn/base/debug.h:9-43) ---------------------
// "[n]: a0 a1 ... " with the first and last m entries when n > 2m
template <typename V>
std::string DebugStr(const V* data, int64_t n, int m = 5) {
  std::string s = "[" + std::to_string(n) + "]: ";
  auto put = [&](int64_t i) {
    std::ostringstream o;
    o << data[i];
    s += o.str() + " ";
  };
  if (n <= 2 * m) {
    for (int64_t i = 0; i < n; ++i) put(i);
  } else {
    for (int64_t i = 0; i < m; ++i) put(i);
    s += "... ";
    for (int64_t i = n - m; i < n; ++i) put(i);
  }
  return s;
}

inline std::string DebugStr(const RowBlock& b) {
  const int64_t n = (int64_t)b.size(), nnz = (int64_t)b.nnz();
  std::string s = "label: " + DebugStr(b.label.data(), n) + "\n" +
                  "offset: " + DebugStr(b.offset.data(), n + 1) + "\n" +
                  "index: " + DebugStr(b.index.data(), nnz);
  if (!b.value.empty()) s += "\nvalue: " + DebugStr(b.value.data(), nnz);
  return s;
}

// ---- hashing / codecs ------------------------------------------------------
uint64_t CityHash64(const char* s, size_t len);
int LZ4CompressBound(int n);
int LZ4Compress(const char* src, char* dst, int srcSize, int dstCap);
int LZ4Decompress(const char* src, char* dst, int compressedSize, int dstCap);

}  // namespace host
}  // namespace wh
