// Shared host-side types of the native runtime.
#pragma once
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <sstream>
#include <string>
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
struct RowBlock {
  std::vector<float> label;
  std::vector<int64_t> offset{0};
  std::vector<uint64_t> index;
  std::vector<float> value;
  std::vector<float> weight;

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
