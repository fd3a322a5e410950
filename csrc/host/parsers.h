#pragma once
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>

#include "common.h"
#include "io.h"

namespace wh {
namespace host {

void ParseLibSVM(const char* p, const char* end, RowBlock* blk);
void ParseCriteo(const char* p, const char* end, bool is_train, RowBlock* blk);
void ParseAdfea(const char* p, const char* end, RowBlock* blk);
std::string CRBEncode(const RowBlock& b);
void CRBDecode(const char* data, size_t size, RowBlock* blk);

// parse part k/n of a file chunk by chunk
class BlockReader {
 public:
  BlockReader(const std::string& path, int part, int nparts, const std::string& fmt);
  bool Next(RowBlock* blk);

 private:
  std::string fmt_;
  std::unique_ptr<InputSplit> split_;
};

// BlockReader on a background thread with a bounded queue (dmlc ThreadedParser)
class ThreadedReader {
 public:
  ThreadedReader(const std::string& path, int part, int nparts, const std::string& fmt,
                 size_t depth = 4);
  ~ThreadedReader();
  bool Next(RowBlock* out);

 private:
  void Run();
  BlockReader reader_;
  size_t depth_;
  std::deque<RowBlock> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool done_ = false, stop_ = false;
  std::string err_;
  std::thread th_;
};

class MinibatchIter {
 public:
  MinibatchIter(const std::string& path, int part, int nparts, const std::string& fmt,
                size_t mb_size, size_t shuf_buf = 0, float neg_sampling = 1.f,
                uint64_t seed = 0);
  bool Next();
  const RowBlock& Value() const { return mb_; }

 private:
  size_t mb_size_, shuf_buf_;
  float neg_;
  std::mt19937_64 rng_;
  std::unique_ptr<ThreadedReader> reader_;
  std::unique_ptr<MinibatchIter> inner_;
  RowBlock in_, mb_;
  size_t start_ = 0, end_ = 0;
  std::vector<size_t> perm_;
};

}  // namespace host
}  // namespace wh
