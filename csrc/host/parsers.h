#pragma once
#include <condition_variable>
#include <deque>
#include <map>
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

// A CRB record with its sections located but not decoded, and its row
// offsets decoded: the unit of the direct CRB reader (registry.cc
// BlockIter), which decodes every section straight into its place in the
// output block instead of into a RowBlock that is then copied.
struct CRBRecord {
  std::string spill;        // the bytes of a re-assembled record (else a view)
  const char* view = nullptr;
  size_t at[5] = {};        // label, offset, index, value, weight: byte offset
  int csz[5] = {};          // compressed size (<= 0: absent)
  int nrows = 0, isz = 8;
  hvec<int64_t> off;        // nrows + 1 row offsets from 0 (CRBDecodeOffsets)
  const char* base() const { return spill.empty() ? view : spill.data(); }
  int64_t nnz() const { return off.back(); }
};
void CRBLocate(const char* data, size_t size, CRBRecord* r);
void CRBDecodeOffsets(CRBRecord* r);
// rows [r0, r1) of section sec (0 label, 2 index, 3 value, 4 weight) into
// dst (index as uint64, the others float); false when the record has no
// such section (dst untouched). tmp: scratch for partial ranges / widening.
bool CRBDecodeRows(const CRBRecord& r, int sec, int64_t r0, int64_t r1, void* dst,
                   std::vector<char>* tmp);

// parse part k/n of a file chunk by chunk
class BlockReader {
 public:
  BlockReader(const std::string& path, int part, int nparts, const std::string& fmt);
  bool Next(RowBlock* blk);
  // I/O only: the next raw chunk (text: whole lines; crb: one record)
  bool NextRaw(std::string* buf);
  // crb: the next record as a view into the split's mapping (see
  // InputSplit::NextRecordView)
  bool NextRecordView(const char** data, size_t* size, std::string* spill) {
    return split_->NextRecordView(data, size, spill);
  }
  // CPU only: parse a raw chunk of format fmt
  static void ParseRaw(const std::string& fmt, const std::string& buf, RowBlock* blk);
  const std::string& fmt() const { return fmt_; }

 private:
  std::string fmt_;
  std::unique_ptr<InputSplit> split_;
};

// Parser threads over one split (dmlc ThreadedParser + the reference's
// OpenMP LibSVMParser): chunks are read in order under a lock, parsed by
// nthreads workers in parallel, and handed out IN READ ORDER (results do not
// depend on the thread count). nthreads = 0 picks WH_PARSE_THREADS or
// min(16, hardware threads).
class ThreadedReader {
 public:
  ThreadedReader(const std::string& path, int part, int nparts, const std::string& fmt,
                 int nthreads = 0, size_t depth = 4);
  ~ThreadedReader();
  // the next block in read order; *out's previous buffers are recycled
  bool Next(RowBlock* out);
  static int DefaultThreads();

 private:
  void Work();
  BlockReader reader_;
  size_t window_;
  std::mutex io_mu_, mu_;
  std::condition_variable cv_;
  int64_t next_read_ = 0, next_out_ = 0, total_ = -1;  // total_: chunks once EOF is seen
  std::map<int64_t, RowBlock> ready_;
  // blocks handed back by Next (the consumer's previous one): their buffers
  // are reused by the decoders -- fresh multi-MB vectors per record were
  // mmap / munmap pairs, and the munmaps' TLB shootdowns across the decoder
  // threads made 8 threads slower than 2 until malloc's threshold adapted
  std::vector<RowBlock> spare_;
  bool stop_ = false;
  std::string err_;
  std::vector<std::thread> th_;
};

class MinibatchIter {
 public:
  MinibatchIter(const std::string& path, int part, int nparts, const std::string& fmt,
                size_t mb_size, size_t shuf_buf = 0, float neg_sampling = 1.f,
                uint64_t seed = 0, int nthreads = 0);
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
  std::vector<size_t> perm_, sel_;
};

}  // namespace host
}  // namespace wh
