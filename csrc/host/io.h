#pragma once
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include "common.h"

namespace wh {
namespace host {

constexpr uint32_t kRecordIOMagic = 0xced7230a;

// URI -> local path (file://, plain paths; other schemes through the mount
// named by WH_FS_MOUNT_<SCHEME>; throws when none is configured). hdfs://,
// viewfs:// and s3:// without a mount are read and written natively
// (remote_fs.h) by the functions and classes below.
std::string ResolvePath(const std::string& uri);
std::vector<std::string> ListDirectory(const std::string& dir);
std::vector<std::string> MatchFile(const std::string& pattern);
int64_t FileSize(const std::string& path);

// Part `part` of `nparts` of one file, snapped to line (text) or record
// (RecordIO) boundaries so every record belongs to exactly one part.
class RemoteReader;

class InputSplit {
 public:
  InputSplit(const std::string& path, int part, int nparts, bool recordio);
  ~InputSplit();
  void BeforeFirst();
  // text: next chunk of whole lines (about `hint` bytes)
  bool NextChunk(std::string* out, size_t hint = 4 << 20);
  // recordio: next (re-assembled) record
  bool NextRecord(std::string* out);
  // recordio, zero-copy: the next record as a view into the part's memory
  // mapping (valid while this split lives); a record the writer split at
  // embedded magic words is re-assembled into *spill and the view points
  // there. Callers serialise the calls; the views can be read concurrently.
  bool NextRecordView(const char** data, size_t* size, std::string* spill);
  int64_t begin() const { return begin_; }
  int64_t end() const { return end_; }
  int64_t bytes_read() const { return pos_ - begin_; }

 private:
  int64_t Align(int64_t pos, int64_t size);
  void src_seek(int64_t off);
  int src_getc();
  size_t src_read(void* buf, size_t n);
  std::string path_;
  bool recordio_;
  std::FILE* fp_ = nullptr;                // local file
  std::unique_ptr<RemoteReader> remote_;  // or a remote one
  std::string own_;                        // a remote recordio part, fetched whole
  int64_t begin_ = 0, end_ = 0, pos_ = 0;
  std::string carry_;
  // recordio parts are memory-mapped (map_ = file bytes [map_off_,
  // map_off_ + map_len_) covering [begin_, end_)); null: stdio reads
  const char* map_ = nullptr;
  int64_t map_off_ = 0;
  size_t map_len_ = 0;
};

class RecordIOWriter {
 public:
  explicit RecordIOWriter(const std::string& path);
  ~RecordIOWriter();
  void WriteRecord(const char* buf, size_t size);
  void WriteRecord(const std::string& s) { WriteRecord(s.data(), s.size()); }
  size_t bytes_written() const { return bytes_; }
  void Close();

 private:
  std::FILE* fp_ = nullptr;
  size_t bytes_ = 0;
  // a remote target: the FILE streams into it (fopencookie), one part at a time
  std::unique_ptr<class RemoteWriter> remote_;
};

}  // namespace host
}  // namespace wh
