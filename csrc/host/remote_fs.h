// Remote file systems read and written natively: HDFS through its WebHDFS
// REST interface and S3 (or any S3-compatible object store) through the S3
// REST API, over HTTP/1.1 (TLS through OpenSSL for https endpoints, AWS
// Signature Version 4 when credentials are set).
//
// Replaces the dmlc-core HDFS / S3 file systems the reference streams its
// data and models through (doc/common/input.rst:53-115: train_data =
// "hdfs://..." / "s3://...", model_out likewise). The data path reads byte
// ranges (InputSplit parts, the device text reader), the control path lists
// directories and stats files (MatchFile), models are written whole.
//
// Addressing (no mount configured for the scheme: WH_FS_MOUNT_<SCHEME> still
// takes precedence, csrc/host/io.cc ResolvePath):
//   hdfs://host[:port]/path, viewfs://...   WebHDFS at http://host:<port>/webhdfs/v1/path
//       <port>: WH_WEBHDFS_PORT (default 9870, the name node's HTTP port --
//       the port in the URI is the RPC port); WH_WEBHDFS_URL=http[s]://h:p
//       overrides host and port; user: HADOOP_USER_NAME, else USER
//   s3://bucket/key                          path-style requests to
//       WH_S3_ENDPOINT (default https://s3.<AWS_REGION or us-east-1>.amazonaws.com);
//       signed with AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY (and
//       AWS_SESSION_TOKEN) when set, anonymous otherwise
#pragma once
#include <cstdint>
#include <future>
#include <string>
#include <vector>

namespace wh {
namespace host {

struct RemoteEntry {
  std::string uri;  // the file's full URI (same scheme and authority as the listing)
  int64_t size = 0;
};

// A URI served by this module: an hdfs / viewfs / s3 scheme with no local
// mount configured for it.
bool IsRemote(const std::string& uri);
// The files directly under `dir_uri` (sorted by URI); a file URI lists itself.
std::vector<RemoteEntry> RemoteList(const std::string& dir_uri);
// Size in bytes, -1 when the object does not exist.
int64_t RemoteSize(const std::string& uri);
// Bytes [off, off + len) (fewer at the end of the object).
std::string RemoteRead(const std::string& uri, int64_t off, int64_t len);
// Create / overwrite the object with `data` (a RemoteWriter).
void RemoteWrite(const std::string& uri, const std::string& data);

// Streaming writes of one remote object, memory bounded by one part: S3
// multipart upload (CreateMultipartUpload / UploadPart / Complete, aborted
// if the writer is dropped unclosed; an object smaller than one part is a
// single PUT), WebHDFS CREATE with the first part then APPEND per part.
// part_bytes: 0 = 64 MiB (S3 wants parts of >= 5 MiB but the last).
class RemoteWriter {
 public:
  explicit RemoteWriter(const std::string& uri, int64_t part_bytes = 0);
  ~RemoteWriter();
  RemoteWriter(const RemoteWriter&) = delete;
  RemoteWriter& operator=(const RemoteWriter&) = delete;
  void Write(const char* p, size_t n);
  void Close();  // uploads what is left and finishes the object
  int64_t parts() const { return nparts_; }

 private:
  void Part(bool last);
  std::string uri_, buf_, upload_id_;
  std::vector<std::string> etags_;
  int64_t part_ = 0, nparts_ = 0;
  bool hdfs_ = false, created_ = false, closed_ = false;
};

// Sequential reads of one remote object through a read-ahead window; once
// two windows were read back to back, the next one is fetched in the
// background while the current one is consumed (a seek elsewhere drops it).
class RemoteReader {
 public:
  explicit RemoteReader(const std::string& uri, int64_t window = 8 << 20);
  ~RemoteReader();
  int64_t size() const { return size_; }
  void Seek(int64_t off) { pos_ = off; }
  int64_t tell() const { return pos_; }
  size_t Read(char* buf, size_t n);
  int GetC();  // EOF (-1) at the end
  int64_t prefetched() const { return prefetched_; }  // windows taken from the read-ahead

 private:
  void Fill();
  std::string uri_;
  int64_t size_ = 0, pos_ = 0, win_;
  std::string buf_;
  int64_t buf_off_ = 0;
  std::future<std::string> next_;  // the read-ahead window at next_off_
  int64_t next_off_ = -1, prefetched_ = 0;
  bool sequential_ = false;
};

// (tests) SigV4 of a request: returns the Authorization header value for
// the given method, host, canonical path (already URI-encoded), sorted
// canonical query, x-amz-date, payload SHA-256 hex, region and credentials.
std::string SigV4Authorization(const std::string& method, const std::string& host,
                               const std::string& path, const std::string& query,
                               const std::string& amz_date, const std::string& payload_sha256,
                               const std::string& region, const std::string& key_id,
                               const std::string& secret, const std::string& token);

}  // namespace host
}  // namespace wh
