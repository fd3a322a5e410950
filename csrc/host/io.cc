// File-system and split I/O (replaces the dmlc-core Stream / InputSplit /
// FileSystem / RecordIO pieces wormhole uses; SURVEY §2.2 "dmlc-core I/O").
//   * ListDirectory + MatchFile: reference learn/base/match_file.h:12-45
//     (POSIX extended regex ".*<file part>", unanchored search)
//   * InputSplit: part k of n of a file as a byte range snapped to record
//     boundaries (text lines or RecordIO records)
//   * RecordIO: dmlc-compatible framing (magic 0xced7230a, 29-bit length,
//     3-bit continuation flag, 4-byte alignment)
#include "io.h"

#include "remote_fs.h"

#include <dirent.h>
#include <regex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>

namespace wh {
namespace host {

// Local paths / file:// directly; any other scheme through the local mount
// named by WH_FS_MOUNT_<SCHEME> (hdfs/viewfs drop the name-node authority,
// object stores keep their bucket). Mirrors wormhole_amd/utils/fs.py.
std::string ResolvePath(const std::string& p) {
  const size_t sep = p.find("://");
  if (sep == std::string::npos) return p;
  std::string scheme = p.substr(0, sep);
  std::string rest = p.substr(sep + 3);
  for (auto& c : scheme) c = (char)std::tolower((unsigned char)c);
  if (scheme == "file") return rest;
  std::string var = "WH_FS_MOUNT_";
  for (char c : scheme) var += (char)std::toupper((unsigned char)c);
  const char* root = std::getenv(var.c_str());
  if (!root || !*root)
    throw std::runtime_error("no filesystem for '" + scheme + "://' (" + p + "): set " + var +
                             " to a local mount of it");
  if (scheme == "hdfs" || scheme == "viewfs") {
    const size_t slash = rest.find('/');
    rest = slash == std::string::npos ? "" : rest.substr(slash + 1);
  }
  std::string out = root;
  if (!out.empty() && out.back() != '/') out += "/";
  return out + rest;
}

namespace {
std::string strip_scheme(const std::string& p) { return ResolvePath(p); }
}  // namespace

std::vector<std::string> ListDirectory(const std::string& dir_in) {
  if (IsRemote(dir_in)) {  // WebHDFS / S3 (csrc/host/remote_fs.cc)
    std::vector<std::string> out;
    for (const auto& e : RemoteList(dir_in)) out.push_back(e.uri);
    return out;
  }
  const std::string dir = strip_scheme(dir_in);
  std::vector<std::string> out;
  struct stat st;
  if (stat(dir.c_str(), &st) != 0) return out;
  if (!S_ISDIR(st.st_mode)) {
    out.push_back(dir);
    return out;
  }
  DIR* d = opendir(dir.c_str());
  if (!d) return out;
  while (struct dirent* e = readdir(d)) {
    std::string name = e->d_name;
    if (name == "." || name == "..") continue;
    std::string full = dir;
    if (!full.empty() && full.back() != '/') full += "/";
    full += name;
    struct stat fs;
    if (stat(full.c_str(), &fs) == 0 && S_ISREG(fs.st_mode)) out.push_back(full);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<std::string> MatchFile(const std::string& pattern_in) {
  const std::string pattern = IsRemote(pattern_in) ? pattern_in : strip_scheme(pattern_in);
  // directory = up to the last '/' (not '\\': a backslash escapes the regex,
  // e.g. "part-[0-9]\\.txt")
  const size_t pos = pattern.find_last_of('/');
  std::string path = "./";
  if (pos != std::string::npos) path = pattern.substr(0, pos);
  std::string file = pos == std::string::npos ? pattern : pattern.substr(pos + 1);
  file = ".*" + file;
  regex_t re;
  int status = regcomp(&re, file.c_str(), REG_EXTENDED | REG_NEWLINE);
  if (status != 0) {
    char msg[512];
    regerror(status, &re, msg, sizeof(msg));
    throw std::runtime_error("error regex '" + pattern + "': " + msg);
  }
  std::vector<std::string> out;
  for (const auto& f : ListDirectory(path)) {
    std::string name = f;
    if (pos == std::string::npos && name.rfind("./", 0) == 0) name = name.substr(2);
    regmatch_t m[1];
    if (regexec(&re, name.c_str(), 1, m, 0) == 0) out.push_back(name);
  }
  regfree(&re);
  return out;
}

int64_t FileSize(const std::string& path) {
  if (IsRemote(path)) return RemoteSize(path);
  struct stat st;
  if (stat(strip_scheme(path).c_str(), &st) != 0) return -1;
  return (int64_t)st.st_size;
}

// ------------------------------------------------------------------ split
InputSplit::InputSplit(const std::string& path, int part, int nparts, bool recordio)
    : path_(IsRemote(path) ? path : strip_scheme(path)), recordio_(recordio) {
  if (IsRemote(path_)) {
    remote_ = std::make_unique<RemoteReader>(path_);
  } else {
    fp_ = std::fopen(path_.c_str(), "rb");
    if (!fp_) throw std::runtime_error("cannot open " + path_);
  }
  const int64_t size = remote_ ? remote_->size() : FileSize(path_);
  WH_CHECK(nparts >= 1 && part >= 0 && part < nparts, "bad part index");
  const int64_t nstep = (size + nparts - 1) / nparts;
  int64_t b = std::min<int64_t>(size, nstep * part);
  int64_t e = std::min<int64_t>(size, nstep * (part + 1));
  begin_ = Align(b, size);
  end_ = Align(e, size);
  if (recordio_ && end_ > begin_ && remote_) {
    // a remote CRB part is fetched whole (one ranged read) and decoded from
    // memory like a mapping
    own_ = RemoteRead(path_, begin_, end_ - begin_);
    WH_CHECK((int64_t)own_.size() == end_ - begin_, "short read of " + path_);
    map_off_ = begin_;
    map_len_ = own_.size();
    map_ = own_.data();
  } else if (recordio_ && end_ > begin_) {
    // CRB parts are read through a mapping: a record is decoded straight
    // from the page cache by whichever reader thread takes it (a stdio read
    // per record under the readers' lock copied every byte once more, on
    // one thread: ~20 M Criteo rows/s, below the text path)
    const int64_t pg = (int64_t)sysconf(_SC_PAGESIZE);
    map_off_ = begin_ / pg * pg;
    map_len_ = (size_t)(end_ - map_off_);
    void* m = mmap(nullptr, map_len_, PROT_READ, MAP_SHARED, fileno(fp_), map_off_);
    if (m != MAP_FAILED) {
      map_ = static_cast<const char*>(m);
      madvise(m, map_len_, MADV_SEQUENTIAL);
      madvise(m, map_len_, MADV_WILLNEED);
    }
  }
  BeforeFirst();
}

InputSplit::~InputSplit() {
  if (map_ && own_.empty()) munmap(const_cast<char*>(map_), map_len_);
  if (fp_) std::fclose(fp_);
}

int64_t InputSplit::Align(int64_t pos, int64_t size) {
  if (pos <= 0) return 0;
  if (pos >= size) return size;
  if (!recordio_) {
    // a line belongs to the part holding its first byte
    src_seek(pos - 1);
    int c;
    int64_t p = pos - 1;
    while ((c = src_getc()) != EOF) {
      ++p;
      if (c == '\n' || c == '\r') {
        // swallow a "\r\n" pair
        int c2 = src_getc();
        if (c2 != EOF && (c2 == '\n' || c2 == '\r') && c2 != c) ++p;
        return p;
      }
    }
    return size;
  }
  // recordio: first 4-aligned magic whose cflag is 0 (full) or 1 (start),
  // scanned in 1 MB blocks (a record can be megabytes long; one fseek+fread
  // per 4-byte step made every part boundary cost ~0.3 s)
  int64_t p = (pos + 3) & ~int64_t(3);
  constexpr int64_t kBlock = 1 << 20;
  std::vector<uint32_t> w(kBlock / 4 + 2);
  while (p + 8 <= size) {
    src_seek(p);
    const int64_t want = std::min<int64_t>(kBlock + 8, size - p) / 4;
    const size_t got = src_read(w.data(), 4 * (size_t)want) / 4;
    if (got < 2) break;
    for (size_t i = 0; i + 1 < got; ++i) {
      if (w[i] == kRecordIOMagic) {
        const uint32_t cflag = w[i + 1] >> 29;
        if (cflag == 0 || cflag == 1) return p + 4 * (int64_t)i;
      }
    }
    p += 4 * (int64_t)(got - 1);  // the last word may start a header
  }
  return size;
}

void InputSplit::src_seek(int64_t off) {
  if (remote_) remote_->Seek(off);
  else std::fseek(fp_, off, SEEK_SET);
}
int InputSplit::src_getc() { return remote_ ? remote_->GetC() : std::fgetc(fp_); }
size_t InputSplit::src_read(void* buf, size_t n) {
  return remote_ ? remote_->Read(static_cast<char*>(buf), n) : std::fread(buf, 1, n, fp_);
}

void InputSplit::BeforeFirst() {
  src_seek(begin_);
  pos_ = begin_;
  carry_.clear();
}

bool InputSplit::NextChunk(std::string* out, size_t hint) {
  out->clear();
  if (recordio_) throw std::runtime_error("NextChunk on a recordio split");
  if (pos_ >= end_ && carry_.empty()) return false;
  const int64_t want = std::min<int64_t>((int64_t)hint, end_ - pos_);
  std::string buf = carry_;
  carry_.clear();
  if (want > 0) {
    const size_t old = buf.size();
    buf.resize(old + want);
    const size_t got = src_read(&buf[old], want);
    buf.resize(old + got);
    pos_ += got;
  }
  if (pos_ < end_) {
    // keep the trailing partial line for the next chunk
    size_t cut = buf.find_last_of("\n\r");
    if (cut == std::string::npos) {
      carry_ = buf;
      return NextChunk(out, hint * 2);
    }
    carry_ = buf.substr(cut + 1);
    buf.resize(cut + 1);
  }
  out->swap(buf);
  return !out->empty() || pos_ < end_;
}

bool InputSplit::NextRecordView(const char** data, size_t* size, std::string* spill) {
  if (!recordio_) throw std::runtime_error("NextRecordView on a text split");
  if (!map_) {
    if (!NextRecord(spill)) return false;
    *data = spill->data();
    *size = spill->size();
    return true;
  }
  spill->clear();
  bool joined = false;
  while (true) {
    if (pos_ >= end_ || pos_ + 8 > end_) return false;
    const char* h = map_ + (pos_ - map_off_);
    uint32_t hdr[2];
    std::memcpy(hdr, h, 8);
    WH_CHECK(hdr[0] == kRecordIOMagic, "invalid recordio stream in " + path_);
    const uint32_t cflag = hdr[1] >> 29, len = hdr[1] & ((1u << 29) - 1);
    const uint32_t padded = (len + 3u) & ~3u;
    if (pos_ + 8 + (int64_t)padded > end_)
      throw std::runtime_error("truncated recordio record in " + path_);
    const char* body = h + 8;
    pos_ += 8 + padded;
    if (cflag == 0) {
      *data = body;
      *size = len;
      return true;
    }
    if (cflag == 1) {
      spill->assign(body, len);
      joined = true;
      continue;
    }
    // 2 = middle, 3 = end: the writer split at an embedded magic word
    WH_CHECK(joined, "recordio continuation without a start in " + path_);
    const uint32_t m = kRecordIOMagic;
    spill->append(reinterpret_cast<const char*>(&m), 4);
    spill->append(body, len);
    if (cflag == 3) {
      *data = spill->data();
      *size = spill->size();
      return true;
    }
  }
}

bool InputSplit::NextRecord(std::string* out) {
  out->clear();
  if (!recordio_) throw std::runtime_error("NextRecord on a text split");
  if (map_) {
    std::string spill;
    const char* p;
    size_t n;
    if (!NextRecordView(&p, &n, &spill)) return false;
    if (p == spill.data()) out->swap(spill);
    else out->assign(p, n);
    return true;
  }
  while (true) {
    if (pos_ >= end_) return false;
    uint32_t hdr[2];
    if (src_read(hdr, 8) != 8) return false;
    WH_CHECK(hdr[0] == kRecordIOMagic, "invalid recordio stream in " + path_);
    const uint32_t cflag = hdr[1] >> 29, len = hdr[1] & ((1u << 29) - 1);
    const uint32_t padded = (len + 3u) & ~3u;
    std::string data(padded, '\0');
    if (padded && src_read(&data[0], padded) != padded)
      throw std::runtime_error("truncated recordio record in " + path_);
    pos_ += 8 + padded;
    data.resize(len);
    if (cflag == 0) {
      *out = std::move(data);
      return true;
    }
    if (cflag == 1) {
      *out = std::move(data);
      continue;
    }
    // 2 = middle, 3 = end: the writer split at an embedded magic word
    const uint32_t m = kRecordIOMagic;
    out->append(reinterpret_cast<const char*>(&m), 4);
    out->append(data);
    if (cflag == 3) return true;
  }
}

// --------------------------------------------------------------- recordio
namespace {
// a FILE* whose writes stream into a RemoteWriter (its parts upload as they fill)
ssize_t remote_cookie_write(void* c, const char* buf, size_t n) {
  try {
    static_cast<RemoteWriter*>(c)->Write(buf, n);
    return (ssize_t)n;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "remote write: %s\n", e.what());
    return -1;
  }
}
}  // namespace

RecordIOWriter::RecordIOWriter(const std::string& path_in) {
  if (IsRemote(path_in)) {
    remote_ = std::make_unique<RemoteWriter>(path_in);
    cookie_io_functions_t io{};
    io.write = remote_cookie_write;
    fp_ = fopencookie(remote_.get(), "w", io);
    if (!fp_) throw std::runtime_error("cannot stream to " + path_in);
    return;
  }
  const std::string path = ResolvePath(path_in);
  fp_ = std::fopen(path.c_str(), "wb");
  if (!fp_) throw std::runtime_error("cannot open " + path + " for writing");
}
RecordIOWriter::~RecordIOWriter() {
  try {
    Close();
  } catch (...) {
  }
}
void RecordIOWriter::Close() {
  const bool failed = fp_ && std::fclose(fp_) != 0;
  fp_ = nullptr;
  if (remote_) {
    std::unique_ptr<RemoteWriter> w = std::move(remote_);
    if (failed) throw std::runtime_error("remote RecordIO write failed");
    w->Close();
  }
}

void RecordIOWriter::WriteRecord(const char* buf, size_t size) {
  WH_CHECK(size < (1u << 29), "record too large");
  const uint32_t magic = kRecordIOMagic;
  const size_t lower = (size >> 2) << 2, upper = ((size + 3) >> 2) << 2;
  size_t dptr = 0;
  auto emit = [&](uint32_t cflag, size_t from, size_t len) {
    const uint32_t lrec = (cflag << 29) | (uint32_t)len;
    std::fwrite(&magic, 4, 1, fp_);
    std::fwrite(&lrec, 4, 1, fp_);
    if (len) std::fwrite(buf + from, 1, len, fp_);
    bytes_ += 8 + len;
  };
  for (size_t i = 0; i < lower; i += 4) {
    uint32_t w;
    std::memcpy(&w, buf + i, 4);
    if (w == magic) {
      emit(dptr == 0 ? 1 : 2, dptr, i - dptr);
      dptr = i + 4;
    }
  }
  emit(dptr != 0 ? 3 : 0, dptr, size - dptr);
  const size_t pad = upper - size;
  static const char zeros[4] = {0, 0, 0, 0};
  if (pad) std::fwrite(zeros, 1, pad, fp_);
  bytes_ += pad;
}

}  // namespace host
}  // namespace wh
