#include "convert_lib.h"

#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>

#include "host/io.h"
#include "host/parsers.h"

namespace wh {
namespace host {
namespace {

// text chunks of whole lines from a file (InputSplit 0/1) or from stdin
class ChunkSource {
 public:
  ChunkSource(const std::string& in, bool recordio) : recordio_(recordio) {
    if (in == "stdin") {
      WH_CHECK(!recordio, "crb input from stdin is not supported");
      fp_ = stdin;
    } else {
      split_.reset(new InputSplit(in, 0, 1, recordio));
    }
  }
  bool Next(std::string* out) {
    if (split_) return recordio_ ? split_->NextRecord(out) : split_->NextChunk(out, 4 << 20);
    if (eof_ && carry_.empty()) return false;
    std::string buf = carry_;
    carry_.clear();
    char tmp[1 << 16];
    while (!eof_ && buf.size() < (4u << 20)) {
      size_t n = std::fread(tmp, 1, sizeof(tmp), fp_);
      if (n == 0) { eof_ = true; break; }
      buf.append(tmp, n);
    }
    if (!eof_) {
      size_t cut = buf.rfind('\n');
      if (cut == std::string::npos) cut = buf.size() - 1;
      carry_ = buf.substr(cut + 1);
      buf.resize(cut + 1);
    }
    *out = std::move(buf);
    return !out->empty() || !eof_;
  }

 private:
  bool recordio_;
  std::unique_ptr<InputSplit> split_;
  std::FILE* fp_ = nullptr;
  bool eof_ = false;
  std::string carry_;
};

void ParseChunk(const std::string& fmt, const std::string& chunk, RowBlock* blk) {
  blk->clear();
  const char* p = chunk.data();
  const char* e = p + chunk.size();
  if (fmt == "libsvm") ParseLibSVM(p, e, blk);
  else if (fmt == "criteo") ParseCriteo(p, e, true, blk);
  else if (fmt == "criteo_test") ParseCriteo(p, e, false, blk);
  else if (fmt == "adfea") ParseAdfea(p, e, blk);
  else if (fmt == "crb") CRBDecode(chunk.data(), chunk.size(), blk);
  else throw std::runtime_error("unknown format " + fmt);
}

// libsvm text exactly as the reference's ostream writer lays it out
void WriteLibSVM(const RowBlock& b, std::string* s) {
  char num[64];
  for (size_t i = 0; i < b.size(); ++i) {
    std::snprintf(num, sizeof(num), "%g ", b.label[i]);
    s->append(num);
    for (int64_t j = b.offset[i]; j < b.offset[i + 1]; ++j) {
      if (b.value.empty())
        std::snprintf(num, sizeof(num), "%llu ", (unsigned long long)b.index[j]);
      else
        std::snprintf(num, sizeof(num), "%llu:%g ", (unsigned long long)b.index[j], b.value[j]);
      s->append(num);
    }
    s->push_back('\n');
  }
}

}  // namespace

ConvertStats Convert(const std::string& in, const std::string& out, const std::string& fmt_in,
                     const std::string& fmt_out, int64_t part_size_bytes) {
  WH_CHECK(fmt_out == "libsvm" || fmt_out == "crb", "unknown output format: " + fmt_out);
  ConvertStats st;
  ChunkSource src(in, fmt_in == "crb");
  const size_t part = part_size_bytes < 0 ? (size_t)-1 : (size_t)part_size_bytes;
  size_t nwrite = (size_t)-1;
  std::FILE* fp = nullptr;
  std::unique_ptr<RecordIOWriter> crb;
  const std::string target = out == "stdout" ? std::string("/dev/stdout") : out;
  std::string chunk, buf;
  RowBlock blk;
  while (src.Next(&chunk)) {
    ParseChunk(fmt_in, chunk, &blk);
    if (blk.size() == 0) continue;
    if (nwrite >= part) {  // open the first / next output part
      std::string name = target;
      if (part != (size_t)-1) {
        char suf[32];
        std::snprintf(suf, sizeof(suf), "-part_%02d", (int)st.parts);
        name += suf;
      }
      ++st.parts;
      crb.reset();
      if (fp) std::fclose(fp);
      fp = nullptr;
      if (fmt_out == "crb") {
        crb.reset(new RecordIOWriter(name));
      } else {
        fp = std::fopen(ResolvePath(name).c_str(), "wb");
        WH_CHECK(fp != nullptr, "cannot open " + name);
      }
      nwrite = 0;
    }
    if (fmt_out == "crb") {
      const std::string rec = CRBEncode(blk);
      crb->WriteRecord(rec);
      nwrite += rec.size();
    } else {
      buf.clear();
      WriteLibSVM(blk, &buf);
      WH_CHECK(std::fwrite(buf.data(), 1, buf.size(), fp) == buf.size(), "write failed");
      nwrite += buf.size();
    }
    st.rows += (int64_t)blk.size();
    st.nnz += (int64_t)blk.nnz();
  }
  crb.reset();
  if (fp) std::fclose(fp);
  return st;
}

}  // namespace host
}  // namespace wh
