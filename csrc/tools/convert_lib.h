// Shared core of the data conversion tools (reference learn/tool/convert.cc,
// learn/tool/text2crb.cc): parse {libsvm, criteo, criteo_test, adfea, crb}
// with the native parsers and write libsvm text or CRB (RecordIO of
// LZ4-compressed row blocks), optionally rotating the output into
// "<out>-part_%02d" files of at most part_size bytes.
#pragma once
#include <cstdint>
#include <string>

namespace wh {
namespace host {

struct ConvertStats {
  int64_t rows = 0, nnz = 0, parts = 0;
};

// part_size_bytes < 0: one output file named `out`. in == "stdin" reads
// standard input; out == "stdout" writes standard output.
ConvertStats Convert(const std::string& in, const std::string& out, const std::string& fmt_in,
                     const std::string& fmt_out, int64_t part_size_bytes);

}  // namespace host
}  // namespace wh
