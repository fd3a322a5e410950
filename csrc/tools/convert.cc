// bin/convert.dmlc: convert data between formats (reference
// learn/tool/convert.cc). Flags (gflags syntax: -name=value, --name value):
//   -data_in     input file or stdin            (default stdin)
//   -data_out    output file or stdout          (default stdout)
//   -format_in   libsvm|criteo|criteo_test|adfea|crb   (default libsvm)
//   -format_out  libsvm|crb                     (default crb)
//   -part_size   split output into parts of <= part_size MB (default -1)
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>

#include "convert_lib.h"

int main(int argc, char** argv) {
  std::map<std::string, std::string> f = {{"data_in", "stdin"},   {"data_out", "stdout"},
                                          {"format_in", "libsvm"}, {"format_out", "crb"},
                                          {"part_size", "-1"}};
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "-help" || a == "--help") {
      std::printf("usage: %s -data_in F -data_out F -format_in FMT -format_out FMT "
                  "[-part_size MB]\n", argv[0]);
      return 0;
    }
    size_t k = a.find_first_not_of('-');
    if (k == 0 || k == std::string::npos) {
      std::fprintf(stderr, "unexpected argument %s\n", a.c_str());
      return 1;
    }
    std::string name = a.substr(k), val;
    size_t eq = name.find('=');
    if (eq != std::string::npos) {
      val = name.substr(eq + 1);
      name = name.substr(0, eq);
    } else if (i + 1 < argc) {
      val = argv[++i];
    }
    if (!f.count(name)) {
      std::fprintf(stderr, "unknown flag -%s\n", name.c_str());
      return 1;
    }
    f[name] = val;
  }
  try {
    const long long mb = std::atoll(f["part_size"].c_str());
    auto st = wh::host::Convert(f["data_in"], f["data_out"], f["format_in"], f["format_out"],
                                mb < 0 ? -1 : mb * 1000000LL);
    std::fprintf(stderr, "converted %lld rows, %lld nnz into %lld file(s)\n", (long long)st.rows,
                 (long long)st.nnz, (long long)st.parts);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "convert: %s\n", e.what());
    return 1;
  }
  return 0;
}
