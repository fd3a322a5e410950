// bin/text2crb.dmlc: input output format [part_size MB]  (reference
// learn/tool/text2crb.cc): text -> CRB, optionally split into parts.
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "convert_lib.h"

int main(int argc, char** argv) {
  if (argc < 4) {
    std::printf("Usage: input output format [part_size] \n");
    std::printf(" - input: a input file name or stdin\n");
    std::printf(" - output: a output file name or stdout\n");
    std::printf(" - format: libsvm, criteo, adfea, ... \n");
    std::printf(" - part_size: split the output into multiple parts, with each part <= "
                "part_size MB \n");
    return 0;
  }
  try {
    const long long mb = argc > 4 ? std::atoll(argv[4]) : -1;
    wh::host::Convert(argv[1], argv[2], argv[3], "crb", mb < 0 ? -1 : mb * 1000000LL);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "text2crb: %s\n", e.what());
    return 1;
  }
  return 0;
}
