#pragma once
#include <vector>

#include "common.h"

namespace wh {
namespace host {

struct LocalizeResult {
  std::vector<uint64_t> uniq;
  std::vector<int32_t> ucnt;
  std::vector<int64_t> owner_cnt;
  std::vector<int32_t> lid;
  std::vector<int64_t> csc_off;
  std::vector<int32_t> csc_row;
  std::vector<float> csc_val;
};

void LocalizeCPU(const uint64_t* keys, size_t nnz, const int64_t* offset, size_t nrows,
                 const float* val, int nshard, int nthreads, LocalizeResult* r);

}  // namespace host
}  // namespace wh
