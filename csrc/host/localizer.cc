// CPU localizer (reference learn/base/localizer.h:96-221 + ParallelSort,
// learn/base/parallel_sort.h:14-41): the GPU-free execution path of
// `localize`. Sorts (owner, key, position) triples with a thread-parallel
// sort + merge, run-length encodes unique keys (grouped by owner shard, so
// local-id order is the key-exchange send order), and emits the per-key
// occurrence lists (CSC) in row order.
#include "localizer.h"

#include <algorithm>
#include <thread>

namespace wh {
namespace host {

namespace {
inline uint64_t mix64b(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

struct Item {
  uint32_t owner;
  uint32_t pos;
  uint64_t key;
};
inline bool item_less(const Item& a, const Item& b) {
  if (a.owner != b.owner) return a.owner < b.owner;
  if (a.key != b.key) return a.key < b.key;
  return a.pos < b.pos;
}

template <typename It, typename Cmp>
void parallel_sort(It begin, It end, int nthreads, Cmp cmp) {
  const size_t n = end - begin;
  const size_t grain = std::max<size_t>(n / std::max(nthreads, 1) + 5, 1 << 14);
  if (nthreads <= 1 || n <= grain) {
    std::sort(begin, end, cmp);
    return;
  }
  It mid = begin + n / 2;
  std::thread t([&] { parallel_sort(begin, mid, nthreads / 2, cmp); });
  parallel_sort(mid, end, nthreads - nthreads / 2, cmp);
  t.join();
  std::inplace_merge(begin, mid, end, cmp);
}
}  // namespace

void LocalizeCPU(const uint64_t* keys, size_t nnz, const int64_t* offset, size_t nrows,
                 const float* val, int nshard, int nthreads, LocalizeResult* r) {
  std::vector<Item> items(nnz);
  for (size_t j = 0; j < nnz; ++j)
    items[j] = Item{nshard <= 1 ? 0u : (uint32_t)(mix64b(keys[j]) % (uint64_t)nshard),
                    (uint32_t)j, keys[j]};
  parallel_sort(items.begin(), items.end(), nthreads, item_less);
  std::vector<int32_t> row_of(nnz);
  for (size_t i = 0; i < nrows; ++i)
    for (int64_t j = offset[i]; j < offset[i + 1]; ++j) row_of[j] = (int32_t)i;
  r->uniq.clear();
  r->ucnt.clear();
  r->owner_cnt.assign(std::max(nshard, 1), 0);
  r->lid.assign(nnz, 0);
  r->csc_row.resize(nnz);
  if (val) r->csc_val.resize(nnz);
  else r->csc_val.clear();
  r->csc_off.assign(1, 0);
  for (size_t j = 0; j < nnz; ++j) {
    const Item& it = items[j];
    if (j == 0 || it.key != items[j - 1].key) {  // owner is a function of key
      r->uniq.push_back(it.key);
      r->ucnt.push_back(0);
      r->owner_cnt[it.owner] += 1;
      if (j > 0) r->csc_off.push_back((int64_t)j);
    }
    r->ucnt.back() += 1;
    r->lid[it.pos] = (int32_t)(r->uniq.size() - 1);
    r->csc_row[j] = row_of[it.pos];
    if (val) r->csc_val[j] = val[it.pos];
  }
  r->csc_off.push_back((int64_t)nnz);
  if (nnz == 0) r->csc_off.assign(1, 0);
}

}  // namespace host
}  // namespace wh
