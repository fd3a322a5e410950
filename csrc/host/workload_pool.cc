// Thread-safe pool of (file, virtual part) tasks with per-node affinity,
// failure reset and a straggler re-queue thread.
// Reference: learn/base/workload_pool.h:17-254. Fixes the
// reference defects listed in SURVEY §2.9 item 1: the shuffle flag is
// initialised and configurable; the straggler knobs are honoured.
#include "workload_pool.h"

#include <algorithm>
#include <chrono>
#include <cstdio>

namespace wh {
namespace host {

static double now_sec() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

WorkloadPool::WorkloadPool(bool shuffle, uint64_t seed, double straggler_factor,
                           double straggler_min_sec, int straggler_min_done, double period)
    : shuffle_(shuffle), rng_(seed), factor_(straggler_factor), min_sec_(straggler_min_sec),
      min_done_(straggler_min_done), period_(period) {
  if (period_ > 0) killer_ = std::thread([this] { Loop(); });
}

WorkloadPool::~WorkloadPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    done_ = true;
  }
  cv_.notify_all();
  if (killer_.joinable()) killer_.join();
}

void WorkloadPool::Loop() {
  std::unique_lock<std::mutex> lk(mu_);
  while (!done_) {
    // (system_clock deadline: libstdc++ implements steady-clock waits with
    // pthread_cond_clockwait, which ThreadSanitizer does not intercept)
    cv_.wait_until(lk, std::chrono::system_clock::now() +
                           std::chrono::duration_cast<std::chrono::system_clock::duration>(
                               std::chrono::duration<double>(period_)));
    if (done_) break;
    RemoveStragglerLocked();
  }
}

void WorkloadPool::Add(const std::vector<std::string>& files, int npart, const std::string& node) {
  std::lock_guard<std::mutex> lk(mu_);
  inited_ = true;
  for (const auto& f : files) {
    auto it = task_.find(f);
    if (it == task_.end()) {
      order_.push_back(f);
      it = task_.emplace(f, Task()).first;
    }
    Task& t = it->second;
    if (t.track.empty()) t.track.assign(npart, 0);
    if (!node.empty()) t.node.insert(node);
  }
}

void WorkloadPool::Clear() {
  std::lock_guard<std::mutex> lk(mu_);
  task_.clear();
  order_.clear();
  assigned_.clear();
  inited_ = false;
  time_.clear();
  num_finished_ = 0;
}

bool WorkloadPool::Get(const std::string& node, Assignment* out) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::pair<std::string, int>> avail;
  for (const auto& f : order_) {
    auto it = task_.find(f);
    if (it == task_.end()) continue;
    const Task& t = it->second;
    if (!t.node.empty() && !t.node.count(node)) continue;
    for (size_t k = 0; k < t.track.size(); ++k)
      if (t.track[k] == 0) {
        avail.emplace_back(f, (int)k);
        if (!shuffle_) break;
      }
    if (!shuffle_ && !avail.empty()) break;
  }
  if (avail.empty()) return false;
  size_t pick = 0;
  if (shuffle_) pick = std::uniform_int_distribution<size_t>(0, avail.size() - 1)(rng_);
  Task& t = task_[avail[pick].first];
  Assigned a;
  a.filename = avail[pick].first;
  a.k = avail[pick].second;
  a.n = (int)t.track.size();
  a.node = node;
  a.start = now_sec();
  t.track[a.k] = 1;
  assigned_.push_back(a);
  out->filename = a.filename;
  out->k = a.k;
  out->n = a.n;
  if (verbose_)
    std::fprintf(stderr, "[pool] assign %s job %s %d / %d. %zu #jobs on processing.\n",
                 node.c_str(), a.filename.c_str(), a.k, a.n, assigned_.size());
  return true;
}

void WorkloadPool::Set(const std::string& node, bool done) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto it = assigned_.begin(); it != assigned_.end();) {
    if (it->node != node) {
      ++it;
      continue;
    }
    if (done) {
      time_.push_back(now_sec() - it->start);
      Mark(it->filename, it->k, 2);
    } else {
      Mark(it->filename, it->k, 0);
      if (verbose_)
        std::fprintf(stderr, "[pool] %s failed to finish %s %d / %d\n", node.c_str(),
                     it->filename.c_str(), it->k, it->n);
    }
    it = assigned_.erase(it);
  }
}

void WorkloadPool::FinishOne(const std::string& node, const std::string& file, int k) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto it = assigned_.begin(); it != assigned_.end(); ++it) {
    if (it->node == node && it->filename == file && it->k == k) {
      time_.push_back(now_sec() - it->start);
      Mark(it->filename, it->k, 2);
      assigned_.erase(it);
      return;
    }
  }
}

void WorkloadPool::Mark(const std::string& f, int k, int mark) {
  auto it = task_.find(f);
  if (it == task_.end()) return;
  Task& t = it->second;
  if (k < 0 || k >= (int)t.track.size()) return;
  if (mark == 2 && t.track[k] != 2) {
    ++num_finished_;
    ++t.done;
  }
  t.track[k] = mark;
  if (t.done == t.track.size()) task_.erase(it);
}

void WorkloadPool::RemoveStragglerLocked() {
  if ((int)time_.size() < min_done_) return;
  double mean = 0;
  for (double x : time_) mean += x;
  mean /= time_.size();
  const double cur = now_sec();
  for (auto it = assigned_.begin(); it != assigned_.end();) {
    const double t = cur - it->start;
    if (t > std::max(mean * factor_, min_sec_)) {
      if (verbose_)
        std::fprintf(stderr,
                     "[pool] %s is processing %s %d / %d for %.1f sec (mean %.1f): reassign\n",
                     it->node.c_str(), it->filename.c_str(), it->k, it->n, t, mean);
      Mark(it->filename, it->k, 0);
      ++num_requeued_;
      it = assigned_.erase(it);
    } else {
      ++it;
    }
  }
}

void WorkloadPool::RemoveStraggler() {
  std::lock_guard<std::mutex> lk(mu_);
  RemoveStragglerLocked();
}

bool WorkloadPool::IsFinished() {
  std::lock_guard<std::mutex> lk(mu_);
  return inited_ && task_.empty() && assigned_.empty();
}
int WorkloadPool::num_finished() {
  std::lock_guard<std::mutex> lk(mu_);
  return num_finished_;
}
int WorkloadPool::num_assigned() {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)assigned_.size();
}
int WorkloadPool::num_requeued() {
  std::lock_guard<std::mutex> lk(mu_);
  return num_requeued_;
}

}  // namespace host
}  // namespace wh
