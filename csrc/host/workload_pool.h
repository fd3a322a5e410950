#pragma once
#include <condition_variable>
#include <list>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace wh {
namespace host {

struct Assignment {
  std::string filename;
  int k = 0, n = 1;
};

class WorkloadPool {
 public:
  WorkloadPool(bool shuffle = false, uint64_t seed = 0, double straggler_factor = 2.0,
               double straggler_min_sec = 5.0, int straggler_min_done = 10,
               double period = 2.0);
  ~WorkloadPool();
  void Add(const std::vector<std::string>& files, int npart, const std::string& node = "");
  void Clear();
  bool Get(const std::string& node, Assignment* out);
  void Finish(const std::string& node) { Set(node, true); }
  // finish ONE workload of node (a worker that prefetches its next workload
  // has two assigned; Finish(node) would mark both)
  void FinishOne(const std::string& node, const std::string& file, int k);
  void Reset(const std::string& node) { Set(node, false); }
  void RemoveStraggler();
  bool IsFinished();
  int num_finished();
  int num_assigned();
  int num_requeued();
  void set_verbose(bool v) { verbose_ = v; }

 private:
  struct Task {
    std::set<std::string> node;
    std::vector<int> track;  // 0 available, 1 assigned, 2 done
    size_t done = 0;
  };
  struct Assigned {
    std::string filename, node;
    int k = 0, n = 1;
    double start = 0;
  };
  void Set(const std::string& node, bool done);
  void Mark(const std::string& f, int k, int mark);
  void RemoveStragglerLocked();
  void Loop();

  bool shuffle_;
  std::mt19937_64 rng_;
  double factor_, min_sec_;
  int min_done_;
  double period_;
  bool verbose_ = false;
  std::map<std::string, Task> task_;
  std::vector<std::string> order_;
  std::list<Assigned> assigned_;
  std::vector<double> time_;
  int num_finished_ = 0, num_requeued_ = 0;
  bool inited_ = false, done_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread killer_;
};

}  // namespace host
}  // namespace wh
