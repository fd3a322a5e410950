// Native parameter-server scheduler (reference learn/solver/: the
// MinibatchScheduler epoch loop, minibatch_solver.h:10-195, over the
// IterScheduler load/save fan-out, iter_solver.h:32-71, over the
// DataParScheduler dispatch, data_parallel.h:32-170).
#pragma once
#include <string>
#include <vector>

#include "json.h"
#include "van.h"
#include "workload_pool.h"

namespace wh {
namespace host {

struct SchedulerConf {
  std::string app = "linear";  // linear | difacto (progress layout, stop rule)
  std::string train_data, val_data, data_format = "libsvm";
  std::string model_in, model_out, predict_out;
  int max_data_pass = 10, save_iter = -1, load_iter = -1, num_parts_per_file = 10;
  double print_sec = 1;
  bool local_data = false;
  // restart of a failed job (launcher --max-restart): model_in / load_iter
  // name the newest complete checkpoint and training resumes right after it
  bool resume = false;
  // difacto stop rules (learn/difacto/async_sgd.h:14-55)
  bool early_stop = false;
  double min_objv_decr = 1e-5;
  bool has_max_objv = false;
  double max_objv = 0;
};

class Scheduler {
 public:
  Scheduler(const SchedulerConf& conf, int num_workers, int num_servers, Van* van);
  // the whole job; throws std::runtime_error when a worker dies
  void Run();

 private:
  struct Printer;
  void WaitWorkers(double timeout_s);
  void Broadcast(const std::string& msg);
  bool Recv(double timeout_s, std::string* who, Json* d);
  void OnDead(const std::string& who);
  void Command(const std::string& cmd, const std::string& file, int iter, bool resume = false);
  bool Iterate(int it, int wtype);
  int MatchOnWorkers(const std::string& pattern);
  bool Show(Printer* p, const std::vector<double>& agg, bool train);
  bool StopRule(const std::vector<double>& agg, bool train);

  SchedulerConf c_;
  int nw_, ns_;
  Van* van_;
  std::vector<std::string> workers_;
  std::vector<std::string> dead_;
  WorkloadPool* pool_ = nullptr;
  double start_ = 0, pre_objv_ = 100.0;
};

}  // namespace host
}  // namespace wh
