// Native parameter-server scheduler. Semantics follow the reference solver
// stack:
//   * epoch loop: [load model_in + predict pass] -> per data pass: train,
//     validate, save every save_iter passes -> final save
//     (minibatch_solver.h:85-136);
//   * each pass matches the data files (or has the workers match their own
//     with local_data), splits every file into num_parts_per_file virtual
//     parts in a WorkloadPool and hands them out one request at a time; a
//     worker's response marks its part done (data_parallel.h:93-158);
//   * progress vectors from the workers are sum-merged and printed every
//     print_sec in the reference table layout (linear/difacto progress.h);
//   * a dead worker's connection re-queues its parts and fails the job; the
//     launcher restarts it (--max-restart) and the restarted scheduler
//     resumes from the newest checkpoint whose save completed on every
//     shard (each worker seals its shard file with a `.ok` marker once it
//     and its optimizer-state side file are written; SURVEY §5.3, reference
//     data_parallel.h:131-135 + minibatch_solver.h:96-109);
//   * DiFacto stop rules: training objective above max_objv, or a validation
//     decrease below min_objv_decr with early_stop (difacto/async_sgd.h:14-55).
// Messages are JSON objects over the Van (csrc/host/van.cc).
#include "scheduler.h"

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>

#include "io.h"
#include "json.h"

namespace wh {
namespace host {

namespace {

double now_sec() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

enum { kTrain = 0, kVal = 1, kPred = 2 };

void out(const std::string& s) {
  std::fputs(s.c_str(), stdout);
  std::fputc('\n', stdout);
  std::fflush(stdout);
}

void err(const std::string& s) {
  std::fputs(s.c_str(), stderr);
  std::fputc('\n', stderr);
  std::fflush(stderr);
}

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, f);
  std::vsnprintf(buf, sizeof(buf), f, ap);
  va_end(ap);
  return buf;
}

void merge(std::vector<double>* agg, const std::vector<double>& d) {
  if (agg->empty()) {
    *agg = d;
    return;
  }
  for (size_t i = 0; i < agg->size() && i < d.size(); ++i) (*agg)[i] += d[i];
}

}  // namespace

// Progress tables (learn/linear/progress.h:8-36, learn/difacto/progress.h:8-42)
struct Scheduler::Printer {
  bool difacto;
  double ttl_ex = 0, nnz_w = 0, nnz_v = 0;
  explicit Printer(bool d) : difacto(d) {}
  std::string head() const {
    return difacto ? "  ttl #ex   inc #ex |  |w|_0  logloss_w |   |V|_0    logloss    AUC"
                   : "  ttl #ex   inc #ex    |w|_0       logloss  accuracy     AUC";
  }
  std::string line(const std::vector<double>& d) {
    if (!difacto) {  // objv, acc, auc, count, new_ex, new_w
      if (d.size() < 6) return "";
      ttl_ex += d[4];
      nnz_w += d[5];
      if (d[4] == 0) return "";
      return fmt("%8.3g  %8.3g  %11.6g  %8.6f  %8.6f  %8.6f", ttl_ex, d[4], nnz_w, d[0] / d[4],
                 d[1] / d[3], d[2] / d[3]);
    }
    // objv, auc, objv_w, copc, count, new_ex, new_w, new_V
    if (d.size() < 8) return "";
    ttl_ex += d[5];
    nnz_w += d[6];
    nnz_v += d[7];
    if (d[5] == 0) return "";
    return fmt("%9.4g  %7.2g | %9.4g  %6.4f | %9.4g  %7.5f  %7.5f ", ttl_ex, d[5], nnz_w,
               d[2] / d[5], nnz_v, d[0] / d[5], d[1] / d[4]);
  }
};

Scheduler::Scheduler(const SchedulerConf& conf, int num_workers, int num_servers, Van* van)
    : c_(conf), nw_(num_workers), ns_(num_servers), van_(van) {}

bool Scheduler::Recv(double timeout_s, std::string* who, Json* d) {
  std::string raw;
  if (!van_->Recv(timeout_s, who, &raw)) return false;
  if (raw == "__closed__") {
    *d = Json::Obj().set("msg", Json::Str("__closed__"));
    return true;
  }
  *d = Json::Parse(raw);
  return true;
}

void Scheduler::Broadcast(const std::string& msg) {
  for (const auto& w : workers_) van_->Send(w, msg);
}

void Scheduler::WaitWorkers(double timeout_s) {
  const double t0 = now_sec();
  while ((int)workers_.size() < nw_) {
    std::string who;
    Json d;
    if (!Recv(1.0, &who, &d)) {
      if (now_sec() - t0 > timeout_s)
        throw std::runtime_error(fmt("only %d of %d workers connected", (int)workers_.size(),
                                     nw_));
      continue;
    }
    if (d["msg"].kind() == Json::kStr && d["msg"].str() == "ready") workers_.push_back(who);
  }
  // "worker-<rank>": order by rank
  std::sort(workers_.begin(), workers_.end(), [](const std::string& a, const std::string& b) {
    return std::atoi(a.c_str() + a.find('-') + 1) < std::atoi(b.c_str() + b.find('-') + 1);
  });
}

void Scheduler::OnDead(const std::string& who) {
  if (std::find(dead_.begin(), dead_.end(), who) != dead_.end()) return;
  dead_.push_back(who);
  err("[scheduler] node " + who + " died");
  if (pool_) pool_->Reset(who);  // re-queue its workload (data_parallel.h:131-135)
  throw std::runtime_error("worker " + who +
                           " failed; its workload was re-queued, restart from the last saved "
                           "model (model_in / load_iter)");
}

void Scheduler::Command(const std::string& cmd, const std::string& file, int iter,
                        bool resume) {
  Broadcast(Json::Obj()
                .set("cmd", Json::Str(cmd))
                .set("file", Json::Str(file))
                .set("iter", Json::Num(iter))
                .set("resume", Json::Bool(resume))
                .Dump());
  int acks = 0;
  while (acks < (int)workers_.size()) {
    std::string who;
    Json d;
    if (!Recv(1.0, &who, &d)) continue;
    const std::string m = d["msg"].kind() == Json::kStr ? d["msg"].str() : "";
    if (m == "__closed__") OnDead(who);
    if (m == "ack") ++acks;
  }
}

int Scheduler::MatchOnWorkers(const std::string& pattern) {
  Broadcast(Json::Obj().set("cmd", Json::Str("match")).set("data", Json::Str(pattern)).Dump());
  int got = 0, nfiles = 0;
  while (got < (int)workers_.size()) {
    std::string who;
    Json d;
    if (!Recv(1.0, &who, &d)) continue;
    const std::string m = d["msg"].kind() == Json::kStr ? d["msg"].str() : "";
    if (m == "__closed__") OnDead(who);
    if (m == "matched") {
      ++got;
      const auto files = d["files"].strs();
      if (!files.empty()) {
        nfiles += (int)files.size();
        pool_->Add(files, c_.num_parts_per_file, who);
      }
    }
  }
  return nfiles;
}

bool Scheduler::StopRule(const std::vector<double>& agg, bool train) {
  if (c_.app != "difacto" || agg.size() < 6) return false;
  const double cur = agg[5] ? agg[0] / agg[5] : 0.0;
  if (train) return c_.has_max_objv && cur > c_.max_objv;
  const double diff = pre_objv_ - cur;
  pre_objv_ = cur;
  if (c_.early_stop && diff < c_.min_objv_decr) {
    out(fmt("The decrease of validation objective is smaller than the minimal requirement: "
            "%g vs %g", diff, c_.min_objv_decr));
    return true;
  }
  return false;
}

bool Scheduler::Show(Printer* p, const std::vector<double>& agg, bool train) {
  const std::string line = p->line(agg);
  if (line.empty()) return false;
  out(fmt("%5.0f  ", now_sec() - start_) + line);
  return StopRule(agg, train);
}

bool Scheduler::Iterate(int it, int wtype) {
  const bool train = wtype == kTrain;
  std::string data;
  if (train) {
    data = c_.train_data;
    out(fmt("Training: iter = %d", it));
  } else {
    data = c_.val_data;
    if (wtype == kPred) {
      out("Predicting");
    } else {
      out(fmt("Validating: iter = %d", it));
      if (data.empty()) return false;
    }
  }
  // straggler knobs (defaults = the reference's: 2x the mean part time, at
  // least 5 s, after 10 finished parts) can be tuned per job from the env
  auto envd = [](const char* k, double d) {
    const char* v = std::getenv(k);
    return v && *v ? std::atof(v) : d;
  };
  std::unique_ptr<WorkloadPool> pool(new WorkloadPool(
      train, (uint64_t)it + 1, envd("WH_STRAGGLER_FACTOR", 2.0), envd("WH_STRAGGLER_MIN_SEC", 5.0),
      (int)envd("WH_STRAGGLER_MIN_DONE", 10)));
  pool->set_verbose(envd("WH_POOL_VERBOSE", 0) != 0);
  pool_ = pool.get();
  if (c_.local_data) {
    // every worker matches the pattern on its own file system and its parts
    // are preferably handed to it (data_parallel.h:96-101 + node affinity)
    if (MatchOnWorkers(data) == 0)
      throw std::runtime_error("no worker has a file matching '" + data + "'");
  } else {
    const auto files = MatchFile(data);
    if (files.empty()) throw std::runtime_error("no file matches '" + data + "'");
    if (c_.num_parts_per_file * (int)files.size() < nw_)
      err(fmt("[scheduler] #parts (%d) < #workers (%d): some workers idle; increase "
              "num_parts_per_file", c_.num_parts_per_file * (int)files.size(), nw_));
    pool->Add(files, c_.num_parts_per_file);
  }
  Printer printer(c_.app == "difacto");
  out("  sec " + printer.head());
  Broadcast(Json::Obj()
                .set("cmd", Json::Str("iterate"))
                .set("type", Json::Num(wtype))
                .set("data_pass", Json::Num(it))
                .set("fmt", Json::Str(c_.data_format))
                .Dump());
  int done = 0;
  std::vector<double> agg;
  bool stop = false;
  double last = now_sec();
  const std::string none = Json::Obj().set("cmd", Json::Str("workload"))
                               .set("file", Json::Null()).Dump();
  while (done < (int)workers_.size()) {
    std::string who;
    Json d;
    if (Recv(0.05, &who, &d)) {
      const std::string m = d["msg"].kind() == Json::kStr ? d["msg"].str() : "";
      if (m == "__closed__") {
        OnDead(who);
      } else if (m == "finished") {
        const Json& f = d["finished"];
        pool->FinishOne(who, f["file"].str(), (int)f["k"].num());
      } else if (m == "request") {
        const Json& f = d["finished"];
        if (f.kind() == Json::kObj) {  // one specific workload (prefetching worker)
          pool->FinishOne(who, f["file"].str(), (int)f["k"].num());
        } else if (f.truthy()) {
          pool->Finish(who);
        }
        Assignment a;
        if (stop || !pool->Get(who, &a)) {
          van_->Send(who, none);
        } else {
          van_->Send(who, Json::Obj()
                              .set("cmd", Json::Str("workload"))
                              .set("file", Json::Str(a.filename))
                              .set("k", Json::Num(a.k))
                              .set("n", Json::Num(a.n))
                              .Dump());
        }
      } else if (m == "progress") {
        merge(&agg, d["data"].nums());
      } else if (m == "pass_done") {
        ++done;
        if (d["progress"].kind() == Json::kArr) merge(&agg, d["progress"].nums());
      }
    }
    if (train && now_sec() - last >= c_.print_sec) {
      last = now_sec();
      if (!agg.empty()) {
        const bool s = Show(&printer, agg, true);
        agg.clear();
        if (s && !stop) {
          stop = true;
          pool->Clear();  // reference StopDispatch
        }
      }
    }
  }
  if (!agg.empty()) stop = Show(&printer, agg, train) || stop;
  pool_ = nullptr;
  return stop;
}

void Scheduler::Run() {
  WaitWorkers(600);
  out(fmt("Connected %d servers and %d workers", ns_, nw_));
  start_ = now_sec();
  const bool is_pred = !c_.predict_out.empty();
  if (is_pred && c_.model_in.empty())
    throw std::runtime_error("should provide model_in for predicting");
  int cur = 0;
  if (c_.resume && !c_.model_in.empty()) {
    out(fmt("Resuming from the model saved at iter = %d", c_.load_iter));
    Command("load", c_.model_in, c_.load_iter, true);
    cur = c_.load_iter + 1;
  } else if (!c_.model_in.empty()) {
    if (c_.load_iter > 0) {
      out(fmt("Loading model from iter = %d", c_.load_iter));
      cur = c_.load_iter;
    } else {
      out("Loading the last model");
      cur = -1;
    }
    Command("load", c_.model_in, cur);
    Iterate(cur, kPred);
    ++cur;
  }
  auto shutdown = [&] { Broadcast(Json::Obj().set("cmd", Json::Str("exit")).Dump()); };
  if (is_pred) {
    out("Prediction is finished!");
    shutdown();
    return;
  }
  while (cur < c_.max_data_pass) {
    if (Iterate(cur, kTrain) || Iterate(cur, kVal)) {
      out("Hit stop critera");
      break;
    }
    if (cur == c_.max_data_pass - 1) {
      out(fmt("Hit max number of data passes %d", c_.max_data_pass));
      break;
    }
    if (!c_.model_out.empty() && c_.save_iter > 0 && (cur + 1) % c_.save_iter == 0) {
      out(fmt("Saving model for iter = %d", cur));
      Command("save", c_.model_out, cur);
    }
    ++cur;
  }
  if (!c_.model_out.empty()) {
    out("Saving the final model");
    Command("save", c_.model_out, -1);
  }
  out("Training is finished!");
  shutdown();
}

}  // namespace host
}  // namespace wh
