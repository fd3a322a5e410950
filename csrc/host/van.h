#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace wh {
namespace host {

class Van {
 public:
  Van() = default;
  ~Van();
  int Listen(int port);  // scheduler side; returns the bound port
  void Connect(const std::string& host, int port, const std::string& my_id, double timeout_s);
  bool Send(const std::string& to, const std::string& msg);
  bool Recv(double timeout_s, std::string* from, std::string* msg);
  std::vector<std::string> Peers();
  void Close();
  int port() const { return port_; }

 private:
  void AcceptLoop(int lfd);
  void ReadLoop(int fd, std::string id);
  void Push(const std::string& from, const std::string& msg);

  int lfd_ = -1, port_ = 0;
  std::atomic<bool> closing_{false};
  std::mutex mu_, send_mu_;
  std::condition_variable cv_;
  std::map<std::string, int> peers_;
  std::deque<std::pair<std::string, std::string>> q_;
  std::thread accept_th_;
  std::vector<std::thread> readers_;
};

}  // namespace host
}  // namespace wh
