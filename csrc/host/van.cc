// Control-plane transport (replaces ps-lite's ZeroMQ van for the scheduler
// <-> worker plane: workloads, progress reports, save/load commands,
// liveness). Length-prefixed frames over TCP; one reader thread per peer
// feeds a single receive queue. A peer's disconnect is delivered as a
// message with kind "__closed__" so the scheduler can re-queue its work
// (the reference's AddNodeFailureHandler hook, learn/solver/data_parallel.h:131-135).
#include "van.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstring>

namespace wh {
namespace host {

namespace {
bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w <= 0) {
      if (w < 0 && errno == EINTR) continue;
      return false;
    }
    c += w;
    n -= (size_t)w;
  }
  return true;
}
bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}
bool send_frame(int fd, const std::string& s) {
  uint64_t n = s.size();
  return write_all(fd, &n, 8) && write_all(fd, s.data(), s.size());
}
bool recv_frame(int fd, std::string* s) {
  uint64_t n;
  if (!read_all(fd, &n, 8)) return false;
  if (n > (1ull << 34)) return false;
  s->resize(n);
  return n == 0 || read_all(fd, &(*s)[0], n);
}
void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}
}  // namespace

Van::~Van() { Close(); }

int Van::Listen(int port) {
  lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  WH_CHECK(lfd_ >= 0, "socket() failed");
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  WH_CHECK(::bind(lfd_, (sockaddr*)&a, sizeof(a)) == 0,
           "bind() failed on port " + std::to_string(port));
  WH_CHECK(::listen(lfd_, 1024) == 0, "listen() failed");
  socklen_t len = sizeof(a);
  getsockname(lfd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  const int lfd = lfd_;
  accept_th_ = std::thread([this, lfd] { AcceptLoop(lfd); });
  return port_;
}

// lfd is the accept thread's own copy: Close() shuts the socket down (which
// wakes accept), joins this thread, and only then closes the descriptor, so
// accept() can never run on a closed or reused fd number.
void Van::AcceptLoop(int lfd) {
  while (!closing_) {
    sockaddr_in a{};
    socklen_t len = sizeof(a);
    int fd = ::accept(lfd, (sockaddr*)&a, &len);
    if (fd < 0) {
      if (closing_) return;
      continue;
    }
    tune(fd);
    std::string hello;
    if (!recv_frame(fd, &hello)) {
      ::close(fd);
      continue;
    }
    std::lock_guard<std::mutex> lk(mu_);
    peers_[hello] = fd;
    readers_.emplace_back([this, fd, hello] { ReadLoop(fd, hello); });
  }
}

void Van::ReadLoop(int fd, std::string id) {
  std::string msg;
  while (recv_frame(fd, &msg)) Push(id, msg);
  if (!closing_) Push(id, "__closed__");
}

void Van::Push(const std::string& from, const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.emplace_back(from, msg);
  }
  cv_.notify_one();
}

void Van::Connect(const std::string& host, int port, const std::string& my_id, double timeout_s) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  WH_CHECK(getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0,
           "cannot resolve " + host);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  int fd = -1;
  while (true) {
    fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (::connect(fd, res->ai_addr, res->ai_addrlen) == 0) break;
    ::close(fd);
    fd = -1;
    if (std::chrono::steady_clock::now() > deadline) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  freeaddrinfo(res);
  WH_CHECK(fd >= 0, "cannot connect to " + host + ":" + std::to_string(port));
  tune(fd);
  WH_CHECK(send_frame(fd, my_id), "hello failed");
  std::lock_guard<std::mutex> lk(mu_);
  peers_["scheduler"] = fd;
  readers_.emplace_back([this, fd] { ReadLoop(fd, "scheduler"); });
}

bool Van::Send(const std::string& to, const std::string& msg) {
  int fd;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = peers_.find(to);
    if (it == peers_.end()) return false;
    fd = it->second;
  }
  std::lock_guard<std::mutex> lk(send_mu_);
  return send_frame(fd, msg);
}

bool Van::Recv(double timeout_s, std::string* from, std::string* msg) {
  std::unique_lock<std::mutex> lk(mu_);
  // system_clock deadline (see WorkloadPool::Loop: steady-clock waits use
  // pthread_cond_clockwait, invisible to ThreadSanitizer)
  const auto until = std::chrono::system_clock::now() +
                     std::chrono::duration_cast<std::chrono::system_clock::duration>(
                         std::chrono::duration<double>(timeout_s));
  if (!cv_.wait_until(lk, until, [&] { return !q_.empty(); })) return false;
  *from = q_.front().first;
  *msg = q_.front().second;
  q_.pop_front();
  return true;
}

std::vector<std::string> Van::Peers() {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> v;
  for (auto& p : peers_) v.push_back(p.first);
  return v;
}

void Van::Close() {
  if (closing_.exchange(true)) return;
  if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);  // wakes accept()
  if (accept_th_.joinable()) accept_th_.join();
  if (lfd_ >= 0) {
    ::close(lfd_);
    lfd_ = -1;
  }
  std::vector<std::thread> readers;
  {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& p : peers_) ::shutdown(p.second, SHUT_RDWR);
    readers.swap(readers_);
  }
  for (auto& t : readers)
    if (t.joinable()) t.join();
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& p : peers_) ::close(p.second);
  peers_.clear();
}

}  // namespace host
}  // namespace wh
