// Native TCP key-value store: cluster rendezvous and control plane.
//
// Replaces the coordination the reference gets from TF's gRPC master/worker
// services (tf.train.Server, example.py:38-40; Supervisor's chief/non-chief
// handshake, example.py:139-145) and implements the ps shutdown protocol the
// reference left commented out (lr2.py:337-346: every worker enqueues a token,
// the ps waits for num_workers tokens and exits).  Uses: RCCL unique-id
// exchange, barriers, chief-init-done flags, done tokens, heartbeats.
//
// Wire format (little endian): request  = u8 op | u32 nargs | nargs x (u64 len | bytes)
//                              response = u8 status | u32 nvals | nvals x (u64 len | bytes)
// A thread per client connection; blocking GET/WAIT park on a condition
// variable with a deadline.  The Python side may also wrap it as a
// torch.distributed Store so gloo bootstraps through the same server.
#include <torch/extension.h>
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>

#include "cv_wait.h"
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dtf {
namespace store {

enum Op : uint8_t { SET = 1, GET = 2, ADD = 3, CHECK = 4, WAIT = 5, DEL = 6, NUMKEYS = 7, KEYS = 8, CAS = 9, PING = 10 };
enum Status : uint8_t { OK = 0, TIMEOUT = 1, ERR = 2, MISSING = 3 };

static bool send_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}
static bool recv_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    c += k;
    n -= (size_t)k;
  }
  return true;
}
static bool send_msg(int fd, uint8_t head, const std::vector<std::string>& parts) {
  std::string buf;
  buf.push_back((char)head);
  uint32_t n = (uint32_t)parts.size();
  buf.append(reinterpret_cast<const char*>(&n), 4);
  for (auto& s : parts) {
    uint64_t l = s.size();
    buf.append(reinterpret_cast<const char*>(&l), 8);
    buf.append(s);
  }
  return send_all(fd, buf.data(), buf.size());
}
static bool recv_msg(int fd, uint8_t& head, std::vector<std::string>& parts) {
  uint32_t n;
  if (!recv_all(fd, &head, 1) || !recv_all(fd, &n, 4)) return false;
  if (n > (1u << 20)) return false;
  parts.resize(n);
  for (auto& s : parts) {
    uint64_t l;
    if (!recv_all(fd, &l, 8)) return false;
    if (l > (1ull << 34)) return false;
    s.resize(l);
    if (l && !recv_all(fd, &s[0], l)) return false;
  }
  return true;
}

static int64_t to_i64(const std::string& s) {
  if (s.empty()) return 0;
  return std::stoll(s);
}

class Server {
 public:
  Server(const std::string& host, int port) {
    fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd_ < 0) throw std::runtime_error("socket() failed");
    int one = 1;
    setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (host.empty() || host == "0.0.0.0" || host == "*") a.sin_addr.s_addr = INADDR_ANY;
    else if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) {
      hostent* he = gethostbyname(host.c_str());
      if (!he) { ::close(fd_); throw std::runtime_error("cannot resolve " + host); }
      memcpy(&a.sin_addr, he->h_addr, sizeof(a.sin_addr));
    }
    if (::bind(fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      ::close(fd_);
      throw std::runtime_error("bind failed on " + host + ":" + std::to_string(port) + ": " + strerror(errno));
    }
    socklen_t len = sizeof(a);
    getsockname(fd_, reinterpret_cast<sockaddr*>(&a), &len);
    port_ = ntohs(a.sin_port);
    if (::listen(fd_, 128) != 0) { ::close(fd_); throw std::runtime_error("listen failed"); }
    acceptor_ = std::thread([this] { accept_loop(); });
  }
  ~Server() { stop(); }
  int port() const { return port_; }
  void stop() {
    // serialised: a second caller (e.g. the destructor racing an explicit
    // stop() from another thread) waits until the threads are joined instead
    // of returning early and destroying joinable std::threads (-> terminate)
    std::lock_guard<std::mutex> g(stop_mu_);
    if (stopping_.exchange(true)) return;
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    {
      std::lock_guard<std::mutex> lk(mu_);
      cv_.notify_all();
      for (int c : clients_) ::shutdown(c, SHUT_RDWR);
    }
    if (acceptor_.joinable()) acceptor_.join();
    for (auto& t : workers_) if (t.joinable()) t.join();
  }

 private:
  void accept_loop() {
    while (!stopping_) {
      pollfd p{fd_, POLLIN, 0};
      int r = ::poll(&p, 1, 200);
      if (r <= 0) continue;
      int c = ::accept(fd_, nullptr, nullptr);
      if (c < 0) continue;
      int one = 1;
      setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> lk(mu_);
      clients_.push_back(c);
      workers_.emplace_back([this, c] { serve(c); });
    }
  }
  void serve(int c) {
    uint8_t op;
    std::vector<std::string> args;
    while (!stopping_ && recv_msg(c, op, args)) {
      uint8_t st = OK;
      std::vector<std::string> out;
      std::unique_lock<std::mutex> lk(mu_);
      switch (op) {
        case SET:
          if (args.size() != 2) { st = ERR; break; }
          kv_[args[0]] = args[1];
          cv_.notify_all();
          break;
        case GET: {  // args: key, timeout_ms
          auto deadline = std::chrono::steady_clock::now() +
                          std::chrono::milliseconds(args.size() > 1 ? to_i64(args[1]) : 0);
          bool ok = cv_wait_until(cv_, lk, deadline, [&] { return stopping_ || kv_.count(args[0]); });
          if (!ok || !kv_.count(args[0])) st = TIMEOUT;
          else out.push_back(kv_[args[0]]);
          break;
        }
        case ADD: {
          int64_t v = to_i64(kv_.count(args[0]) ? kv_[args[0]] : "0") + to_i64(args[1]);
          kv_[args[0]] = std::to_string(v);
          out.push_back(kv_[args[0]]);
          cv_.notify_all();
          break;
        }
        case CHECK: {
          bool all = true;
          for (auto& k : args) all = all && kv_.count(k);
          out.push_back(all ? "1" : "0");
          break;
        }
        case WAIT: {  // args: timeout_ms, keys...
          auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(to_i64(args[0]));
          auto have = [&] {
            for (size_t i = 1; i < args.size(); ++i) if (!kv_.count(args[i])) return false;
            return true;
          };
          if (!cv_wait_until(cv_, lk, deadline, [&] { return stopping_ || have(); }) || !have()) st = TIMEOUT;
          break;
        }
        case DEL:
          out.push_back(kv_.erase(args[0]) ? "1" : "0");
          break;
        case NUMKEYS:
          out.push_back(std::to_string(kv_.size()));
          break;
        case KEYS: {
          const std::string& pre = args.empty() ? std::string() : args[0];
          for (auto it = kv_.lower_bound(pre); it != kv_.end() && it->first.compare(0, pre.size(), pre) == 0; ++it)
            out.push_back(it->first);
          break;
        }
        case CAS: {  // key, expected, desired ("" expected == absent)
          auto it = kv_.find(args[0]);
          const bool absent = it == kv_.end();
          if ((absent && args[1].empty()) || (!absent && it->second == args[1])) {
            kv_[args[0]] = args[2];
            cv_.notify_all();
          }
          out.push_back(kv_[args[0]]);
          break;
        }
        case PING:
          out.push_back("pong");
          break;
        default:
          st = ERR;
      }
      lk.unlock();
      if (!send_msg(c, st, out)) break;
    }
    ::close(c);
  }

  int fd_ = -1, port_ = 0;
  std::atomic<bool> stopping_{false};
  std::mutex stop_mu_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
  std::vector<int> clients_;
  std::vector<std::thread> workers_;
  std::thread acceptor_;
};

class Client {
 public:
  Client(const std::string& host, int port, double timeout_s) : timeout_ms_((int64_t)(timeout_s * 1000)) {
    auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms_);
    std::string last;
    while (true) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
        int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
        if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          fd_ = fd;
          freeaddrinfo(res);
          return;
        }
        last = strerror(errno);
        if (fd >= 0) ::close(fd);
        freeaddrinfo(res);
      } else {
        last = "cannot resolve " + host;
      }
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("store connect to " + host + ":" + std::to_string(port) + " timed out: " + last);
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
  ~Client() { close(); }
  void close() {
    if (fd_ >= 0) { ::close(fd_); fd_ = -1; }
  }

  std::vector<std::string> call(uint8_t op, const std::vector<std::string>& args, uint8_t* status) {
    std::lock_guard<std::mutex> lk(mu_);
    if (fd_ < 0) throw std::runtime_error("store client closed");
    if (!send_msg(fd_, op, args)) throw std::runtime_error("store connection lost (send)");
    uint8_t st;
    std::vector<std::string> out;
    if (!recv_msg(fd_, st, out)) throw std::runtime_error("store connection lost (recv)");
    if (status) *status = st;
    if (st == ERR) throw std::runtime_error("store error");
    return out;
  }
  int64_t timeout_ms() const { return timeout_ms_; }

 private:
  int fd_ = -1;
  int64_t timeout_ms_;
  std::mutex mu_;
};

// Python-facing store: optionally hosts the server, always owns a client.
class TCPStore {
 public:
  TCPStore(const std::string& host, int port, bool is_server, double timeout_s)
      : host_(host), timeout_s_(timeout_s) {
    if (is_server) {
      server_ = std::make_unique<Server>(host, port);
      port = server_->port();
    }
    port_ = port;
    client_ = std::make_unique<Client>(is_server ? std::string("127.0.0.1") : host, port, timeout_s);
  }
  int port() const { return port_; }
  bool is_server() const { return server_ != nullptr; }
  void set(const std::string& k, py::bytes v) {
    std::string s = v;
    py::gil_scoped_release nogil;
    client_->call(SET, {k, s}, nullptr);
  }
  py::bytes get(const std::string& k, double timeout_s) {
    std::vector<std::string> out;
    uint8_t st;
    {
      py::gil_scoped_release nogil;
      const int64_t ms = timeout_s < 0 ? client_->timeout_ms() : (int64_t)(timeout_s * 1000);
      out = client_->call(GET, {k, std::to_string(ms)}, &st);
    }
    if (st == TIMEOUT) throw std::runtime_error("store get timed out: " + k);
    return py::bytes(out.at(0));
  }
  int64_t add(const std::string& k, int64_t d) {
    py::gil_scoped_release nogil;
    return to_i64(client_->call(ADD, {k, std::to_string(d)}, nullptr).at(0));
  }
  bool check(const std::vector<std::string>& keys) {
    py::gil_scoped_release nogil;
    return client_->call(CHECK, keys, nullptr).at(0) == "1";
  }
  void wait(const std::vector<std::string>& keys, double timeout_s) {
    uint8_t st;
    {
      py::gil_scoped_release nogil;
      std::vector<std::string> a;
      a.push_back(std::to_string(timeout_s < 0 ? client_->timeout_ms() : (int64_t)(timeout_s * 1000)));
      a.insert(a.end(), keys.begin(), keys.end());
      client_->call(WAIT, a, &st);
    }
    if (st == TIMEOUT) throw std::runtime_error("store wait timed out");
  }
  bool del(const std::string& k) {
    py::gil_scoped_release nogil;
    return client_->call(DEL, {k}, nullptr).at(0) == "1";
  }
  int64_t num_keys() {
    py::gil_scoped_release nogil;
    return to_i64(client_->call(NUMKEYS, {}, nullptr).at(0));
  }
  std::vector<std::string> keys(const std::string& prefix) {
    py::gil_scoped_release nogil;
    return client_->call(KEYS, {prefix}, nullptr);
  }
  py::bytes compare_set(const std::string& k, py::bytes expected, py::bytes desired) {
    std::string e = expected, d = desired;
    std::vector<std::string> out;
    {
      py::gil_scoped_release nogil;
      out = client_->call(CAS, {k, e, d}, nullptr);
    }
    return py::bytes(out.at(0));
  }
  // All `world` participants call barrier(name); returns when all arrived.
  void barrier(const std::string& name, int world, double timeout_s) {
    py::gil_scoped_release nogil;
    const int64_t n = to_i64(client_->call(ADD, {"__barrier/" + name, "1"}, nullptr).at(0));
    if (n == world) client_->call(SET, {"__barrier_done/" + name, "1"}, nullptr);
    uint8_t st;
    const int64_t ms = timeout_s < 0 ? client_->timeout_ms() : (int64_t)(timeout_s * 1000);
    client_->call(WAIT, {std::to_string(ms), "__barrier_done/" + name}, &st);
    if (st == TIMEOUT) throw std::runtime_error("barrier timed out: " + name);
  }
  bool ping() {
    py::gil_scoped_release nogil;
    try {
      return client_->call(PING, {}, nullptr).at(0) == "pong";
    } catch (...) {
      return false;
    }
  }
  void close() {
    py::gil_scoped_release nogil;
    if (client_) client_->close();
    if (server_) server_->stop();
  }

 private:
  std::string host_;
  int port_ = 0;
  double timeout_s_;
  std::unique_ptr<Server> server_;
  std::unique_ptr<Client> client_;
};

}  // namespace store

void init_store(py::module& m) {
  using store::TCPStore;
  py::class_<TCPStore>(m, "TCPStore")
      .def(py::init<const std::string&, int, bool, double>(), py::arg("host"), py::arg("port"),
           py::arg("is_server") = false, py::arg("timeout") = 300.0)
      .def_property_readonly("port", &TCPStore::port)
      .def_property_readonly("is_server", &TCPStore::is_server)
      .def("set", &TCPStore::set)
      .def("get", &TCPStore::get, py::arg("key"), py::arg("timeout") = -1.0)
      .def("add", &TCPStore::add)
      .def("check", &TCPStore::check)
      .def("wait", &TCPStore::wait, py::arg("keys"), py::arg("timeout") = -1.0)
      .def("delete_key", &TCPStore::del)
      .def("num_keys", &TCPStore::num_keys)
      .def("keys", &TCPStore::keys, py::arg("prefix") = "")
      .def("compare_set", &TCPStore::compare_set)
      .def("barrier", &TCPStore::barrier, py::arg("name"), py::arg("world"), py::arg("timeout") = -1.0)
      .def("ping", &TCPStore::ping)
      .def("close", &TCPStore::close);
}

}  // namespace dtf
