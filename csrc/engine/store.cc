#include "store.h"

#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <stdexcept>

#include "wire.h"

namespace mvcore {

namespace {
enum Status : uint8_t { kOk = 0, kTimeout = 1, kError = 2 };

std::chrono::steady_clock::time_point deadline_after(double s) {
  return std::chrono::steady_clock::now() +
         std::chrono::duration_cast<std::chrono::steady_clock::duration>(
             std::chrono::duration<double>(s < 0 ? 3.0e7 : s));
}
}  // namespace

// --------------------------------------------------------------------- server
KVServer::KVServer(const std::string& host, int port) {
  port_ = port;
  lfd_ = tcp_listen(host, &port_);
  acceptor_ = std::thread([this] { accept_loop(); });
}

KVServer::~KVServer() {
  try {
    close();
  } catch (...) {
  }
}

void KVServer::accept_loop() {
  while (!stop_) {
    int fd;
    try {
      fd = tcp_accept(lfd_, 0.2);
    } catch (...) {
      continue;   // timeout tick: re-check stop_
    }
    std::lock_guard<std::mutex> g(conn_mu_);
    if (stop_) {
      close_fd(fd);
      break;
    }
    fds_.push_back(fd);
    conns_.emplace_back([this, fd] { serve(fd); });
  }
}

void KVServer::serve(int fd) {
  try {
    while (!stop_) {
      std::string req = recv_msg(fd);
      ++requests_;
      send_msg(fd, handle(req));
    }
  } catch (...) {
    // client gone (or shutdown): this connection's thread ends
  }
}

std::string KVServer::handle(const std::string& req) {
  Reader r(req);
  Writer w;
  const uint8_t op = r.u8();
  std::unique_lock<std::mutex> lk(mu_);
  switch (op) {
    case kSet: {
      std::string k = r.str();
      kv_[k] = r.str();
      cv_.notify_all();
      w.u8(kOk);
      break;
    }
    case kGet: {
      std::string k = r.str();
      const double t = r.f64();
      if (!cv_.wait_until(lk, deadline_after(t), [&] { return stop_ || kv_.count(k) > 0; }) ||
          stop_) {
        w.u8(kTimeout);
        w.str("timed out after " + std::to_string(t) + " s waiting for key '" + k + "'");
        break;
      }
      w.u8(kOk);
      w.str(kv_[k]);
      break;
    }
    case kAdd: {
      std::string k = r.str();
      const int64_t d = r.i64();
      int64_t v = 0;
      auto it = kv_.find(k);
      if (it != kv_.end()) {
        try {
          v = std::stoll(it->second);
        } catch (...) {
          w.u8(kError);
          w.str("add: key '" + k + "' does not hold an integer");
          break;
        }
      }
      v += d;
      kv_[k] = std::to_string(v);
      cv_.notify_all();
      w.u8(kOk);
      w.i64(v);
      break;
    }
    case kCheck:
    case kWait: {
      const uint32_t n = r.u32();
      std::vector<std::string> keys(n);
      for (auto& k : keys) k = r.str();
      auto all = [&] {
        for (auto& k : keys)
          if (!kv_.count(k)) return false;
        return true;
      };
      if (op == kCheck) {
        w.u8(kOk);
        w.u8(all() ? 1 : 0);
        break;
      }
      const double t = r.f64();
      if (!cv_.wait_until(lk, deadline_after(t), [&] { return stop_ || all(); }) || stop_) {
        w.u8(kTimeout);
        w.str("timed out after " + std::to_string(t) + " s waiting for " + std::to_string(n) +
              " key(s)");
        break;
      }
      w.u8(kOk);
      break;
    }
    case kDelete: {
      std::string k = r.str();
      w.u8(kOk);
      w.u8(kv_.erase(k) ? 1 : 0);
      break;
    }
    case kNumKeys:
      w.u8(kOk);
      w.i64((int64_t)kv_.size());
      break;
    case kCompareSet: {
      std::string k = r.str(), expected = r.str(), desired = r.str();
      auto it = kv_.find(k);
      if ((it == kv_.end() && expected.empty()) || (it != kv_.end() && it->second == expected)) {
        kv_[k] = desired;
        cv_.notify_all();
        w.u8(kOk);
        w.str(desired);
      } else {
        w.u8(kOk);
        w.str(it == kv_.end() ? expected : it->second);
      }
      break;
    }
    case kPing:
      w.u8(kOk);
      break;
    default:
      w.u8(kError);
      w.str("unknown store op " + std::to_string(op));
  }
  return w.buf;
}

void KVServer::close() {
  if (stop_.exchange(true)) return;
  cv_.notify_all();
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int fd : fds_) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : conns_)
    if (t.joinable()) t.join();
  for (int fd : fds_) close_fd(fd);
  fds_.clear();
  conns_.clear();
  close_fd(lfd_);
  lfd_ = -1;
}

// --------------------------------------------------------------------- client
KVClient::KVClient(const std::string& host, int port, double timeout_s) : timeout_s_(timeout_s) {
  fd_ = tcp_connect(host, port, timeout_s);
}

KVClient::~KVClient() { close(); }

void KVClient::close() {
  std::lock_guard<std::mutex> g(mu_);
  close_fd(fd_);
  fd_ = -1;
}

std::string KVClient::call(const std::string& req) {
  std::lock_guard<std::mutex> g(mu_);
  if (fd_ < 0) throw std::runtime_error("mivod store: client closed");
  send_msg(fd_, req);
  return recv_msg(fd_);
}

static void check_status(Reader& r) {
  const uint8_t s = r.u8();
  if (s == 0) return;
  std::string msg = r.str();
  if (s == kTimeout) throw std::runtime_error("mivod store: " + msg);
  throw std::runtime_error("mivod store: " + msg);
}

void KVClient::set(const std::string& key, const std::string& value) {
  Writer w;
  w.u8(kSet);
  w.str(key);
  w.str(value);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
}

std::string KVClient::get(const std::string& key) {
  Writer w;
  w.u8(kGet);
  w.str(key);
  w.f64(timeout_s_);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.str();
}

int64_t KVClient::add(const std::string& key, int64_t delta) {
  Writer w;
  w.u8(kAdd);
  w.str(key);
  w.i64(delta);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.i64();
}

bool KVClient::check(const std::vector<std::string>& keys) {
  Writer w;
  w.u8(kCheck);
  w.u32((uint32_t)keys.size());
  for (auto& k : keys) w.str(k);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.u8() != 0;
}

void KVClient::wait(const std::vector<std::string>& keys, double timeout_s) {
  Writer w;
  w.u8(kWait);
  w.u32((uint32_t)keys.size());
  for (auto& k : keys) w.str(k);
  w.f64(timeout_s);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
}

bool KVClient::remove(const std::string& key) {
  Writer w;
  w.u8(kDelete);
  w.str(key);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.u8() != 0;
}

int64_t KVClient::num_keys() {
  Writer w;
  w.u8(kNumKeys);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.i64();
}

std::string KVClient::compare_set(const std::string& key, const std::string& expected,
                                  const std::string& desired) {
  Writer w;
  w.u8(kCompareSet);
  w.str(key);
  w.str(expected);
  w.str(desired);
  std::string resp = call(w.buf);
  Reader r(resp);
  check_status(r);
  return r.str();
}

}  // namespace mvcore
