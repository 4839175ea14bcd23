// mivod rendezvous key-value store (SURVEY.md §1 N1 "C++ TCP rendezvous KV store",
// §2.4 "Process launch / bootstrap"; the role of horovodrun's Gloo rendezvous HTTP
// server, horovod/run/gloo_run.py, that HOROVOD_GLOO_RENDEZVOUS_ADDR/PORT point to).
//
// The launcher (mivod.run) hosts one KVServer; every rank connects a KVClient and
// bootstraps through it: the gloo world (mivod.run.store.NativeStore is a
// torch.distributed.Store backed by this client), mivod's RCCL unique id, the
// xGMI mesh's IPC handles, the TCP rings' addresses.
//
// Protocol: one persistent TCP connection per client, length-prefixed request /
// response records (wire.h Writer/Reader): [u8 op][args...] -> [u8 status][result].
// The server runs a thread per connection over one mutex-guarded map + condition
// variable, so a GET / WAIT blocks on the server until the key exists (bounded by the
// client's timeout) and never polls.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace mvcore {

enum StoreOp : uint8_t {
  kSet = 1,
  kGet = 2,          // blocks until the key exists (timeout)
  kAdd = 3,          // int64 counter (created at 0), returns the new value
  kCheck = 4,        // all keys exist?
  kWait = 5,         // blocks until all keys exist (timeout)
  kDelete = 6,
  kNumKeys = 7,
  kCompareSet = 8,   // set if current == expected (or absent and expected == ""), returns current
  kPing = 9,
};

class KVServer {
 public:
  // port 0 = ephemeral; host "" / "0.0.0.0" = all interfaces
  KVServer(const std::string& host, int port);
  ~KVServer();
  KVServer(const KVServer&) = delete;
  KVServer& operator=(const KVServer&) = delete;
  int port() const { return port_; }
  int64_t requests() const { return requests_; }
  void close();

 private:
  void accept_loop();
  void serve(int fd);
  std::string handle(const std::string& req);

  int lfd_ = -1, port_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> requests_{0};
  std::thread acceptor_;
  std::mutex conn_mu_;
  std::vector<std::thread> conns_;
  std::vector<int> fds_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<std::string, std::string> kv_;
};

class KVClient {
 public:
  KVClient(const std::string& host, int port, double timeout_s);
  ~KVClient();
  KVClient(const KVClient&) = delete;
  KVClient& operator=(const KVClient&) = delete;

  void set(const std::string& key, const std::string& value);
  std::string get(const std::string& key);
  int64_t add(const std::string& key, int64_t delta);
  bool check(const std::vector<std::string>& keys);
  void wait(const std::vector<std::string>& keys, double timeout_s);
  bool remove(const std::string& key);
  int64_t num_keys();
  std::string compare_set(const std::string& key, const std::string& expected,
                          const std::string& desired);
  void set_timeout(double s) { timeout_s_ = s; }
  double timeout() const { return timeout_s_; }
  void close();

 private:
  std::string call(const std::string& req);
  int fd_ = -1;
  double timeout_s_;
  std::mutex mu_;   // one request in flight per connection
};

}  // namespace mvcore
