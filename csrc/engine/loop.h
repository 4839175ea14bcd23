// mivod background engine loop: the negotiation cycle in a native thread.
//
// Parity: horovod 0.18.1 common/operations.cc BackgroundThreadLoop / RunLoopOnce
// (SURVEY.md §2.2 U2): a background thread wakes every cycle (HOROVOD_CYCLE_TIME)
// or as soon as a request is queued, ships this rank's new requests to the
// coordinator (Controller::negotiate: TCP star, response cache, stall inspector),
// and hands the coordinator's response list to the executor.  The loop, its
// timing and all control-plane I/O run here without the Python GIL; Python only
// enqueues requests (a short critical section) and executes the responses, which
// need torch tensors (mivod/parallel/engine.py, the executor thread blocks in
// wait() with the GIL released).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "controller.h"

namespace mvcore {

struct CycleResult {
  std::vector<Response> responses;
  bool all_shutdown = false;
  int64_t exec_at = 0;     // issue-order point of this cycle's GPU responses
  std::string error;       // control-plane failure (the loop has stopped)
};

class EngineLoop {
 public:
  // cycle_s <= 0 or a 1-rank world: negotiate as soon as a request arrives
  EngineLoop(std::shared_ptr<Controller> ctl, int size, double cycle_s);
  ~EngineLoop();
  EngineLoop(const EngineLoop&) = delete;
  EngineLoop& operator=(const EngineLoop&) = delete;

  void submit(std::vector<Request> reqs);
  // this rank's issue-order position Q (parallel/order.py), read at every cycle
  void set_position(int64_t q) { position_.store(q, std::memory_order_release); }
  // ask every rank to shut down; the loop ends once all ranks did
  void request_shutdown();
  // next cycle with responses (or the final / error one); false on timeout
  bool wait(double timeout_s, CycleResult* out);
  bool finished() const { return finished_.load(); }
  int64_t cycles() const { return cycles_.load(); }
  int64_t requests() const { return requests_.load(); }
  void join();

 private:
  void run();

  std::shared_ptr<Controller> ctl_;
  int size_;
  double cycle_s_;
  std::mutex mu_;
  std::condition_variable cv_;        // producer -> loop
  std::condition_variable out_cv_;    // loop -> executor
  std::vector<Request> queue_;
  std::deque<CycleResult> out_;
  bool shutdown_ = false;
  std::atomic<int64_t> position_{0};
  std::atomic<bool> finished_{false};
  std::atomic<int64_t> cycles_{0};
  std::atomic<int64_t> requests_{0};
  std::thread thread_;
};

}  // namespace mvcore
