#include "loop.h"

#include <chrono>

namespace mvcore {

EngineLoop::EngineLoop(std::shared_ptr<Controller> ctl, int size, double cycle_s)
    : ctl_(std::move(ctl)), size_(size), cycle_s_(cycle_s) {
  if (!ctl_) throw std::invalid_argument("mivod EngineLoop: controller required");
  thread_ = std::thread([this] { run(); });
}

EngineLoop::~EngineLoop() {
  request_shutdown();
  join();
}

void EngineLoop::join() {
  if (thread_.joinable()) thread_.join();
}

void EngineLoop::submit(std::vector<Request> reqs) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (shutdown_) throw std::runtime_error("mivod engine is shutting down");
    requests_ += (int64_t)reqs.size();
    for (auto& r : reqs) queue_.push_back(std::move(r));
  }
  cv_.notify_all();
}

void EngineLoop::request_shutdown() {
  {
    std::lock_guard<std::mutex> g(mu_);
    shutdown_ = true;
  }
  cv_.notify_all();
}

bool EngineLoop::wait(double timeout_s, CycleResult* out) {
  std::unique_lock<std::mutex> lk(mu_);
  auto ready = [&] { return !out_.empty() || finished_.load(); };
  if (timeout_s < 0) out_cv_.wait(lk, ready);
  else out_cv_.wait_for(lk, std::chrono::duration<double>(timeout_s), ready);
  if (out_.empty()) return false;
  *out = std::move(out_.front());
  out_.pop_front();
  return true;
}

void EngineLoop::run() {
  const bool timed = size_ > 1 && cycle_s_ > 0;
  const auto cycle = std::chrono::duration<double>(cycle_s_ > 0 ? cycle_s_ : 0.0);
  while (true) {
    std::vector<Request> batch;
    bool stopping;
    {
      std::unique_lock<std::mutex> lk(mu_);
      if (!shutdown_ && queue_.empty()) {
        // a multi-rank world negotiates every cycle even with nothing queued:
        // other ranks' requests (and their stall state) need this rank's answer
        if (timed) cv_.wait_for(lk, cycle, [&] { return shutdown_ || !queue_.empty(); });
        else cv_.wait(lk, [&] { return shutdown_ || !queue_.empty(); });
      }
      batch.swap(queue_);
      stopping = shutdown_;
    }
    CycleResult res;
    try {
      res.responses = ctl_->negotiate(batch, stopping, &res.all_shutdown,
                                      position_.load(std::memory_order_acquire), &res.exec_at);
    } catch (const std::exception& e) {
      res.error = e.what();
      res.all_shutdown = true;
    }
    ++cycles_;
    const bool last = !res.error.empty() || (stopping && res.all_shutdown);
    if (!res.responses.empty() || last) {
      std::lock_guard<std::mutex> g(mu_);
      out_.push_back(std::move(res));
    }
    if (last) break;
    out_cv_.notify_all();
  }
  finished_.store(true);
  out_cv_.notify_all();
}

}  // namespace mvcore
