// Horovod-compatible chrome://tracing timeline writer (HOROVOD_TIMELINE).
// Parity: horovod common/timeline.cc.  Producers (engine
// thread, hook threads, the coordinator) enqueue events under a mutex; a
// dedicated writer thread formats and appends them, so recording never blocks
// on file I/O.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>

namespace mvcore {

class Timeline {
 public:
  Timeline(const std::string& path, bool mark_cycles);
  ~Timeline();
  void start(const std::string& name, const std::string& phase, const std::string& args = "");
  void activity(const std::string& name, const std::string& phase) { start(name, phase); }
  void end(const std::string& name);
  void instant(const std::string& name, const std::string& what);
  // complete ("X") event with explicit start / duration in this timeline's clock
  // (GPU phases of the static gradient schedule, timed by hipEvents)
  void complete(const std::string& name, const std::string& phase, int64_t ts_us, int64_t dur_us);
  void mark_cycle();
  int64_t now_us() const;
  void close();
  bool mark_cycles() const { return mark_cycles_; }
  int64_t events_written() const { return written_; }

 private:
  struct Ev {
    char ph;
    std::string name, phase, args;
    int64_t ts;
    int64_t dur = 0;
  };
  void push(Ev e);
  void run();
  int pid_for(const std::string& name, std::string* meta);

  FILE* f_ = nullptr;
  bool mark_cycles_;
  std::chrono::steady_clock::time_point t0_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Ev> q_;
  bool stop_ = false;
  std::thread writer_;
  std::unordered_map<std::string, int> pids_;
  std::unordered_map<std::string, bool> open_;
  int64_t written_ = 0;
};

}  // namespace mvcore
