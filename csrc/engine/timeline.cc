#include "timeline.h"

#include <stdexcept>

namespace mvcore {

static std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (char c : s) {
    if (c == '"' || c == '\\') { o.push_back('\\'); o.push_back(c); }
    else if ((unsigned char)c < 0x20) { char b[8]; snprintf(b, sizeof b, "\\u%04x", c); o += b; }
    else o.push_back(c);
  }
  return o;
}

Timeline::Timeline(const std::string& path, bool mark_cycles)
    : mark_cycles_(mark_cycles), t0_(std::chrono::steady_clock::now()) {
  f_ = fopen(path.c_str(), "w");
  if (!f_) throw std::runtime_error("mivod timeline: cannot open " + path);
  fputs("[\n", f_);
  writer_ = std::thread([this] { run(); });
}

Timeline::~Timeline() { close(); }

int64_t Timeline::now_us() const {
  return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() -
                                                               t0_).count();
}

void Timeline::push(Ev e) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    q_.push_back(std::move(e));
  }
  cv_.notify_one();
}

void Timeline::start(const std::string& name, const std::string& phase, const std::string& args) {
  push(Ev{'B', name, phase, args, now_us()});
}
void Timeline::end(const std::string& name) { push(Ev{'E', name, "", "", now_us()}); }
void Timeline::instant(const std::string& name, const std::string& what) {
  push(Ev{'i', name, what, "", now_us()});
}
void Timeline::complete(const std::string& name, const std::string& phase, int64_t ts_us,
                        int64_t dur_us) {
  Ev e{'X', name, phase, "", ts_us};
  e.dur = dur_us < 0 ? 0 : dur_us;
  push(std::move(e));
}
void Timeline::mark_cycle() {
  if (mark_cycles_) instant("cycle", "CYCLE_START");
}

int Timeline::pid_for(const std::string& name, std::string* meta) {
  auto it = pids_.find(name);
  if (it != pids_.end()) return it->second;
  int pid = (int)pids_.size() + 1;
  pids_[name] = pid;
  char b[512];
  snprintf(b, sizeof b,
           "{\"name\": \"process_name\", \"ph\": \"M\", \"pid\": %d, \"args\": {\"name\": \"%s\"}},\n"
           "{\"name\": \"process_sort_index\", \"ph\": \"M\", \"pid\": %d, \"args\": {\"sort_index\": %d}},\n",
           pid, json_escape(name).c_str(), pid, pid);
  *meta = b;
  return pid;
}

void Timeline::run() {
  std::unique_lock<std::mutex> lk(mu_);
  while (true) {
    cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
    std::deque<Ev> batch;
    batch.swap(q_);
    bool done = stop_;
    lk.unlock();
    std::string out;
    for (auto& e : batch) {
      std::string meta;
      int pid = pid_for(e.name, &meta);
      out += meta;
      char b[256];
      if (e.ph == 'B') {
        if (open_[e.name]) {
          snprintf(b, sizeof b, "{\"ph\": \"E\", \"pid\": %d, \"tid\": 1, \"ts\": %lld},\n", pid,
                   (long long)e.ts);
          out += b;
        }
        out += "{\"name\": \"" + json_escape(e.phase) + "\", \"ph\": \"B\", \"pid\": " +
               std::to_string(pid) + ", \"tid\": 1, \"ts\": " + std::to_string(e.ts);
        if (!e.args.empty()) out += ", \"args\": {\"detail\": \"" + json_escape(e.args) + "\"}";
        out += "},\n";
        open_[e.name] = true;
      } else if (e.ph == 'E') {
        if (open_[e.name]) {
          snprintf(b, sizeof b, "{\"ph\": \"E\", \"pid\": %d, \"tid\": 1, \"ts\": %lld},\n", pid,
                   (long long)e.ts);
          out += b;
          open_[e.name] = false;
        }
      } else if (e.ph == 'X') {
        out += "{\"name\": \"" + json_escape(e.phase) + "\", \"ph\": \"X\", \"pid\": " +
               std::to_string(pid) + ", \"tid\": 2, \"ts\": " + std::to_string(e.ts) +
               ", \"dur\": " + std::to_string(e.dur) + "},\n";
      } else {
        out += "{\"name\": \"" + json_escape(e.phase) + "\", \"ph\": \"i\", \"s\": \"p\", \"pid\": " +
               std::to_string(pid) + ", \"tid\": 1, \"ts\": " + std::to_string(e.ts) + "},\n";
      }
      ++written_;
    }
    if (!out.empty()) {
      fputs(out.c_str(), f_);
      fflush(f_);
    }
    lk.lock();
    if (done && q_.empty()) break;
  }
}

void Timeline::close() {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) return;
    stop_ = true;
  }
  cv_.notify_one();
  if (writer_.joinable()) writer_.join();
  if (f_) {
    fputs("{}]\n", f_);
    fclose(f_);
    f_ = nullptr;
  }
}

}  // namespace mvcore
