// Native tier-1 test of the coordinator (built with -fsanitize=thread or
// address,undefined by tests/test_native_sanitizers.py): N ranks as threads,
// each with its own Controller over localhost TCP.  Every rank submits the same
// names in a different order, spread over several cycles, with one mismatched
// tensor; all ranks must receive the identical ordered, fused response stream,
// the mismatch must come back as an error on every rank, and shutdown must
// complete.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <random>
#include <thread>
#include <vector>

#include "../controller.h"

using namespace mvcore;

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 4;
  const int T = 40;  // tensors
  std::atomic<int> port{0};
  std::vector<std::vector<std::string>> streams(N);
  std::vector<int> errors(N, 0);
  std::vector<std::thread> th;
  for (int r = 0; r < N; ++r) {
    th.emplace_back([&, r] {
      ControllerConfig cfg;
      cfg.rank = r;
      cfg.size = N;
      cfg.fusion_threshold = 64 * 10;   // fuse at most 10 x 64-byte tensors
      cfg.stall_check_s = 5;
      Controller c(cfg);
      if (r == 0) port = c.listen();
      while (port.load() == 0) std::this_thread::yield();
      c.connect("127.0.0.1", port.load());
      std::vector<int> order(T);
      for (int i = 0; i < T; ++i) order[i] = i;
      std::mt19937 g(1234 + r);
      std::shuffle(order.begin(), order.end(), g);
      size_t next = 0;
      int done = 0;
      bool all = false;
      for (int cycle = 0; cycle < 10000 && !all; ++cycle) {
        std::vector<Request> reqs;
        for (int k = 0; k < 7 && next < order.size(); ++k, ++next) {
          Request q;
          q.name = "t" + std::to_string(order[next]);
          q.kind = ALLREDUCE;
          q.dtype = "f32";
          q.shape = {16};
          if (order[next] == 7 && r == N - 1) q.shape = {17};  // mismatch
          q.nbytes = 64;
          q.device = 0;
          reqs.push_back(q);
        }
        bool want_shutdown = next == order.size() && done >= T;
        auto resp = c.negotiate(reqs, want_shutdown, &all);
        for (auto& rs : resp) {
          std::string s;
          for (auto& n : rs.names) s += n + ",";
          if (!rs.error.empty()) {
            errors[r]++;
            s = "ERR:" + s;
          }
          streams[r].push_back(s);
          done += (int)rs.names.size();
        }
      }
      c.close();
    });
  }
  for (auto& t : th) t.join();
  int rc = 0;
  for (int r = 1; r < N; ++r)
    if (streams[r] != streams[0]) {
      fprintf(stderr, "rank %d saw a different response stream\n", r);
      rc = 1;
    }
  int total = 0;
  bool fused = false;
  for (auto& s : streams[0]) {
    total += (int)std::count(s.begin(), s.end(), ',');
    fused |= std::count(s.begin(), s.end(), ',') > 1;
  }
  if (total != T) { fprintf(stderr, "expected %d names, got %d\n", T, total); rc = 1; }
  if (!fused) { fprintf(stderr, "no fused response seen\n"); rc = 1; }
  for (int r = 0; r < N; ++r)
    if (errors[r] != 1) { fprintf(stderr, "rank %d errors=%d (want 1)\n", r, errors[r]); rc = 1; }
  printf(rc ? "FAIL\n" : "OK %zu responses\n", streams[0].size());
  return rc;
}
