// Native test of the CPU ring data plane: N ranks as threads over loopback TCP.
// Built and run under ThreadSanitizer and AddressSanitizer+UBSan by
// tests/test_native_sanitizers.py.  Usage: test_ring <nranks>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../ring.h"

using namespace mvcore;

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                                \
  do {                                                                          \
    if (!(c)) {                                                                 \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                                 \
    }                                                                           \
  } while (0)

int main(int argc, char** argv) {
  const int N = argc > 1 ? std::atoi(argv[1]) : 4;
  std::vector<Ring*> rings(N);
  std::vector<int> ports(N);
  for (int r = 0; r < N; ++r) {
    rings[r] = new Ring(r, N, 30.0);
    ports[r] = rings[r]->listen();
  }
  std::vector<std::thread> th;
  for (int r = 0; r < N; ++r) {
    th.emplace_back([&, r] {
      Ring& R = *rings[r];
      R.connect("127.0.0.1", ports[(r + 1) % N]);
      // fp32 sum, uneven chunking
      for (int64_t cnt : {0L, 1L, 5L, 1000L, 262147L}) {
        std::vector<float> v(cnt);
        for (int64_t i = 0; i < cnt; ++i) v[i] = (float)(r + 1) * (float)(i % 7);
        R.allreduce(v.data(), cnt, kF32, false);
        const float tot = (float)(N * (N + 1) / 2);
        for (int64_t i = 0; i < cnt; ++i) CHECK(v[i] == tot * (float)(i % 7));
      }
      std::vector<double> d(33, (double)r);
      R.allreduce(d.data(), 33, kF64, true);
      for (double x : d) CHECK(std::fabs(x - (N - 1) / 2.0) < 1e-12);
      std::vector<int64_t> k(9, r);
      R.allreduce(k.data(), 9, kI64, false);
      for (int64_t x : k) CHECK(x == (int64_t)N * (N - 1) / 2);
      // broadcast from every root, 2.5 MiB (spans pipeline segments)
      for (int root = 0; root < N; ++root) {
        std::vector<int32_t> b((5 << 20) / 8, r == root ? 7 + root : -1);
        R.broadcast(b.data(), (int64_t)b.size() * 4, root);
        for (int32_t x : b) CHECK(x == 7 + root);
      }
      // ragged allgather
      std::vector<int64_t> bytes(N);
      int64_t total = 0;
      for (int q = 0; q < N; ++q) {
        bytes[q] = 3 * (q + 1);
        total += bytes[q];
      }
      std::vector<char> in(bytes[r], (char)('a' + r)), out(total);
      R.allgatherv(in.data(), out.data(), bytes);
      int64_t o = 0;
      for (int q = 0; q < N; ++q)
        for (int64_t i = 0; i < bytes[q]; ++i) CHECK(out[o++] == (char)('a' + q));
      R.barrier();
    });
  }
  for (auto& t : th) t.join();
  for (auto* p : rings) delete p;
  // host reducer: fp16 / bf16 spot checks (1 + 2 = 3 exactly representable)
  uint16_t h1[9], h2[9];
  for (int i = 0; i < 9; ++i) {
    h1[i] = 0x3c00;  // fp16 1.0
    h2[i] = 0x4000;  // fp16 2.0
  }
  ring_reduce_sum(h1, h2, 9, kF16);
  for (int i = 0; i < 9; ++i) CHECK(h1[i] == 0x4200);  // 3.0
  uint16_t b1[3] = {0x3f80, 0x3f80, 0x3f80}, b2[3] = {0x4000, 0x4000, 0x4000};  // bf16 1, 2
  ring_reduce_sum(b1, b2, 3, kBF16);
  for (int i = 0; i < 3; ++i) CHECK(b1[i] == 0x4040);  // 3.0
  if (g_fail) {
    std::printf("FAILED %d\n", g_fail.load());
    return 1;
  }
  std::printf("OK ring %d ranks\n", N);
  return 0;
}
