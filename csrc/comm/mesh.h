// mivod xGMI mesh allreduce (SURVEY.md §2.5 K7, §2.4 "XgmiMeshTransport").
//
// For small and medium buckets a ring is latency-bound (2(N-1) hops); on a node
// whose GPUs are all point-to-point connected by xGMI every rank can instead
// read its peers' copies directly.  Each rank owns, in device memory allocated
// uncached (stores reach HBM, remote readers never see stale lines) and
// exported with HIP IPC:
//   * a double-buffered STAGING area (the bucket's input; the pack kernel can
//     write straight into it — stage_ptr() — so no extra copy is made),
//   * a double-buffered RESULT area (two-shot only),
//   * an N-slot FLAG array: slot p holds the last barrier sequence number rank
//     p has published to this rank.
// Every rank maps every peer's three areas.
//
// Barrier (inside a kernel): block 0 publishes `seq` into slot [rank] of every
// peer's flag array (system-scope release); every block then waits until its
// own flag array shows >= seq from every peer.  The wait is bounded by a
// wall-clock timeout (wall_clock64 ticks): a peer that does not arrive makes
// the kernel write NaN into the output (never the local gradient), set a
// host-mapped status word, and exit — a watcher thread sees that word within
// ~20 ms and, by default, ends the process with a diagnosis (the epochs of the
// ranks are out of step after a timeout, so there is nothing to resume).
//
// one-shot (small buckets): barrier; every rank sums the N staging copies in
//   FIXED rank order 0..N-1 in fp32 — each link carries the whole bucket once.
// two-shot (medium buckets): barrier; rank r reduces only its 1/N chunk (same
//   fixed order) into its RESULT area and the output  [kernel boundary]
//   barrier; rank r copies every peer's reduced chunk from the peer's RESULT
//   area — each link carries 2/N of the bucket (reduce-scatter + all-gather
//   over the mesh).
// Both produce the same bits as each other and on every rank (deterministic).
//
// Slot reuse is safe without extra barriers: call e+2 reuses slot e&1 only after
// this rank's call e+1 saw every peer publish a sequence number of call e+1,
// which each peer does after its own call-e kernels (same stream) finished
// reading this rank's areas.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <string>
#include <thread>
#include <vector>

namespace mvcomm {

class Mesh {
 public:
  // timeout_s: how long a kernel waits for a peer before failing loudly;
  // exit_on_timeout: the watcher ends the process (default) instead of only
  // marking the mesh failed (then every later call throws).
  Mesh(int rank, int size, int device, size_t capacity_bytes, double timeout_s = 30.0,
       bool exit_on_timeout = true);
  ~Mesh();
  Mesh(const Mesh&) = delete;
  Mesh& operator=(const Mesh&) = delete;

  static constexpr int kMaxRanks = 16;
  // this rank's exported IPC handles (staging, result, flags): 3 x 64 bytes
  std::string handles() const;
  // every rank's handles, indexed by rank (own entry ignored)
  void open(const std::vector<std::string>& all);

  // Device address of the staging slot the NEXT allreduce reads: a producer
  // (the bucket pack kernel) that writes its output here saves the copy.
  uintptr_t stage_ptr() const;

  // dtype: 0 fp32, 1 bf16, 2 fp16.  out = scale * sum over ranks of in.
  // algo: 0 auto (one-shot up to oneshot_max_bytes, two-shot above), 1 one-shot,
  // 2 two-shot.  `in` may be stage_ptr() (no staging copy).
  void allreduce(const void* in, void* out, size_t count, int dtype, float scale,
                 uintptr_t stream, int algo = 0);
  // 0 = ok; 1 = a peer did not arrive within the timeout (host-mapped word, no sync)
  int status() const;
  bool failed() const { return failed_; }

  size_t capacity() const { return cap_; }
  int rank() const { return rank_; }
  int size() const { return size_; }
  int64_t calls() const { return calls_; }
  int64_t bytes() const { return bytes_; }
  int64_t copies_saved() const { return copies_saved_; }
  int64_t two_shot_calls() const { return two_shot_; }
  size_t oneshot_max_bytes() const { return oneshot_max_; }
  void set_oneshot_max_bytes(size_t b) { oneshot_max_ = b; }
  double timeout_s() const { return timeout_s_; }
  void close();

 private:
  void watch();

  int rank_, size_, device_;
  size_t cap_;
  size_t oneshot_max_ = 1u << 20;
  double timeout_s_;
  bool exit_on_timeout_;
  int64_t timeout_ticks_ = 0;
  char* stage_ = nullptr;        // 2 * cap_ bytes, uncached, exported
  char* result_ = nullptr;       // 2 * cap_ bytes, uncached, exported (two-shot)
  uint64_t* flags_ = nullptr;    // kMaxRanks slots, uncached, exported
  int* status_host_ = nullptr;   // host-mapped, coherent: written by the kernels
  int* status_dev_ = nullptr;    // its device address
  std::vector<char*> peer_stage_, peer_result_;
  std::vector<uint64_t*> peer_flags_;
  char** d_peer_stage_ = nullptr;     // device copies of the pointer tables
  char** d_peer_result_ = nullptr;
  uint64_t** d_peer_flags_ = nullptr;
  uint64_t epoch_ = 0;                // calls issued (slot parity)
  uint64_t seq_ = 0;                  // barrier sequence numbers issued
  int64_t calls_ = 0, bytes_ = 0, copies_saved_ = 0, two_shot_ = 0;
  bool opened_ = false;
  std::atomic<bool> failed_{false};
  std::atomic<bool> stop_{false};
  std::thread watcher_;
};

}  // namespace mvcomm
