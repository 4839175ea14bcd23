// mivod xGMI mesh one-shot allreduce (SURVEY.md §2.5 K7, §2.4 "XgmiMeshTransport").
//
// For small buckets a ring is latency-bound (2(N-1) hops); on a node whose GPUs
// are all point-to-point connected by xGMI, every rank can instead read every
// peer's copy directly and reduce locally — one hop.  Each rank owns a
// double-buffered staging area and an N-slot flag array in device memory
// allocated uncached (stores reach HBM, remote reads never see stale lines) and
// exported with HIP IPC; every rank maps every peer's area.
//
// allreduce(epoch e):
//   1. copy the input into this rank's staging slot e&1 (kernel boundary);
//   2. the reduce kernel's block 0 publishes e into slot [rank] of every peer's
//      flag array (system-scope release);
//   3. every block waits (bounded spin, s_sleep backoff) until its own flag
//      array shows e from every peer (system-scope acquire), then sums the N
//      staging copies in FIXED rank order 0..N-1 in fp32 and writes the result —
//      so every rank produces bit-identical output, deterministically.
// Slot reuse is safe without a second barrier: epoch e+2 reuses slot e&1 only
// after this rank's e+1 reduce saw every peer arrive at e+1, which each peer
// signals after its own e reduce (same stream) finished reading.
// A spin that exceeds the bound writes a status word and exits (no GPU hang).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace mvcomm {

class Mesh {
 public:
  Mesh(int rank, int size, int device, size_t capacity_bytes);
  ~Mesh();
  Mesh(const Mesh&) = delete;
  Mesh& operator=(const Mesh&) = delete;

  static constexpr int kMaxRanks = 16;
  // this rank's exported IPC handles (staging area, flag array): 2 x 64 bytes
  std::string handles() const;
  // every rank's handles, indexed by rank (own entry ignored)
  void open(const std::vector<std::string>& all);

  // dtype: 0 fp32, 1 bf16, 2 fp16.  out = scale * sum over ranks of in.
  void allreduce(const void* in, void* out, size_t count, int dtype, float scale,
                 uintptr_t stream);
  // 0 = ok; 1 = a peer did not arrive within the spin bound (synchronous read)
  int status() const;

  size_t capacity() const { return cap_; }
  int rank() const { return rank_; }
  int size() const { return size_; }
  int64_t calls() const { return calls_; }
  int64_t bytes() const { return bytes_; }
  void close();

 private:
  int rank_, size_, device_;
  size_t cap_;
  char* stage_ = nullptr;        // 2 * cap_ bytes, uncached, exported
  uint64_t* flags_ = nullptr;    // size_ slots, uncached, exported
  int* status_ = nullptr;        // device status word
  std::vector<char*> peer_stage_;
  std::vector<uint64_t*> peer_flags_;
  char** d_peer_stage_ = nullptr;     // device copies of the pointer tables
  uint64_t** d_peer_flags_ = nullptr;
  uint64_t epoch_ = 0;
  int64_t calls_ = 0, bytes_ = 0;
  bool opened_ = false;
};

}  // namespace mvcomm
