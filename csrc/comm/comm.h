// mivod GPU data plane: an RCCL communicator owned by mivod (not torch's
// ProcessGroupNCCL), driven from C++ on mivod's HIP comm stream.
//
// Parity: horovod 0.18.1 ops/nccl_operations.cc NCCLAllreduce /
// NCCLHierarchicalAllreduce + the lazily created NCCL communicator
// (call sites C1/C5/C6), re-designed for MI355X:
//   * one communicator per process, created eagerly at mivod.init() from a
//     unique id that rank 0 publishes through the rendezvous store;
//   * every collective is enqueued on the caller's HIP stream (the high-priority
//     comm stream) — the host never waits;
//   * Average is ncclAvg, a folded 1/N pre-scale is ncclRedOpCreatePreMulSum;
//   * Adasum's vector-halving exchange is grouped ncclSend/ncclRecv;
//   * hierarchical allreduce uses ncclCommSplit intra-/cross-node comms;
//   * a watchdog thread polls ncclCommGetAsyncError and the age of the oldest
//     unfinished collective (hipEvent per op) and calls ncclCommAbort after the
//     stall-shutdown time, so a dead peer ends the job instead of hanging it.
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace mvcomm {

std::string unique_id();   // 128 raw bytes (NCCL_UNIQUE_ID_BYTES)
int rccl_version();
// "" when the RCCL library loaded at run time matches the header this module was
// compiled against (major.minor), else a one-line description of the skew
std::string version_note();
// features gated on the run-time library version (not the header's)
bool runtime_has_ctas_config();   // ncclConfig_t minCTAs / maxCTAs (NCCL >= 2.17)
bool runtime_has_fp8();           // ncclFloat8e4m3 / e5m2 codes 10 / 11 (NCCL >= 2.24)

struct CommStats {
  int64_t calls = 0;
  int64_t bytes = 0;          // payload bytes handed to RCCL (per rank, not wire bytes)
  int64_t completed = 0;
};

class Comm {
 public:
  // Collective: every rank of the communicator calls it with the same arguments.
  // min_ctas / max_ctas > 0: ncclCommInitRankConfig with that CTA (channel) range
  Comm(const std::string& uid, int rank, int size, int device, double timeout_s,
       bool exit_on_abort, int min_ctas = 0, int max_ctas = 0);
  ~Comm();
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;

  int rank() const { return rank_; }

  int min_ctas() const { return min_ctas_; }

  int max_ctas() const { return max_ctas_; }
  int size() const { return size_; }
  int device() const { return device_; }
  // ncclCommCount: the number of ranks RCCL itself sees in this communicator
  int count() const;

  // op: ncclRedOp_t value (ncclSum/ncclProd/ncclMax/ncclMin/ncclAvg).
  void allreduce(const void* in, void* out, size_t count, int dtype, int op, uintptr_t stream);
  // sum of (scale * x) across ranks: the averaging factor rides inside RCCL.
  void allreduce_premul(const void* in, void* out, size_t count, int dtype, double scale,
                        uintptr_t stream);
  void reduce_scatter(const void* in, void* out, size_t recvcount, int dtype, int op,
                      uintptr_t stream);
  void allgather(const void* in, void* out, size_t sendcount, int dtype, uintptr_t stream);
  void broadcast(const void* in, void* out, size_t count, int dtype, int root, uintptr_t stream);
  // one grouped send+recv with `peer` (Adasum level exchange)
  void sendrecv(const void* sbuf, size_t scount, void* rbuf, size_t rcount, int dtype, int peer,
                uintptr_t stream);
  // all-to-all with per-peer counts / element displacements
  void alltoallv(const void* sbuf, const std::vector<size_t>& scounts,
                 const std::vector<size_t>& sdispls, void* rbuf,
                 const std::vector<size_t>& rcounts, const std::vector<size_t>& rdispls,
                 int dtype, uintptr_t stream);

  // ncclCommSplit: collective over this comm; ranks with equal `color` form a comm.
  std::unique_ptr<Comm> split(int color, int key);

  // raise if the watchdog / RCCL reported an error
  void check() const;
  std::string error() const;
  void abort(const std::string& why);
  void destroy();     // ncclCommDestroy after the streams drained (shutdown)

  CommStats stats() const;
  int outstanding() const;

 private:
  Comm() = default;
  void track(hipStream_t s, size_t bytes, const char* what);
  void start_watchdog();
  void watchdog_loop();
  static size_t dtype_size(int dtype);

  ncclComm_t comm_ = nullptr;
  int rank_ = 0, size_ = 1, device_ = 0;
  int min_ctas_ = 0, max_ctas_ = 0;
  double timeout_s_ = 0.0;
  bool exit_on_abort_ = false;

  struct Pending {
    hipEvent_t ev;
    std::chrono::steady_clock::time_point t;
    const char* what;
  };
  mutable std::mutex mu_;
  std::deque<Pending> pending_;
  std::vector<hipEvent_t> free_events_;
  CommStats stats_;
  std::string error_;
  std::atomic<bool> aborted_{false};
  std::atomic<bool> stop_{false};
  std::condition_variable cv_;
  std::thread watchdog_;
};

}  // namespace mvcomm
