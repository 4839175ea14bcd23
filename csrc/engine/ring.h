// mivod native CPU data plane: bandwidth-optimal ring collectives over TCP.
//
// Parity: horovod 0.18.1 ops/mpi_operations.cc (MPIAllreduce / MPIAllgather /
// MPIBroadcast for CPU tensors) and common/half.cc (the float16 MPI sum op),
// SURVEY.md §2.2 U9/U12 and §2.4 "CPU data plane: TcpRingTransport".  No MPI:
// every rank keeps two persistent sockets (to its ring successor, from its
// predecessor); allreduce is reduce-scatter + allgather around the ring
// (2(N-1)/N of the buffer on the wire per rank), with each step full-duplex
// (poll-driven non-blocking send + receive).  fp16 is summed through F16C
// (8 lanes per instruction, fp32 accumulate), bf16 through fp32 with
// round-to-nearest-even.  Used for CPU tensors (the gloo-free world that runs
// the multi-rank tests on GPU-less hosts); GPU tensors ride RCCL.
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

namespace mvcore {

enum RingDtype : int { kF32 = 0, kF64 = 1, kF16 = 2, kBF16 = 3, kI32 = 4, kI64 = 5, kU8 = 6, kI8 = 7 };

int ring_dtype_size(int dtype);

class Ring {
 public:
  // per-step I/O timeout once connected (HOROVOD_STALL_SHUTDOWN_TIME_SECONDS):
  // a dead or stalled peer raises on every surviving rank instead of hanging
  void set_timeout(double s) { timeout_s_ = s; }
  Ring(int rank, int size, double timeout_s = 300.0);
  ~Ring();
  Ring(const Ring&) = delete;
  Ring& operator=(const Ring&) = delete;

  // bind an ephemeral port on all interfaces; returns it (publish to the ring)
  int listen();
  // connect to the successor, then accept the predecessor (listen() first, on all ranks)
  void connect(const std::string& next_host, int next_port);

  // in-place sum over all ranks of `count` elements (average: divide floats by size)
  void allreduce(void* data, int64_t count, int dtype, bool average);
  // out = concat over ranks of each rank's block; bytes[r] = size of rank r's block
  void allgatherv(const void* in, void* out, const std::vector<int64_t>& bytes);
  // root's `bytes` bytes to every rank (pipelined along the ring)
  void broadcast(void* data, int64_t bytes, int root);
  void barrier();
  void close();

  int rank() const { return rank_; }
  int size() const { return size_; }
  int64_t bytes_sent() const { return bytes_sent_; }

 private:
  void sendrecv(const void* sbuf, size_t sbytes, void* rbuf, size_t rbytes);
  void send_all(const void* buf, size_t n);
  void recv_all(void* buf, size_t n);

  int rank_, size_;
  double timeout_s_;
  int lfd_ = -1, next_fd_ = -1, prev_fd_ = -1;
  std::vector<char> tmp_;
  int64_t bytes_sent_ = 0;
  std::mutex mu_;
};

// dst[i] += src[i] for `count` elements of `dtype` (exposed for tests)
void ring_reduce_sum(void* dst, const void* src, int64_t count, int dtype);

}  // namespace mvcore
