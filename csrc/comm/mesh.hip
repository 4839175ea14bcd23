// xGMI mesh allreduce (one-shot / two-shot): see mesh.h for the protocol.
#include "mesh.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>

#include "../kernels/mv_common.h"

namespace mvcomm {

#define MESH_HIP(call)                                                                   \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess)                                                                \
      throw std::runtime_error(std::string("mivod mesh: ") + #call + ": " +              \
                               hipGetErrorString(e_));                                   \
  } while (0)

namespace {

using mv::kVec;
constexpr int kThreads = 256;
constexpr int kMaxGrid = 256;

struct Peers {
  char* const* stage;      // [n] staging base of every rank (own included)
  char* const* result;     // [n] result base of every rank
  uint64_t* const* flags;  // [n] flag array of every rank
  uint64_t* mine;          // this rank's flag array
  int* status;             // host-mapped status word
  int rank, n;
  int64_t timeout_ticks;
};

// Publish `seq` to every peer (block 0), then wait (every block, thread 0) until
// every peer has published >= seq to us, bounded by the wall-clock timeout.
// Returns false on timeout (status word set).
__device__ bool mesh_barrier(const Peers& P, uint64_t seq) {
  if (blockIdx.x == 0 && (int)threadIdx.x < P.n && (int)threadIdx.x != P.rank) {
    __threadfence_system();
    __hip_atomic_store(&P.flags[threadIdx.x][P.rank], seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    int good = 1;
    for (int p = 0; p < P.n && good; ++p) {
      if (p == P.rank) continue;
      while (__hip_atomic_load(&P.mine[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
        __builtin_amdgcn_s_sleep(8);
        if (wall_clock64() - t0 > P.timeout_ticks) {
          good = 0;
          break;
        }
      }
    }
    if (!good) __hip_atomic_store(P.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

// out[v*8 .. v*8+8) for v in [v0, v1) (+ the scalar tail [t0, t1)) = NaN: a
// failed barrier never leaves the local gradient in the output.
template <typename T>
__device__ void poison(T* out, int64_t v0, int64_t v1, int64_t t0, int64_t t1) {
  float nan8[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) nan8[j] = __builtin_nanf("");
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t v = v0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; v < v1; v += stride)
    mv::store8(out + v * kVec, nan8);
  if (blockIdx.x == 0)
    for (int64_t i = t0 + threadIdx.x; i < t1; i += kThreads) mv::st1(out + i, nan8[0]);
}

// fixed-order (rank 0..n-1) fp32 sum of the staged copies over vectors [v0, v1)
// and the scalar tail [t0, t1); written to out (and to res when non-null)
template <typename T>
__device__ void reduce_range(const Peers& P, size_t slot, float scale, T* out, T* res,
                             int64_t v0, int64_t v1, int64_t t0, int64_t t1) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t v = v0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; v < v1; v += stride) {
    const int64_t i = v * kVec;
    float acc[8], x[8];
    mv::load8(reinterpret_cast<const T*>(P.stage[0] + slot) + i, acc);
    for (int p = 1; p < P.n; ++p) {
      mv::load8(reinterpret_cast<const T*>(P.stage[p] + slot) + i, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= scale;
    mv::store8(out + i, acc);
    if (res != nullptr) mv::store8(res + i, acc);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = t0 + threadIdx.x; i < t1; i += kThreads) {
      float acc = 0.f;
      for (int p = 0; p < P.n; ++p) acc += mv::ld1(reinterpret_cast<const T*>(P.stage[p] + slot) + i);
      mv::st1(out + i, acc * scale);
      if (res != nullptr) mv::st1(res + i, acc * scale);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void mesh_oneshot_kernel(Peers P, uint64_t seq,
                                                                 size_t slot, T* __restrict__ out,
                                                                 int64_t count, float scale) {
  const int64_t nvec = count / kVec;
  if (!mesh_barrier(P, seq)) {
    poison(out, 0, nvec, nvec * kVec, count);
    return;
  }
  reduce_range<T>(P, slot, scale, out, nullptr, 0, nvec, nvec * kVec, count);
}

// rank r's chunk, in whole 8-element vectors: [r*cv, min((r+1)*cv, nvec)); the
// last rank also owns the scalar tail
__device__ __forceinline__ void chunk_of(int r, int n, int64_t count, int64_t& v0, int64_t& v1,
                                         int64_t& t0, int64_t& t1) {
  const int64_t nvec = count / kVec;
  const int64_t cv = (nvec + n - 1) / n;
  v0 = std::min<int64_t>((int64_t)r * cv, nvec);
  v1 = std::min<int64_t>(v0 + cv, nvec);
  t0 = t1 = nvec * kVec;
  if (r == n - 1) t1 = count;
}

template <typename T>
__global__ __launch_bounds__(kThreads) void mesh_rs_kernel(Peers P, uint64_t seq, size_t slot,
                                                            T* __restrict__ out, int64_t count,
                                                            float scale) {
  if (!mesh_barrier(P, seq)) {
    const int64_t nvec = count / kVec;
    poison(out, 0, nvec, nvec * kVec, count);
    return;
  }
  int64_t v0, v1, t0, t1;
  chunk_of(P.rank, P.n, count, v0, v1, t0, t1);
  reduce_range<T>(P, slot, scale, out, reinterpret_cast<T*>(P.result[P.rank] + slot), v0, v1,
                  t0, t1);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void mesh_ag_kernel(Peers P, uint64_t seq, size_t slot,
                                                            T* __restrict__ out, int64_t count) {
  const int64_t nvec = count / kVec;
  if (!mesh_barrier(P, seq)) {
    poison(out, 0, nvec, nvec * kVec, count);
    return;
  }
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int p = 0; p < P.n; ++p) {
    if (p == P.rank) continue;
    int64_t v0, v1, t0, t1;
    chunk_of(p, P.n, count, v0, v1, t0, t1);
    const T* src = reinterpret_cast<const T*>(P.result[p] + slot);
    for (int64_t v = v0 + (int64_t)blockIdx.x * kThreads + threadIdx.x; v < v1; v += stride) {
      const int64_t i = v * kVec;
      *reinterpret_cast<uint4*>(out + i) = *reinterpret_cast<const uint4*>(src + i);
      if (sizeof(T) == 4)
        *reinterpret_cast<uint4*>(out + i + 4) = *reinterpret_cast<const uint4*>(src + i + 4);
    }
    if (blockIdx.x == 0)
      for (int64_t i = t0 + threadIdx.x; i < t1; i += kThreads) out[i] = src[i];
  }
}

void* alloc_shared(size_t bytes) {
  void* p = nullptr;
  // uncached: stores reach memory, remote readers never hit stale cache lines
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) return p;
  (void)hipGetLastError();
  MESH_HIP(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
  return p;
}

int grid_for(int64_t nvec) {
  return (int)std::min<int64_t>(kMaxGrid, std::max<int64_t>(1, (nvec + kThreads - 1) / kThreads));
}

}  // namespace

Mesh::Mesh(int rank, int size, int device, size_t capacity_bytes, double timeout_s,
           bool exit_on_timeout)
    : rank_(rank),
      size_(size),
      device_(device),
      cap_((capacity_bytes + 255) / 256 * 256),
      timeout_s_(timeout_s > 0 ? timeout_s : 30.0),
      exit_on_timeout_(exit_on_timeout) {
  if (size < 1 || size > kMaxRanks || rank < 0 || rank >= size)
    throw std::invalid_argument("mivod mesh: 1 <= size <= 16 ranks");
  MESH_HIP(hipSetDevice(device));
  int khz = 0;
  MESH_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  if (khz <= 0) khz = 100000;   // 100 MHz, the CDNA constant-rate clock
  timeout_ticks_ = (int64_t)(timeout_s_ * 1000.0 * khz);
  stage_ = static_cast<char*>(alloc_shared(2 * cap_));
  result_ = static_cast<char*>(alloc_shared(2 * cap_));
  flags_ = static_cast<uint64_t*>(alloc_shared(kMaxRanks * sizeof(uint64_t)));
  MESH_HIP(hipMemset(flags_, 0, kMaxRanks * sizeof(uint64_t)));
  // finite contents from the start: the arena's alignment gaps between a
  // bucket's tensors are never packed, so they reduce whatever the slot held
  // before (identically on every rank) — zeros or earlier finite gradients
  MESH_HIP(hipMemset(stage_, 0, 2 * cap_));
  MESH_HIP(hipMemset(result_, 0, 2 * cap_));
  MESH_HIP(hipHostMalloc(reinterpret_cast<void**>(&status_host_), sizeof(int),
                         hipHostMallocMapped | hipHostMallocCoherent));
  *reinterpret_cast<volatile int*>(status_host_) = 0;
  MESH_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&status_dev_), status_host_, 0));
  MESH_HIP(hipDeviceSynchronize());
  watcher_ = std::thread([this] { watch(); });
}

Mesh::~Mesh() {
  try {
    close();
  } catch (...) {
  }
}

void Mesh::watch() {
  // the kernels never block the host: this thread turns a timed-out barrier
  // into a diagnosis (and, by default, a non-zero exit) within ~20 ms
  while (!stop_) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    if (status_host_ == nullptr) break;
    if (*reinterpret_cast<volatile int*>(status_host_) != 0 && !failed_.exchange(true)) {
      fprintf(stderr,
              "[mivod] rank %d: xGMI mesh allreduce: a peer did not arrive within %.1f s "
              "(dead, stalled or out of step); the output was poisoned with NaN%s\n",
              rank_, timeout_s_, exit_on_timeout_ ? "; exiting" : "");
      fflush(stderr);
      if (exit_on_timeout_) std::_Exit(1);
    }
  }
}

void Mesh::close() {
  stop_ = true;
  if (watcher_.joinable()) watcher_.join();
  if (stage_ == nullptr) return;
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (int p = 0; p < (int)peer_stage_.size(); ++p) {
    if (p == rank_) continue;
    if (peer_stage_[p]) hipIpcCloseMemHandle(peer_stage_[p]);
    if (peer_result_[p]) hipIpcCloseMemHandle(peer_result_[p]);
    if (peer_flags_[p]) hipIpcCloseMemHandle(peer_flags_[p]);
  }
  peer_stage_.clear();
  peer_result_.clear();
  peer_flags_.clear();
  if (d_peer_stage_) hipFree(d_peer_stage_);
  if (d_peer_result_) hipFree(d_peer_result_);
  if (d_peer_flags_) hipFree(d_peer_flags_);
  hipFree(stage_);
  hipFree(result_);
  hipFree(flags_);
  hipHostFree(status_host_);
  stage_ = result_ = nullptr;
  flags_ = nullptr;
  status_host_ = status_dev_ = nullptr;
  d_peer_stage_ = d_peer_result_ = nullptr;
  d_peer_flags_ = nullptr;
  opened_ = false;
}

std::string Mesh::handles() const {
  hipIpcMemHandle_t h[3];
  MESH_HIP(hipIpcGetMemHandle(&h[0], stage_));
  MESH_HIP(hipIpcGetMemHandle(&h[1], result_));
  MESH_HIP(hipIpcGetMemHandle(&h[2], flags_));
  std::string s(sizeof(h), '\0');
  std::memcpy(&s[0], h, sizeof(h));
  return s;
}

void Mesh::open(const std::vector<std::string>& all) {
  if ((int)all.size() != size_) throw std::invalid_argument("mivod mesh: one handle per rank");
  MESH_HIP(hipSetDevice(device_));
  peer_stage_.assign(size_, nullptr);
  peer_result_.assign(size_, nullptr);
  peer_flags_.assign(size_, nullptr);
  for (int p = 0; p < size_; ++p) {
    if (p == rank_) {
      peer_stage_[p] = stage_;
      peer_result_[p] = result_;
      peer_flags_[p] = flags_;
      continue;
    }
    hipIpcMemHandle_t h[3];
    if (all[p].size() != sizeof(h)) throw std::invalid_argument("mivod mesh: bad handle size");
    std::memcpy(h, all[p].data(), sizeof(h));
    void* q[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3; ++k)
      MESH_HIP(hipIpcOpenMemHandle(&q[k], h[k], hipIpcMemLazyEnablePeerAccess));
    peer_stage_[p] = static_cast<char*>(q[0]);
    peer_result_[p] = static_cast<char*>(q[1]);
    peer_flags_[p] = static_cast<uint64_t*>(q[2]);
  }
  MESH_HIP(hipMalloc(&d_peer_stage_, size_ * sizeof(char*)));
  MESH_HIP(hipMalloc(&d_peer_result_, size_ * sizeof(char*)));
  MESH_HIP(hipMalloc(&d_peer_flags_, size_ * sizeof(uint64_t*)));
  MESH_HIP(hipMemcpy(d_peer_stage_, peer_stage_.data(), size_ * sizeof(char*),
                     hipMemcpyHostToDevice));
  MESH_HIP(hipMemcpy(d_peer_result_, peer_result_.data(), size_ * sizeof(char*),
                     hipMemcpyHostToDevice));
  MESH_HIP(hipMemcpy(d_peer_flags_, peer_flags_.data(), size_ * sizeof(uint64_t*),
                     hipMemcpyHostToDevice));
  opened_ = true;
}

uintptr_t Mesh::stage_ptr() const {
  if (!opened_) throw std::logic_error("mivod mesh: open() first");
  return reinterpret_cast<uintptr_t>(stage_ + ((epoch_ + 1) & 1) * cap_);
}

template <typename T>
static void launch(const Peers& P, bool two_shot, uint64_t seq, size_t slot, void* out,
                   int64_t count, float scale, hipStream_t st) {
  T* o = static_cast<T*>(out);
  const int64_t nvec = count / kVec;
  if (!two_shot) {
    hipLaunchKernelGGL((mesh_oneshot_kernel<T>), dim3(grid_for(nvec)), dim3(kThreads), 0, st, P,
                       seq, slot, o, count, scale);
    return;
  }
  const int64_t cv = (nvec + P.n - 1) / P.n;
  hipLaunchKernelGGL((mesh_rs_kernel<T>), dim3(grid_for(cv)), dim3(kThreads), 0, st, P, seq, slot,
                     o, count, scale);
  hipLaunchKernelGGL((mesh_ag_kernel<T>), dim3(grid_for(cv * (P.n - 1))), dim3(kThreads), 0, st,
                     P, seq + 1, slot, o, count);
}

void Mesh::allreduce(const void* in, void* out, size_t count, int dtype, float scale,
                     uintptr_t stream, int algo) {
  if (!opened_) throw std::logic_error("mivod mesh: open() first");
  if (failed_)
    throw std::runtime_error("mivod mesh: a previous allreduce timed out waiting for a peer");
  if (dtype < 0 || dtype > 2) throw std::invalid_argument("mivod mesh: dtype must be fp32 / bf16 / fp16");
  const size_t es = dtype == 0 ? 4 : 2;
  const size_t bytes = count * es;
  if (bytes > cap_) throw std::invalid_argument("mivod mesh: bucket exceeds the staging capacity");
  if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0)
    throw std::invalid_argument("mivod mesh: output must be 16-byte aligned");
  if (count == 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t e = ++epoch_;
  const size_t slot_off = (e & 1) * cap_;
  if (in == stage_ + slot_off) {
    ++copies_saved_;            // the producer wrote straight into the staging slot
  } else {
    MESH_HIP(hipMemcpyAsync(stage_ + slot_off, in, bytes, hipMemcpyDeviceToDevice, st));
  }
  const bool two_shot = size_ > 1 && (algo == 2 || (algo == 0 && bytes > oneshot_max_));
  Peers P{d_peer_stage_, d_peer_result_, d_peer_flags_, flags_, status_dev_, rank_, size_,
          timeout_ticks_};
  const uint64_t seq = seq_ + 1;
  seq_ += two_shot ? 2 : 1;
  switch (dtype) {
    case 0: launch<float>(P, two_shot, seq, slot_off, out, (int64_t)count, scale, st); break;
    case 1: launch<__bf16>(P, two_shot, seq, slot_off, out, (int64_t)count, scale, st); break;
    default: launch<_Float16>(P, two_shot, seq, slot_off, out, (int64_t)count, scale, st); break;
  }
  MESH_HIP(hipGetLastError());
  ++calls_;
  if (two_shot) ++two_shot_;
  bytes_ += (int64_t)bytes;
}

int Mesh::status() const {
  return status_host_ ? *reinterpret_cast<volatile int*>(status_host_) : 0;
}

}  // namespace mvcomm
