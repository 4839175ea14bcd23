// xGMI mesh one-shot allreduce: see mesh.h for the protocol.
#include "mesh.h"

#include <algorithm>
#include <cstring>
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
// ~30 s of s_sleep(8) polls: far beyond any legitimate skew between ranks
// (a peer still running its backward), short enough that a dead peer ends the
// kernel instead of the GPU.
constexpr uint64_t kSpinLimit = 120000000ull;

template <typename T>
__global__ __launch_bounds__(kThreads) void mesh_reduce_kernel(
    char* const* __restrict__ peer_stage, uint64_t* const* __restrict__ peer_flags,
    uint64_t* __restrict__ my_flags, int* __restrict__ status, int rank, int n, uint64_t epoch,
    size_t slot_off, T* __restrict__ out, int64_t count, float scale) {
  // 1. publish this rank's arrival into every peer's flag array
  if (blockIdx.x == 0 && threadIdx.x < n && (int)threadIdx.x != rank) {
    __threadfence_system();
    __hip_atomic_store(&peer_flags[threadIdx.x][rank], epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 2. wait until every peer has published this epoch (bounded)
  __shared__ int ok;
  if (threadIdx.x == 0) {
    int good = 1;
    for (int p = 0; p < n && good; ++p) {
      if (p == rank) continue;
      uint64_t spins = 0;
      while (__hip_atomic_load(&my_flags[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) <
             epoch) {
        __builtin_amdgcn_s_sleep(8);
        if (++spins > kSpinLimit) {
          good = 0;
          break;
        }
      }
    }
    if (!good) status[0] = 1;
    __threadfence_system();
    ok = good;
  }
  __syncthreads();
  if (!ok) return;
  // 3. fixed-order fp32 sum of the N staged copies
  const int64_t nvec = count / kVec;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t v = (int64_t)blockIdx.x * kThreads + threadIdx.x; v < nvec; v += stride) {
    const int64_t i = v * kVec;
    float acc[8], x[8];
    mv::load8(reinterpret_cast<const T*>(peer_stage[0] + slot_off) + i, acc);
    for (int p = 1; p < n; ++p) {
      mv::load8(reinterpret_cast<const T*>(peer_stage[p] + slot_off) + i, x);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] *= scale;
    mv::store8(out + i, acc);
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nvec * kVec + threadIdx.x; i < count; i += kThreads) {
      float acc = 0.f;
      for (int p = 0; p < n; ++p) acc += mv::ld1(reinterpret_cast<const T*>(peer_stage[p] + slot_off) + i);
      mv::st1(out + i, acc * scale);
    }
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

}  // namespace

Mesh::Mesh(int rank, int size, int device, size_t capacity_bytes)
    : rank_(rank), size_(size), device_(device), cap_((capacity_bytes + 255) / 256 * 256) {
  if (size < 1 || size > kMaxRanks || rank < 0 || rank >= size)
    throw std::invalid_argument("mivod mesh: 1 <= size <= 16 ranks");
  MESH_HIP(hipSetDevice(device));
  stage_ = static_cast<char*>(alloc_shared(2 * cap_));
  flags_ = static_cast<uint64_t*>(alloc_shared(kMaxRanks * sizeof(uint64_t)));
  MESH_HIP(hipMemset(flags_, 0, kMaxRanks * sizeof(uint64_t)));
  MESH_HIP(hipMalloc(&status_, sizeof(int)));
  MESH_HIP(hipMemset(status_, 0, sizeof(int)));
  MESH_HIP(hipDeviceSynchronize());
}

Mesh::~Mesh() {
  try {
    close();
  } catch (...) {
  }
}

void Mesh::close() {
  if (stage_ == nullptr) return;
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (int p = 0; p < (int)peer_stage_.size(); ++p) {
    if (p == rank_) continue;
    if (peer_stage_[p]) hipIpcCloseMemHandle(peer_stage_[p]);
    if (peer_flags_[p]) hipIpcCloseMemHandle(peer_flags_[p]);
  }
  peer_stage_.clear();
  peer_flags_.clear();
  if (d_peer_stage_) hipFree(d_peer_stage_);
  if (d_peer_flags_) hipFree(d_peer_flags_);
  hipFree(stage_);
  hipFree(flags_);
  hipFree(status_);
  stage_ = nullptr;
  flags_ = nullptr;
  status_ = nullptr;
  d_peer_stage_ = nullptr;
  d_peer_flags_ = nullptr;
  opened_ = false;
}

std::string Mesh::handles() const {
  hipIpcMemHandle_t a, b;
  MESH_HIP(hipIpcGetMemHandle(&a, stage_));
  MESH_HIP(hipIpcGetMemHandle(&b, flags_));
  std::string s(sizeof(a) + sizeof(b), '\0');
  std::memcpy(&s[0], &a, sizeof(a));
  std::memcpy(&s[sizeof(a)], &b, sizeof(b));
  return s;
}

void Mesh::open(const std::vector<std::string>& all) {
  if ((int)all.size() != size_) throw std::invalid_argument("mivod mesh: one handle per rank");
  MESH_HIP(hipSetDevice(device_));
  peer_stage_.assign(size_, nullptr);
  peer_flags_.assign(size_, nullptr);
  for (int p = 0; p < size_; ++p) {
    if (p == rank_) {
      peer_stage_[p] = stage_;
      peer_flags_[p] = flags_;
      continue;
    }
    hipIpcMemHandle_t a, b;
    if (all[p].size() != sizeof(a) + sizeof(b))
      throw std::invalid_argument("mivod mesh: bad handle size");
    std::memcpy(&a, all[p].data(), sizeof(a));
    std::memcpy(&b, all[p].data() + sizeof(a), sizeof(b));
    void* sp = nullptr;
    void* fp = nullptr;
    MESH_HIP(hipIpcOpenMemHandle(&sp, a, hipIpcMemLazyEnablePeerAccess));
    MESH_HIP(hipIpcOpenMemHandle(&fp, b, hipIpcMemLazyEnablePeerAccess));
    peer_stage_[p] = static_cast<char*>(sp);
    peer_flags_[p] = static_cast<uint64_t*>(fp);
  }
  MESH_HIP(hipMalloc(&d_peer_stage_, size_ * sizeof(char*)));
  MESH_HIP(hipMalloc(&d_peer_flags_, size_ * sizeof(uint64_t*)));
  MESH_HIP(hipMemcpy(d_peer_stage_, peer_stage_.data(), size_ * sizeof(char*),
                     hipMemcpyHostToDevice));
  MESH_HIP(hipMemcpy(d_peer_flags_, peer_flags_.data(), size_ * sizeof(uint64_t*),
                     hipMemcpyHostToDevice));
  opened_ = true;
}

void Mesh::allreduce(const void* in, void* out, size_t count, int dtype, float scale,
                     uintptr_t stream) {
  if (!opened_) throw std::logic_error("mivod mesh: open() first");
  const size_t es = dtype == 0 ? 4 : 2;
  const size_t bytes = count * es;
  if (bytes > cap_) throw std::invalid_argument("mivod mesh: bucket exceeds the staging capacity");
  if ((reinterpret_cast<uintptr_t>(out) & 15u) != 0)
    throw std::invalid_argument("mivod mesh: output must be 16-byte aligned");
  if (count == 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint64_t e = ++epoch_;
  const size_t slot_off = (e & 1) * cap_;
  MESH_HIP(hipMemcpyAsync(stage_ + slot_off, in, bytes, hipMemcpyDeviceToDevice, st));
  const int64_t nvec = (int64_t)(count / kVec);
  int grid = (int)std::min<int64_t>(256, std::max<int64_t>(1, (nvec + kThreads - 1) / kThreads));
  switch (dtype) {
    case 0:
      hipLaunchKernelGGL((mesh_reduce_kernel<float>), dim3(grid), dim3(kThreads), 0, st,
                         d_peer_stage_, d_peer_flags_, flags_, status_, rank_, size_, e, slot_off,
                         (float*)out, (int64_t)count, scale);
      break;
    case 1:
      hipLaunchKernelGGL((mesh_reduce_kernel<__bf16>), dim3(grid), dim3(kThreads), 0, st,
                         d_peer_stage_, d_peer_flags_, flags_, status_, rank_, size_, e, slot_off,
                         (__bf16*)out, (int64_t)count, scale);
      break;
    case 2:
      hipLaunchKernelGGL((mesh_reduce_kernel<_Float16>), dim3(grid), dim3(kThreads), 0, st,
                         d_peer_stage_, d_peer_flags_, flags_, status_, rank_, size_, e, slot_off,
                         (_Float16*)out, (int64_t)count, scale);
      break;
    default:
      throw std::invalid_argument("mivod mesh: dtype must be fp32 / bf16 / fp16");
  }
  MESH_HIP(hipGetLastError());
  ++calls_;
  bytes_ += (int64_t)bytes;
}

int Mesh::status() const {
  int s = 0;
  MESH_HIP(hipMemcpy(&s, status_, sizeof(int), hipMemcpyDeviceToHost));
  return s;
}

}  // namespace mvcomm
