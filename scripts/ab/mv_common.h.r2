// mivod CDNA4 (gfx950) kernel helpers: dtype tags, 8-wide vector load/store
// with fused conversion, wave64 reductions.
//
// Every memory-bound mivod kernel moves 8 elements per lane per step: 16 B for
// bf16/fp16 (one global_load_dwordx4) and 32 B for fp32 (two dwordx4).  The
// conversion to/from bf16 uses gfx950's v_cvt_pk_bf16_f32 (RNE), emitted by
// clang for a plain (__bf16) cast on this target.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mv {

enum Dtype : int { F32 = 0, BF16 = 1, F16 = 2 };

constexpr int kWave = 64;
constexpr int kVec = 8;            // elements per lane per step
constexpr int kBlock = 256;        // 4 waves
constexpr int kChunk = 4096;       // elements per workgroup (2 steps of 256x8)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

template <typename T> struct DT;
template <> struct DT<float> { static constexpr Dtype v = F32; };
template <> struct DT<__bf16> { static constexpr Dtype v = BF16; };
template <> struct DT<_Float16> { static constexpr Dtype v = F16; };

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f32(_Float16 x) { return (float)x; }

template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float x) { return (__bf16)x; }
template <> __device__ __forceinline__ _Float16 from_f32<_Float16>(float x) { return (_Float16)x; }

// ---- 8-wide vector load (aligned) -> fp32 registers ----
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  f32x4 a = *reinterpret_cast<const f32x4*>(p);
  f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
__device__ __forceinline__ void load8(const __bf16* p, float (&v)[8]) {
  u16x8 a = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(((uint32_t)a[j]) << 16);
}
// non-temporal (last-use) streaming load: the line is not kept in L2 / MALL
__device__ __forceinline__ void load8_nt(const __bf16* p, float (&v)[8]) {
  u16x8 a = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(p));
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = __uint_as_float(((uint32_t)a[j]) << 16);
}
__device__ __forceinline__ void load8(const _Float16* p, float (&v)[8]) {
  u16x8 a = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    unsigned short s = a[j];
    v[j] = (float)__builtin_bit_cast(_Float16, s);
  }
}

// ---- fp32 registers -> 8-wide vector store (aligned), with conversion ----
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  f32x4 a = {v[0], v[1], v[2], v[3]};
  f32x4 b = {v[4], v[5], v[6], v[7]};
  *reinterpret_cast<f32x4*>(p) = a;
  *reinterpret_cast<f32x4*>(p + 4) = b;
}
// Packed RNE f32x2 -> bf16x2 on gfx950 (lo <- a, hi <- b).  Written as inline
// asm: ROCm 7.2 clang mis-lowers __builtin_convertvector(f32x2 -> bf16x2) inside
// unrolled loops (it converted only the even elements: caught by
// tests/test_kernels_gpu.py::test_pack_unpack_cast_scale).
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ void store8(__bf16* p, const float (&v)[8]) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 o = {cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]), cvt_pk_bf16(v[4], v[5]),
             cvt_pk_bf16(v[6], v[7])};
  *reinterpret_cast<u32x4*>(p) = o;
}
__device__ __forceinline__ void store8(_Float16* p, const float (&v)[8]) {
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = __builtin_bit_cast(unsigned short, (_Float16)v[j]);
  *reinterpret_cast<u16x8*>(p) = o;
}

// scalar tail helpers
template <typename T>
__device__ __forceinline__ float ld1(const T* p) { return to_f32(*p); }
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) { *p = from_f32<T>(v); }

__device__ __forceinline__ bool aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

// wave64 sum via DPP-backed shuffles
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Block (256 threads = 4 waves) sum of NV values; result valid in thread 0.
template <int NV>
__device__ __forceinline__ void block_sum(float (&v)[NV]) {
  __shared__ float red[NV][kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int w = threadIdx.x / kWave;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    v[i] = wave_sum(v[i]);
    if (lane == 0) red[i][w] = v[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < kBlock / kWave; ++j) s += red[i][j];  // fixed order: deterministic
      v[i] = s;
    }
  }
}

}  // namespace mv
