// Host-side declarations of the mivod gfx950 kernel launchers (mv_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Multi-tensor table passed by value in the kernel arguments (<= 2 KB).
constexpr int kMvMaxTensors = 64;
struct MtArgs {
  void* ptr[kMvMaxTensors];            // tensor-side pointers
  int64_t numel[kMvMaxTensors];
  int64_t flat_off[kMvMaxTensors];     // element offset in the flat buffer
  int32_t chunk_start[kMvMaxTensors + 1];  // prefix sum of 4096-element chunks
  int32_t ntensors;
};

// Static segment/chunk table of a flat bucket (device pointers).
struct ChunkTable {
  const int64_t* begin;   // [nchunks] element offset of each chunk
  const int32_t* len;     // [nchunks]
  const int32_t* seg;     // [nchunks] owning segment
  const int32_t* seg_c0;  // [nseg] first chunk of segment
  const int32_t* seg_nc;  // [nseg] chunk count of segment
  int32_t nchunks;
  int32_t nseg;
};

void mv_launch_mt_copy(const MtArgs& a, int tensor_dtype, void* flat, int flat_dtype, bool to_flat,
                       float scale, int* found_nonfinite, hipStream_t st);
// flag |= any(!isfinite(x)) (read-only)
void mv_launch_nonfinite_scan(const void* x, int dtype, int64_t n, int* flag, hipStream_t st);
void mv_launch_flat_cast(const void* src, int sd, void* dst, int dd, int64_t n, float scale,
                         int* found_nonfinite, hipStream_t st);
void mv_launch_sgd(const void* g, int gd, float* w, float* mom, void* model, int md, int64_t n,
                   float lr, float momentum, float dampening, float wd, float gscale, int nesterov,
                   int first, const float* dyn, const int* skip, hipStream_t st);
// skip (nullable): device int32; nonzero => the kernel returns without updating
// (fp16-wire overflow guard, identical on every rank after the flag allreduce)
// dyn (nullable): device [lr, first, bc1, bc2] read by the kernel instead of the
// scalar arguments — HIP-graph replayable hyperparameters (mivod/torch/graphs.py)
void mv_launch_adam(const void* g, int gd, float* w, float* m, float* v, void* model, int md,
                    int64_t n, float lr, float b1, float b2, float eps, float wd, float gscale,
                    float bc1, float bc2, int adamw, int keras_eps, const float* dyn,
                    const int* skip, hipStream_t st);
void mv_launch_adadelta(const void* g, int gd, float* w, float* sq, float* acc, void* model, int md,
                        int64_t n, float lr, float rho, float eps, float wd, float gscale,
                        const float* dyn, const int* skip, hipStream_t st);
void mv_launch_lars(const void* g, int gd, float* w, float* mom, void* model, int md,
                    const ChunkTable& ct, const int32_t* sflag, float* partial, float* norms,
                    float lr, float momentum, float wd, float eta, float gscale, float eps,
                    int first, const float* dyn, const int* skip, hipStream_t st);
void mv_launch_seg_dot3(const void* a, const void* b, int dt, const ChunkTable& ct, float* partial,
                        float* out, hipStream_t st);
void mv_launch_adasum_combine(void* a, const void* b, int dt, const ChunkTable& ct,
                              const float* dots, hipStream_t st);
// Adasum (vector halving): per-segment (a.b, |a|^2, |b|^2) with a fp32 and b any dtype
void mv_launch_seg_dot3_f(const float* a, const void* b, int bdt, const ChunkTable& ct,
                          float* partial, float* out, hipStream_t st);
// f <- cf*f + cr*r on the fp32 running merge (swap: f holds b instead of a)
void mv_launch_adasum_fcombine(float* f, const void* r, int rdt, const ChunkTable& ct,
                               const float* dots, int swap, hipStream_t st);
