// Host declarations of mv_stem.hip (ResNet 7x7/2 stem conv with BN statistics epilogue).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// number of [2][64] statistics partial rows mv_stem_fwd writes for batch N
int mv_stem_partials(int N);
// z [N, 112, 112, 64] = conv7x7/2/pad3(x [N, 224, 224, 4], w [64, 7, 7, 4] (OHWC)), bf16
// NHWC; partial [P][2][64] = per-channel (sum, sum^2) of bf16(z) - shift (shift may be null)
// grid > 0 overrides the occupancy-sized grid (tests): partial then has `grid` rows
// cin: channels of the NHWC input x — 4 (zero-padded RGB) or 3 (raw RGB, read directly)
void mv_stem_fwd(const void* x, const void* w, void* z, const float* shift, float* partial, int N,
                 hipStream_t st, int grid = 0, int cin = 4);
// dw [64, 7, 7, 4] (OHWC bf16) = the stem conv's weight gradient from x [N, 224, 224, 4] and
// dz [N, 112, 112, 64]; work: fp32 [mv_stem_wgrad_blocks(N) * 64 * 224]
int mv_stem_wgrad_blocks(int N);
void mv_stem_wgrad(const void* x, const void* dz, void* dw, float* work, int N, hipStream_t st,
                   int cin = 4);

// The stem's BN+ReLU + 3x3/2/pad-1 maxpool backward fused into the weight gradient: dz is
// never written — each output row's dz is rebuilt while it is staged, from the conv output
// z and the pooled gradients, with mv_pool.hip's maxpool_bwd_k3s2_kernel<true> math and
// summation order (the same bf16 dz bits).  ca, cb, cc: the BN backward coefficients
// (dz = ca * relu'(z) * g + cb * z + cc, from mv_pool_bn_reduce + mv_bn_bwd_from_partials).
struct MvStemPoolBwd {
  const void* z;            // [N, 112, 112, 64] bf16, the stem conv output
  const void* dy;           // [N, 56, 56, 64] bf16 pooled gradient
  const void* dy2;          // second pooled gradient stream or null
  const uint8_t* idx;       // [N, 56, 56, 64] window argmax (0..8)
  const float* scale;       // the BN's saved scale / bias (ReLU gate)
  const float* bias;
  const float* ca;
  const float* cb;
  const float* cc;
};
void mv_stem_wgrad_pool_bn(const void* x, const MvStemPoolBwd& pb, void* dw, float* work, int N,
                           hipStream_t st, int cin = 4);
