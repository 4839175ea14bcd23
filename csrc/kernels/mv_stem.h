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
