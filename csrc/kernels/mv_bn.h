// Host launchers for the fused NHWC BatchNorm(+add)(+ReLU) kernels (mv_bn.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// number of row-partials the reduction passes produce (size the [P][2][C] workspace)
int mv_bn_partials(int64_t M, int C);

// y == nullptr: statistics + running-stat update + scale/bias only (no apply pass)
void mv_bn_fwd_train(const void* x, const void* res, void* y, int64_t M, int C, float* rmean,
                     float* rvar, const float* gamma, const float* beta, float momentum, float eps,
                     bool relu, float* partial, int P, float* save_mean, float* save_invstd,
                     float* scale, float* bias, hipStream_t st, void* mask = nullptr);

// finalize + apply from [P][2][C] statistics partials produced by the conv GEMM epilogue
void mv_bn_fwd_from_partials(const void* x, const void* res, void* y, int64_t M, int C,
                             float* rmean, float* rvar, const float* gamma, const float* beta,
                             float momentum, float eps, bool relu, const float* partial, int P,
                             float* save_mean, float* save_invstd, float* scale, float* bias,
                             hipStream_t st, void* mask = nullptr);
// finalize + dx pass of a BN backward whose reduce ran in the producing GEMM's epilogue
void mv_bn_bwd_from_partials(const void* dz, const void* x, void* dx, int64_t M, int C,
                             const float* save_mean, const float* save_invstd,
                             const float* gamma, const float* scale, const float* bias,
                             float* dgamma, float* dbeta, const float* partial, int P, float* ca,
                             float* cb, float* cc, hipStream_t st);

void mv_bn_apply(const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
                 const float* bias, bool relu, hipStream_t st, void* mask = nullptr);
// mask (add+ReLU only, may be null): [M, C/8] bytes, bit j of byte (r, c/8) = y[r, c+j] > 0

// mode 0: plain BN, 1: BN+ReLU (mask from x), 2: BN+add+ReLU (mask from y, writes dz),
// 3: as 2 with y = the forward's [M, C/8] bitmask.
// dy2 (mode 2 only, may be null): second gradient stream added to dy on the fly.
void mv_bn_bwd(int mode, const void* dy, const void* dy2, const void* x, const void* y, void* dz, void* dx,
               int64_t M, int C, const float* save_mean, const float* save_invstd,
               const float* gamma, const float* scale, const float* bias, float* dgamma,
               float* dbeta, float* partial, int P, float* ca, float* cb, float* cc,
               int dy2_stride, int H, int W, hipStream_t st);
// dy2_stride > 1: dy2 is [N, ceil(H/s), ceil(W/s), C] (gradient of a stride-s 1x1 conv's
// input at its output resolution), added only on rows of the stride grid

// y = relu(x * scale + bias) with [P][C] column-sum partials of the bf16 y (P returned,
// <= mv_bn_partials(M, C))
int mv_bn_apply_colsum(const void* x, void* y, int64_t M, int C, const float* scale,
                       const float* bias, float* partial, hipStream_t st);

// statistics of the stride-ds grid rows of x [Nb, H, W, C] (what a stride-ds 1x1 conv reads):
// saved {mean, invstd, scale, bias} with gamma = 1, beta = 0; partial: [P][2][C] workspace,
// P = mv_bn_partials(rows, C)
void mv_bn_stats_strided(const void* x, int Nb, int H, int W, int C, int ds, float* partial,
                         int P, float* save_mean, float* save_invstd, float* scale, float* bias,
                         hipStream_t st);
