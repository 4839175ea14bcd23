// Implicit-GEMM 3x3 convolution (pad 1, stride 1/2), NHWC bf16, gfx950 MFMA (mv_conv.hip)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// partial rows [P][2][K] of the fused BN-statistics epilogue for an M-pixel output
int64_t mv_conv3x3_partials(int64_t M, int K);
// y[N, Ho, Wo, K] = conv3x3(x[N, H, W, C], w[K, 3, 3, C]); C, K multiples of 64.
// partial != null: BN statistics of the bf16 outputs around shift (may be null = 0).
// Returns false for an unsupported shape (nothing launched).
// bn_x != null (requires partial): the epilogue instead runs the mode-1 (BN+ReLU)
// backward reduce of the BN whose output x is (y = its data gradient): bn_x = that BN's
// input [.., K], bn_vec = its saved [4][K] (mean, invstd, scale, bias).
bool mv_conv3x3(const void* x, const void* w, void* y, int N, int H, int W, int C, int K,
                int stride, const float* shift, float* partial, hipStream_t st,
                const void* bn_x = nullptr, const float* bn_vec = nullptr);

// same kernel for ks = 1 (pad 0) or 3 (pad 1): y[N, Ho, Wo, K] = conv(x[N, H, W, C], w[K, ks, ks, C])
// in_scale / in_bias ([C] each, the 64 -> 64 row-patch kernel only — false elsewhere): x is
// the producing BN's INPUT and relu(x * in_scale + in_bias) is convolved
bool mv_conv_nhwc(const void* x, const void* w, void* y, int N, int H, int W, int C, int K, int ks,
                  int stride, const float* shift, float* partial, hipStream_t st,
                  const void* bn_x = nullptr, const float* bn_vec = nullptr,
                  const float* in_scale = nullptr, const float* in_bias = nullptr);

// 3x3 weight gradient: dw[K, 3, 3, C] (bf16, channels_last [K, C, 3, 3]) of
// y = conv3x3(x, w, stride, pad 1) given dy; work: fp32 [mv_wgrad3x3_workspace(M, K, C)]
int64_t mv_wgrad3x3_workspace(int64_t M, int K, int C);
// (in_scale / in_bias: as mv_conv_nhwc's — the weight gradient w.r.t. relu(x * in_scale +
// in_bias); the 64 -> 64 row-patch kernel only)
bool mv_wgrad3x3(const void* x, const void* dy, void* dw, float* work, int N, int H, int W, int C,
                 int K, int stride, hipStream_t st, const float* in_scale = nullptr,
                 const float* in_bias = nullptr);

// 1x1 (pad 0, stride 1/2) weight gradient: dw[K, C] (bf16) of y = conv1x1(x, w, stride)
// given dy; work: fp32 [mv_wgrad1x1_workspace(M, K, C)], M = N * Ho * Wo
int64_t mv_wgrad1x1_workspace(int64_t M, int K, int C);
// (dw_fp32: dw is fp32 instead of bf16)
// dy2 != null: dy's channels [k1, K) come from dy2 ([N, Ho, Wo, K - k1]) — dw = [dy | dy2]^T . x
bool mv_wgrad1x1(const void* x, const void* dy, void* dw, float* work, int N, int H, int W, int C,
                 int K, int stride, hipStream_t st, bool dw_fp32 = false,
                 const void* dy2 = nullptr, int k1 = 0, bool dy2_gather = false);
// (dy2_gather: dy2 is [N, H, W, K - k1] at the input resolution, read at each output row's
// strided input pixel — stride 2 only)

// 64 -> 64 channel 3x3 / stride 1 "row patch" kernel (mv_conv64.hip): filter resident in
// LDS, 8-row input patches staged once for all 9 taps.  W <= 62.  grid = persistent
// workgroups (= the partial-row count when partial != null).  Same epilogues as
// mv_conv3x3 (statistics / BN+ReLU backward reduce).
bool mv_conv64_supported(int N, int H, int W, int C, int K, int ks, int stride);
// in_scale / in_bias (64 each): x is the producing BN's INPUT and relu(x * in_scale +
// in_bias) is convolved (applied while staging the patch; the BN output never exists)
bool mv_conv64(const void* x, const void* w, void* y, int N, int H, int W, const float* shift,
               float* partial, int grid, hipStream_t st, const void* bn_x = nullptr,
               const float* bn_vec = nullptr, const float* in_scale = nullptr,
               const float* in_bias = nullptr);
// weight gradient of the 64 -> 64 3x3 / stride 1 conv on the row-patch scheme
// (mv_conv64.hip): W % 4 == 0, W <= 56; writes fp32 partial [grid][9][64][64] rows for
// mv_conv.hip's wgrad reduce
bool mv_wgrad64_supported(int N, int H, int W, int C, int K, int stride);
bool mv_wgrad64(const void* x, const void* dy, float* partial, int grid, int N, int H, int W,
                hipStream_t st, const float* in_scale = nullptr, const float* in_bias = nullptr);

// Stride-2 3x3 (pad 1) data gradient as four output-parity-class gather GEMMs (no zero
// fill, no structurally-zero products): dy [Nb, H/2, W/2, K], wt = the transposed flipped
// filter [C][3][3][K], dx [Nb, H, W, C]; H, W even, C, K % 64 == 0 (C % 256 == 0 runs on
// mv_gemm256.hip AMODE 4, else conv3x3_kernel's DG mode)
bool mv_conv3x3_s2_dgrad_supported(int Nb, int H, int W, int C, int K);
bool mv_conv3x3_s2_dgrad(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C,
                         int K, hipStream_t st);

// The data-gradient filters of n convs in one launch (see mv_conv.hip): w [K][ks][ks][C] ->
// wt [C][ks][ks][K], taps rotated.  The caller builds the table once (host image of
// mv_transpose_filters_table_bytes bytes, copied to device memory) and reuses it while the
// filter and output pointers stay put.
int64_t mv_transpose_filters_blocks(const int* K, const int* C, const int* ks, int n);
int64_t mv_transpose_filters_table_bytes(int n, int64_t blocks);
void mv_transpose_filters_table(const void* const* src, void* const* dst, const int* K,
                                const int* C, const int* ks, int n, void* host_image);
void mv_transpose_filters(const void* table, int n, int64_t blocks, hipStream_t st);
