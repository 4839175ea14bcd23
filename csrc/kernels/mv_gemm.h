// Host-side declarations of the gfx950 MFMA NT GEMM (mv_gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// number of [2][N] statistics partial rows gemm_nt writes for this problem
int64_t mv_gemm_partials(int64_t M, int N, int K);
// C[M,N] = A[M,K] . B[N,K]^T (bf16 in/out, fp32 accumulate); K % 64 == 0, N % 64 == 0.
// partial != null: fused BN statistics of C around shift -> partial[ceil(M/BM)][2][N];
// C == null (with partial): statistics only, C is not written (streamed shapes)
void mv_gemm_nt(const void* A, const void* B, void* C, int64_t M, int N, int K,
                const float* shift, float* partial, hipStream_t st);

// Data-gradient GEMM with the following BN+add+ReLU backward reduce fused (EPI 2 of
// the streaming kernel; K in {64, 128, 256} only — returns false otherwise):
// dy = A . B^T (bf16-rounded), d = mask ? dy + dy2 : 0 -> DZ, partial[P][2][N] =
// (sum d, sum d * (x - mean)) with P = mv_gemm_bwd_partials(M, N, K, bn); bn = the
// column-tile width (0: default)
int64_t mv_gemm_bwd_partials(int64_t M, int N, int K, int bn);
// dy2_stride > 1: dy2 is [*, ceil(H/s), ceil(W/s), N] on the stride grid of the [*, H, W]
// rows (added where h and w are multiples of s)
bool mv_gemm_nt_bn_bwd(const void* A, const void* B, void* DZ, int64_t M, int N, int K,
                       const void* dy2, const void* mask, const void* x, const float* mean,
                       float* partial, int bn, hipStream_t st, int dy2_stride = 1, int H = 1,
                       int W = 1);

// BN(+residual)+ReLU apply fused into the GEMM epilogue (EPI 3 of the streaming kernel):
// z = bf16(A . B^T), Y = relu(z * scale + bias + res) and the [M, N/8] bitmask of Y > 0 —
// bit-identical to gemm_nt's z followed by mv_bn.hip's apply (ops.bn._Conv1x1BNFold's
// recompute forward: statistics pass with C == null, finalize, then this)
bool mv_gemm_apply_supported(int N, int K);
// rscale != null: res is the shortcut BN's INPUT and bf16(res * rscale + rbias) is added
bool mv_gemm_nt_apply(const void* A, const void* B, void* Y, int64_t M, int N, int K,
                      const void* res, const float* scale, const float* bias, void* mask,
                      hipStream_t st, const float* rscale = nullptr, const float* rbias = nullptr);

// The BN3 fold's data gradient (ops.bn._Conv1x1BNFold) with the producing BN2's ReLU
// backward reduce (EPI 4): dx = [A1 | A2] . B^T + badd (A1 = dz [M, K1], A2 = x [M, K2],
// B = [K2, K1 + K2]), d = (fma(xb, scale, bias) > 0) ? bf16(dx) : 0 -> D [M, K2], partials
// [P][2][K2] = (sum d, sum d (xb - mean)); (K1, K2) in {(256, 64), (512, 128)}.
int64_t mv_gemm_fold_dx_partials(int64_t M, int K1, int K2);   // -1: unsupported
bool mv_gemm_fold_dx(const void* A1, const void* A2, const void* B, const float* badd,
                     void* D, int64_t M, int K1, int K2, const void* xb, const float* mean,
                     const float* scale, const float* bias, float* partial, hipStream_t st);

// D[M, K2] = [A1 | A2] . B^T + badd (EPI 6: the dual-source GEMM of mv_gemm_fold_dx with a
// plain store) — the projection-shortcut fold's input gradient; (K1, K2) = (256, 64) only
bool mv_gemm_dual_supported(int K1, int K2);
bool mv_gemm_dual_bias(const void* A1, const void* A2, const void* B, const float* badd, void* D,
                       int64_t M, int K1, int K2, hipStream_t st);

// EPI 7: mv_gemm_nt_apply with the residual recomputed in the same kernel — y = relu(
// bf16(A . B^T) * scale + bias + bf16(bf16(A2 . B2^T) * rscale + rbias)) (a stride-1
// projection shortcut conv + BN on the block input A2 [M, K]; K == 64 only)
bool mv_gemm_apply_dual_supported(int N, int K);
bool mv_gemm_nt_apply_dual(const void* A, const void* B, const void* A2, const void* B2, void* Y,
                           int64_t M, int N, int K, const float* scale, const float* bias,
                           const float* rscale, const float* rbias, void* mask, hipStream_t st);

// 256 x 256 tile, 8-wave glds pipeline (mv_gemm256.hip): N % 256 == 0, K % 64 == 0;
// partial rows = mv_gemm256_partials(M, N).  mv_gemm_nt routes its tiled shapes here.
bool mv_gemm256_supported(int64_t M, int N, int K);
int64_t mv_gemm256_partials(int64_t M, int N);
bool mv_gemm256_nt(const void* A, const void* B, void* C, int64_t M, int N, int K,
                   const float* shift, float* partial, hipStream_t st);
// The strided 1x1 conv (stride ds) on the same kernel: X [Nb, H, W, K] NHWC, C [Nb * Ho *
// Wo, N]; optional BN statistics (partial rows = mv_gemm256_partials(Nb * Ho * Wo, N)).
bool mv_gemm256_strided(const void* X, const void* B, void* C, int Nb, int H, int W, int K, int N,
                        int ds, const float* shift, float* partial, hipStream_t st);
// D = [A1 | A2] . B^T + badd (A1 [M, K1], A2 [M, K2], B [N, K1 + K2]); with partial: the
// BN fold's data-gradient epilogue (mv_gemm_fold_dx's, any N % 256 == 0): d = fma(xb,
// scale, bias) > 0 ? bf16(D) : 0 is stored, partials [mv_gemm256_partials(M, N)][2][N] =
// (sum d, sum d (xb - mean)); without: plain store
bool mv_gemm256_dual(const void* A1, const void* A2, const void* B, const float* badd, void* D,
                     int64_t M, int K1, int K2, int N, const void* xb, const float* mean,
                     const float* scale, const float* bias, float* partial, hipStream_t st,
                     int ds = 1, int H = 0, int W = 0);
// (ds > 1: A2 is [Nb, H, W, K2] read at each output row's stride-ds pixel — M = Nb Ho Wo)
// 1x1 weight gradient on the 256 x 256 pipeline (stride 1): partial[S][K][C] fp32 with
// S = mv_wgrad256_splits(M, C, K); DY channels [k1, K) from DY2 ([M, K - k1]) when k1 < K
bool mv_wgrad256_supported(int64_t M, int C, int K, int k1);
int64_t mv_wgrad256_splits(int64_t M, int C, int K);
bool mv_wgrad256(const void* X, const void* DY, const void* DY2, float* partial, int64_t M, int C,
                 int K, int k1, hipStream_t st);
// Implicit ks x ks convolution (pad ks / 2, stride 1-2, ks = 1 or 3) on the same pipeline
// (AMODE 3): X [Nb, H, W, Cin] NHWC, Wt [Cout][ks][ks][Cin], Y [Nb * Ho * Wo, Cout];
// Cout % 256 == 0.  partial: BN statistics of Y around shift (rows = mv_gemm256_partials(M, Cout));
// bn_x (+ partial, bn_vec = [4][Cout] mean, -, scale, bias): Y is the data gradient of a
// BN+ReLU output and d = fma(bn_x, scale, bias) > 0 ? bf16(Y) : 0 is stored with the
// partials (sum d, sum d (bn_x - mean)) — mv_conv.hip's EPI 2.
bool mv_conv256_supported(int N, int H, int W, int Cin, int Cout, int ks, int stride);
bool mv_conv256(const void* X, const void* Wt, void* Y, int Nb, int H, int W, int Cin, int Cout,
                int ks, int stride, const float* shift, float* partial, const void* bn_x,
                const float* bn_vec, hipStream_t st);
// 3x3 (pad 1, stride 1-2) weight gradient on the same pipeline: partial[S][K][9 C] fp32
// ([K][3][3][C] per split, the channels_last filter layout), S = mv_wgrad256_3x3_splits;
// C % 256 == 0, K % 256 == 0
bool mv_wgrad256_3x3_supported(int N, int H, int W, int C, int K, int stride);
int64_t mv_wgrad256_3x3_splits(int N, int H, int W, int C, int K, int stride);
bool mv_wgrad256_3x3(const void* X, const void* DY, float* partial, int N, int H, int W, int C,
                     int K, int stride, hipStream_t st);
// Stride-2 3x3 (pad 1) data gradient on the same pipeline (AMODE 4, one launch per output
// parity class): dy [Nb, H/2, W/2, Cout], wt = the transposed, flipped filter [Cin][3][3][Cout],
// dx [Nb, H, W, Cin] (every pixel written); H, W even, Cin % 256 == 0.
bool mv_dgrad256_s2_supported(int Nb, int H, int W, int Cin, int Cout);
bool mv_dgrad256_s2(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int Cin,
                    int Cout, hipStream_t st);
