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
bool mv_gemm_nt_apply(const void* A, const void* B, void* Y, int64_t M, int N, int K,
                      const void* res, const float* scale, const float* bias, void* mask,
                      hipStream_t st);
