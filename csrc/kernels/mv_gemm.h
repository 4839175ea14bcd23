// Host-side declarations of the gfx950 MFMA NT GEMM (mv_gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// number of [2][N] statistics partial rows gemm_nt writes for this problem
int64_t mv_gemm_partials(int64_t M, int N, int K);
// C[M,N] = A[M,K] . B[N,K]^T (bf16 in/out, fp32 accumulate); K % 64 == 0, N % 64 == 0.
// partial != null: fused BN statistics of C around shift -> partial[ceil(M/BM)][2][N]
void mv_gemm_nt(const void* A, const void* B, void* C, int64_t M, int N, int K,
                const float* shift, float* partial, hipStream_t st);
