// Small-matrix math of the BN fold (ops/bn.py _Conv1x1BNFold) in two launches.
//
// The folded backward of a 1x1 conv (weight W [cout, cin], input x [m, cin]) followed by
// a training BatchNorm needs, per step and block, only [cout] / [cout, cin] / [cin, cin]
// sized quantities once the big products are done (g = dz^T x and gram = x^T x by
// wgrad1x1, column sums of x, the consumer's reduce partials).  In eager PyTorch that
// is ~22 tiny kernels per block (reductions, outer products, p x p matmuls, casts, a
// concat) — ~400 launches per ResNet-50 step at 5-8 us each.  Here:
//
//   fold_coeffs_kernel (one workgroup per output channel c, then one per input channel):
//     sdz[c]  = sum_p part[p][0][c]                 (the consumer epilogue's sum dz)
//     sdzx[c] = sum_k W[c][k] g[c][k] - mean[c] sdz[c]     (sum dz (z - mean), z = x W^T)
//     dgamma, dbeta, ca, cb, cc exactly as mv_bn.hip finalize_bwd_kernel
//     xsum[k] = sum_p colsum[p][k]  (or taken as given)
//   fold_products_kernel (16x16 LDS-tiled small GEMMs, then elementwise jobs):
//     dW[c][k]        = ca[c] g[c][k] + cb[c] (W gram)[c][k] + cc[c] xsum[k]   -> bf16
//     bcat[k][c]      = ca[c] W[c][k]                      (c < cout)           -> bf16
//     bcat[k][cout+j] = sum_c W[c][k] cb[c] W[c][j]        (j < cin)            -> bf16
//     badd[k]         = sum_c cc[c] W[c][k]                                      fp32
// so dx = [dz | x] . bcat^T + badd and dW as above.  All sums run in a fixed order
// (deterministic, identical on every rank).
#include "mv_common.h"
#include "mv_fold.h"

namespace mv {
namespace fold {

constexpr int kThreads = 256;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(kThreads) void fold_coeffs_kernel(
    const float* __restrict__ part, int P, const __bf16* __restrict__ w,
    const float* __restrict__ g, const float* __restrict__ vec, const float* __restrict__ gamma,
    int64_t M, int cout, int cin, const float* __restrict__ colsum, int P2,
    float* __restrict__ co, float* __restrict__ xsum) {
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x;
  if (b >= cout) {                    // column sums of x (block-uniform branch)
    const int k = b - cout;
    if (!colsum) return;
    float s = 0.f;
    for (int p = threadIdx.x; p < P2; p += kThreads) s += colsum[(int64_t)p * cin + k];
    s = block_sum(s, red);
    if (threadIdx.x == 0) xsum[k] = s;
    return;
  }
  const int c = b;
  float s1 = 0.f, s2 = 0.f;
  for (int p = threadIdx.x; p < P; p += kThreads) s1 += part[(int64_t)p * 2 * cout + c];
  for (int k = threadIdx.x; k < cin; k += kThreads)
    s2 += (float)w[(int64_t)c * cin + k] * g[(int64_t)c * cin + k];
  const float sdz = block_sum(s1, red);
  const float rowdot = block_sum(s2, red);
  if (threadIdx.x != 0) return;
  const float mean = vec[c], is = vec[cout + c];
  const float sdzx = rowdot - mean * sdz;
  co[c] = sdzx * is;                   // dgamma
  co[cout + c] = sdz;                  // dbeta
  const float gm = gamma ? gamma[c] : 1.f;
  const float inv_m = 1.f / (float)M;
  const float a = gm * is;
  const float bb = -a * is * is * sdzx * inv_m;
  co[2 * cout + c] = a;
  co[3 * cout + c] = bb;
  co[4 * cout + c] = -a * sdz * inv_m - bb * mean;
}

// 16x16 output tiles (one per workgroup, one element per lane) for the two small GEMMs,
// staged through LDS in 16-deep chunks; then elementwise jobs.  Block ranges:
//   [0, n1)            dW tiles   (cout/16 x cin/16):  (W gram)[c][k]
//   [n1, n1 + n2)      Q tiles    (cin/16 x cin/16):   sum_c W[c][k] cb[c] W[c][j]
//   [n1 + n2, grid)    bcat[:, :cout] and badd, grid-stride
constexpr int kT = 16;

__global__ __launch_bounds__(kThreads) void fold_products_kernel(
    const __bf16* __restrict__ w, const float* __restrict__ g, const float* __restrict__ gram,
    const float* __restrict__ co, const float* __restrict__ xsum, int cout, int cin,
    __bf16* __restrict__ dw, __bf16* __restrict__ bcat, float* __restrict__ badd, int n1,
    int n2) {
  const float* ca = co + 2 * cout;
  const float* cb = co + 3 * cout;
  const float* cc = co + 4 * cout;
  const int ldb = cout + cin;
  const int ty = threadIdx.x / kT, tx = threadIdx.x % kT;
  __shared__ float ta[kT][kT + 1], tb[kT][kT + 1];
  const int b = blockIdx.x;
  if (b < n1) {                                       // dW tile
    const int tiles_k = cin / kT;
    const int c0 = (b / tiles_k) * kT, k0 = (b % tiles_k) * kT;
    float s = 0.f;
    for (int j0 = 0; j0 < cin; j0 += kT) {
      ta[ty][tx] = (float)w[(int64_t)(c0 + ty) * cin + j0 + tx];
      tb[ty][tx] = gram[(int64_t)(j0 + ty) * cin + k0 + tx];
      __syncthreads();
#pragma unroll
      for (int jj = 0; jj < kT; ++jj) s += ta[ty][jj] * tb[jj][tx];
      __syncthreads();
    }
    const int c = c0 + ty, k = k0 + tx;
    const int64_t i = (int64_t)c * cin + k;
    dw[i] = (__bf16)(ca[c] * g[i] + cb[c] * s + cc[c] * xsum[k]);
    return;
  }
  if (b < n1 + n2) {                                  // Q tile -> bcat[k][cout + j]
    const int tiles_j = cin / kT, t = b - n1;
    const int k0 = (t / tiles_j) * kT, j0 = (t % tiles_j) * kT;
    float s = 0.f;
    for (int c0 = 0; c0 < cout; c0 += kT) {
      const int c = c0 + ty;
      ta[ty][tx] = (float)w[(int64_t)c * cin + k0 + tx] * cb[c];
      tb[ty][tx] = (float)w[(int64_t)c * cin + j0 + tx];
      __syncthreads();
#pragma unroll
      for (int q = 0; q < kT; ++q) s += ta[q][ty] * tb[q][tx];
      __syncthreads();
    }
    bcat[(int64_t)(k0 + ty) * ldb + cout + j0 + tx] = (__bf16)s;
    return;
  }
  const int64_t n_bl = (int64_t)cin * cout, total = n_bl + cin;
  const int nb3 = gridDim.x - n1 - n2;
  for (int64_t i = (int64_t)(b - n1 - n2) * kThreads + threadIdx.x; i < total;
       i += (int64_t)nb3 * kThreads) {
    if (i < n_bl) {                                   // bcat[k][c], c fastest
      const int k = (int)(i / cout), c = (int)(i % cout);
      bcat[(int64_t)k * ldb + c] = (__bf16)(ca[c] * (float)w[(int64_t)c * cin + k]);
    } else {                                          // badd[k]
      const int k = (int)(i - n_bl);
      float s = 0.f;
      for (int c = 0; c < cout; ++c) s += cc[c] * (float)w[(int64_t)c * cin + k];
      badd[k] = s;
    }
  }
}

}  // namespace fold
}  // namespace mv

void mv_fold_coeffs(const float* part, int P, const void* w, const float* g, const float* vec,
                    const float* gamma, int64_t M, int cout, int cin, const float* colsum, int P2,
                    float* co, float* xsum, hipStream_t st) {
  const int blocks = cout + (colsum ? cin : 0);
  hipLaunchKernelGGL(mv::fold::fold_coeffs_kernel, dim3(blocks), dim3(mv::fold::kThreads), 0, st,
                     part, P, (const __bf16*)w, g, vec, gamma, M, cout, cin, colsum, P2, co, xsum);
}

void mv_fold_products(const void* w, const float* g, const float* gram, const float* co,
                      const float* xsum, int cout, int cin, void* dw, void* bcat, float* badd,
                      hipStream_t st) {
  using mv::fold::kT;
  const int n1 = dw ? (cout / kT) * (cin / kT) : 0;
  const int n2 = (cin / kT) * (cin / kT);
  const int64_t rest = (int64_t)cin * cout + cin;
  int n3 = (int)((rest + mv::fold::kThreads - 1) / mv::fold::kThreads);
  if (n3 > 1024) n3 = 1024;
  hipLaunchKernelGGL(mv::fold::fold_products_kernel, dim3((unsigned)(n1 + n2 + n3)),
                     dim3(mv::fold::kThreads), 0, st, (const __bf16*)w, g, gram, co, xsum, cout,
                     cin, (__bf16*)dw, (__bf16*)bcat, badd, n1, n2);
}
