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

// The two small GEMMs as 64 x 64 output tiles per workgroup, 4 x 4 outputs per lane
// (register-tiled fp32 FMA, operands staged through LDS 16 deep), then the GEMV and the
// elementwise jobs.  Block ranges:
//   [0, n1)                 dW tiles (cout/64 x cin/64):  (W gram)[c][k]
//   [n1, n1 + n2)           Q tiles  (cin/64 x cin/64):   sum_c W[c][k] cb[c] W[c][j]
//   [n1 + n2, n1 + n2 + n4) badd, 64 k per block (the 4 waves split c, fixed-order sum)
//   [n1 + n2 + n4, grid)    bcat[:, :cout], grid-stride
// (The first version staged 16 x 16 tiles with one output per lane and ran the GEMV as one
// serial loop per k: ~67 us per launch, 1.0 ms/step at ResNet-50 bs2048.)
constexpr int kBT = 64, kKC = 16;

__global__ __launch_bounds__(kThreads) void fold_products_kernel(
    const __bf16* __restrict__ w, const float* __restrict__ g, const float* __restrict__ gram,
    const float* __restrict__ co, const float* __restrict__ xsum, int cout, int cin,
    __bf16* __restrict__ dw, __bf16* __restrict__ bcat, float* __restrict__ badd, int n1,
    int n2, int n4) {
  const float* ca = co + 2 * cout;
  const float* cb = co + 3 * cout;
  const float* cc = co + 4 * cout;
  const int ldb = cout + cin;
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  if (b < n1 + n2) {
    // sa[kk][r] = A[r][k0 + kk], sb[kk][col] = B[k0 + kk][col] (A row-tile, B column-tile)
    __shared__ __attribute__((aligned(16))) float sa[kKC][kBT + 4], sb[kKC][kBT + 4];
    const bool is_dw = b < n1;
    const int t = is_dw ? b : b - n1;
    const int tiles_n = cin / kBT;
    const int r0 = (t / tiles_n) * kBT, n0 = (t % tiles_n) * kBT;
    const int K = is_dw ? cin : cout;
    const int ty = tid >> 4, tx = tid & 15;          // outputs rows 4 ty.., cols 4 tx..
    // staging: 4 elements of each tile per lane
    const int lr = tid >> 2, lk = (tid & 3) * 4;     // A: row lr, k lk..lk+3 / B: k, col
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) acc[i][jj] = 0.f;
    for (int k0 = 0; k0 < K; k0 += kKC) {
      if (is_dw) {
        // A = W [cout][cin] (row c, k contiguous); B = gram [cin][cin]
#pragma unroll
        for (int q = 0; q < 4; ++q)
          sa[lk + q][lr] = (float)w[(int64_t)(r0 + lr) * cin + k0 + lk + q];
        const int bk = tid >> 4, bc = (tid & 15) * 4;
        const float4 v = *reinterpret_cast<const float4*>(gram + (int64_t)(k0 + bk) * cin + n0 + bc);
        sb[bk][bc] = v.x;
        sb[bk][bc + 1] = v.y;
        sb[bk][bc + 2] = v.z;
        sb[bk][bc + 3] = v.w;
      } else {
        // A[k][c] = W[c][k] cb[c] (row k = r0.., c = k0..); B[c][j] = W[c][j]
        const int ck = tid >> 4, cr = (tid & 15) * 4;
        const int c = k0 + ck;
        const float cbc = cb[c];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          sa[ck][cr + q] = (float)w[(int64_t)c * cin + r0 + cr + q] * cbc;
          sb[ck][cr + q] = (float)w[(int64_t)c * cin + n0 + cr + q];
        }
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < kKC; ++kk) {
        const float4 a = *reinterpret_cast<const float4*>(&sa[kk][4 * ty]);
        const float4 bv = *reinterpret_cast<const float4*>(&sb[kk][4 * tx]);
        const float av[4] = {a.x, a.y, a.z, a.w}, bw[4] = {bv.x, bv.y, bv.z, bv.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) acc[i][jj] = __builtin_fmaf(av[i], bw[jj], acc[i][jj]);
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + 4 * ty + i;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int n = n0 + 4 * tx + jj;
        if (is_dw) {
          const int64_t e = (int64_t)r * cin + n;
          dw[e] = (__bf16)(ca[r] * g[e] + cb[r] * acc[i][jj] + cc[r] * xsum[n]);
        } else {
          bcat[(int64_t)r * ldb + cout + n] = (__bf16)acc[i][jj];
        }
      }
    }
    return;
  }
  if (b < n1 + n2 + n4) {                            // badd[k] = sum_c cc[c] W[c][k]
    __shared__ float red[4][kBT];
    const int k = (b - n1 - n2) * kBT + (tid & 63), wv = tid >> 6;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int c = wv;
    for (; c + 12 < cout; c += 16) {
      s0 += cc[c] * (float)w[(int64_t)c * cin + k];
      s1 += cc[c + 4] * (float)w[(int64_t)(c + 4) * cin + k];
      s2 += cc[c + 8] * (float)w[(int64_t)(c + 8) * cin + k];
      s3 += cc[c + 12] * (float)w[(int64_t)(c + 12) * cin + k];
    }
    for (; c < cout; c += 4) s0 += cc[c] * (float)w[(int64_t)c * cin + k];
    red[wv][tid & 63] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (wv == 0) badd[k] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    return;
  }
  const int64_t n_bl = (int64_t)cin * cout;
  const int nb3 = gridDim.x - n1 - n2 - n4;
  for (int64_t i = (int64_t)(b - n1 - n2 - n4) * kThreads + tid; i < n_bl;
       i += (int64_t)nb3 * kThreads) {
    const int k = (int)(i / cout), c = (int)(i % cout);     // bcat[k][c], c fastest
    bcat[(int64_t)k * ldb + c] = (__bf16)(ca[c] * (float)w[(int64_t)c * cin + k]);
  }
}

// BN statistics partials of z = x W^T from the Gram matrix G = x^T x (ops.bn._gram_stats):
//   part[0][c] = sum_k W[c][k] xsum[k] - m shift[c]                        = sum (z - shift)
//   part[1][c] = sum_k W[c][k] (G W^T)[k][c] - 2 shift[c] u[c] + m shift[c]^2  = sum (z - shift)^2
// One workgroup per 16 output channels: W's rows in LDS (fp32), thread t owns Gram rows
// k = t, t + 256, .. and reads G[j][k] (= G[k][j]: coalesced across threads) for all j,
// then a fixed-order block reduction per channel.
constexpr int kGsCh = 16;

__global__ __launch_bounds__(kThreads) void gram_stats_kernel(
    const __bf16* __restrict__ w, const float* __restrict__ gram, const float* __restrict__ xsum,
    const float* __restrict__ shift, int64_t m, int cout, int cin, float* __restrict__ part) {
  extern __shared__ float gs_smem[];
  float* wl = gs_smem;                              // [cin][kGsCh]: W^T rows, 4 x 16-byte reads
  float* red = gs_smem + kGsCh * cin;               // [2][kGsCh][kThreads / 64]
  const int c0 = blockIdx.x * kGsCh, tid = threadIdx.x;
  for (int q = tid; q < kGsCh * cin; q += kThreads) {
    const int r = q / cin, k = q - r * cin;
    wl[k * kGsCh + r] = (float)w[(int64_t)(c0 + r) * cin + k];
  }
  __syncthreads();
  float qs[kGsCh], us[kGsCh];
#pragma unroll
  for (int r = 0; r < kGsCh; ++r) { qs[r] = 0.f; us[r] = 0.f; }
  for (int k = tid; k < cin; k += kThreads) {
    float t[kGsCh];
#pragma unroll
    for (int r = 0; r < kGsCh; ++r) t[r] = 0.f;
    // 8 Gram loads in flight per thread (a serial chain of L2 round trips otherwise)
#pragma unroll 8
    for (int j = 0; j < cin; ++j) {
      const float g = gram[(int64_t)j * cin + k];
      const f32x4* wj = reinterpret_cast<const f32x4*>(wl + j * kGsCh);
#pragma unroll
      for (int h = 0; h < kGsCh / 4; ++h) {
        const f32x4 wv = wj[h];
#pragma unroll
        for (int e = 0; e < 4; ++e) t[4 * h + e] = __builtin_fmaf(g, wv[e], t[4 * h + e]);
      }
    }
    const float xs = xsum[k];
#pragma unroll
    for (int r = 0; r < kGsCh; ++r) {
      qs[r] = __builtin_fmaf(wl[k * kGsCh + r], t[r], qs[r]);
      us[r] = __builtin_fmaf(wl[k * kGsCh + r], xs, us[r]);
    }
  }
  const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int r = 0; r < kGsCh; ++r) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      qs[r] += __shfl_xor(qs[r], o, 64);
      us[r] += __shfl_xor(us[r], o, 64);
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int r = 0; r < kGsCh; ++r) {
      red[(0 * kGsCh + r) * (kThreads / 64) + wv] = qs[r];
      red[(1 * kGsCh + r) * (kThreads / 64) + wv] = us[r];
    }
  }
  __syncthreads();
  if (tid < kGsCh) {
    float q = 0.f, u = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) {
      q += red[(0 * kGsCh + tid) * (kThreads / 64) + i];
      u += red[(1 * kGsCh + tid) * (kThreads / 64) + i];
    }
    const int c = c0 + tid;
    const float sh = shift ? shift[c] : 0.f, mf = (float)m;
    part[c] = u - mf * sh;
    part[cout + c] = q - 2.f * sh * u + mf * sh * sh;
  }
}

}  // namespace fold
}  // namespace mv

bool mv_gram_stats(const void* w, const float* gram, const float* xsum, const float* shift,
                   int64_t m, int cout, int cin, float* part, hipStream_t st) {
  using namespace mv::fold;
  if (cout % kGsCh || cin < 1 || cin > 1024) return false;
  const size_t lds = (size_t)(kGsCh * cin + 2 * kGsCh * (kThreads / 64)) * sizeof(float);
  hipLaunchKernelGGL(gram_stats_kernel, dim3(cout / kGsCh), dim3(kThreads), lds, st,
                     (const __bf16*)w, gram, xsum, shift, m, cout, cin, part);
  return true;
}

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
  using mv::fold::kBT;
  const int n1 = dw ? (cout / kBT) * (cin / kBT) : 0;
  const int n2 = (cin / kBT) * (cin / kBT);
  const int n4 = cin / kBT;
  const int64_t rest = (int64_t)cin * cout;
  int n3 = (int)((rest + mv::fold::kThreads - 1) / mv::fold::kThreads);
  if (n3 > 1024) n3 = 1024;
  hipLaunchKernelGGL(mv::fold::fold_products_kernel, dim3((unsigned)(n1 + n2 + n4 + n3)),
                     dim3(mv::fold::kThreads), 0, st, (const __bf16*)w, g, gram, co, xsum, cout,
                     cin, (__bf16*)dw, (__bf16*)bcat, badd, n1, n2, n4);
}
