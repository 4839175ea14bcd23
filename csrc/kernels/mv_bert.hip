// Fused transformer elementwise kernels (BERT) for gfx950.
//
//  * bias_gelu       y = gelu(x + b)             (x = GEMM output without bias)
//    backward        dx = dy * gelu'(x + b), dbias = sum_rows dx  (one pass)
//  * bias_dropout_add_ln
//                    v = res + dropout(z + b);  y = LN(v) * gamma + beta
//    backward        dv = LN'(dy) (the residual's grad), dz = dropout'(dv),
//                    dgamma / dbeta / dbias column sums            (one pass)
//
// Replaces, per BERT layer, torch's separate bias-add (inside the GEMM), GELU,
// dropout, residual add, LayerNorm and their backward kernels plus the
// bias-gradient reductions (profiles/r1_bert_large_fused_attention.md).
// Dropout masks come from a counter hash of (seed, row, col) — no mask tensor.
//
// Row kernels: one wave per row (wave64, 8 bf16 per lane per 512-column chunk,
// all chunks held in registers, H <= 4096, H % 512 == 0 or H % 8 == 0 with
// guards); row statistics by wave shuffles.  Column sums: each lane owns fixed
// columns across the rows its wave processes, waves combine through LDS in a
// fixed order, one partial row per workgroup, then a fixed-order finalize
// kernel — deterministic.
#include "mv_bert.h"
#include "mv_common.h"

#include <cstdlib>

namespace mv {
namespace tx {

constexpr int kRowsPerBlock = 32;      // 4 waves x 8 rows
constexpr float kSqrt1_2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ bool keep(uint32_t seed, uint32_t row, uint32_t col, uint32_t th) {
  return mix32(mix32(seed + row * 0x9E3779B1u) + col * 0x85EBCA6Bu) >= th;
}

// Exact-erf GELU (BERT's), with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7,
// far below bf16's 4e-3 resolution): one reciprocal, a 5-term polynomial and ONE
// exponential, exp(-v^2 / 2), which gelu'(v) reuses for the Gaussian pdf term.  ocml's
// erff is a branchy piecewise rational approximation; with it the bias-GELU passes were
// VALU-bound at ~2.4 TB/s (profiles/r2_bert_large_bs512_short_attn_bwd.md).
__device__ __forceinline__ void gelu_parts(float v, float* cdf, float* e) {
  const float z = fabsf(v) * kSqrt1_2;
  const float t = __builtin_amdgcn_rcpf(__builtin_fmaf(0.3275911f, z, 1.f));
  float p = __builtin_fmaf(1.061405429f, t, -1.453152027f);
  p = __builtin_fmaf(p, t, 1.421413741f);
  p = __builtin_fmaf(p, t, -0.284496736f);
  p = __builtin_fmaf(p, t, 0.254829592f);
  p *= t;
  *e = __expf(-z * z);                               // exp(-v^2 / 2)
  const float erf_abs = __builtin_fmaf(-p, *e, 1.f);
  *cdf = 0.5f + 0.5f * __builtin_copysignf(erf_abs, v);
}
__device__ __forceinline__ float gelu(float v) {
  float cdf, e;
  gelu_parts(v, &cdf, &e);
  return v * cdf;
}
__device__ __forceinline__ float gelu_grad(float v) {
  float cdf, e;
  gelu_parts(v, &cdf, &e);
  return __builtin_fmaf(v * kInvSqrt2Pi, e, cdf);
}

// --------------------------------------------------------------- bias + GELU
// 2-D geometry: a workgroup owns columns [c0, c0 + 2048) (256 lanes x 8) and
// a range of rows; each lane keeps its 8 columns' bias and partial sums.
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const __bf16* __restrict__ x,
                                                             const __bf16* __restrict__ b,
                                                             __bf16* __restrict__ y, int64_t M,
                                                             int N, int64_t rows_per_block) {
  const int c = blockIdx.y * 2048 + threadIdx.x * 8;
  if (c >= N) return;
  float bv[8];
  load8(b + c, bv);
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  int64_t r = r0;
  // 4 rows per step: 4 independent 16-B loads in flight per lane (one row at a time
  // left the lane waiting on each load's full latency: ~4 TB/s)
  for (; r + 3 < r1; r += 4) {
    float v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8(x + (r + u) * N + c, v[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[u][j] = gelu(v[u][j] + bv[j]);
      store8(y + (r + u) * N + c, v[u]);
    }
  }
  for (; r < r1; ++r) {
    float v[8];
    load8(x + r * N + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = gelu(v[j] + bv[j]);
    store8(y + r * N + c, v);
  }
}

__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const __bf16* __restrict__ dy,
                                                             const __bf16* __restrict__ x,
                                                             const __bf16* __restrict__ b,
                                                             __bf16* __restrict__ dx,
                                                             float* __restrict__ partial,
                                                             int64_t M, int N,
                                                             int64_t rows_per_block) {
  const int c = blockIdx.y * 2048 + threadIdx.x * 8;
  if (c >= N) return;
  float bv[8], acc[8];
  load8(b + c, bv);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  const int64_t r0 = blockIdx.x * rows_per_block;
  const int64_t r1 = r0 + rows_per_block < M ? r0 + rows_per_block : M;
  int64_t r = r0;
  for (; r + 1 < r1; r += 2) {   // 2 rows x 2 tensors = 4 loads in flight per lane
    float v[2][8], g[2][8];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      load8(x + (r + u) * N + c, v[u]);
      load8(dy + (r + u) * N + c, g[u]);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        g[u][j] *= gelu_grad(v[u][j] + bv[j]);
        acc[j] += g[u][j];
      }
      store8(dx + (r + u) * N + c, g[u]);
    }
  }
  for (; r < r1; ++r) {
    float v[8], g[8];
    load8(x + r * N + c, v);
    load8(dy + r * N + c, g);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] *= gelu_grad(v[j] + bv[j]);
      acc[j] += g[j];
    }
    store8(dx + r * N + c, g);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) partial[(int64_t)blockIdx.x * N + c + j] = acc[j];
}

// Column sums of fp32 partials -> bf16.  Partial row p of set `y` lives at
// partial + y*set_off + p*stride.  A workgroup owns 16 columns x 16 row groups
// (64 B coalesced per row, >= 192 workgroups for BERT's shapes); the 16 group
// sums combine through LDS in a fixed order: deterministic.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ partial, int P,
                                                      int N, int64_t stride, int64_t set_off,
                                                      __bf16* __restrict__ out0,
                                                      __bf16* __restrict__ out1,
                                                      __bf16* __restrict__ out2) {
  __bf16* out = blockIdx.y == 0 ? out0 : (blockIdx.y == 1 ? out1 : out2);
  if (!out) return;                                    // uniform per workgroup
  const int tc = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + tc;
  const float* base = partial + blockIdx.y * set_off + c;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < N) {
    int p = g;
    for (; p + 48 < P; p += 64) {
      s0 += base[(int64_t)p * stride];
      s1 += base[(int64_t)(p + 16) * stride];
      s2 += base[(int64_t)(p + 32) * stride];
      s3 += base[(int64_t)(p + 48) * stride];
    }
    for (; p < P; p += 16) s0 += base[(int64_t)p * stride];
  }
  __shared__ float red[16][17];
  red[g][tc] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][tc];
    out[c] = (__bf16)t;
  }
}

// ------------------------------------------------- bias + dropout + add + LN
struct LnArgs {
  const __bf16* z;      // [M, H] GEMM output (no bias)
  const __bf16* bias;   // [H] or null
  const __bf16* res;    // [M, H] residual or null
  const __bf16* gamma;  // [H]
  const __bf16* beta;   // [H]
  __bf16* v;            // [M, H] saved pre-LN sum
  __bf16* y;            // [M, H]
  float* mean;          // [M]
  float* rstd;          // [M]
  int64_t M;
  int H;
  float eps;
  float p_drop;
  uint32_t seed;
  uint32_t thresh;
};

template <int NCH>
__global__ __launch_bounds__(256) void ln_fwd_kernel(LnArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.M) return;
  const float inv_keep = a.p_drop > 0.f ? 1.f / (1.f - a.p_drop) : 1.f;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = k * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[k][j] = 0.f;
    if (c < a.H) {
      float z[8], bb[8], rr[8];
      load8(a.z + row * a.H + c, z);
      if (a.bias) load8(a.bias + c, bb);
      if (a.res) load8(a.res + row * a.H + c, rr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = z[j] + (a.bias ? bb[j] : 0.f);
        if (a.p_drop > 0.f)
          t = keep(a.seed, (uint32_t)row, (uint32_t)(c + j), a.thresh) ? t * inv_keep : 0.f;
        t += a.res ? rr[j] : 0.f;
        v[k][j] = (float)(__bf16)t;     // stats on the stored (bf16) value
        s += v[k][j];
      }
      if (a.v) store8(a.v + row * a.H + c, v[k]);
    }
  }
  const float mean = wave_sum(s) / (float)a.H;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    if (k * 512 + lane * 8 < a.H) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        q += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / (float)a.H + a.eps);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = k * 512 + lane * 8;
    if (c < a.H) {
      float gm[8], bt[8], o[8];
      load8(a.gamma + c, gm);
      load8(a.beta + c, bt);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * gm[j] + bt[j];
      store8(a.y + row * a.H + c, o);
    }
  }
  if (lane == 0) {
    a.mean[row] = mean;
    a.rstd[row] = rstd;
  }
}

struct LnBwdArgs {
  const __bf16* dy;     // [M, H]
  const __bf16* v;      // [M, H] saved pre-LN sum
  const float* mean;    // [M]
  const float* rstd;    // [M]
  const __bf16* gamma;  // [H]
  __bf16* dv;           // [M, H] grad of the sum (= residual grad)
  __bf16* dz;           // [M, H] grad of z (dropout backward), or null
  float* partial;       // [P][3][H]: dgamma, dbeta, dbias(= sum dz)
  int64_t M;
  int H;
  float p_drop;
  uint32_t seed;
  uint32_t thresh;
  const __bf16* dy2;    // [M, H] second gradient stream of y, added on load, or null
};

// Write one wave-partial set (this wave's 8 x NCH columns) into LDS slot w, then
// combine the 4 waves in fixed order into partial row `which` of this block.
template <int NCH>
__device__ __forceinline__ void block_colsum(const float (&src)[NCH][8], float (*red)[512],
                                             float* __restrict__ dst, int H) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) red[w][lane * 8 + j] = src[k][j];
    __syncthreads();
    for (int t = threadIdx.x; t < 512; t += 256) {
      const int c = k * 512 + t;
      if (c < H) dst[c] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    }
  }
}

template <int NCH>
__global__ __launch_bounds__(256) void ln_bwd_kernel(LnBwdArgs a) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float inv_keep = a.p_drop > 0.f ? 1.f / (1.f - a.p_drop) : 1.f;
  float dg[NCH][8], db[NCH][8], dzs[NCH][8], gm[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = k * 512 + lane * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) dg[k][j] = db[k][j] = dzs[k][j] = gm[k][j] = 0.f;
    if (c < a.H) load8(a.gamma + c, gm[k]);       // once per kernel, not per row
  }
  // the next row's dy / dy2 / v are loaded (raw 16-byte vectors) while the current
  // row is reduced and written: a wave keeps two rows of loads in flight instead of
  // waiting a full memory latency at the top of every row
  struct Raw {
    u32x4 dy[NCH], d2[NCH], v[NCH];
  };
  auto ld = [&](int64_t row, Raw& R) {
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 512 + lane * 8;
      R.dy[k] = R.d2[k] = R.v[k] = u32x4{0u, 0u, 0u, 0u};
      if (c < a.H && row < a.M) {
        R.dy[k] = *reinterpret_cast<const u32x4*>(a.dy + row * a.H + c);
        if (a.dy2) R.d2[k] = *reinterpret_cast<const u32x4*>(a.dy2 + row * a.H + c);
        R.v[k] = *reinterpret_cast<const u32x4*>(a.v + row * a.H + c);
      }
    }
  };
  auto unpack = [](const u32x4& r, float (&o)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[2 * j] = __uint_as_float(r[j] << 16);
      o[2 * j + 1] = __uint_as_float(r[j] & 0xffff0000u);
    }
  };
  const int64_t rbeg = (int64_t)blockIdx.x * kRowsPerBlock + w * (kRowsPerBlock / 4);
  constexpr bool PF = NCH <= 2;         // wider rows: no room for a second row of loads
  Raw cur, nxt;
  if (PF) ld(rbeg, cur);
  for (int rr = 0; rr < kRowsPerBlock / 4; ++rr) {
    const int64_t row = rbeg + rr;
    if (row >= a.M) break;
    if (!PF) ld(row, cur);
    else if (rr + 1 < kRowsPerBlock / 4) ld(row + 1, nxt);
    const float mean = a.mean[row], rstd = a.rstd[row];
    float xh[NCH][8], g[NCH][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 512 + lane * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) xh[k][j] = g[k][j] = 0.f;
      if (c < a.H) {
        float dy[8], vv[8];
        unpack(cur.dy[k], dy);
        if (a.dy2) {   // residual use of y (mivod.ops.bn.tap): no separate autograd add
          float e[8];
          unpack(cur.d2[k], e);
#pragma unroll
          for (int j = 0; j < 8; ++j) dy[j] += e[j];
        }
        unpack(cur.v[k], vv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (vv[j] - mean) * rstd;
          g[k][j] = dy[j] * gm[k][j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
          dg[k][j] += dy[j] * xh[k][j];
          db[k][j] += dy[j];
        }
      }
    }
    s1 = wave_sum(s1) / (float)a.H;
    s2 = wave_sum(s2) / (float)a.H;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = k * 512 + lane * 8;
      if (c < a.H) {
        float d[8], z[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          d[j] = rstd * (g[k][j] - s1 - xh[k][j] * s2);
          float t = d[j];
          if (a.p_drop > 0.f)
            t = keep(a.seed, (uint32_t)row, (uint32_t)(c + j), a.thresh) ? t * inv_keep : 0.f;
          z[j] = t;
          dzs[k][j] += t;
        }
        store8(a.dv + row * a.H + c, d);
        if (a.dz) store8(a.dz + row * a.H + c, z);
      }
    }
    if (PF) cur = nxt;
  }
  __shared__ float red[4][512];
  float* base = a.partial + (int64_t)blockIdx.x * 3 * a.H;
  block_colsum<NCH>(dg, red, base, a.H);
  block_colsum<NCH>(db, red, base + a.H, a.H);
  block_colsum<NCH>(dzs, red, base + 2 * a.H, a.H);
}

}  // namespace tx
}  // namespace mv

using namespace mv::tx;

static int64_t rows_per_block_for(int64_t M, int N, int64_t* P) {
  const int gy = (N + 2047) / 2048;
  static const int64_t total = [] {      // workgroups per pass (A/B knob MIVOD_TX_BLOCKS)
    const char* e = std::getenv("MIVOD_TX_BLOCKS");
    const int64_t v = e ? std::atoll(e) : 0;
    return v > 0 ? v : (int64_t)1024;
  }();
  int64_t blocks = total / gy;
  if (blocks < 1) blocks = 1;
  int64_t rpb = (M + blocks - 1) / blocks;
  if (rpb < 8) rpb = 8;
  *P = (M + rpb - 1) / rpb;
  return rpb;
}

int64_t mv_bias_gelu_partials(int64_t M, int N) {
  int64_t P;
  rows_per_block_for(M, N, &P);
  return P;
}

void mv_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t M, int N, hipStream_t st) {
  int64_t P;
  const int64_t rpb = rows_per_block_for(M, N, &P);
  hipLaunchKernelGGL(bias_gelu_fwd_kernel, dim3((unsigned)P, (N + 2047) / 2048), dim3(256), 0, st,
                     (const __bf16*)x, (const __bf16*)b, (__bf16*)y, M, N, rpb);
}

void mv_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, float* partial,
                      void* dbias, int64_t M, int N, hipStream_t st) {
  int64_t P;
  const int64_t rpb = rows_per_block_for(M, N, &P);
  hipLaunchKernelGGL(bias_gelu_bwd_kernel, dim3((unsigned)P, (N + 2047) / 2048), dim3(256), 0, st,
                     (const __bf16*)dy, (const __bf16*)x, (const __bf16*)b, (__bf16*)dx, partial,
                     M, N, rpb);
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 15) / 16, 1), dim3(256), 0, st,
                     (const float*)partial, (int)P, N, (int64_t)N, (int64_t)0, (__bf16*)dbias,
                     (__bf16*)nullptr, (__bf16*)nullptr);
}

int64_t mv_ln_partials(int64_t M) { return (M + kRowsPerBlock - 1) / kRowsPerBlock; }

void mv_ln_fwd(const LnFwdParams& p, hipStream_t st) {
  LnArgs a{(const __bf16*)p.z, (const __bf16*)p.bias, (const __bf16*)p.res,
           (const __bf16*)p.gamma, (const __bf16*)p.beta, (__bf16*)p.v, (__bf16*)p.y, p.mean,
           p.rstd, p.M, p.H, p.eps, p.p_drop, p.seed, p.thresh};
  const dim3 g((unsigned)((p.M + 3) / 4));
  if (p.H <= 512) hipLaunchKernelGGL(ln_fwd_kernel<1>, g, dim3(256), 0, st, a);
  else if (p.H <= 1024) hipLaunchKernelGGL(ln_fwd_kernel<2>, g, dim3(256), 0, st, a);
  else if (p.H <= 2048) hipLaunchKernelGGL(ln_fwd_kernel<4>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ln_fwd_kernel<8>, g, dim3(256), 0, st, a);
}

void mv_ln_bwd(const LnBwdParams& p, void* dgamma, void* dbeta, void* dbias, hipStream_t st) {
  LnBwdArgs a{(const __bf16*)p.dy, (const __bf16*)p.v, p.mean, p.rstd, (const __bf16*)p.gamma,
              (__bf16*)p.dv, (__bf16*)p.dz, p.partial, p.M, p.H, p.p_drop, p.seed, p.thresh,
              (const __bf16*)p.dy2};
  const int64_t P = mv_ln_partials(p.M);
  const dim3 g((unsigned)P);
  if (p.H <= 512) hipLaunchKernelGGL(ln_bwd_kernel<1>, g, dim3(256), 0, st, a);
  else if (p.H <= 1024) hipLaunchKernelGGL(ln_bwd_kernel<2>, g, dim3(256), 0, st, a);
  else if (p.H <= 2048) hipLaunchKernelGGL(ln_bwd_kernel<4>, g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(ln_bwd_kernel<8>, g, dim3(256), 0, st, a);
  // partial layout [P][3][H]: set stride H, row stride 3H; one launch for all three
  hipLaunchKernelGGL(colsum_kernel, dim3((p.H + 15) / 16, 3), dim3(256), 0, st,
                     (const float*)p.partial, (int)P, p.H, (int64_t)3 * p.H, (int64_t)p.H,
                     (__bf16*)dgamma, (__bf16*)dbeta, (__bf16*)dbias);
}
