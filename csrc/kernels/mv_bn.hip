// Fused NHWC BatchNorm (+ residual add) (+ ReLU) for bf16 activations on gfx950.
//
// Why: on ResNet-50 bf16 (bs 256, 1x MI355X) MIOpen's BatchNorm kernels plus the
// separate ReLU / residual-add / threshold-backward elementwise kernels took
// ~22 of 39 ms per step at ~3 TB/s (profiles/r1_resnet50_bs256_baseline_miopen_bn.md).
// Fusing them cuts HBM passes per BN layer from 5 to 3 (fwd, ReLU) / 8 to 4 (fwd,
// add+ReLU) and from 8 to 5 (bwd, ReLU) / 8 to 7 (bwd, add+ReLU), and every
// pass streams 16-byte lanes.
//
// Layout: x is [M, C] (channels_last, M = N*H*W), C % 8 == 0.  A workgroup owns
// a slab of CB = min(C, 256) channels (blockIdx.y) and a range of rows
// (blockIdx.x); each lane owns 8 consecutive channels of one row per step, so
// the per-channel coefficients stay in registers for the whole slab.
//
// Statistics are reduced deterministically (fixed-order block partials, then a
// fixed-order finalize) so every DP rank computes bit-identical results.
// Sums are taken around a per-channel shift (the running mean) to limit
// cancellation in E[x^2] - E[x]^2.
#include "mv_common.h"
#include "mv_bn.h"

#include <cstdlib>
#include <mutex>
#include <unordered_map>

namespace mv {
namespace bn {

constexpr int kCB = 256;    // channels per workgroup slab
constexpr int kTPR = kCB / kVec;  // 32 lanes per row (when C >= 256)
constexpr int kFinCh = 2;   // finalize: channels per workgroup
constexpr int kFinSub = kBlock / kFinCh;  // 128 partial-subsets per channel

struct Geo {
  int64_t M;
  int C;
  int CB;    // channels in this launch's slab width (<= kCB)
  int TPR;   // lanes per row
  int RPI;   // rows per iteration (per workgroup)
  int64_t RB;  // rows per workgroup
  // stats_kernel only: ds > 1 reads row r of the stride-ds grid of a [*, H, W, C] input
  // (the rows a stride-ds 1x1 conv reads) instead of row r of x
  int ds = 1, H = 1, W = 1;
};

__device__ __forceinline__ int64_t src_row(const Geo& g, int64_t r) {
  if (g.ds == 1) return r;
  const uint32_t Ho = (uint32_t)((g.H - 1) / g.ds + 1), Wo = (uint32_t)((g.W - 1) / g.ds + 1);
  const uint32_t r32 = (uint32_t)r, t = r32 / Wo, wo = r32 - t * Wo;
  const uint32_t n = t / Ho, ho = t - n * Ho;
  return ((int64_t)n * g.H + ho * g.ds) * g.W + wo * g.ds;
}

__device__ __forceinline__ void lane_map(const Geo& g, int* tc, int* tr, int* c, bool* valid) {
  *tc = threadIdx.x % g.TPR;
  *tr = threadIdx.x / g.TPR;
  *c = blockIdx.y * g.CB + *tc * kVec;
  *valid = (*tr < g.RPI) && (*c < g.C);
}

// Last read of a streamed activation (apply / dx passes: the statistics pass already
// read it): non-temporal, so it does not push reusable lines out of L2 / MALL.
// MIVOD_BN_NT=0 at run time selects default-policy loads (A/B switch).
template <bool NT>
__device__ __forceinline__ void ldlast(const __bf16* p, float (&v)[8]) {
  if (NT) load8_nt(p, v);
  else load8(p, v);
}

// Second gradient stream of row r.  ds == 1: same [M, C] layout as dy.  ds > 1: dy2
// is the gradient of a stride-ds 1x1 conv's input computed at the OUTPUT resolution
// ([N, ceil(H/ds), ceil(W/ds), C]); rows off the stride grid get zero (the shortcut
// downsample of a ResNet stage: no full-resolution zero-filled tensor exists).
template <bool NT>
__device__ __forceinline__ void ld_dy2(const __bf16* dy2, int64_t r, int c, int C, int ds,
                                       int H, int W, float (&v)[8]) {
  if (ds == 1) {
    ldlast<NT>(dy2 + r * C + c, v);
    return;
  }
  // 32-bit index math (the launcher guarantees M < 2^32): a 64-bit divide per row
  // costs ~100 ALU instructions per lane, comparable to the load itself
  const uint32_t r32 = (uint32_t)r, W32 = (uint32_t)W, H32 = (uint32_t)H;
  const uint32_t t = r32 / W32, w = r32 - t * W32;
  const uint32_t n = t / H32, h = t - n * H32;
  if ((h % (uint32_t)ds) | (w % (uint32_t)ds)) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    return;
  }
  const uint32_t Ho = (H32 + ds - 1) / ds, Wo = (W32 + ds - 1) / ds;
  const int64_t ro = ((int64_t)(n * Ho + h / ds)) * Wo + w / ds;
  ldlast<NT>(dy2 + ro * C + c, v);
}

// First read of a tensor a later pass reads again (statistics / reduce passes):
// non-temporal when RNT (the default, see bn_rnt).  The add+ReLU reduce (DZ) keeps x
// default-policy: its reduce time is unchanged either way, and the dx pass that follows
// runs ~8% faster on the lines it leaves (micro_bn: 491 -> 454 us at [6.4M, 64])
template <bool RNT>
__device__ __forceinline__ void ldfirst(const __bf16* p, float (&v)[8]) {
  if (RNT) load8_nt(p, v);
  else load8(p, v);
}

__device__ __forceinline__ void load8f(const float* p, float (&v)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = p[j];
}

// ---------------------------------------------------------------- forward
// U rows in flight per lane per iteration (16-byte loads)
template <int U, bool RNT = false>
__global__ __launch_bounds__(kBlock) void stats_kernel(const __bf16* __restrict__ x,
                                                        const float* __restrict__ shift,
                                                        float* __restrict__ partial, Geo g) {
  int tc, tr, c;
  bool valid;
  lane_map(g, &tc, &tr, &c, &valid);
  float s1[8], s2[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; sh[j] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * g.RB;
  const int64_t r1 = (r0 + g.RB < g.M) ? r0 + g.RB : g.M;
  if (valid) {
    if (shift) load8f(shift + c, sh);
    int64_t r = r0 + tr;
    for (; r + (U - 1) * g.RPI < r1; r += U * g.RPI) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) ldfirst<RNT>(x + src_row(g, r + u * g.RPI) * g.C + c, v[u]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float a = v[u][j] - sh[j];
          a1 += a;
          a2 += a * a;
        }
        s1[j] += a1;
        s2[j] += a2;
      }
    }
    for (; r < r1; r += g.RPI) {
      float v0[8];
      ldfirst<RNT>(x + src_row(g, r) * g.C + c, v0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = v0[j] - sh[j];
        s1[j] += a;
        s2[j] += a * a;
      }
    }
  }
  __shared__ float red[2][kBlock * kVec];   // [k][tr * CB + tc*8 + j]
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * kVec + j] = s1[j];
    red[1][threadIdx.x * kVec + j] = s2[j];
  }
  __syncthreads();
  const int cb_eff = min(g.CB, g.C - (int)blockIdx.y * g.CB);
  for (int v = threadIdx.x; v < 2 * cb_eff; v += kBlock) {
    const int k = v / cb_eff, cc = v % cb_eff;
    float s = 0.f;
    for (int t = 0; t < g.RPI; ++t) s += red[k][t * g.TPR * kVec + cc];
    partial[((int64_t)blockIdx.x * 2 + k) * g.C + blockIdx.y * g.CB + cc] = s;
  }
}

// Fixed-order reduction of [P][2][C] partials for kFinCh channels per block.
__device__ __forceinline__ void fin_reduce(const float* __restrict__ partial, int P, int C, int ch,
                                           float* o1, float* o2) {
  const int lc = threadIdx.x % kFinCh, sub = threadIdx.x / kFinCh;
  // 4 independent accumulator pairs keep 8 loads in flight per lane; the
  // combination order is fixed, so the result is deterministic.
  float a0 = 0.f, b0 = 0.f, a1 = 0.f, b1 = 0.f, a2 = 0.f, b2 = 0.f, a3 = 0.f, b3 = 0.f;
  if (ch < C) {
    const int64_t st = (int64_t)2 * C;
    const float* q = partial + ch;
    int p = sub;
    for (; p + 3 * kFinSub < P; p += 4 * kFinSub) {
      a0 += q[(int64_t)p * st];
      b0 += q[(int64_t)p * st + C];
      a1 += q[(int64_t)(p + kFinSub) * st];
      b1 += q[(int64_t)(p + kFinSub) * st + C];
      a2 += q[(int64_t)(p + 2 * kFinSub) * st];
      b2 += q[(int64_t)(p + 2 * kFinSub) * st + C];
      a3 += q[(int64_t)(p + 3 * kFinSub) * st];
      b3 += q[(int64_t)(p + 3 * kFinSub) * st + C];
    }
    for (; p < P; p += kFinSub) {
      a0 += q[(int64_t)p * st];
      b0 += q[(int64_t)p * st + C];
    }
  }
  float a = (a0 + a1) + (a2 + a3), b = (b0 + b1) + (b2 + b3);
  // fixed xor-tree across the 32 lanes of a wave that share this channel
  // (lane = sub*kFinCh + lc), then 4 wave partials combined in order via LDS
#pragma unroll
  for (int o = kFinCh; o < kWave; o <<= 1) {
    a += __shfl_xor(a, o, kWave);
    b += __shfl_xor(b, o, kWave);
  }
  __shared__ float red[2][kBlock / kWave][kFinCh];
  const int w = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  if (lane < kFinCh) {
    red[0][w][lane] = a;
    red[1][w][lane] = b;
  }
  __syncthreads();
  if (sub == 0) {
    float x = 0.f, y = 0.f;
#pragma unroll
    for (int k = 0; k < kBlock / kWave; ++k) { x += red[0][k][lc]; y += red[1][k][lc]; }
    *o1 = x;
    *o2 = y;
  }
}

__global__ __launch_bounds__(kBlock) void finalize_fwd_kernel(
    const float* __restrict__ partial, int P, int64_t M, int C, float* __restrict__ rmean,
    float* __restrict__ rvar, const float* __restrict__ gamma, const float* __restrict__ beta,
    float momentum, float eps, float* __restrict__ save_mean, float* __restrict__ save_invstd,
    float* __restrict__ scale, float* __restrict__ bias) {
  const int ch = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  float s1 = 0.f, s2 = 0.f;
  fin_reduce(partial, P, C, ch, &s1, &s2);
  if (threadIdx.x / kFinCh != 0 || ch >= C) return;
  const float inv_m = 1.f / (float)M;
  const float sh = rmean ? rmean[ch] : 0.f;
  const float ms = s1 * inv_m;
  float var = fmaxf(s2 * inv_m - ms * ms, 0.f);
  const float mean = sh + ms;
  const float invstd = 1.f / sqrtf(var + eps);
  save_mean[ch] = mean;
  save_invstd[ch] = invstd;
  if (rmean) {
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    rmean[ch] = (1.f - momentum) * sh + momentum * mean;
    rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * unb;
  }
  const float sc = (gamma ? gamma[ch] : 1.f) * invstd;
  scale[ch] = sc;
  bias[ch] = (beta ? beta[ch] : 0.f) - mean * sc;
}

// bit j set <=> output channel c+j of the row is > 0 (the add+ReLU backward mask:
// 1 byte per 8 channels instead of re-reading the 16-byte bf16 output)
__device__ __forceinline__ uint8_t relu_bits(const float (&v)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) m |= (v[j] > 0.f ? 1u : 0u) << j;
  return (uint8_t)m;
}

// U rows in flight per lane per iteration (U = 2 by default; MIVOD_BN_APPLY_U=4)
template <bool RELU, bool RES, bool NT = true, int U = 4>
__global__ __launch_bounds__(kBlock) void apply_kernel(const __bf16* __restrict__ x,
                                                        const __bf16* __restrict__ res,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ bias,
                                                        __bf16* __restrict__ y, Geo g,
                                                        uint8_t* __restrict__ mask) {
  int tc, tr, c;
  bool valid;
  lane_map(g, &tc, &tr, &c, &valid);
  if (!valid) return;
  const int C8 = g.C / kVec;
  float sc[8], bi[8];
  load8f(scale + c, sc);
  load8f(bias + c, bi);
  const int64_t r0 = (int64_t)blockIdx.x * g.RB;
  const int64_t r1 = (r0 + g.RB < g.M) ? r0 + g.RB : g.M;
  int64_t r = r0 + tr;
  for (; r + (U - 1) * g.RPI < r1; r += U * g.RPI) {
    float v[U][8], q[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) ldlast<NT>(x + (r + u * g.RPI) * g.C + c, v[u]);
    if (RES) {
#pragma unroll
      for (int u = 0; u < U; ++u) ldlast<NT>(res + (r + u * g.RPI) * g.C + c, q[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = __builtin_fmaf(v[u][j], sc[j], bi[j]);
        if (RES) a += q[u][j];
        if (RELU) a = fmaxf(a, 0.f);
        v[u][j] = a;
      }
      store8(y + (r + u * g.RPI) * g.C + c, v[u]);
      if (RELU && RES && mask) mask[(r + u * g.RPI) * C8 + c / kVec] = relu_bits(v[u]);
    }
  }
  for (; r < r1; r += g.RPI) {
    float v0[8], q0[8];
    const int64_t o0 = r * g.C + c;
    ldlast<NT>(x + o0, v0);
    if (RES) ldlast<NT>(res + o0, q0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a = __builtin_fmaf(v0[j], sc[j], bi[j]);
      if (RES) a += q0[j];
      if (RELU) a = fmaxf(a, 0.f);
      v0[j] = a;
    }
    store8(y + o0, v0);
    if (RELU && RES && mask) mask[r * C8 + c / kVec] = relu_bits(v0);
  }
}

// BN + ReLU apply that also emits per-column sums of the bf16 OUTPUT (fixed-order
// [P][C] partials): the colsum(x) term of a consumer 1x1 conv's folded BN backward
// (ops.bn._Conv1x1BNFold: dW = ... + cc (x) colsum(x)) without a statistics pass over x.
// No early return: every lane reaches the block reduction's barrier.
template <int U>
__global__ __launch_bounds__(kBlock) void apply_colsum_kernel(const __bf16* __restrict__ x,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ bias,
                                                               __bf16* __restrict__ y, Geo g,
                                                               float* __restrict__ partial) {
  int tc, tr, c;
  bool valid;
  lane_map(g, &tc, &tr, &c, &valid);
  float cs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = 0.f;
  if (valid) {
    float sc[8], bi[8];
    load8f(scale + c, sc);
    load8f(bias + c, bi);
    const int64_t r0 = (int64_t)blockIdx.x * g.RB;
    const int64_t r1 = (r0 + g.RB < g.M) ? r0 + g.RB : g.M;
    int64_t r = r0 + tr;
    for (; r + (U - 1) * g.RPI < r1; r += U * g.RPI) {
      float v[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) ldlast<true>(x + (r + u * g.RPI) * g.C + c, v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[u][j] = fmaxf(__builtin_fmaf(v[u][j], sc[j], bi[j]), 0.f);
          cs[j] += (float)(__bf16)v[u][j];
        }
        store8(y + (r + u * g.RPI) * g.C + c, v[u]);
      }
    }
    for (; r < r1; r += g.RPI) {
      float v0[8];
      ldlast<true>(x + r * g.C + c, v0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v0[j] = fmaxf(__builtin_fmaf(v0[j], sc[j], bi[j]), 0.f);
        cs[j] += (float)(__bf16)v0[j];
      }
      store8(y + r * g.C + c, v0);
    }
  }
  __shared__ float red[kBlock * kVec];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * kVec + j] = cs[j];
  __syncthreads();
  const int cb_eff = min(g.CB, g.C - (int)blockIdx.y * g.CB);
  for (int cc = threadIdx.x; cc < cb_eff; cc += kBlock) {
    float t = 0.f;
    for (int q = 0; q < g.RPI; ++q) t += red[q * g.TPR * kVec + cc];
    partial[(int64_t)blockIdx.x * g.C + blockIdx.y * g.CB + cc] = t;
  }
}

// ---------------------------------------------------------------- backward
// MODE 0: no activation (d = dy)
// MODE 1: ReLU, mask recomputed from x:  d = (fma(x, scale, bias) > 0) ? dy : 0
// MODE 2: add + ReLU, mask from the saved output y: d = (y > 0) ? dy : 0; d is
//         written out (it is also the residual branch's gradient)
// MODE 3: MODE 2 with the forward's 1-bit-per-channel mask ([M, C/8] bytes) in place
//         of y: one byte per lane-row instead of a 16-byte bf16 load (~1/5 of the
//         pass's HBM traffic)
template <int MODE>
__device__ __forceinline__ void masked(const float (&dy)[8], const float (&x)[8],
                                       const float (&yv)[8], const float (&sc)[8],
                                       const float (&bi)[8], float (&d)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (MODE == 3) d[j] = (__float_as_uint(yv[0]) >> j) & 1u ? dy[j] : 0.f;
    else if (MODE == 0) d[j] = dy[j];
    else if (MODE == 1) d[j] = __builtin_fmaf(x[j], sc[j], bi[j]) > 0.f ? dy[j] : 0.f;
    else d[j] = yv[j] > 0.f ? dy[j] : 0.f;
  }
}

// last-use reads (dy2, the saved output y, and dy in MODE 2 where the dx pass reads dz)
// are non-temporal
template <int MODE, bool NT = true, bool RNT = false>
__global__ __launch_bounds__(kBlock) void bwd_reduce_kernel(
    const __bf16* __restrict__ dy, const __bf16* __restrict__ dy2, const __bf16* __restrict__ x,
    const __bf16* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ scale,
    const float* __restrict__ bias, __bf16* __restrict__ dz, float* __restrict__ partial, Geo g,
    int ds, int H, int W) {
  int tc, tr, c;
  bool valid;
  lane_map(g, &tc, &tr, &c, &valid);
  constexpr bool DZ = MODE >= 2;   // writes the masked gradient (residual branch)
  const uint8_t* mk = (const uint8_t*)y;
  const int C8 = g.C / kVec;
  float s1[8], s2[8], mu[8], sc[8], bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; mu[j] = 0.f; sc[j] = 0.f; bi[j] = 0.f; }
  const int64_t r0 = (int64_t)blockIdx.x * g.RB;
  const int64_t r1 = (r0 + g.RB < g.M) ? r0 + g.RB : g.M;
  if (valid) {
    load8f(mean + c, mu);
    if (MODE == 1) { load8f(scale + c, sc); load8f(bias + c, bi); }
    int64_t r = r0 + tr;
    for (; r + g.RPI < r1; r += 2 * g.RPI) {
      float a0[8], a1[8], x0[8], x1[8], y0[8], y1[8], d0[8], d1[8];
      const int64_t o0 = r * g.C + c, o1 = (r + g.RPI) * g.C + c;
      if (DZ) ldlast<NT>(dy + o0, a0); else ldfirst<RNT>(dy + o0, a0);
      if (DZ) ldlast<NT>(dy + o1, a1); else ldfirst<RNT>(dy + o1, a1);
      if (dy2) {   // second gradient stream of a tapped output (uniform branch)
        float b0[8], b1[8];
        ld_dy2<NT>(dy2, r, c, g.C, ds, H, W, b0);
        ld_dy2<NT>(dy2, r + g.RPI, c, g.C, ds, H, W, b1);
#pragma unroll
        for (int j = 0; j < 8; ++j) { a0[j] += b0[j]; a1[j] += b1[j]; }
      }
      ldfirst<RNT && !DZ>(x + o0, x0);
      ldfirst<RNT && !DZ>(x + o1, x1);
      if (MODE == 2) { ldlast<NT>(y + o0, y0); ldlast<NT>(y + o1, y1); }
      if (MODE == 3) {
        y0[0] = __uint_as_float((uint32_t)mk[r * C8 + c / kVec]);
        y1[0] = __uint_as_float((uint32_t)mk[(r + g.RPI) * C8 + c / kVec]);
      }
      masked<MODE>(a0, x0, y0, sc, bi, d0);
      masked<MODE>(a1, x1, y1, sc, bi, d1);
      if (DZ) { store8(dz + o0, d0); store8(dz + o1, d1); }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += d0[j] + d1[j];
        s2[j] += d0[j] * (x0[j] - mu[j]) + d1[j] * (x1[j] - mu[j]);
      }
    }
    for (; r < r1; r += g.RPI) {
      float a0[8], x0[8], y0[8], d0[8];
      const int64_t o0 = r * g.C + c;
      if (DZ) ldlast<NT>(dy + o0, a0); else ldfirst<RNT>(dy + o0, a0);
      if (dy2) {
        float b0[8];
        ld_dy2<NT>(dy2, r, c, g.C, ds, H, W, b0);
#pragma unroll
        for (int j = 0; j < 8; ++j) a0[j] += b0[j];
      }
      ldfirst<RNT && !DZ>(x + o0, x0);
      if (MODE == 2) ldlast<NT>(y + o0, y0);
      if (MODE == 3) y0[0] = __uint_as_float((uint32_t)mk[r * C8 + c / kVec]);
      masked<MODE>(a0, x0, y0, sc, bi, d0);
      if (DZ) store8(dz + o0, d0);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += d0[j];
        s2[j] += d0[j] * (x0[j] - mu[j]);
      }
    }
  }
  __shared__ float red[2][kBlock * kVec];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][threadIdx.x * kVec + j] = s1[j];
    red[1][threadIdx.x * kVec + j] = s2[j];
  }
  __syncthreads();
  const int cb_eff = min(g.CB, g.C - (int)blockIdx.y * g.CB);
  for (int v = threadIdx.x; v < 2 * cb_eff; v += kBlock) {
    const int k = v / cb_eff, cc = v % cb_eff;
    float s = 0.f;
    for (int t = 0; t < g.RPI; ++t) s += red[k][t * g.TPR * kVec + cc];
    partial[((int64_t)blockIdx.x * 2 + k) * g.C + blockIdx.y * g.CB + cc] = s;
  }
}

__global__ __launch_bounds__(kBlock) void finalize_bwd_kernel(
    const float* __restrict__ partial, int P, int64_t M, int C, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ ca,
    float* __restrict__ cb, float* __restrict__ cc) {
  const int ch = blockIdx.x * kFinCh + threadIdx.x % kFinCh;
  float sdz = 0.f, sdzx = 0.f;
  fin_reduce(partial, P, C, ch, &sdz, &sdzx);
  if (threadIdx.x / kFinCh != 0 || ch >= C) return;
  const float is = invstd[ch];
  if (dgamma) dgamma[ch] = sdzx * is;
  if (dbeta) dbeta[ch] = sdz;
  const float gm = gamma ? gamma[ch] : 1.f;
  const float inv_m = 1.f / (float)M;
  const float a = gm * is;
  const float b = -a * is * is * sdzx * inv_m;
  ca[ch] = a;
  cb[ch] = b;
  cc[ch] = -a * sdz * inv_m - b * mean[ch];
}

template <int MODE, bool NT = true, int U = 4>
__global__ __launch_bounds__(kBlock) void bwd_dx_kernel(
    const __bf16* __restrict__ d_in, const __bf16* __restrict__ x,
    const float* __restrict__ scale, const float* __restrict__ bias, const float* __restrict__ ca,
    const float* __restrict__ cb, const float* __restrict__ cc, __bf16* __restrict__ dx, Geo g) {
  int tc, tr, c;
  bool valid;
  lane_map(g, &tc, &tr, &c, &valid);
  if (!valid) return;
  float a[8], b[8], k[8], sc[8], bi[8];
  load8f(ca + c, a);
  load8f(cb + c, b);
  load8f(cc + c, k);
  if (MODE == 1) { load8f(scale + c, sc); load8f(bias + c, bi); }
  const int64_t r0 = (int64_t)blockIdx.x * g.RB;
  const int64_t r1 = (r0 + g.RB < g.M) ? r0 + g.RB : g.M;
  int64_t r = r0 + tr;
  for (; r + (U - 1) * g.RPI < r1; r += U * g.RPI) {
    float d[U][8], xv[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) ldlast<NT>(d_in + (r + u * g.RPI) * g.C + c, d[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) ldlast<NT>(x + (r + u * g.RPI) * g.C + c, xv[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float e = d[u][j];
        if (MODE == 1) e = __builtin_fmaf(xv[u][j], sc[j], bi[j]) > 0.f ? e : 0.f;
        d[u][j] = a[j] * e + (b[j] * xv[u][j] + k[j]);
      }
      store8(dx + (r + u * g.RPI) * g.C + c, d[u]);
    }
  }
  for (; r < r1; r += g.RPI) {
    float d0[8], x0[8];
    const int64_t o0 = r * g.C + c;
    ldlast<NT>(d_in + o0, d0);
    ldlast<NT>(x + o0, x0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float e0 = d0[j];
      if (MODE == 1) e0 = __builtin_fmaf(x0[j], sc[j], bi[j]) > 0.f ? e0 : 0.f;
      d0[j] = a[j] * e0 + (b[j] * x0[j] + k[j]);
    }
    store8(dx + o0, d0);
  }
}

static Geo make_geo(int64_t M, int C, int64_t rows_per_block) {
  Geo g;
  g.M = M;
  g.C = C;
  g.CB = C < kCB ? C : kCB;
  g.TPR = g.CB / kVec;
  g.RPI = kBlock / g.TPR;
  int64_t rb = rows_per_block;
  if (rb < g.RPI) rb = g.RPI;
  rb = (rb + g.RPI - 1) / g.RPI * g.RPI;
  g.RB = rb;
  return g;
}

static dim3 grid_of(const Geo& g) {
  const int64_t gx = (g.M + g.RB - 1) / g.RB;
  const int gy = (g.C + g.CB - 1) / g.CB;
  return dim3((unsigned)gx, (unsigned)gy);
}

// ---------------------------------------------------------------- launch shape
// Every BN pass is one round of exactly the workgroups the chip holds at once
// (occupancy x CUs, from the HIP occupancy API): with a fixed 2048/4096-block
// grid the kernels whose VGPR count allows 7 (not 8) workgroups per CU ran a
// second, 1/7-full round as a tail — the stats pass sat at ~4.6 TB/s
// (scripts/micro_bn.py).  Each workgroup streams one contiguous row range.
static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  return n;
}

static int resident_blocks(const void* fn) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(fn);
  if (it != cache.end()) return it->second;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, kBlock, 0) != hipSuccess || per < 1)
    per = 1;
  const int r = per * num_cus();
  cache.emplace(fn, r);
  return r;
}

// one resident round of workgroups, >= min_rows rows each, <= cap row blocks
static Geo round_geo(int64_t M, int C, const void* fn, int64_t min_rows, int64_t cap) {
  Geo g0 = make_geo(M, C, min_rows);
  const int gy = (C + g0.CB - 1) / g0.CB;
  int64_t bx = resident_blocks(fn) / gy;
  if (bx < 1) bx = 1;
  const int64_t by_rows = (M + min_rows - 1) / min_rows;
  if (bx > by_rows) bx = by_rows;
  if (bx > cap) bx = cap;
  if (bx < 1) bx = 1;
  return make_geo(M, C, (M + bx - 1) / bx);
}

}  // namespace bn
}  // namespace mv

using namespace mv;
using namespace mv::bn;

// Upper bound on the row-partials a reduction pass produces (sizes the
// [P][2][C] workspace); the launchers pick the actual count <= this.
int mv_bn_partials(int64_t M, int C) {
  Geo g = make_geo(M, C, 64);
  const int gy = (C + g.CB - 1) / g.CB;
  int64_t p = (M + 63) / 64;
  const int64_t cap = 2048 / gy > 0 ? 2048 / gy : 1;
  if (p > cap) p = cap;
  if (p < 1) p = 1;
  return (int)p;
}

// MIVOD_BN_NT (default 1): non-temporal last-use loads in the apply / dx passes
static bool bn_nt() {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_BN_NT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Non-temporal loads in the statistics / reduce passes too (MIVOD_BN_RNT=0: default
// policy).  scripts/micro_bn.py, bs512 shapes: stats 202 -> 125 us and reduce(ReLU)
// 335 -> 257 us at [1.6M, 256]; the following apply / dx pass loses ~50 us of that
// (it no longer finds lines the reduce pass left behind), net ~4% per BN layer.
static bool bn_rnt() {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_BN_RNT");
    return !(e && e[0] == '0');
  }();
  return on;
}

static Geo reduce_geo(int64_t M, int C, int P, const void* fn) {
  return round_geo(M, C, fn, 64, P);
}

static Geo apply_geo(int64_t M, int C, const void* fn) {
  return round_geo(M, C, fn, 64, 1 << 30);
}

void mv_bn_fwd_train(const void* x, const void* res, void* y, int64_t M, int C, float* rmean,
                     float* rvar, const float* gamma, const float* beta, float momentum, float eps,
                     bool relu, float* partial, int P, float* save_mean, float* save_invstd,
                     float* scale, float* bias, hipStream_t st, void* mask) {
  dim3 grr;
  if (bn_rnt()) {
    Geo gr = reduce_geo(M, C, P, (const void*)&stats_kernel<8, true>);
    grr = grid_of(gr);
    hipLaunchKernelGGL((stats_kernel<8, true>), grr, dim3(kBlock), 0, st, (const __bf16*)x, rmean,
                       partial, gr);
  } else {
    Geo gr = reduce_geo(M, C, P, (const void*)&stats_kernel<8>);
    grr = grid_of(gr);
    hipLaunchKernelGGL(stats_kernel<8>, grr, dim3(kBlock), 0, st, (const __bf16*)x, rmean, partial, gr);
  }
  hipLaunchKernelGGL(finalize_fwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kBlock), 0, st,
                     partial, (int)grr.x, M, C, rmean, rvar, gamma, beta, momentum, eps, save_mean,
                     save_invstd, scale, bias);
  if (y) mv_bn_apply(x, res, y, M, C, scale, bias, relu, st, mask);   // y == null: statistics only
}

// Statistics (no running-stat update, no apply) of the rows a stride-ds 1x1 conv reads
// from x [Nb, H, W, C]: mean / invstd over Nb * ceil(H/ds) * ceil(W/ds) rows, no strided copy
void mv_bn_stats_strided(const void* x, int Nb, int H, int W, int C, int ds, float* partial,
                         int P, float* save_mean, float* save_invstd, float* scale, float* bias,
                         hipStream_t st) {
  const int64_t M = (int64_t)Nb * ((H - 1) / ds + 1) * ((W - 1) / ds + 1);
  Geo gr = reduce_geo(M, C, P, (const void*)&stats_kernel<8, true>);
  gr.ds = ds;
  gr.H = H;
  gr.W = W;
  const dim3 grr = grid_of(gr);
  hipLaunchKernelGGL((stats_kernel<8, true>), grr, dim3(kBlock), 0, st, (const __bf16*)x,
                     (const float*)nullptr, partial, gr);
  hipLaunchKernelGGL(finalize_fwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kBlock), 0, st,
                     partial, (int)grr.x, M, C, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f,
                     save_mean, save_invstd, scale, bias);
}

// The statistics were produced elsewhere (the 1x1 conv GEMM's fused epilogue,
// mv_gemm.hip): [P][2][C] partials around shift = running mean, same layout as
// stats_kernel's.  Finalize (+ running-stat update) and apply only.
void mv_bn_fwd_from_partials(const void* x, const void* res, void* y, int64_t M, int C,
                             float* rmean, float* rvar, const float* gamma, const float* beta,
                             float momentum, float eps, bool relu, const float* partial, int P,
                             float* save_mean, float* save_invstd, float* scale, float* bias,
                             hipStream_t st, void* mask) {
  hipLaunchKernelGGL(finalize_fwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kBlock), 0, st,
                     partial, P, M, C, rmean, rvar, gamma, beta, momentum, eps, save_mean,
                     save_invstd, scale, bias);
  if (y) mv_bn_apply(x, res, y, M, C, scale, bias, relu, st, mask);
}

// apply / dx passes: 4 rows in flight per lane (ResNet-50 bs2048 bench A/B, two boxes:
// +0.2% / +0.4% over 2; equal on the bs512 shapes, scripts/micro_bn.py);
// MIVOD_BN_APPLY_U=2 selects 2
static bool apply_u2() {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_BN_APPLY_U");
    return e && e[0] == '2';
  }();
  return on;
}

template <bool RELU, bool RES, bool NT, int U>
static void launch_apply_u(const __bf16* x, const __bf16* r, const float* scale,
                           const float* bias, __bf16* y, int64_t M, int C, hipStream_t st,
                           uint8_t* mask) {
  Geo ga = apply_geo(M, C, (const void*)&apply_kernel<RELU, RES, NT, U>);
  hipLaunchKernelGGL((apply_kernel<RELU, RES, NT, U>), grid_of(ga), dim3(kBlock), 0, st, x, r,
                     scale, bias, y, ga, mask);
}

template <bool RELU, bool RES>
static void launch_apply(const __bf16* x, const __bf16* r, const float* scale, const float* bias,
                         __bf16* y, int64_t M, int C, hipStream_t st, uint8_t* mask) {
  if (bn_nt()) {
    if (apply_u2()) launch_apply_u<RELU, RES, true, 2>(x, r, scale, bias, y, M, C, st, mask);
    else launch_apply_u<RELU, RES, true, 4>(x, r, scale, bias, y, M, C, st, mask);
  } else {
    launch_apply_u<RELU, RES, false, 2>(x, r, scale, bias, y, M, C, st, mask);
  }
}

void mv_bn_apply(const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
                 const float* bias, bool relu, hipStream_t st, void* mask) {
  uint8_t* mk = (uint8_t*)mask;   // add+ReLU only
  const __bf16* xp = (const __bf16*)x;
  const __bf16* rp = (const __bf16*)res;
  __bf16* yp = (__bf16*)y;
  if (res) {
    if (relu) launch_apply<true, true>(xp, rp, scale, bias, yp, M, C, st, mk);
    else launch_apply<false, true>(xp, rp, scale, bias, yp, M, C, st, nullptr);
  } else {
    if (relu) launch_apply<true, false>(xp, rp, scale, bias, yp, M, C, st, nullptr);
    else launch_apply<false, false>(xp, rp, scale, bias, yp, M, C, st, nullptr);
  }
}

template <int MODE>
static int launch_bwd_reduce(const __bf16* dy, const __bf16* dy2, const __bf16* x,
                             const __bf16* y, const float* mean, const float* scale,
                             const float* bias, __bf16* dz, float* partial, int P, int64_t M,
                             int C, int ds, int H, int W, hipStream_t st) {
  if (bn_nt() && bn_rnt()) {
    Geo gr = reduce_geo(M, C, P, (const void*)&bwd_reduce_kernel<MODE, true, true>);
    dim3 grr = grid_of(gr);
    hipLaunchKernelGGL((bwd_reduce_kernel<MODE, true, true>), grr, dim3(kBlock), 0, st, dy, dy2, x,
                       y, mean, scale, bias, dz, partial, gr, ds, H, W);
    return (int)grr.x;
  }
  if (bn_nt()) {
    Geo gr = reduce_geo(M, C, P, (const void*)&bwd_reduce_kernel<MODE, true>);
    dim3 grr = grid_of(gr);
    hipLaunchKernelGGL((bwd_reduce_kernel<MODE, true>), grr, dim3(kBlock), 0, st, dy, dy2, x, y,
                       mean, scale, bias, dz, partial, gr, ds, H, W);
    return (int)grr.x;
  }
  Geo gr = reduce_geo(M, C, P, (const void*)&bwd_reduce_kernel<MODE, false>);
  dim3 grr = grid_of(gr);
  hipLaunchKernelGGL((bwd_reduce_kernel<MODE, false>), grr, dim3(kBlock), 0, st, dy, dy2, x, y,
                     mean, scale, bias, dz, partial, gr, ds, H, W);
  return (int)grr.x;
}

template <int MODE, bool NT, int U>
static void launch_bwd_dx_u(const __bf16* d, const __bf16* x, const float* scale,
                            const float* bias, const float* ca, const float* cb, const float* cc,
                            __bf16* dx, int64_t M, int C, hipStream_t st) {
  Geo ga = apply_geo(M, C, (const void*)&bwd_dx_kernel<MODE, NT, U>);
  hipLaunchKernelGGL((bwd_dx_kernel<MODE, NT, U>), grid_of(ga), dim3(kBlock), 0, st, d, x, scale,
                     bias, ca, cb, cc, dx, ga);
}

template <int MODE>
static void launch_bwd_dx(const __bf16* d, const __bf16* x, const float* scale, const float* bias,
                          const float* ca, const float* cb, const float* cc, __bf16* dx, int64_t M,
                          int C, hipStream_t st) {
  if (bn_nt()) {
    if (apply_u2()) launch_bwd_dx_u<MODE, true, 2>(d, x, scale, bias, ca, cb, cc, dx, M, C, st);
    else launch_bwd_dx_u<MODE, true, 4>(d, x, scale, bias, ca, cb, cc, dx, M, C, st);
  } else {
    launch_bwd_dx_u<MODE, false, 2>(d, x, scale, bias, ca, cb, cc, dx, M, C, st);
  }
}

void mv_bn_bwd(int mode, const void* dy, const void* dy2, const void* x, const void* y, void* dz, void* dx,
               int64_t M, int C, const float* save_mean, const float* save_invstd,
               const float* gamma, const float* scale, const float* bias, float* dgamma,
               float* dbeta, float* partial, int P, float* ca, float* cb, float* cc,
               int dy2_stride, int H, int W, hipStream_t st) {
  const __bf16* dyp = (const __bf16*)dy;
  const __bf16* dy2p = (const __bf16*)dy2;
  const __bf16* xp = (const __bf16*)x;
  const __bf16* yp = (const __bf16*)y;
  __bf16* dzp = (__bf16*)dz;
  int pa;
  switch (mode) {
    case 0: pa = launch_bwd_reduce<0>(dyp, dy2p, xp, yp, save_mean, scale, bias, dzp, partial, P, M, C, dy2_stride, H, W, st); break;
    case 1: pa = launch_bwd_reduce<1>(dyp, dy2p, xp, yp, save_mean, scale, bias, dzp, partial, P, M, C, dy2_stride, H, W, st); break;
    case 2: pa = launch_bwd_reduce<2>(dyp, dy2p, xp, yp, save_mean, scale, bias, dzp, partial, P, M, C, dy2_stride, H, W, st); break;
    default: pa = launch_bwd_reduce<3>(dyp, dy2p, xp, yp, save_mean, scale, bias, dzp, partial, P, M, C, dy2_stride, H, W, st); break;
  }
  hipLaunchKernelGGL(finalize_bwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kBlock), 0, st,
                     partial, pa, M, C, save_mean, save_invstd, gamma, dgamma, dbeta, ca, cb, cc);
  __bf16* dxp = (__bf16*)dx;
  switch (mode) {
    case 0: launch_bwd_dx<0>(dyp, xp, scale, bias, ca, cb, cc, dxp, M, C, st); break;
    case 1: launch_bwd_dx<1>(dyp, xp, scale, bias, ca, cb, cc, dxp, M, C, st); break;
    default: launch_bwd_dx<0>((const __bf16*)dzp, xp, scale, bias, ca, cb, cc, dxp, M, C, st); break;
  }
}

// BN backward whose reduce pass ran inside the producing data-gradient GEMM
// (mv_gemm_nt_bn_bwd): dz and its [P][2][C] partials (sum dz, sum dz (x - mean)) are
// given, so only the finalize and the dx pass remain.
void mv_bn_bwd_from_partials(const void* dz, const void* x, void* dx, int64_t M, int C,
                             const float* save_mean, const float* save_invstd,
                             const float* gamma, const float* scale, const float* bias,
                             float* dgamma, float* dbeta, const float* partial, int P, float* ca,
                             float* cb, float* cc, hipStream_t st) {
  hipLaunchKernelGGL(finalize_bwd_kernel, dim3((C + kFinCh - 1) / kFinCh), dim3(kBlock), 0, st,
                     partial, P, M, C, save_mean, save_invstd, gamma, dgamma, dbeta, ca, cb, cc);
  if (dx)   // dx == nullptr: coefficients only (ops.conv._Conv1x1BNFold folds dx into its GEMMs)
    launch_bwd_dx<0>((const __bf16*)dz, (const __bf16*)x, scale, bias, ca, cb, cc, (__bf16*)dx, M,
                     C, st);
}

// y = relu(x * scale + bias) + [P][C] column-sum partials of y; returns P (<= mv_bn_partials)
int mv_bn_apply_colsum(const void* x, void* y, int64_t M, int C, const float* scale,
                       const float* bias, float* partial, hipStream_t st) {
  Geo g = reduce_geo(M, C, mv_bn_partials(M, C), (const void*)&apply_colsum_kernel<2>);
  const dim3 grid = grid_of(g);
  hipLaunchKernelGGL(apply_colsum_kernel<2>, grid, dim3(kBlock), 0, st, (const __bf16*)x, scale,
                     bias, (__bf16*)y, g, partial);
  return (int)grid.x;
}
