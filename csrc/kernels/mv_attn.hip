// Fused multi-head attention (forward + backward) for BERT on gfx950 MFMA.
//
// Shapes: qkv [b, s, 3, h, 64] bf16 (the fused QKV projection), out [b, s, h, 64]
// bf16, optional additive key bias [b, s] fp32, attention-probability dropout.
// Head dim is fixed at 64 (BERT base/large).  All products run on
// v_mfma_f32_16x16x32_bf16 (wave64; lane l holds A[l&15][8(l>>4)+j],
// B[8(l>>4)+j][l&15], C/D row (l>>4)*4+r, col l&15).
//
// The k-major operands (V^T, Q^T, dO^T, K^T) are read from row-major LDS images with
// gfx950's transposed LDS read (ds_read_b64_tr_b16, tr8 below): no element-wise
// transposed LDS copies.
//
// Forward (one workgroup = 4 waves = 64 queries of one (b, h)): each wave keeps
// its 16 query rows as MFMA B fragments, streams K / V^T blocks of 64 keys
// through LDS, computes S^T = K Q^T so that every lane owns ONE query column
// (softmax max/sum reduce with two xor-shuffles), keeps the running max / sum
// online (exp2 domain), and feeds P straight from the accumulators into P.V as
// the A operand — the MFMA k order is permuted (keys 4g+r of two 16-key tiles)
// and V^T is read from LDS in that same order, so no transpose is needed.
// The log-sum-exp per query is saved for the backward pass.
//
// Backward (FlashAttention-2 style, one workgroup per 64-key block): each wave
// keeps K and V fragments of its 16 keys in registers, recomputes P from the
// saved LSE for every 64-query block, and accumulates dV^T += dO^T Z and
// dK^T += Q^T dS with the accumulator-as-operand trick (products that sum over
// the query = row index of the S tile need no data movement); dQ = dS K sums
// over keys, so dS goes through LDS once and each key block writes its own fp32
// dQ partial (plain stores, no atomics: deterministic), reduced by a small
// kernel — or, for s <= 128, bwd_short_kernel: one 8-wave workgroup per (b, h)
// covering every key, dQ written once in bf16 and delta computed in-kernel.
// Dropout masks are regenerated from a counter hash of
// (seed, b*h, query, key) in both passes.
#include "mv_common.h"
#include "mv_attn.h"

namespace mv {
namespace attn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int D = 64;
constexpr int KB = 64;     // keys per block
constexpr int QB = 64;     // queries per block
constexpr int PAD = 8;     // LDS row padding (elements): 144-B rows spread banks
constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// counter-based dropout decision, identical in forward and backward
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t bh, uint32_t q, uint32_t k,
                                          uint32_t thresh) {
  return mix32(mix32(mix32(seed + bh * 0x9E3779B1u) + q) + k * 0x85EBCA6Bu) >= thresh;
}

__device__ __forceinline__ f32x4v mfma(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, (__bf16)x);
}

__device__ __forceinline__ bf16x8 pack8(const float (&v)[8]) {
  bf16x8 o;
  uint32_t* w = reinterpret_cast<uint32_t*>(&o);
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = cvt_pk_bf16(v[2 * i], v[2 * i + 1]);
  return o;
}

__device__ __forceinline__ bf16x8 ld_b128(const __bf16* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));

// gfx950 transposed LDS read (ds_read_b64_tr_b16): each 16-lane group reads a 4-row x
// 16-column block of a row-major bf16 LDS array and lane c receives column col0 + c of
// rows r0 .. r0 + 3 — the k-major MFMA operand straight from a row-major image, no
// transposed copy.  Lane c supplies the address of row r0 + c/4, columns 4(c%4) ...
__device__ __forceinline__ s16x4 tr4(const __bf16* base, int stride, int r0, int col0, int c) {
  const __bf16* p = base + (r0 + (c >> 2)) * stride + col0 + 4 * (c & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

// 8 k-values: rows ra .. ra+3 then rb .. rb+3 of column col0 + c
__device__ __forceinline__ bf16x8 tr8(const __bf16* base, int stride, int ra, int rb, int col0,
                                      int c) {
  const s16x4 a = tr4(base, stride, ra, col0, c);
  const s16x4 b = tr4(base, stride, rb, col0, c);
  bf16x8 o;
  short* q = reinterpret_cast<short*>(&o);
  q[0] = a[0]; q[1] = a[1]; q[2] = a[2]; q[3] = a[3];
  q[4] = b[0]; q[5] = b[1]; q[6] = b[2]; q[7] = b[3];
  return o;
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
  uint32_t* w = reinterpret_cast<uint32_t*>(&z);
  w[0] = w[1] = w[2] = w[3] = 0u;
  return z;
}

// ---------------------------------------------------------------- forward
__global__ __launch_bounds__(256) void fwd_kernel(AttnParams p) {
  const int bh = blockIdx.y;
  const int bi = bh / p.h, hi = bh % p.h;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const int q0 = blockIdx.x * QB + w * 16;
  const int64_t tok = 3LL * p.h * D;
  const __bf16* Qb = ((const __bf16*)p.qkv) + (int64_t)bi * p.s * tok + (int64_t)hi * D;
  const __bf16* Kb = Qb + (int64_t)p.h * D;
  const __bf16* Vb = Qb + 2LL * p.h * D;
  __shared__ __attribute__((aligned(16))) __bf16 Ks[KB][D + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 Vs[KB][D + PAD];   // row-major; V^T via tr8

  bf16x8 qf[2];
  {
    const int q = q0 + c;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[ks] = q < p.s ? ld_b128(Qb + (int64_t)q * tok + 32 * ks + 8 * g) : zero8();
  }
  f32x4v O[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) O[n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  const float inv_keep = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;

  for (int kb0 = 0; kb0 < p.s; kb0 += KB) {
    __syncthreads();
    {  // cooperative K / V^T block load: thread -> (key, 16 dims)
      const int t = threadIdx.x, key = t >> 2, d0 = (t & 3) * 16;
      const int kg = kb0 + key;
      bf16x8 k0 = zero8(), k1 = zero8(), v0 = zero8(), v1 = zero8();
      if (kg < p.s) {
        k0 = ld_b128(Kb + (int64_t)kg * tok + d0);
        k1 = ld_b128(Kb + (int64_t)kg * tok + d0 + 8);
        v0 = ld_b128(Vb + (int64_t)kg * tok + d0);
        v1 = ld_b128(Vb + (int64_t)kg * tok + d0 + 8);
      }
      *reinterpret_cast<bf16x8*>(&Ks[key][d0]) = k0;
      *reinterpret_cast<bf16x8*>(&Ks[key][d0 + 8]) = k1;
      *reinterpret_cast<bf16x8*>(&Vs[key][d0]) = v0;
      *reinterpret_cast<bf16x8*>(&Vs[key][d0 + 8]) = v1;
    }
    __syncthreads();
    // S^T tiles: st[t][r] = score(key kb0 + 16t + 4g + r, query q0 + c)
    float sv[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) acc = mfma(ld_b128(&Ks[16 * t + c][32 * ks + 8 * g]), qf[ks], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb0 + 16 * t + 4 * g + r;
        float v = acc[r] * p.scale_log2;
        if (p.mask) v += (key < p.s ? p.mask[(int64_t)bi * p.s + key] : 0.f) * LOG2E;
        sv[t][r] = key < p.s ? v : -INFINITY;
      }
    }
    float mb = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) mb = fmaxf(mb, sv[t][r]);
    mb = fmaxf(mb, __shfl_xor(mb, 16, 64));
    mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
    const float m_new = fmaxf(m_run, mb);
    const float alpha = (m_new == -INFINITY) ? 1.f : exp2f(m_run - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = (m_new == -INFINITY) ? 0.f : exp2f(sv[t][r] - m_new);
        sv[t][r] = e;
        lsum += e;
      }
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    // rescale the O rows (query 4g+r lives in lane 4g+r's column)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float ar = __shfl(alpha, 4 * g + r, 64);
#pragma unroll
      for (int n = 0; n < 4; ++n) O[n][r] *= ar;
    }
    if (p.p_drop > 0.f) {
      const uint32_t qg = (uint32_t)(q0 + c);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const uint32_t key = (uint32_t)(kb0 + 16 * t + 4 * g + r);
          sv[t][r] = keep_elem(p.seed, bh, qg, key, p.thresh) ? sv[t][r] * inv_keep : 0.f;
        }
    }
    // O += P V  (two 32-key chunks; k order = keys 16*t0+4g+r, 16*t1+4g+r)
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
      const int t0 = 2 * ch, t1 = 2 * ch + 1;
      float a8[8] = {sv[t0][0], sv[t0][1], sv[t0][2], sv[t0][3],
                     sv[t1][0], sv[t1][1], sv[t1][2], sv[t1][3]};
      const bf16x8 af = pack8(a8);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 bfr = tr8(&Vs[0][0], D + PAD, 16 * t0 + 4 * g, 16 * t1 + 4 * g, 16 * n, c);
        O[n] = mfma(af, bfr, O[n]);
      }
    }
  }
  float l_tot = l_run + __shfl_xor(l_run, 16, 64);
  l_tot += __shfl_xor(l_tot, 32, 64);
  if (g == 0 && q0 + c < p.s)
    p.lse[(int64_t)bh * p.s + q0 + c] = m_run + log2f(l_tot);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float lr = __shfl(l_tot, 4 * g + r, 64);
    const float inv = lr > 0.f ? 1.f / lr : 0.f;
    const int q = q0 + 4 * g + r;
    if (q < p.s) {
      __bf16* o = ((__bf16*)p.out) + ((int64_t)bi * p.s + q) * p.h * D + (int64_t)hi * D;
#pragma unroll
      for (int n = 0; n < 4; ++n) o[16 * n + c] = (__bf16)(O[n][r] * inv);
    }
  }
}

// ---------------------------------------------------------------- backward
// delta[bh, q] = sum_d dO * O
__global__ __launch_bounds__(256) void delta_kernel(const __bf16* __restrict__ out,
                                                     const __bf16* __restrict__ dout,
                                                     float* __restrict__ delta, int b, int s,
                                                     int h) {
  // 8 lanes per (b, s, h) row, 16 B each: a wave reads 8 whole 128-B rows per load
  // (one-thread-per-row touched 64 lines per instruction and ran at ~1 TB/s)
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  const int j8 = (threadIdx.x & 7) * 8;
  const int64_t rows = (int64_t)b * s * h;
  float acc = 0.f;
  if (i < rows) {
    float a[8], e[8];
    load8(out + i * D + j8, a);
    load8(dout + i * D + j8, e);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * e[j];
  }
  acc += __shfl_xor(acc, 1, 64);
  acc += __shfl_xor(acc, 2, 64);
  acc += __shfl_xor(acc, 4, 64);
  if (i < rows && j8 == 0) {
    const int hi = (int)(i % h);
    const int64_t bs = i / h;
    const int q = (int)(bs % s), bi = (int)(bs / s);
    delta[((int64_t)bi * h + hi) * s + q] = acc;
  }
}

__global__ __launch_bounds__(256) void bwd_kernel(AttnParams p, const __bf16* __restrict__ dout,
                                                   const float* __restrict__ delta,
                                                   float* __restrict__ dq_part,
                                                   __bf16* __restrict__ dqkv) {
  const int bh = blockIdx.y;
  const int bi = bh / p.h, hi = bh % p.h;
  const int kb = blockIdx.x;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const int k0 = kb * KB + w * 16;
  const int64_t tok = 3LL * p.h * D;
  const int64_t otok = (int64_t)p.h * D;
  const __bf16* Qb = ((const __bf16*)p.qkv) + (int64_t)bi * p.s * tok + (int64_t)hi * D;
  const __bf16* Kb = Qb + (int64_t)p.h * D;
  const __bf16* Vb = Qb + 2LL * p.h * D;
  const __bf16* dOb = dout + (int64_t)bi * p.s * otok + (int64_t)hi * D;

  __shared__ __attribute__((aligned(16))) __bf16 Qs[QB][D + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 dOs[QB][D + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 dSs[QB][KB + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 Ks[KB][D + PAD];     // K^T via tr8
  __shared__ float lse_s[QB], del_s[QB];

  // this wave's 16 keys as MFMA B fragments (K^T / V^T columns)
  bf16x8 kf[2], vf[2];
  {
    const int key = k0 + c;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = key < p.s ? ld_b128(Kb + (int64_t)key * tok + 32 * ks + 8 * g) : zero8();
      vf[ks] = key < p.s ? ld_b128(Vb + (int64_t)key * tok + 32 * ks + 8 * g) : zero8();
    }
  }
  {  // this block's keys, row-major, for dQ = dS K
    const int t = threadIdx.x, key = t >> 2, d0 = (t & 3) * 16;
    const int kg = kb * KB + key;
    bf16x8 a = zero8(), b2 = zero8();
    if (kg < p.s) {
      a = ld_b128(Kb + (int64_t)kg * tok + d0);
      b2 = ld_b128(Kb + (int64_t)kg * tok + d0 + 8);
    }
    *reinterpret_cast<bf16x8*>(&Ks[key][d0]) = a;
    *reinterpret_cast<bf16x8*>(&Ks[key][d0 + 8]) = b2;
  }
  f32x4v dVt[4], dKt[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    dVt[n] = f32x4v{0.f, 0.f, 0.f, 0.f};
    dKt[n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  }
  const float inv_keep = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
  const int keyc = k0 + c;
  const float kbias = (p.mask && keyc < p.s) ? p.mask[(int64_t)bi * p.s + keyc] * LOG2E : 0.f;
  const int nkb = (p.s + KB - 1) / KB;

  for (int qb0 = 0; qb0 < p.s; qb0 += QB) {
    __syncthreads();
    {
      const int t = threadIdx.x, row = t >> 2, d0 = (t & 3) * 16;
      const int qg = qb0 + row;
      bf16x8 q0v = zero8(), q1v = zero8(), o0 = zero8(), o1 = zero8();
      if (qg < p.s) {
        q0v = ld_b128(Qb + (int64_t)qg * tok + d0);
        q1v = ld_b128(Qb + (int64_t)qg * tok + d0 + 8);
        o0 = ld_b128(dOb + (int64_t)qg * otok + d0);
        o1 = ld_b128(dOb + (int64_t)qg * otok + d0 + 8);
      }
      *reinterpret_cast<bf16x8*>(&Qs[row][d0]) = q0v;
      *reinterpret_cast<bf16x8*>(&Qs[row][d0 + 8]) = q1v;
      *reinterpret_cast<bf16x8*>(&dOs[row][d0]) = o0;
      *reinterpret_cast<bf16x8*>(&dOs[row][d0 + 8]) = o1;
      if (t < QB) {
        const int qq = qb0 + t;
        lse_s[t] = qq < p.s ? p.lse[(int64_t)bh * p.s + qq] : INFINITY;
        del_s[t] = qq < p.s ? delta[(int64_t)bh * p.s + qq] : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {         // 32-query chunks
      float zc[2][4], dsc[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * ch + u;
        f32x4v sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sacc = mfma(ld_b128(&Qs[16 * qt + c][32 * ks + 8 * g]), kf[ks], sacc);
          pacc = mfma(ld_b128(&dOs[16 * qt + c][32 * ks + 8 * g]), vf[ks], pacc);
        }
        // sacc[r] = S(q = qb0+16qt+4g+r, key = keyc); pacc[r] = dZ(q, key)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qt + 4 * g + r;
          float pr = 0.f;
          if (keyc < p.s) pr = exp2f(sacc[r] * p.scale_log2 + kbias - lse_s[ql]);
          float z = pr, dzd = pacc[r];
          if (p.p_drop > 0.f) {
            const bool kp = keep_elem(p.seed, bh, (uint32_t)(qb0 + ql), (uint32_t)keyc, p.thresh);
            z = kp ? pr * inv_keep : 0.f;
            dzd = kp ? dzd * inv_keep : 0.f;
          }
          const float ds = pr * (dzd - del_s[ql]);
          zc[u][r] = z;
          dsc[u][r] = ds;
          dSs[ql][w * 16 + c] = (__bf16)ds;
        }
      }
      float zb[8] = {zc[0][0], zc[0][1], zc[0][2], zc[0][3], zc[1][0], zc[1][1], zc[1][2], zc[1][3]};
      float sb[8] = {dsc[0][0], dsc[0][1], dsc[0][2], dsc[0][3],
                     dsc[1][0], dsc[1][1], dsc[1][2], dsc[1][3]};
      const bf16x8 zf = pack8(zb), sf = pack8(sb);
      const int qa = 32 * ch + 4 * g, qbb = 32 * ch + 16 + 4 * g;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        dVt[n] = mfma(tr8(&dOs[0][0], D + PAD, qa, qbb, 16 * n, c), zf, dVt[n]);
        dKt[n] = mfma(tr8(&Qs[0][0], D + PAD, qa, qbb, 16 * n, c), sf, dKt[n]);
      }
    }
    __syncthreads();
    // dQ partial for 16 queries (this wave's q tile) over this block's 64 keys
    {
      const int qt = w;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc = mfma(ld_b128(&dSs[16 * qt + c][32 * ks + 8 * g]),
                     tr8(&Ks[0][0], D + PAD, 32 * ks + 8 * g, 32 * ks + 8 * g + 4, 16 * n, c),
                     acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qb0 + 16 * qt + 4 * g + r;
          if (q < p.s)
            dq_part[(((int64_t)kb * p.b + bi) * p.s + q) * otok + (int64_t)hi * D + 16 * n + c] =
                acc[r];
        }
      }
    }
  }
  // dK, dV: dKt[n][r] = dK^T(d = 16n+4g+r, key = keyc)
  if (keyc < p.s) {
    const float sc = p.scale_log2 / LOG2E;   // 1/sqrt(D)
    __bf16* dk = dqkv + ((int64_t)bi * p.s + keyc) * tok + (int64_t)p.h * D + (int64_t)hi * D;
    __bf16* dv = dk + (int64_t)p.h * D;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dk[16 * n + 4 * g + r] = (__bf16)(dKt[n][r] * sc);
        dv[16 * n + 4 * g + r] = (__bf16)dVt[n][r];
      }
  }
  (void)nkb;
}

// Short sequences (s <= 128, BERT pre-training's 128): ONE workgroup of 8 waves per
// (b, h) owns all (up to 2) key blocks — waves 0-3 keys 0-63, waves 4-7 keys 64-127 —
// so dQ = dS K sums over every key inside the workgroup and is written once in bf16
// (no fp32 partials, no dq_reduce pass), delta = rowsum(dO * O) is computed in the
// query-block prologue (no delta pass), and each Q / dO block is staged once for both
// key halves.
__global__ __launch_bounds__(512) void bwd_short_kernel(AttnParams p,
                                                         const __bf16* __restrict__ out,
                                                         const __bf16* __restrict__ dout,
                                                         __bf16* __restrict__ dqkv) {
  constexpr int SK = 2 * KB;     // keys per workgroup
  const int bh = blockIdx.x;
  const int bi = bh / p.h, hi = bh % p.h;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, g = l >> 4, c = l & 15;
  const int kh = w >> 2, wq = w & 3;
  const int k0 = kh * KB + wq * 16;
  const int64_t tok = 3LL * p.h * D;
  const int64_t otok = (int64_t)p.h * D;
  const __bf16* Qb = ((const __bf16*)p.qkv) + (int64_t)bi * p.s * tok + (int64_t)hi * D;
  const __bf16* Kb = Qb + (int64_t)p.h * D;
  const __bf16* Vb = Qb + 2LL * p.h * D;
  const __bf16* dOb = dout + (int64_t)bi * p.s * otok + (int64_t)hi * D;
  const __bf16* Ob = out + (int64_t)bi * p.s * otok + (int64_t)hi * D;

  // row-major images only: the k-major operands (Q^T, dO^T, K^T) come from them through
  // transposed LDS reads (tr8), so no element-wise transposed copies are written
  __shared__ __attribute__((aligned(16))) __bf16 Qs[QB][D + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 dOs[QB][D + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 dSs[QB][SK + PAD];
  __shared__ __attribute__((aligned(16))) __bf16 Ks[SK][D + PAD];
  __shared__ float lse_s[QB], del_s[QB];

  bf16x8 kf[2], vf[2];
  {
    const int key = k0 + c;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = key < p.s ? ld_b128(Kb + (int64_t)key * tok + 32 * ks + 8 * g) : zero8();
      vf[ks] = key < p.s ? ld_b128(Vb + (int64_t)key * tok + 32 * ks + 8 * g) : zero8();
    }
  }
  {  // all SK keys, row-major, for dQ = dS K
    const int t = threadIdx.x, key = t >> 2, d0 = (t & 3) * 16;
    bf16x8 a = zero8(), b2 = zero8();
    if (key < p.s) {
      a = ld_b128(Kb + (int64_t)key * tok + d0);
      b2 = ld_b128(Kb + (int64_t)key * tok + d0 + 8);
    }
    *reinterpret_cast<bf16x8*>(&Ks[key][d0]) = a;
    *reinterpret_cast<bf16x8*>(&Ks[key][d0 + 8]) = b2;
  }
  f32x4v dVt[4], dKt[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    dVt[n] = f32x4v{0.f, 0.f, 0.f, 0.f};
    dKt[n] = f32x4v{0.f, 0.f, 0.f, 0.f};
  }
  const float inv_keep = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
  const float qscale = p.scale_log2 / LOG2E;   // 1/sqrt(D)
  const int keyc = k0 + c;
  const float kbias = (p.mask && keyc < p.s) ? p.mask[(int64_t)bi * p.s + keyc] * LOG2E : 0.f;

  for (int qb0 = 0; qb0 < p.s; qb0 += QB) {
    __syncthreads();
    if (threadIdx.x < 256) {   // Q / dO tiles, row-major and transposed
      const int t = threadIdx.x, row = t >> 2, d0 = (t & 3) * 16;
      const int qg = qb0 + row;
      bf16x8 q0v = zero8(), q1v = zero8(), o0 = zero8(), o1 = zero8();
      if (qg < p.s) {
        q0v = ld_b128(Qb + (int64_t)qg * tok + d0);
        q1v = ld_b128(Qb + (int64_t)qg * tok + d0 + 8);
        o0 = ld_b128(dOb + (int64_t)qg * otok + d0);
        o1 = ld_b128(dOb + (int64_t)qg * otok + d0 + 8);
      }
      *reinterpret_cast<bf16x8*>(&Qs[row][d0]) = q0v;
      *reinterpret_cast<bf16x8*>(&Qs[row][d0 + 8]) = q1v;
      *reinterpret_cast<bf16x8*>(&dOs[row][d0]) = o0;
      *reinterpret_cast<bf16x8*>(&dOs[row][d0 + 8]) = o1;
      if (t < QB) {
        const int qq = qb0 + t;
        lse_s[t] = qq < p.s ? p.lse[(int64_t)bh * p.s + qq] : INFINITY;
      }
    } else {                   // delta = rowsum(dO * O): 4 lanes x 16 dims per query
      const int u = threadIdx.x - 256, row = u >> 2, d0 = (u & 3) * 16;
      const int qg = qb0 + row;
      float acc = 0.f;
      if (qg < p.s) {
        float a[8], e[8];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          load8(Ob + (int64_t)qg * otok + d0 + 8 * hh, a);
          load8(dOb + (int64_t)qg * otok + d0 + 8 * hh, e);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += a[j] * e[j];
        }
      }
      acc += __shfl_xor(acc, 1, 64);
      acc += __shfl_xor(acc, 2, 64);
      if ((u & 3) == 0) del_s[row] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {         // 32-query chunks
      float zc[2][4], dsc[2][4];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qt = 2 * ch + u;
        f32x4v sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          sacc = mfma(ld_b128(&Qs[16 * qt + c][32 * ks + 8 * g]), kf[ks], sacc);
          pacc = mfma(ld_b128(&dOs[16 * qt + c][32 * ks + 8 * g]), vf[ks], pacc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * qt + 4 * g + r;
          float pr = 0.f;
          if (keyc < p.s) pr = exp2f(sacc[r] * p.scale_log2 + kbias - lse_s[ql]);
          float z = pr, dzd = pacc[r];
          if (p.p_drop > 0.f) {
            const bool kp = keep_elem(p.seed, bh, (uint32_t)(qb0 + ql), (uint32_t)keyc, p.thresh);
            z = kp ? pr * inv_keep : 0.f;
            dzd = kp ? dzd * inv_keep : 0.f;
          }
          const float ds = pr * (dzd - del_s[ql]);
          zc[u][r] = z;
          dsc[u][r] = ds;
          dSs[ql][kh * KB + wq * 16 + c] = (__bf16)ds;
        }
      }
      float zb[8] = {zc[0][0], zc[0][1], zc[0][2], zc[0][3], zc[1][0], zc[1][1], zc[1][2], zc[1][3]};
      float sb[8] = {dsc[0][0], dsc[0][1], dsc[0][2], dsc[0][3],
                     dsc[1][0], dsc[1][1], dsc[1][2], dsc[1][3]};
      const bf16x8 zf = pack8(zb), sf = pack8(sb);
      const int qa = 32 * ch + 4 * g, qbb = 32 * ch + 16 + 4 * g;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        dVt[n] = mfma(tr8(&dOs[0][0], D + PAD, qa, qbb, 16 * n, c), zf, dVt[n]);
        dKt[n] = mfma(tr8(&Qs[0][0], D + PAD, qa, qbb, 16 * n, c), sf, dKt[n]);
      }
    }
    __syncthreads();
    // dQ[64 q, 64 d] = dS[64, SK] K[SK, 64]: wave -> query tile w&3, d tiles 2(w>>2)+{0,1}
    {
      const int qt = w & 3;
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) {
        const int n = 2 * (w >> 2) + nn;
        f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < SK / 32; ++ks)
          acc = mfma(ld_b128(&dSs[16 * qt + c][32 * ks + 8 * g]),
                     tr8(&Ks[0][0], D + PAD, 32 * ks + 8 * g, 32 * ks + 8 * g + 4, 16 * n, c), acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = qb0 + 16 * qt + 4 * g + r;
          if (q < p.s)
            dqkv[((int64_t)bi * p.s + q) * tok + (int64_t)hi * D + 16 * n + c] =
                (__bf16)(acc[r] * qscale);
        }
      }
    }
  }
  if (keyc < p.s) {
    __bf16* dk = dqkv + ((int64_t)bi * p.s + keyc) * tok + (int64_t)p.h * D + (int64_t)hi * D;
    __bf16* dv = dk + (int64_t)p.h * D;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dk[16 * n + 4 * g + r] = (__bf16)(dKt[n][r] * qscale);
        dv[16 * n + 4 * g + r] = (__bf16)dVt[n][r];
      }
  }
}

__global__ __launch_bounds__(256) void dq_reduce_kernel(const float* __restrict__ dq_part,
                                                         __bf16* __restrict__ dqkv, int nkb,
                                                         int b, int s, int h, float scale) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;   // element of [b,s,h,D]
  const int64_t n = (int64_t)b * s * h * D;
  if (i >= n) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < nkb; ++k) {
    float v[8];
    load8(dq_part + (int64_t)k * n + i, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] *= scale;
  const int64_t row = i / D, d = i % D;          // row = (b*s + q)*h + hi (D: power of 2)
  const uint32_t r32 = (uint32_t)row, bsq32 = r32 / (uint32_t)h;   // rows < 2^32 (bindings)
  const int64_t bsq = bsq32, hi = r32 - bsq32 * (uint32_t)h;
  store8(dqkv + bsq * 3 * h * D + hi * D + d, acc);
}

}  // namespace attn
}  // namespace mv

using namespace mv::attn;

void mv_attn_fwd(const AttnParams& p, hipStream_t st) {
  dim3 grid((p.s + QB - 1) / QB, p.b * p.h);
  hipLaunchKernelGGL(fwd_kernel, grid, dim3(256), 0, st, p);
}

void mv_attn_bwd(const AttnParams& p, const void* out, const void* dout, float* delta,
                 float* dq_part, void* dqkv, hipStream_t st) {
  if (p.s <= 2 * KB) {   // one workgroup per (b, h): no delta / dq_reduce passes
    hipLaunchKernelGGL(bwd_short_kernel, dim3(p.b * p.h), dim3(512), 0, st, p, (const __bf16*)out,
                       (const __bf16*)dout, (__bf16*)dqkv);
    return;
  }
  const int64_t rows = (int64_t)p.b * p.s * p.h;
  static_assert(D == 64, "delta_kernel maps 8 lanes x 8 elements onto a row");
  hipLaunchKernelGGL(delta_kernel, dim3((unsigned)((rows * 8 + 255) / 256)), dim3(256), 0, st,
                     (const __bf16*)out, (const __bf16*)dout, delta, p.b, p.s, p.h);
  const int nkb = (p.s + KB - 1) / KB;
  hipLaunchKernelGGL(bwd_kernel, dim3(nkb, p.b * p.h), dim3(256), 0, st, p,
                     (const __bf16*)dout, (const float*)delta, dq_part, (__bf16*)dqkv);
  const int64_t n8 = rows * D / 8;
  hipLaunchKernelGGL(dq_reduce_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st,
                     (const float*)dq_part, (__bf16*)dqkv, nkb, p.b, p.s, p.h,
                     p.scale_log2 / LOG2E);
}

namespace mv {
namespace attn {
// debug / test helper: materialise the dropout keep-mask [b, h, s(q), s(k)]
__global__ void mask_kernel(int b, int h, int s, uint32_t seed, uint32_t thresh, uint8_t* keep) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)b * h * s * s;
  if (i >= n) return;
  const int k = (int)(i % s);
  const int q = (int)((i / s) % s);
  const uint32_t bh = (uint32_t)(i / ((int64_t)s * s));
  keep[i] = keep_elem(seed, bh, (uint32_t)q, (uint32_t)k, thresh) ? 1 : 0;
}
}  // namespace attn
}  // namespace mv

void mv_attn_dropout_mask(int b, int h, int s, uint32_t seed, uint32_t thresh, uint8_t* keep,
                          hipStream_t st) {
  const int64_t n = (int64_t)b * h * s * s;
  hipLaunchKernelGGL(mv::attn::mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     b, h, s, seed, thresh, keep);
}
