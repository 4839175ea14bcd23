// NHWC pooling kernels for the ResNet stem / head on gfx950.
//
//  * maxpool_fwd: y = maxpool_kxk/s(act(x)) with an optional fused per-channel
//    affine + ReLU prologue (the stem's BatchNorm apply), argmax stored as one
//    uint8 per output element (window position, k*k <= 255).  torch's NHWC
//    max-pool writes int64 indices (8 B per output element) and needs the BN
//    output materialised first: for ResNet-50 bs512 that is an 822 MB write +
//    read + an 822 MB index write that this kernel never does.
//  * maxpool_bwd: gather form — each input element sums the (<= ceil(k/s)^2)
//    output gradients whose argmax points at it.  No zero-fill, no atomics,
//    deterministic; optional second gradient stream dy2 (tapped output).
//  * gap_fwd / gap_bwd: global average pool over H*W (NHWC) and its broadcast
//    backward (torch's channels_last expand falls back to a non-vectorized
//    elementwise kernel: 160 us per step at bs512).
//
// Every lane handles 8 consecutive channels of one pixel (16 B bf16 vectors);
// C % 8 == 0 is checked on the host.
#include "mv_common.h"
#include "mv_pool.h"

namespace mv {
namespace pool {

struct PoolGeo {
  int N, H, W, C, OH, OW, k, s, p;
};

// KC > 0: compile-time window size (ResNet's 3): the KC*KC loads are unrolled and all in
// flight at once instead of one dependent load per loop trip
template <int KC>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const __bf16* __restrict__ x,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ bias,
                                                          int relu, __bf16* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeo g) {
  const int k = KC > 0 ? KC : g.k;
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.OH * g.OW * cv;
  if (t >= total) return;
  // 32-bit index math (launcher: total < 2^32); 64-bit div/mod per lane is ~100 ALU ops
  const uint32_t t32 = (uint32_t)t, cv32 = (uint32_t)cv;
  const uint32_t pix0 = t32 / cv32;
  const int c = (int)(t32 - pix0 * cv32) * 8;
  const uint32_t pw = pix0 / (uint32_t)g.OW;
  const int ow = (int)(pix0 - pw * (uint32_t)g.OW);
  const uint32_t ph = pw / (uint32_t)g.OH;
  const int oh = (int)(pw - ph * (uint32_t)g.OH);
  const int n = (int)ph;
  float sc[8], bi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = 1.f; bi[j] = 0.f; }
  if (scale) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = scale[c + j]; bi[j] = bias[c + j]; }
  }
  float best[8];
  uint32_t arg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
  const int h0 = oh * g.s - g.p, w0 = ow * g.s - g.p;
#pragma unroll
  for (int kh = 0; kh < k; ++kh) {
    const int ih = h0 + kh;
    if (ih < 0 || ih >= g.H) continue;
#pragma unroll
    for (int kw = 0; kw < k; ++kw) {
      const int iw = w0 + kw;
      if (iw < 0 || iw >= g.W) continue;
      float v[8];
      load8(x + (((int64_t)n * g.H + ih) * g.W + iw) * g.C + c, v);
      const uint32_t pos = kh * k + kw;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a = scale ? __builtin_fmaf(v[j], sc[j], bi[j]) : v[j];
        if (relu) a = a > 0.f ? a : 0.f;
        a = (float)(__bf16)a;                  // compare what torch would have stored
        if (a > best[j] || __builtin_isnan(a)) {   // first maximum wins (torch order)
          best[j] = a;
          arg[j] = pos;
        }
      }
    }
  }
  store8(y + t * 8, best);
  uint32_t lo = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
  uint32_t hi = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  *reinterpret_cast<u32x2*>(idx + t * 8) = u32x2{lo, hi};
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const __bf16* __restrict__ dy,
                                                          const __bf16* __restrict__ dy2,
                                                          const uint8_t* __restrict__ idx,
                                                          __bf16* __restrict__ dx, PoolGeo g) {
  const int cv = g.C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)g.N * g.H * g.W * cv;
  if (t >= total) return;
  // 32-bit index math (launcher: total < 2^32): 64-bit div/mod per lane was the
  // kernel's bottleneck (~2 TB/s)
  const uint32_t t32 = (uint32_t)t, cv32 = (uint32_t)cv;
  const uint32_t pix0 = t32 / cv32;
  const int c = (int)(t32 - pix0 * cv32) * 8;
  const uint32_t pw = pix0 / (uint32_t)g.W;
  const int iw = (int)(pix0 - pw * (uint32_t)g.W);
  const uint32_t ph = pw / (uint32_t)g.H;
  const int ih = (int)(pw - ph * (uint32_t)g.H);
  const int n = (int)ph;
  // output windows containing ih: oh*s - p <= ih <= oh*s - p + k - 1
  const int ohl = max(0, (ih + g.p - g.k + g.s) / g.s);
  const int ohh = min(g.OH - 1, (ih + g.p) / g.s);
  const int owl = max(0, (iw + g.p - g.k + g.s) / g.s);
  const int owh = min(g.OW - 1, (iw + g.p) / g.s);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int oh = ohl; oh <= ohh; ++oh) {
    const int kh = ih - (oh * g.s - g.p);
    if (kh < 0 || kh >= g.k) continue;
    for (int ow = owl; ow <= owh; ++ow) {
      const int kw = iw - (ow * g.s - g.p);
      if (kw < 0 || kw >= g.k) continue;
      const uint32_t pos = kh * g.k + kw;
      const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c;
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 a = *reinterpret_cast<const u32x2*>(idx + o);
      float d[8];
      load8(dy + o, d);
      if (dy2) {
        float e[8];
        load8(dy2 + o, e);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] += e[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = j < 4 ? a[0] : a[1];
        const uint32_t id = (w >> (8 * (j & 3))) & 0xffu;
        if (id == pos) acc[j] += d[j];
      }
    }
  }
  store8(dx + t * 8, acc);
}

// k = 3, s = 2, p = 1 (ResNet) with even H, W: one lane per 2x2 block of input pixels
// x 8 channels.  The block (2a.., 2b..) belongs to exactly the windows oh in {a, a+1},
// ow in {b, b+1}, so every lane loads the same 4 windows (no divergent 1/2/4-window
// loops as in the generic kernel, and each window's dy / index is loaded once per block
// instead of once per covered pixel) and writes 4 pixels.
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2_kernel(const __bf16* __restrict__ dy,
                                                               const __bf16* __restrict__ dy2,
                                                               const uint8_t* __restrict__ idx,
                                                               __bf16* __restrict__ dx,
                                                               PoolGeo g) {
  const uint32_t cv = (uint32_t)g.C / 8, hb = (uint32_t)g.H / 2, wb = (uint32_t)g.W / 2;
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const uint32_t total = (uint32_t)g.N * hb * wb * cv;
  if (t >= total) return;
  const uint32_t q0 = t / cv;
  const int c = (int)(t - q0 * cv) * 8;
  const uint32_t q1 = q0 / wb;
  const int b = (int)(q0 - q1 * wb);
  const uint32_t n = q1 / hb;
  const int a = (int)(q1 - n * hb);
  float acc[2][2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[i][jj][e] = 0.f;
#pragma unroll
  for (int da = 0; da < 2; ++da) {
    const int oh = a + da;
    if (oh >= g.OH) continue;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int ow = b + db;
      if (ow >= g.OW) continue;
      const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + c;
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      const u32x2 iw8 = *reinterpret_cast<const u32x2*>(idx + o);
      float d[8];
      load8(dy + o, d);
      if (dy2) {
        float e2[8];
        load8(dy2 + o, e2);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] += e2[e];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kh = i - 2 * da + 1;          // row of input 2a + i inside window oh
        if (kh < 0) continue;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int kw = jj - 2 * db + 1;
          if (kw < 0) continue;
          const uint32_t pos = (uint32_t)(kh * 3 + kw);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t w = e < 4 ? iw8[0] : iw8[1];
            if (((w >> (8 * (e & 3))) & 0xffu) == pos) acc[i][jj][e] += d[e];
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int64_t px = ((int64_t)n * g.H + 2 * a + i) * g.W + 2 * b + jj;
      store8(dx + px * g.C + c, acc[i][jj]);
    }
}

// global average pool: x [N, HW, C] -> y [N, C]; one lane per (n, 8 channels)
__global__ __launch_bounds__(256) void gap_fwd_kernel(const __bf16* __restrict__ x,
                                                      __bf16* __restrict__ y, int N, int HW,
                                                      int C) {
  const int cv = C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * cv) return;
  const int n = (int)(t / cv), c = (int)(t % cv) * 8;
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  const __bf16* base = x + (int64_t)n * HW * C + c;
  for (int i = 0; i < HW; ++i) {
    float v[8];
    load8(base + (int64_t)i * C, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += v[j];
  }
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] *= inv;
  store8(y + (int64_t)n * C + c, s);
}

// dx[n, i, c] = dy[n, c] / HW
__global__ __launch_bounds__(256) void gap_bwd_kernel(const __bf16* __restrict__ dy,
                                                      __bf16* __restrict__ dx, int N, int HW,
                                                      int C) {
  const int cv = C / 8;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= (int64_t)N * HW * cv) return;
  const uint32_t t32 = (uint32_t)t, cv32 = (uint32_t)cv;   // launcher: total < 2^32
  const uint32_t q = t32 / cv32;
  const int c = (int)(t32 - q * cv32) * 8;
  const int n = (int)(q / (uint32_t)HW);
  float v[8];
  load8(dy + (int64_t)n * C + c, v);
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= inv;
  store8(dx + t * 8, v);
}

// Zero-pad the channel dim of an NHWC bf16 tensor, Cin -> Cout (<= 8): the
// ResNet stem's 3-channel image becomes 4 channels, for which MIOpen's 7x7/2
// conv kernels run ~1.4x faster (fwd+wgrad); the zero channel changes nothing.
// One lane per pixel: Cin scalar loads (consecutive lanes read consecutive
// 2*Cin-byte runs) and one 8-byte store when Cout == 4.
__global__ __launch_bounds__(256) void pad_channels_kernel(const uint16_t* __restrict__ x,
                                                           uint16_t* __restrict__ y,
                                                           int64_t pixels, int cin, int cout) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= pixels) return;
  uint16_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (j < cin) ? x[t * cin + j] : (uint16_t)0;
  if (cout == 4) {
    uint2 o;
    o.x = (uint32_t)v[0] | ((uint32_t)v[1] << 16);
    o.y = (uint32_t)v[2] | ((uint32_t)v[3] << 16);
    *reinterpret_cast<uint2*>(y + t * 4) = o;
  } else {
    for (int j = 0; j < cout; ++j) y[t * cout + j] = v[j];
  }
}

}  // namespace pool
}  // namespace mv

using namespace mv::pool;

static unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

void mv_maxpool_fwd(const void* x, const float* scale, const float* bias, bool relu, void* y,
                    uint8_t* idx, int N, int H, int W, int C, int OH, int OW, int k, int s, int p,
                    hipStream_t st) {
  PoolGeo g{N, H, W, C, OH, OW, k, s, p};
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  if (total >= (int64_t(1) << 32)) return;   // bindings reject such shapes first
  if (!total) return;
  if (k == 3)
    hipLaunchKernelGGL(maxpool_fwd_kernel<3>, dim3(blocks_for(total)), dim3(256), 0, st,
                       (const __bf16*)x, scale, bias, relu ? 1 : 0, (__bf16*)y, idx, g);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<0>, dim3(blocks_for(total)), dim3(256), 0, st,
                       (const __bf16*)x, scale, bias, relu ? 1 : 0, (__bf16*)y, idx, g);
}

void mv_maxpool_bwd(const void* dy, const void* dy2, const uint8_t* idx, void* dx, int N, int H,
                    int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st) {
  PoolGeo g{N, H, W, C, OH, OW, k, s, p};
  const int64_t total = (int64_t)N * H * W * (C / 8);
  if (!total) return;
  if (total >= (int64_t(1) << 32)) return;   // bindings reject such shapes first
  if (k == 3 && s == 2 && p == 1 && H % 2 == 0 && W % 2 == 0 && OH == H / 2 && OW == W / 2) {
    const int64_t t4 = total / 4;
    hipLaunchKernelGGL(maxpool_bwd_k3s2_kernel, dim3(blocks_for(t4)), dim3(256), 0, st,
                       (const __bf16*)dy, (const __bf16*)dy2, idx, (__bf16*)dx, g);
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(blocks_for(total)), dim3(256), 0, st,
                     (const __bf16*)dy, (const __bf16*)dy2, idx, (__bf16*)dx, g);
}

void mv_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st) {
  const int64_t total = (int64_t)N * (C / 8);
  if (!total) return;
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(blocks_for(total)), dim3(256), 0, st, (const __bf16*)x,
                     (__bf16*)y, N, HW, C);
}

void mv_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st) {
  const int64_t total = (int64_t)N * HW * (C / 8);
  if (!total || total >= (int64_t(1) << 32)) return;   // bindings reject such shapes first
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(blocks_for(total)), dim3(256), 0, st,
                     (const __bf16*)dy, (__bf16*)dx, N, HW, C);
}

void mv_pad_channels(const void* x, void* y, int64_t pixels, int cin, int cout, hipStream_t st) {
  if (!pixels) return;
  hipLaunchKernelGGL(pad_channels_kernel, dim3(blocks_for(pixels)), dim3(256), 0, st,
                     (const uint16_t*)x, (uint16_t*)y, pixels, cin, cout);
}
