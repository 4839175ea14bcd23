// 3x3 / pad 1 / stride 1 convolution for 64 -> 64 channels (ResNet-50 layer1 conv2 forward
// and its data gradient as a forward conv), NHWC bf16, gfx950 MFMA — the "row patch" kernel.
//
// Why a second 3x3 kernel: the general implicit GEMM (mv_conv.hip) stages one 64-channel
// TAP per K step, so at 64 channels a 256-pixel tile takes 9 short K steps and re-reads
// every input row 9 times (once per tap) from L2; with one stage in flight the loop is
// latency-bound (1.18 ms per bs-2048 launch in the full step, 3x the HBM time).
//
// Here a workgroup keeps the WHOLE filter (64 x 9 x 64 bf16 = 72 KB) resident in LDS and
// walks tiles of R = 8 output rows of one image: the (R + 2) x (W + 2) input patch (halo
// included, zero outside the image) is staged ONCE into LDS and all 9 taps read their
// shifted pixels from it — each input row is fetched from HBM 1.25x instead of 9x from L2.
// The next tile's patch is prefetched into registers while the current one computes.
//
//   LDS: filter [64 out][9 taps][8 chunks of 8 channels] (chunk c of out channel k at
//        c ^ (k & 7): the 16 A-fragment rows of one read hit distinct banks) +
//        patch  [R + 2 rows][64 pixel columns][8 chunks] (chunk c of patch column q at
//        c ^ (q & 7)); 72 + 80 KB, one workgroup (4 waves, 1 per SIMD) per CU.
//   MFMA v_mfma_f32_16x16x32_bf16, A = filter (16 out channels x 32 k), B = pixels
//        (16 pixels x 32 k): each lane's 4 accumulators are 4 consecutive output
//        channels of one pixel (8-byte stores), as in mv_conv.hip.
//   Waves: wave w owns all 64 output channels (4 N tiles) and the pixel tiles 7w .. 7w+6
//        of the tile's R * W = 448 pixels (28 M tiles for W = 56): per 32-wide k step 11
//        fragment reads feed 28 independent MFMAs (0.4 KB of LDS per MFMA, under the LDS
//        rate; 512 registers per wave hold 112 accumulators + the prefetch).
//   EPI 0: plain; 1: + the following BN's statistics (sum, sum^2 of the bf16 outputs
//        around shift) as one [2][64] partial row per workgroup; 2: the mode-1 (BN+ReLU)
//        backward reduce of the BN that produced this conv's input (this conv = its data
//        gradient), exactly mv_conv.hip's EPI 2.
// The bf16 conversions use cvt_pk_bf16_cc (the accumulators may live in VGPRs here).
#include "mv_common.h"
#include "mv_conv.h"

#include <type_traits>

namespace mv {
namespace conv64 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kC = 64;               // input = output channels
constexpr int kR = 8;                // output rows per tile
constexpr int kPR = kR + 2;          // patch rows
constexpr int kPW = 64;              // patch columns (W + 2 <= 64), padded to 64
constexpr int kThreads = 512;        // 8 waves, 2 per SIMD (256 registers each)
constexpr int kTMW = 7;              // pixel (M) tiles per wave
constexpr int kTN = 2;               // output-channel (N) tiles per wave: 32 channels
constexpr int kMaxW = kPW - 2;       // widest image row
constexpr int kMT = 4 * kTMW;        // M tiles per tile (28 -> 448 pixels >= R * W)
constexpr int kFilt = kC * 9 * kC;   // filter elements
constexpr int kPatchChunks = kPR * kPW * 8;
constexpr int kLoads = (kPatchChunks + kThreads - 1) / kThreads;   // 16-byte loads / thread

__device__ __forceinline__ f32x4v mfma(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int fidx(int k, int tap, int c) {      // filter LDS element index
  return ((k * 9 + tap) * 8 + (c ^ (k & 7))) * 8;
}
__device__ __forceinline__ int pidx(int row, int col, int c) {    // patch LDS element index
  return ((row * kPW + col) * 8 + (c ^ (col & 7))) * 8;
}
__device__ __forceinline__ float round_bf16(float x) { return (float)(__bf16)x; }

struct Geo64 {
  int N, H, W;
  int hblocks;          // ceil(H / R)
  int64_t tiles;        // N * hblocks
};

// The producing BN + ReLU applied while staging (xsc != null): X is that BN's INPUT z and
// the patch holds bf16(relu(z * xsc + xbi)) — the BN output is never materialised (padding
// taps stay 0).  Each staging thread owns one fixed 8-channel chunk, so its 16 affine
// coefficients live in registers.
__device__ __forceinline__ void bn_relu8(u32x4& v, const float (&sc)[8], const float (&bi)[8]) {
  uint32_t w[4] = {v[0], v[1], v[2], v[3]};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = fmaxf(__builtin_fmaf(__uint_as_float(w[j] << 16), sc[2 * j], bi[2 * j]), 0.f);
    const float hi =
        fmaxf(__builtin_fmaf(__uint_as_float(w[j] & 0xffff0000u), sc[2 * j + 1], bi[2 * j + 1]), 0.f);
    w[j] = cvt_pk_bf16(lo, hi);
  }
  v = u32x4{w[0], w[1], w[2], w[3]};
}

template <int EPI>
__global__ __launch_bounds__(kThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv64_kernel(
    const __bf16* __restrict__ X, const __bf16* __restrict__ Wt, __bf16* __restrict__ Y,
    Geo64 g, const float* __restrict__ shift, float* __restrict__ partial,
    const __bf16* __restrict__ bnx, const float* __restrict__ bnvec,
    const float* __restrict__ xsc, const float* __restrict__ xbi) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[kFilt + kPR * kPW * kC];   // 152 KB
  __bf16* fs = lds;                 // filter
  __bf16* ps = lds + kFilt;         // patch
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nh = wv & 1, mg = wv >> 1;           // N half (32 channels), M group
  const int gq = lane >> 4, rl = lane & 15;
  const int W = g.W, H = g.H;

  // filter -> LDS (W is [64][3][3][64] = [k][tap][c])
  for (int q = tid; q < kC * 9 * 8; q += kThreads) {
    const int k = q / 72, rem = q - k * 72, tap = rem >> 3, c = rem & 7;
    *reinterpret_cast<u32x4*>(fs + fidx(k, tap, c)) =
        *reinterpret_cast<const u32x4*>(Wt + (int64_t)q * 8);
  }

  // per lane: the patch position of its pixel in each of its 7 M tiles (tap (0,0)):
  // element offset of (row, col) in the patch and the column (for the chunk swizzle)
  int pbase[kTMW], pcol[kTMW];
#pragma unroll
  for (int b = 0; b < kTMW; ++b) {
    const int p = (mg * kTMW + b) * 16 + rl;       // pixel within the tile
    const int r = p / W, c = p - r * W;
    const bool ok = r < kR;
    pbase[b] = ok ? (r * kPW + c) * 64 : 0;
    pcol[b] = ok ? c : 0;
  }

  // next tile's patch -> registers (zero outside the image / the patch).  With 512 threads
  // and 64-pixel patch rows, thread tid stages chunk (tid & 7) of patch column tid >> 3 in
  // every patch row i (load i): one column offset + validity per thread, one row pointer
  // per tile and load.
  static_assert(kThreads == 8 * kPW && kLoads == kPR, "one patch row per load");
  const int scol = tid >> 3, sch = tid & 7;
  const bool colok = scol >= 1 && scol - 1 < W;
  const int64_t coff = (int64_t)(scol - 1) * kC + sch * 8;
  const int soff = pidx(0, scol, sch);              // + row * kPW * 64
  // (never on the data-gradient variant: its input is a gradient)
  const bool bna = EPI != 2 && xsc != nullptr;      // (wave-uniform)
  float asc[8], abi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    asc[j] = bna ? xsc[sch * 8 + j] : 0.f;
    abi[j] = bna ? xbi[sch * 8 + j] : 0.f;
  }
  u32x4 pre[kLoads];
  auto gload = [&](int64_t t) {
    const int n = (int)(t / g.hblocks), h0 = (int)(t - (int64_t)n * g.hblocks) * kR;
    const __bf16* img = X + (int64_t)n * H * W * kC;
#pragma unroll
    for (int i = 0; i < kLoads; ++i) {
      const int ih = h0 + i - 1;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (colok && ih >= 0 && ih < H)
        v = *reinterpret_cast<const u32x4*>(img + (int64_t)ih * W * kC + coff);
      pre[i] = v;
    }
  };

  float s1[kTN][4], s2[kTN][4];
#pragma unroll
  for (int a = 0; a < kTN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[a][r] = 0.f;
      s2[a][r] = 0.f;
    }

  f32x4v acc[kTN][kTMW];
  // epilogue of tile tp (acc): bf16 stores (+ statistics / BN backward reduce).  Its
  // per-channel vectors and (EPI 2) the BN input are loaded up front, all in flight at
  // once (one wait), not one dependent load per element.  The pointers pass through an
  // empty asm per tile so the loads stay here and are not hoisted out of the tile loop
  // (their registers, live across the K loop, would spill).
  auto epilogue = [&](int64_t tp) {
    const float* shp = shift;
    const float* bvp = bnvec;
    asm volatile("" : "+s"(shp));
    asm volatile("" : "+s"(bvp));
    const int n = (int)(tp / g.hblocks), h0 = (int)(tp - (int64_t)n * g.hblocks) * kR;
    float4 cv[EPI == 0 ? 1 : kTN][EPI == 2 ? 3 : 1];
    if constexpr (EPI != 0) {
#pragma unroll
      for (int a = 0; a < kTN; ++a) {
        const int col = nh * 32 + a * 16 + 4 * gq;
        if constexpr (EPI == 1) {
          cv[a][0] = shp ? *reinterpret_cast<const float4*>(shp + col) : float4{0.f, 0.f, 0.f, 0.f};
        } else {
          cv[a][0] = *reinterpret_cast<const float4*>(bvp + col);            // mean
          cv[a][1] = *reinterpret_cast<const float4*>(bvp + 2 * kC + col);   // scale
          cv[a][2] = *reinterpret_cast<const float4*>(bvp + 3 * kC + col);   // bias
        }
      }
    }
    // pixel offsets within the image (int32: < 2^31 elements per image) in two halves of
    // the 7 M tiles, so the EPI-2 input loads of a half are in flight together
    const __bf16* ximg = bnx + (EPI == 2 ? (int64_t)n * H * W * kC : 0);
    __bf16* yimg = Y + (int64_t)n * H * W * kC;
    auto half = [&](auto b0c, auto b1c) {
      constexpr int B0 = decltype(b0c)::value, B1 = decltype(b1c)::value;
      int off[B1 - B0];
      bool ok[B1 - B0];
#pragma unroll
      for (int b = B0; b < B1; ++b) {
        const int p = (mg * kTMW + b) * 16 + rl;
        const int r = p / W;
        ok[b - B0] = r < kR && h0 + r < H;
        off[b - B0] = ((h0 + r) * W + (p - r * W)) * kC;
      }
      u32x2 xw[EPI == 2 ? B1 - B0 : 1][EPI == 2 ? kTN : 1];
      if constexpr (EPI == 2) {
#pragma unroll
        for (int b = B0; b < B1; ++b)
#pragma unroll
          for (int a = 0; a < kTN; ++a)
            xw[b - B0][a] = ok[b - B0] ? *reinterpret_cast<const u32x2*>(
                                             ximg + off[b - B0] + nh * 32 + a * 16 + 4 * gq)
                                       : u32x2{0u, 0u};
      }
#pragma unroll
      for (int b = B0; b < B1; ++b) {
        if (!ok[b - B0]) continue;
#pragma unroll
        for (int a = 0; a < kTN; ++a) {
          const f32x4v v = acc[a][b];
          const int col = nh * 32 + a * 16 + 4 * gq;
          __bf16* yp = yimg + off[b - B0] + col;
          if constexpr (EPI == 2) {
            const u32x2 x2 = xw[b - B0][a];
            const float xv[4] = {__uint_as_float(x2[0] << 16), __uint_as_float(x2[0] & 0xffff0000u),
                                 __uint_as_float(x2[1] << 16), __uint_as_float(x2[1] & 0xffff0000u)};
            const float mus[4] = {cv[a][0].x, cv[a][0].y, cv[a][0].z, cv[a][0].w};
            const float scs[4] = {cv[a][1].x, cv[a][1].y, cv[a][1].z, cv[a][1].w};
            const float bis[4] = {cv[a][2].x, cv[a][2].y, cv[a][2].z, cv[a][2].w};
            float dv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float d = __builtin_fmaf(xv[r], scs[r], bis[r]) > 0.f ? round_bf16(v[r]) : 0.f;
              dv[r] = d;
              s1[a][r] += d;
              s2[a][r] += d * (xv[r] - mus[r]);
            }
            *reinterpret_cast<u32x2*>(yp) =
                u32x2{cvt_pk_bf16_cc(dv[0], dv[1]), cvt_pk_bf16_cc(dv[2], dv[3])};
          } else {
            const uint32_t lo = cvt_pk_bf16_cc(v[0], v[1]), hi = cvt_pk_bf16_cc(v[2], v[3]);
            *reinterpret_cast<u32x2*>(yp) = u32x2{lo, hi};
            if constexpr (EPI == 1) {
              const float vb[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                                   __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
              const float shs[4] = {cv[a][0].x, cv[a][0].y, cv[a][0].z, cv[a][0].w};
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float d = vb[r] - shs[r];
                s1[a][r] += d;
                s2[a][r] += d * d;
              }
            }
          }
        }
      }
    };
    half(std::integral_constant<int, 0>{}, std::integral_constant<int, 4>{});
    half(std::integral_constant<int, 4>{}, std::integral_constant<int, kTMW>{});
  };
  // 18 k steps (9 taps x 2 halves of 32 channels), fully unrolled and software-pipelined:
  // the fragments of step j+1 are read from LDS while step j's 28 MFMAs run (two
  // register sets); the scheduling barriers keep the compiler from hoisting every read
  // of the tile (which spilled) and from rotating the accumulators through copies
  auto frags = [&](int step, bf16x8 (&wf)[kTN], bf16x8 (&xf)[kTMW]) {
    const int tap = step >> 1, ch = (step & 1) * 4 + gq;
    const int dr = tap / 3, dc = tap - dr * 3;
    const int off = dr * kPW * 64 + dc * 64;
#pragma unroll
    for (int a = 0; a < kTN; ++a)
      wf[a] = *reinterpret_cast<const bf16x8*>(fs + fidx(nh * 32 + a * 16 + rl, tap, ch));
#pragma unroll
    for (int b = 0; b < kTMW; ++b)
      xf[b] = *reinterpret_cast<const bf16x8*>(
          ps + pbase[b] + off + ((ch ^ ((pcol[b] + dc) & 7)) << 3));
  };
  auto mmas = [&](const bf16x8 (&wf)[kTN], const bf16x8 (&xf)[kTMW]) {
#pragma unroll
    for (int a = 0; a < kTN; ++a)
#pragma unroll
      for (int b = 0; b < kTMW; ++b) acc[a][b] = mfma(wf[a], xf[b], acc[a][b]);
  };

  // Tile loop: [patch j -> LDS] [epilogue of j-1] [issue loads of j+1] [compute j]: the
  // stores of j-1 and the loads of j+1 fly during j's MFMAs.  The only wait on the memory
  // pipe is for the loads of tile j, issued a whole tile earlier.
  // the producing BN + ReLU on the in-image pixels of tile tt's prefetched patch rows
  auto bn_stage = [&](int64_t tt) {
    const int h0 = (int)(tt - (tt / g.hblocks) * g.hblocks) * kR;
#pragma unroll
    for (int i = 0; i < kLoads; ++i) {
      const int ih = h0 + i - 1;
      if (colok && ih >= 0 && ih < H) bn_relu8(pre[i], asc, abi);
    }
  };
  int64_t t = blockIdx.x;
  int64_t tprev = -1;
  if (t < g.tiles) {
    gload(t);
    if (bna) bn_stage(t);
  }
  for (; t < g.tiles; t += gridDim.x) {
    __syncthreads();                      // previous tile's patch reads done (and filter stored)
#pragma unroll
    for (int i = 0; i < kLoads; ++i)
      *reinterpret_cast<u32x4*>(ps + soff + i * kPW * 64) = pre[i];
    __syncthreads();
    // epilogue of the previous tile first (the prefetch registers are free here), then
    // the loads of the next tile: both drain while this tile's MFMAs run
    if (tprev >= 0) epilogue(tprev);
    __builtin_amdgcn_sched_barrier(0);
    if (t + gridDim.x < g.tiles) gload(t + gridDim.x);
    __builtin_amdgcn_sched_barrier(0);

#pragma unroll
    for (int a = 0; a < kTN; ++a)
#pragma unroll
      for (int b = 0; b < kTMW; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      bf16x8 wA[kTN], xA[kTMW];
      frags(st, wA, xA);
      mmas(wA, xA);
      __builtin_amdgcn_sched_barrier(0);
      // the next tile's BN + ReLU mid-tile: its rows have had half a tile to arrive, and the
      // VALU work overlaps the other wave's MFMAs on this SIMD (at the barrier both waves
      // would be doing it at once)
      if (st == 8 && bna && t + gridDim.x < g.tiles) {
        bn_stage(t + gridDim.x);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    tprev = t;
  }
  if (tprev >= 0) epilogue(tprev);
  if constexpr (EPI == 0) return;
  // fixed-order reduction: the 16 pixel lanes, then the 4 M-group waves of each channel half
#pragma unroll
  for (int a = 0; a < kTN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[a][r] += __shfl_xor(s1[a][r], o, kWave);
        s2[a][r] += __shfl_xor(s2[a][r], o, kWave);
      }
  __syncthreads();
  float* red = reinterpret_cast<float*>(ps);       // [2][4 groups][64]
  if (rl == 0) {
#pragma unroll
    for (int a = 0; a < kTN; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = nh * 32 + a * 16 + 4 * gq + r;
        red[(0 * 4 + mg) * kC + c] = s1[a][r];
        red[(1 * 4 + mg) * kC + c] = s2[a][r];
      }
  }
  __syncthreads();
  for (int v = tid; v < 2 * kC; v += kThreads) {
    const int k = v / kC, c = v - k * kC;
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < 4; ++m) s += red[(k * 4 + m) * kC + c];
    partial[((int64_t)blockIdx.x * 2 + k) * kC + c] = s;
  }
}

}  // namespace conv64
}  // namespace mv

bool mv_conv64_supported(int N, int H, int W, int C, int K, int ks, int stride) {
  return N > 0 && C == 64 && K == 64 && ks == 3 && stride == 1 && H >= 1 && W >= 1 &&
         (int64_t)H * W * 64 < (int64_t(1) << 31) &&
         W <= mv::conv64::kMaxW && (int64_t)mv::conv64::kR * W <= 16 * mv::conv64::kMT;
}

// grid = `grid` persistent workgroups (the caller's partial-row count)
bool mv_conv64(const void* x, const void* w, void* y, int N, int H, int W, const float* shift,
               float* partial, int grid, hipStream_t st, const void* bn_x, const float* bn_vec,
               const float* in_scale, const float* in_bias) {
  using namespace mv::conv64;
  if (!mv_conv64_supported(N, H, W, 64, 64, 3, 1) || grid < 1) return false;
  Geo64 g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.hblocks = (H + kR - 1) / kR;
  g.tiles = (int64_t)N * g.hblocks;
  const __bf16* X = (const __bf16*)x;
  const __bf16* Wt = (const __bf16*)w;
  __bf16* Y = (__bf16*)y;
  if ((in_scale == nullptr) != (in_bias == nullptr) || (bn_x && in_scale)) return false;
  if (bn_x) {
    if (!partial) return false;
    hipLaunchKernelGGL(conv64_kernel<2>, dim3(grid), dim3(kThreads), 0, st, X, Wt, Y, g,
                       nullptr, partial, (const __bf16*)bn_x, bn_vec, in_scale, in_bias);
  } else if (partial) {
    hipLaunchKernelGGL(conv64_kernel<1>, dim3(grid), dim3(kThreads), 0, st, X, Wt, Y, g,
                       shift, partial, nullptr, nullptr, in_scale, in_bias);
  } else {
    hipLaunchKernelGGL(conv64_kernel<0>, dim3(grid), dim3(kThreads), 0, st, X, Wt, Y, g,
                       nullptr, nullptr, nullptr, nullptr, in_scale, in_bias);
  }
  return true;
}

// ===========================================================================
// Weight gradient of the same 64 -> 64 3x3 / stride 1 conv (ResNet-50 layer1), row patch:
//   dW[k][tap][c] = sum_p dy[p][k] . X[pixel(p) + tap][c]
// The general wgrad3x3 kernel stages, per 32-pixel chunk, the dy rows and NINE tap-shifted
// X row tiles (every input row read 9x from L2).  Here a workgroup stages, per tile of
// R = 8 output rows of one image, the dy rows (448 px x 64 k, 56 KB) and the (R + 2)-row
// X patch (80 KB) once, and all 9 taps read their shifted pixels from the patch.  Both
// MFMA operands are pixel(=reduction)-major and come from gfx950's transposed LDS reads
// (ds_read_b64_tr_b16, 4 consecutive pixels per read: W % 4 == 0 keeps a group of 4 in
// one image row, so a tap shift moves it to 4 consecutive patch pixels, and the padded
// patch stride makes every tap a constant offset from tap (0, 0)).  8 waves:
// wave w owns input-channel tile w & 3 (16 c) and output-channel tiles 2 (w >> 2) .. +1
// for all 9 taps (18 accumulators), accumulated over the workgroup's tiles; fp32
// partial [G][9][64][64] rows + mv_conv.hip's fixed-order wgrad reduce.
// ===========================================================================
namespace mv {
namespace conv64 {

typedef short s16x4 __attribute__((ext_vector_type(4)));

constexpr int kWThreads = 512;
constexpr int kDyPix = kR * 56;                   // dy pixels staged per tile (W <= 56)
constexpr int kWLoadsDy = kDyPix * 8 / kWThreads;   // 7
constexpr int kWLoadsX = kPR;                       // 10 (one patch row per load)

// dy tile: [448 px][64 k] bf16, 128-B rows; the 16-B chunk ch of pixel p is stored at
// ch ^ dswz(p).  A transposed read's 32-lane half touches 8 consecutive pixels, 32 B each;
// the 64 banks span 256 B, so the 4 even (odd) pixels must sit in distinct 32-B windows.
__device__ __forceinline__ int dswz(int p) { return ((p >> 1) & 3) << 1; }
// X patch: [10 rows][58 cols] pixels at a 160-B (80-element) stride, unswizzled: 8
// consecutive pixels land on bank offsets 40 j mod 64 = {0, 40, 16, 56, 32, 8, 48, 24}
// dwords, one 8-dword window each, and every tap shift (dr, dc) is the constant offset
// (58 dr + dc) x 160 B from tap (0, 0).
constexpr int kPS = 80;                    // patch pixel stride (elements)
constexpr int kPC = 58;                    // patch columns (W + 2 <= 58)

__device__ __forceinline__ bf16x8 tr8p(const __bf16* pa, const __bf16* pb) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pa);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)pb);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 o = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, o);
}

__global__ __launch_bounds__(kWThreads, 1) __attribute__((amdgpu_waves_per_eu(2, 2)))
void wgrad64_kernel(const __bf16* __restrict__ X, const __bf16* __restrict__ DY,
                    float* __restrict__ partial, Geo64 g, const float* __restrict__ xsc,
                    const float* __restrict__ xbi) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[kDyPix * kC + kPR * kPC * kPS];   // 147 KB
  __bf16* ds = lds;
  __bf16* ps = lds + kDyPix * kC;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = wv & 3, kh = wv >> 2;
  const int gq = lane >> 4, cl = lane & 15;
  const int W = g.W, H = g.H;
  const int npix = kR * W;           // pixels per tile (W % 4 == 0, W <= 56)

  // staging roles.  dy: pixel (tid >> 3) + 64 i, chunk tid & 7.  X: patch column tid >> 3
  // (< 58) of patch row i, chunk tid & 7.
  const int sch = tid & 7, spix = tid >> 3;
  const bool colok = spix >= 1 && spix - 1 < W;
  const int64_t xcoff = (int64_t)(spix - 1) * kC + sch * 8;
  // X = the producing BN's input z when xsc != null: the patch holds relu(z * xsc + xbi)
  const bool bna = xsc != nullptr;
  float asc[8], abi[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    asc[j] = bna ? xsc[sch * 8 + j] : 0.f;
    abi[j] = bna ? xbi[sch * 8 + j] : 0.f;
  }
  u32x4 pdy[kWLoadsDy], px[kWLoadsX];
  auto gload = [&](int64_t t) {
    const int n = (int)(t / g.hblocks), h0 = (int)(t - (int64_t)n * g.hblocks) * kR;
    const __bf16* img = X + (int64_t)n * H * W * kC;
#pragma unroll
    for (int i = 0; i < kWLoadsX; ++i) {
      const int ih = h0 + i - 1;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (colok && ih >= 0 && ih < H)
        v = *reinterpret_cast<const u32x4*>(img + (int64_t)ih * W * kC + xcoff);
      px[i] = v;
    }
    const __bf16* dimg = DY + (int64_t)n * H * W * kC;
#pragma unroll
    for (int i = 0; i < kWLoadsDy; ++i) {
      const int p = spix + 64 * i;
      const int r = p / W;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (p < npix && h0 + r < H)
        v = *reinterpret_cast<const u32x4*>(dimg + ((int64_t)(h0 + r) * W + (p - r * W)) * kC +
                                            sch * 8);
      pdy[i] = v;
    }
  };

  // MFMA k index -> pixel: lane group gq holds pixels 4 gq + {0..3} (first half of its 8)
  // and 16 + 4 gq + {0..3} (second half) of the 32-pixel k step, so each 32-lane half of
  // a transposed read touches 8 consecutive pixels.  dy read addresses (k step 0; the +32
  // pixel step keeps dswz):
  const __bf16* ads[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = 4 * gq + 16 * h + (cl >> 2), e = 16 * (2 * kh + u) + 4 * (cl & 3);
      ads[u][h] = ds + r * 64 + (((e >> 3) ^ dswz(r)) << 3) + (e & 7);
    }
  const __bf16* pbase = ps + (cl >> 2) * kPS + 16 * ct + 4 * (cl & 3);
  f32x4v acc[2][9];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) acc[u][tp] = f32x4v{0.f, 0.f, 0.f, 0.f};

  auto bn_stage = [&](int64_t tt) {      // the producing BN + ReLU on tile tt's patch rows
    const int h0 = (int)(tt - (tt / g.hblocks) * g.hblocks) * kR;
#pragma unroll
    for (int i = 0; i < kWLoadsX; ++i) {
      const int ih = h0 + i - 1;
      if (colok && ih >= 0 && ih < H) bn_relu8(px[i], asc, abi);
    }
  };
  int64_t t = blockIdx.x;
  if (t < g.tiles) gload(t);
  for (; t < g.tiles; t += gridDim.x) {
    __syncthreads();                      // previous tile's reads done
    if (bna) bn_stage(t);                 // (mid-loop placement measured slower here)
    if (spix < kPC) {
#pragma unroll
      for (int i = 0; i < kWLoadsX; ++i)
        *reinterpret_cast<u32x4*>(ps + (i * kPC + spix) * kPS + sch * 8) = px[i];
    }
#pragma unroll
    for (int i = 0; i < kWLoadsDy; ++i) {
      const int p = spix + 64 * i;
      *reinterpret_cast<u32x4*>(ds + p * 64 + ((sch ^ dswz(p)) << 3)) = pdy[i];
    }
    __syncthreads();
    if (t + gridDim.x < g.tiles) gload(t + gridDim.x);
    __builtin_amdgcn_sched_barrier(0);
    // ceil(R W / 32) k steps of 32 pixels.  Pixels >= R W (and rows past H) are zero dy
    // rows: they add nothing, and their patch index is clamped to 0 so every read stays
    // inside the patch.  (row, col) of this lane's two pixel groups advance by 32 a step.
    const int nks = (npix + 31) >> 5;
    int ra = (4 * gq) / W, ca = 4 * gq - ra * W;
    int rb = (4 * gq + 16) / W, cb = 4 * gq + 16 - rb * W;
#pragma unroll 1
    for (int ks = 0; ks < nks; ++ks) {
      const int pa = ks * 32 + 4 * gq;
      const int qa = pa < npix ? ra * kPC + ca : 0;
      const int qb = pa + 16 < npix ? rb * kPC + cb : 0;
      bf16x8 af[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) af[u] = tr8p(ads[u][0] + ks * 32 * 64, ads[u][1] + ks * 32 * 64);
      const __bf16* ba = pbase + qa * kPS;
      const __bf16* bb = pbase + qb * kPS;
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int off = ((tp / 3) * kPC + tp % 3) * kPS;
        const bf16x8 bfr = tr8p(ba + off, bb + off);
#pragma unroll
        for (int u = 0; u < 2; ++u) acc[u][tp] = mfma(af[u], bfr, acc[u][tp]);
      }
      __builtin_amdgcn_sched_barrier(0);
      ca += 32;
      while (ca >= W) {
        ca -= W;
        ++ra;
      }
      cb += 32;
      while (cb >= W) {
        cb -= W;
        ++rb;
      }
    }
  }
  // partial[blockIdx][tap][k][c]; every block writes (zeros without tiles)
  float* pp = partial + (int64_t)blockIdx.x * 9 * kC * kC;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * (2 * kh + u) + 4 * gq + r, c = 16 * ct + cl;
        pp[((int64_t)tp * kC + k) * kC + c] = acc[u][tp][r];
      }
}

}  // namespace conv64
}  // namespace mv

bool mv_wgrad64_supported(int N, int H, int W, int C, int K, int stride) {
  return N > 0 && C == 64 && K == 64 && stride == 1 && H >= 1 && W >= 4 && W % 4 == 0 &&
         W <= 56 && (int64_t)H * W * 64 < (int64_t(1) << 31);
}

bool mv_wgrad64(const void* x, const void* dy, float* partial, int grid, int N, int H, int W,
                hipStream_t st, const float* in_scale, const float* in_bias) {
  using namespace mv::conv64;
  if (!mv_wgrad64_supported(N, H, W, 64, 64, 1) || grid < 1) return false;
  Geo64 g;
  g.N = N;
  g.H = H;
  g.W = W;
  g.hblocks = (H + kR - 1) / kR;
  g.tiles = (int64_t)N * g.hblocks;
  if ((in_scale == nullptr) != (in_bias == nullptr)) return false;
  hipLaunchKernelGGL(wgrad64_kernel, dim3(grid), dim3(kWThreads), 0, st, (const __bf16*)x,
                     (const __bf16*)dy, partial, g, in_scale, in_bias);
  return true;
}
