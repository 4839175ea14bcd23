// ResNet stem: 7x7 / stride 2 / pad 3 conv, 4 (zero-padded RGB) -> 64 channels, NHWC bf16,
// on MFMA with the stem BatchNorm's statistics in the epilogue.
//
// MIOpen runs this shape at ~240 TFLOP/s (2.7 ms per bs-2048 step, K = 7*7*4 is awkward
// for its tilings) and the BN statistics pass reads the 3.3 GB output again.  Here one
// output ROW (112 pixels x 64 channels) is an [112 x 224] . [224 x 64] product whose K
// walks the 7x7 window as (tap row r, tap-column pair, channel): for v_mfma_f32_16x16x32
// k-step r, the 16-byte operand of k-group g is the input pixels (2p + 2g, 2p + 2g + 1) of
// padded row r — 8 contiguous bf16 of an LDS image of the 7 input rows — so the im2col
// operand is read straight from the staged rows (tap column 7 is a zero weight).
//
// Workgroup = 4 waves, persistent over pairs of output rows (n, oh..oh+1); wave w owns output
// channels 16w .. 16w+15 and all 2 x 7 pixel tiles.  The filter (64 x 224, XOR-swizzled 16-byte chunks)
// stays in LDS; the next row's input is prefetched into registers during the MFMAs.
// Epilogue: bf16 store of 4 consecutive channels per lane + per-channel (sum, sum^2)
// around the running mean, reduced to one [2][64] partial row per workgroup (fixed order,
// mv_bn.hip's finalize layout).
#include "mv_common.h"
#include "mv_stem.h"

namespace mv {
namespace stem {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kH = 224, kW = 224, kC = 4, kOH = 112, kOW = 112, kCO = 64;
constexpr int kPW = 232;                    // padded patch row (230 used: cols -3 .. 226)
constexpr int kChunks = 32;                 // filter row: 28 used 16-byte chunks, 32 for the swizzle
// R output rows per iteration share 2R + 5 staged input rows (R = 2: 9 rows for 2 output
// rows instead of 14, and each filter fragment feeds 14 pixel tiles)
#ifndef MV_STEM_ROWS
#define MV_STEM_ROWS 2
#endif
constexpr int kR = MV_STEM_ROWS;
constexpr int kIR = 2 * kR + 5;             // staged input rows
constexpr int kPatch = kIR * kPW;           // pixels in the LDS patch
constexpr int kLoads = (kIR * 230 + 255) / 256;   // 8-byte patch loads per thread

__device__ __forceinline__ f32x4v mfma(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// one input pixel as the 4-channel LDS image wants it: cin = 4 (zero-padded RGB, one 8-byte
// load) or cin = 3 (the raw RGB image, three 2-byte loads, channel 3 = 0 — no padded copy
// of the input is ever written)
__device__ __forceinline__ u32x2 ld_px(const __bf16* x, int64_t pix, int cin) {
  if (cin == 4) return *reinterpret_cast<const u32x2*>(x + pix * 4);
  const uint16_t* p = reinterpret_cast<const uint16_t*>(x) + pix * 3;
  return u32x2{(uint32_t)p[0] | ((uint32_t)p[1] << 16), (uint32_t)p[2]};
}

// 2 waves/SIMD: 236 VGPRs with the MFMA accumulators in VGPRs (1.21 vs 1.53 ms at 1 wave).
// Round 2 saw NaN at this bound: the epilogue's bf16 conversion was inline asm, which
// the compiler's hazard recognizer cannot see into, so it read the VGPR accumulators 0-6
// wait states after the MFMA wrote them (11 needed; no hardware interlock) — the
// epilogue now uses mv_common.h's compiler-selected cvt_pk_bf16_cc; checked by
// scripts/check_mfma_asm_hazards.py; tests/test_conv_gpu.py runs several grid sizes.
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(const __bf16* __restrict__ x,
                                                       const __bf16* __restrict__ w,
                                                       __bf16* __restrict__ z,
                                                       const float* __restrict__ shift,
                                                       float* __restrict__ partial, int N,
                                                       int cin) {
  __shared__ __attribute__((aligned(16))) __bf16 ws[kCO * kChunks * 8];   // 32 KB
  __shared__ __attribute__((aligned(16))) __bf16 ps[kPatch * kC];         // 14.5 KB
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int g = lane >> 4, rl = lane & 15;

  // filter -> LDS: row o, chunk (r, pair) = w[o][r][2 pair .. 2 pair + 1][0..3] (OHWC)
  for (int q = tid; q < kCO * kChunks; q += 256) {
    const int o = q / kChunks, ch = q % kChunks;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (ch < 28) {
      const int r = ch / 4, pr = ch % 4;
      const __bf16* src = w + ((o * 7 + r) * 7 + 2 * pr) * kC;
      const u32x2 a = *reinterpret_cast<const u32x2*>(src);
      v[0] = a[0];
      v[1] = a[1];
      if (pr < 3) {
        const u32x2 b = *reinterpret_cast<const u32x2*>(src + kC);
        v[2] = b[0];
        v[3] = b[1];
      }
    }
    *reinterpret_cast<u32x4*>(ws + (o * kChunks + (ch ^ (o & 7))) * 8) = v;
  }

  const int64_t rows = (int64_t)N * (kOH / kR);      // row groups
  u32x2 pre[kLoads];
  auto gload = [&](int64_t row) {
    const int n = (int)(row / (kOH / kR)), oh = (int)(row % (kOH / kR)) * kR;
#pragma unroll
    for (int i = 0; i < kLoads; ++i) {
      const int q = tid + i * 256;
      const int r = q / 230, pc = q % 230;
      const int ih = 2 * oh + r - 3, iw = pc - 3;
      u32x2 v = {0u, 0u};
      if (q < kIR * 230 && ih >= 0 && ih < kH && iw >= 0 && iw < kW)
        v = ld_px(x, ((int64_t)n * kH + ih) * kW + iw, cin);
      pre[i] = v;
    }
  };

  float sh[4], s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sh[j] = shift ? shift[16 * wv + 4 * g + j] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
  int64_t row = blockIdx.x;
  if (row < rows) gload(row);
  for (; row < rows; row += gridDim.x) {
    __syncthreads();                     // previous row's patch reads (and filter stores) done
#pragma unroll
    for (int i = 0; i < kLoads; ++i) {
      const int q = tid + i * 256;
      if (q < kIR * 230) {
        const int r = q / 230, pc = q % 230;
        *reinterpret_cast<u32x2*>(ps + (r * kPW + pc) * kC) = pre[i];
      }
    }
    __syncthreads();
    if (row + gridDim.x < rows) gload(row + gridDim.x);
    f32x4v acc[kR][7];
#pragma unroll
    for (int j = 0; j < kR; ++j)
#pragma unroll
      for (int t = 0; t < 7; ++t) acc[j][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 7; ++kk) {
      const int o = 16 * wv + rl, ch = kk * 4 + g;
      const bf16x8 wf = *reinterpret_cast<const bf16x8*>(ws + (o * kChunks + (ch ^ (o & 7))) * 8);
#pragma unroll
      for (int j = 0; j < kR; ++j)
#pragma unroll
        for (int t = 0; t < 7; ++t) {
          const int p = t * 16 + rl;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(
              ps + ((2 * j + kk) * kPW + 2 * p + 2 * g) * kC);
          acc[j][t] = mfma(wf, af, acc[j][t]);
        }
    }
#pragma unroll
    for (int j = 0; j < kR; ++j)
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      __bf16* zr = z + (row * kR + j) * (int64_t)kOW * kCO + 16 * wv + 4 * g;
      const int p = t * 16 + rl;
      // raw MFMA accumulators (VGPRs at 2 waves/SIMD): the hazard-safe conversion
      const uint32_t lo = cvt_pk_bf16_cc(acc[j][t][0], acc[j][t][1]);
      const uint32_t hi = cvt_pk_bf16_cc(acc[j][t][2], acc[j][t][3]);
      *reinterpret_cast<u32x2*>(zr + (int64_t)p * kCO) = u32x2{lo, hi};
      const float v[4] = {__uint_as_float(lo << 16), __uint_as_float(lo & 0xffff0000u),
                          __uint_as_float(hi << 16), __uint_as_float(hi & 0xffff0000u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[e] - sh[e];
        s1[e] += d;
        s2[e] += d * d;
      }
    }
  }
  // fixed-order reduction over the 16 pixel lanes that share these 4 channels
#pragma unroll
  for (int j = 0; j < 4; ++j) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[j] += __shfl_xor(s1[j], o, kWave);
      s2[j] += __shfl_xor(s2[j], o, kWave);
    }
  }
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * wv + 4 * g + j;
      partial[((int64_t)blockIdx.x * 2 + 0) * kCO + c] = s1[j];
      partial[((int64_t)blockIdx.x * 2 + 1) * kCO + c] = s2[j];
    }
  }
}

}  // namespace stem
}  // namespace mv

int mv_stem_partials(int N) {
  static int per = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, (const void*)mv::stem::stem_fwd_kernel,
                                                     256, 0) != hipSuccess || v < 1)
      v = 1;
    return v;
  }();
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  const int64_t rows = (int64_t)N * (mv::stem::kOH / mv::stem::kR);
  int64_t g = (int64_t)cus * per;
  if (g > rows) g = rows;
  return (int)g;
}

void mv_stem_fwd(const void* x, const void* w, void* z, const float* shift, float* partial, int N,
                 hipStream_t st, int grid, int cin) {
  if (grid <= 0) grid = mv_stem_partials(N);
  hipLaunchKernelGGL(mv::stem::stem_fwd_kernel, dim3(grid), dim3(256), 0, st, (const __bf16*)x,
                     (const __bf16*)w, (__bf16*)z, shift, partial, N, cin);
}

// ---------------------------------------------------------------- weight gradient
// dW[o][k] = sum over output pixels p of dz[p][o] * patch_p[k], k = (tap row r, tap column
// s in 0..7, channel c) — s = 7 is dropped at the end.  Per output row: dz [112 x 64] staged
// in LDS (rows 112..127 zero, the XOR layout of mv_conv's transposed reads) and the 7 input
// rows; both MFMA operands are pixel(k)-major and come from gfx950 transposed LDS reads —
// for the image operand the "row" of pixel p is the 16 contiguous values patch[r][2p + s0 ..
// 2p + s0 + 3][0..3] (row pitch 16 bytes, overlapping rows).  Wave w owns output channels
// 16w..16w+15 and all 14 k tiles; fp32 partials [G][64][224] + a fixed-order reduce.
namespace mv {
namespace stem {

typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int dswz(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }

// 4 pixels (rows r0 .. r0+3) of column col0 + c of the [128][64] dz tile
__device__ __forceinline__ s16x4 dz_tr4(const __bf16* base, int r0, int col0, int c) {
  const int r = r0 + (c >> 2), e = col0 + 4 * (c & 3);
  const __bf16* p = base + r * 64 + (((e >> 3) ^ dswz(r)) << 3) + (e & 7);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

// 4 pixels (p0 .. p0+3, clamped to 111) of k column c of tile (r, s0) of the patch
__device__ __forceinline__ s16x4 px_tr4(const __bf16* ps, int p0, int r, int s0, int c) {
  int p = p0 + (c >> 2);
  p = p < kOW - 1 ? p : kOW - 1;
  const __bf16* a = ps + (r * kPW + 2 * p + s0) * kC + 4 * (c & 3);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a);
}

__device__ __forceinline__ bf16x8 cat8(const s16x4& a, const s16x4& b) {
  bf16x8 o;
  short* q = reinterpret_cast<short*>(&o);
  q[0] = a[0]; q[1] = a[1]; q[2] = a[2]; q[3] = a[3];
  q[4] = b[0]; q[5] = b[1]; q[6] = b[2]; q[7] = b[3];
  return o;
}


// FUSE: dz comes from the maxpool + BN+ReLU backward (MvStemPoolBwd), built per output row
// while it is staged (512-thread workgroups): thread t < 448 owns 8 channels of the pixel
// pair (2b, 2b + 1) of the row, whose pooled windows are columns b, b + 1 of the 1 (even
// row) or 2 (odd row) pooled rows covering it.  The z pair is prefetched with the next
// row's patch; the 2 windows of a pooled row are loaded together and applied in
// maxpool_bwd_k3s2_kernel's order (same fp32 sums, same fma epilogue -> the same dz bits).
constexpr int kPairs = (kOW / 2) * 8;                 // (pixel pair, 8-channel group) items per row

__device__ __forceinline__ void pool_bn_dz_pair(const MvStemPoolBwd& pb, const float* coef, int n,
                                                int oh, int b, int c, const u32x4 (&zr)[2],
                                                u32x4 (&out)[2]) {
  constexpr int kPH = kOH / 2, kPW2 = kOW / 2;
  float acc[2][8];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  const int a = oh >> 1, i = oh & 1;
  const int nda = i && a + 1 < kPH ? 2 : 1;           // uniform per row
  const bool ok1 = b + 1 < kPW2;
  // one pooled row at a time (both rows' windows in flight spill at 128 VGPRs)
  for (int da = 0; da < nda; ++da) {
    const int kh = i - 2 * da + 1;
    u32x2 iw[2];
    u32x4 dv[2], d2v[2];
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      const int col = db && !ok1 ? b : b + db;        // clamped; masked below
      const int64_t o = (((int64_t)n * kPH + a + da) * kPW2 + col) * kCO + c;
      iw[db] = *reinterpret_cast<const u32x2*>(pb.idx + o);
      dv[db] = *reinterpret_cast<const u32x4*>(reinterpret_cast<const __bf16*>(pb.dy) + o);
      d2v[db] = pb.dy2 ? *reinterpret_cast<const u32x4*>(reinterpret_cast<const __bf16*>(pb.dy2) + o)
                       : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      float d[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        d[2 * q] = __uint_as_float(dv[db][q] << 16);
        d[2 * q + 1] = __uint_as_float(dv[db][q] & 0xffff0000u);
      }
      if (pb.dy2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          d[2 * q] += __uint_as_float(d2v[db][q] << 16);
          d[2 * q + 1] += __uint_as_float(d2v[db][q] & 0xffff0000u);
        }
      }
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int kw = jj - 2 * db + 1;
        if (kw < 0) continue;
        const uint32_t pos = db && !ok1 ? 0xffu : (uint32_t)(kh * 3 + kw);   // 0xff: no index
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t wd = e < 4 ? iw[db][0] : iw[db][1];
          if (((wd >> (8 * (e & 3))) & 0xffu) == pos) acc[jj][e] += d[e];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    float v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __uint_as_float(zr[k][q] << 16);
      v[2 * q + 1] = __uint_as_float(zr[k][q] & 0xffff0000u);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float* kf = coef + c + e;      // [5][64]: scale, bias, ca, cb, cc
      const float d = __builtin_fmaf(v[e], kf[0], kf[64]) > 0.f ? acc[k][e] : 0.f;
      v[e] = __builtin_fmaf(kf[128], d, __builtin_fmaf(kf[192], v[e], kf[256]));
    }
    out[k] = u32x4{cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3]), cvt_pk_bf16(v[4], v[5]),
                   cvt_pk_bf16(v[6], v[7])};
  }
}

// NT threads (NT / 64 waves): wave w owns output channels 16 (w % 4) .. + 15 and the
// 14 / (NT / 256) k tiles from (w / 4) * that on — a tile's products are summed in the same
// order whatever NT is.
template <int NT, bool FUSE>
__global__ __launch_bounds__(NT, FUSE ? 4 : 1) void stem_wgrad_kernel(const __bf16* __restrict__ x,
                                                        const __bf16* __restrict__ dz,
                                                        float* __restrict__ partial, int N,
                                                        int cin, MvStemPoolBwd pb) {
  static_assert(!FUSE || NT >= kPairs, "one pixel pair per thread");
  constexpr int kTPW = 14 / (NT / 256);                // k tiles per wave
  __shared__ __attribute__((aligned(16))) __bf16 ps[7 * kPW * kC];        // 13 KB
  __shared__ __attribute__((aligned(16))) __bf16 ds[128 * 64];            // 16 KB
  __shared__ float coef[FUSE ? 5 * 64 : 1];
  const int tid = threadIdx.x;
  if constexpr (FUSE) {
    for (int q = tid; q < 5 * 64; q += NT) {
      const float* src[5] = {pb.scale, pb.bias, pb.ca, pb.cb, pb.cc};
      coef[q] = src[q / 64][q % 64];
    }
  }
  const int64_t rows = (int64_t)N * kOH;
  f32x4v acc[kTPW];
#pragma unroll
  for (int t = 0; t < kTPW; ++t) acc[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
  // dz rows 112..127 stay zero (written once)
  for (int q = tid; q < 16 * 8; q += NT) {
    const int r = 112 + q / 8, ch = q % 8;
    *reinterpret_cast<u32x4*>(ds + r * 64 + ((ch ^ dswz(r)) << 3)) = u32x4{0u, 0u, 0u, 0u};
  }
  // next row's patch and dz (FUSE: z pair) in registers while the current row computes
  constexpr int kPL = (7 * 230 + NT - 1) / NT;            // 8-byte patch loads per thread
  constexpr int kDz = FUSE ? 2 : (kOW * 8 + NT - 1) / NT;  // 16-byte dz / z chunks per thread
  u32x2 pp[kPL];
  u32x4 pd[kDz];
  auto gload = [&](int64_t row, int tid) {
    const int n = (int)(row / kOH), oh = (int)(row % kOH);
#pragma unroll
    for (int i = 0; i < kPL; ++i) {
      const int q = tid + i * NT;
      const int r = q / 230, pc = q % 230;
      const int ih = 2 * oh + r - 3, iw = pc - 3;
      u32x2 v = {0u, 0u};
      if (q < 7 * 230 && ih >= 0 && ih < kH && iw >= 0 && iw < kW)
        v = ld_px(x, ((int64_t)n * kH + ih) * kW + iw, cin);
      pp[i] = v;
    }
    if constexpr (FUSE) {
      const __bf16* zr = reinterpret_cast<const __bf16*>(pb.z) + row * (int64_t)kOW * kCO;
      const int b = tid / 8, c = (tid % 8) * 8;
#pragma unroll
      for (int k = 0; k < 2; ++k)
        pd[k] = tid < kPairs ? *reinterpret_cast<const u32x4*>(zr + (2 * b + k) * kCO + c)
                             : u32x4{0u, 0u, 0u, 0u};

    } else {
      const __bf16* dzr = dz + row * (int64_t)kOW * kCO;
#pragma unroll
      for (int i = 0; i < kDz; ++i) {
        const int q = tid + i * NT;
        pd[i] = q < kOW * 8 ? *reinterpret_cast<const u32x4*>(dzr + q * 8) : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  int64_t row = blockIdx.x;
  if (row < rows) gload(row, tid);
  for (; row < rows; row += gridDim.x) {
    // FUSE: lane-derived values recomputed per row from an opaque copy of the thread id —
    // hoisted out of the loop, the ~60 loop-invariant LDS / global addresses spill at the
    // 128 VGPRs of 4 waves / SIMD
    int tid = threadIdx.x;
    if constexpr (FUSE) asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wv = tid >> 6, g = lane >> 4, cl = lane & 15;
    const int cw = wv & 3, t0 = (wv >> 2) * kTPW;
    __syncthreads();                        // previous row's LDS reads done
#pragma unroll
    for (int i = 0; i < kPL; ++i) {
      const int q = tid + i * NT;
      if (q < 7 * 230) {
        const int r = q / 230, pc = q % 230;
        *reinterpret_cast<u32x2*>(ps + (r * kPW + pc) * kC) = pp[i];
      }
    }
    if constexpr (FUSE) {
      if (tid < kPairs) {
        const int oh = (int)(row % kOH);
        const int b = tid / 8, ch = tid % 8;
        const u32x4 zr[2] = {pd[0], pd[1]};
        u32x4 o[2];
        // the pooled windows are loaded here, not prefetched with the patch: holding them
        // through the MFMA phase needs 2 waves / SIMD (3.66 vs 2.90 ms/step at bs 2048)
        pool_bn_dz_pair(pb, coef, (int)(row / kOH), oh, b, ch * 8, zr, o);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int r = 2 * b + k;
          *reinterpret_cast<u32x4*>(ds + r * 64 + ((ch ^ dswz(r)) << 3)) = o[k];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < kDz; ++i) {
        const int q = tid + i * NT;
        if (q < kOW * 8) {
          const int r = q / 8, ch = q % 8;
          *reinterpret_cast<u32x4*>(ds + r * 64 + ((ch ^ dswz(r)) << 3)) = pd[i];
        }
      }
    }
    __syncthreads();
    if (row + gridDim.x < rows) gload(row + gridDim.x, tid);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int p0 = ks * 32 + 8 * g;
      const bf16x8 af = cat8(dz_tr4(ds, p0, 16 * cw, cl), dz_tr4(ds, p0 + 4, 16 * cw, cl));
#pragma unroll
      for (int tt = 0; tt < kTPW; ++tt) {
        const int t = t0 + tt, r = t >> 1, s0 = 4 * (t & 1);
        const bf16x8 bf = cat8(px_tr4(ps, p0, r, s0, cl), px_tr4(ps, p0 + 4, r, s0, cl));
        acc[tt] = mfma(af, bf, acc[tt]);
      }
      // FUSE (4 waves / SIMD): keep the fragment reads of one k step together (hoisting
      // all 28 spills at 128 VGPRs)
      if constexpr (FUSE) __builtin_amdgcn_sched_barrier(0);
    }
  }
  const int lane = tid & 63, wv = tid >> 6, g = lane >> 4, cl = lane & 15;
  const int cw = wv & 3, t0 = (wv >> 2) * kTPW;
  float* pout = partial + (int64_t)blockIdx.x * kCO * 224;
#pragma unroll
  for (int tt = 0; tt < kTPW; ++tt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      pout[(16 * cw + 4 * g + r) * 224 + (t0 + tt) * 16 + cl] = acc[tt][r];
}

// dw[o][r][s][c] (OHWC, s < 7) = sum_g partial[g][o][r * 32 + s * 4 + c], fixed order
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ partial,
                                                                int G, __bf16* __restrict__ dw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= kCO * 7 * 7 * kC) return;
  const int c = i % kC, s = (i / kC) % 7, r = (i / (kC * 7)) % 7, o = i / (kC * 49);
  const int k = r * 32 + s * 4 + c;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int gi = 0;
  for (; gi + 3 < G; gi += 4) {
    a0 += partial[((int64_t)gi * kCO + o) * 224 + k];
    a1 += partial[((int64_t)(gi + 1) * kCO + o) * 224 + k];
    a2 += partial[((int64_t)(gi + 2) * kCO + o) * 224 + k];
    a3 += partial[((int64_t)(gi + 3) * kCO + o) * 224 + k];
  }
  for (; gi < G; ++gi) a0 += partial[((int64_t)gi * kCO + o) * 224 + k];
  dw[i] = (__bf16)((a0 + a1) + (a2 + a3));
}

}  // namespace stem
}  // namespace mv

int mv_stem_wgrad_blocks(int N) {
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  int64_t g = (int64_t)cus * 4;
  const int64_t rows = (int64_t)N * mv::stem::kOH;
  if (g > rows) g = rows;
  return (int)g;
}

void mv_stem_wgrad(const void* x, const void* dz, void* dw, float* work, int N, hipStream_t st,
                   int cin) {
  const int G = mv_stem_wgrad_blocks(N);
  hipLaunchKernelGGL((mv::stem::stem_wgrad_kernel<256, false>), dim3(G), dim3(256), 0, st,
                     (const __bf16*)x, (const __bf16*)dz, work, N, cin, MvStemPoolBwd{});
  hipLaunchKernelGGL(mv::stem::stem_wgrad_reduce_kernel, dim3((64 * 196 + 255) / 256), dim3(256), 0,
                     st, work, G, (__bf16*)dw);
}

void mv_stem_wgrad_pool_bn(const void* x, const MvStemPoolBwd& pb, void* dw, float* work, int N,
                           hipStream_t st, int cin) {
  const int G = mv_stem_wgrad_blocks(N);
  hipLaunchKernelGGL((mv::stem::stem_wgrad_kernel<512, true>), dim3(G), dim3(512), 0, st,
                     (const __bf16*)x, (const __bf16*)nullptr, work, N, cin, pb);
  hipLaunchKernelGGL(mv::stem::stem_wgrad_reduce_kernel, dim3((64 * 196 + 255) / 256), dim3(256), 0,
                     st, work, G, (__bf16*)dw);
}
