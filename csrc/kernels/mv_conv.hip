// Implicit-GEMM 3x3 convolution (pad 1, stride 1 or 2) on gfx950 MFMA, NHWC bf16.
//
//   Y[m, k] = sum_{r, s, c} X[n, ho*st - 1 + r, wo*st - 1 + s, c] . W[k, r, s, c]
//   m = (n, ho, wo) — a GEMM with M = N*Ho*Wo, N = Cout, K = 9*Cin whose A operand
//   (im2col(X)) is never materialised: every 64-channel K step of the tile reads one
//   filter tap's rows of X straight into LDS.
//
// Staging: global_load_lds (16 bytes per lane, no VGPR round trip) into a 3-slot
// LDS ring; the loads of the next TWO K steps — across the boundary into the
// workgroup's next output tile — are in flight while the current step runs on the
// matrix cores (counted vmcnt waits + raw s_barrier, so they survive the barrier).  The LDS image is lane-linear (the LDS-DMA writes base + lane*16),
// so the 16-byte-chunk XOR swizzle that keeps the fragment reads conflict-free is
// applied to the per-lane GLOBAL source address (slot (row, c) holds chunk
// c ^ (row & 7)) and undone on the read.  Padding taps read a zero page.
//
// Persistent tiles: a workgroup owns one column tile (BN output channels) and walks
// output-row tiles mt = stream, stream + nstreams, ...; with STATS the following
// BatchNorm's per-channel sums (of the bf16-rounded outputs around shift) accumulate
// in registers over all of them and one [2][BN] partial row per stream is written —
// the layout of the BN finalize (mv_bn.hip), as in mv_gemm.hip.
//
// MFMA mapping as mv_gemm.hip: the filter tile is the A operand, so each lane's 4
// accumulators are 4 consecutive output channels of one output pixel (8-byte stores).
#include "mv_common.h"
#include "mv_conv.h"
#include "mv_gemm.h"

#include <algorithm>
#include <cstdlib>

namespace mv {
namespace conv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 64;              // input channels per K step (one tap)

__device__ __attribute__((aligned(16))) uint32_t g_zero[32];   // zero page for padding taps

__device__ __forceinline__ f32x4v mfma(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int swz(int row, int ch) { return row * BK + ((ch ^ (row & 7)) << 3); }
__device__ __forceinline__ float round_bf16(float x) { return (float)(__bf16)x; }

__device__ __forceinline__ int remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ void glds16(const void* src, __bf16* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

struct Geo {
  int H, W, C, Ho, Wo, K, st;
  int64_t M;
  int ks = 3;        // filter size: 3 (pad 1) or 1 (pad 0) for the forward kernel
  // conv3x3_kernel<..., DG = true>: stride-2 3x3 DATA gradient, output parity class (ph, pw)
  // (mv_gemm256.hip AMODE 4's scheme): rows are the class pixels (n, i, j) of dx [*, H, W, K],
  // the gather reads dy [*, Ho, Wo, C] at (n, i + di, j + dj) for the class's taps
  int ph = 0, pw = 0;
  // wgrad1x1 only: dy channels [k1, K) come from dy2 ([M, K - k1], output rows) — the BN
  // fold's dz^T x and Gram x^T x in one pass over x (k1 = K: single source)
  const __bf16* dy2 = nullptr;
  int k1 = 0;
  // dy2x: dy2 is [*, H, W, K - k1] at the INPUT resolution, read at the strided pixel of
  // each output row like X (the shortcut fold's Gram pass over x0[:, :, ::s, ::s])
  int dy2x = 0;
};

// per-thread state of the A rows it stages (A_CH rows, fixed source chunk): the byte
// address of tap (0, 0) and a 9-bit mask of the taps that fall inside the image —
// per K step only a wave-uniform offset is added (keeps the issue path a few VALU ops)
template <int A_CH>
struct RowInfo {
  uint64_t addr[A_CH];
  uint32_t valid[A_CH];
};

template <int A_CH, int NT, bool DG = false>
__device__ __forceinline__ void row_info(const Geo& g, const __bf16* X, int64_t m0, int tid,
                                         int sc, RowInfo<A_CH>& ri) {
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int64_t m = m0 + i * (NT / 8) + (tid >> 3);
    ri.valid[i] = 0;
    ri.addr[i] = 0;
    if (DG && m < g.M) {
      // class row (n, ci, cj) reads dy (n, ci + di, cj + dj): bit 2 di + dj when inside dy
      // (rows < 2^31: 32-bit unsigned divisions, several times cheaper than 64-bit ones)
      const uint32_t hw = (uint32_t)(g.Ho * g.Wo);
      const int rem = (int)((uint32_t)m % hw);
      const int ci = (int)((uint32_t)rem / (uint32_t)g.Wo), cj = rem - ci * g.Wo;
      const bool r1 = ci + 1 < g.Ho, c1 = cj + 1 < g.Wo;
      ri.valid[i] = 1u | (c1 ? 2u : 0u) | (r1 ? 4u : 0u) | (r1 && c1 ? 8u : 0u);
      ri.addr[i] = (uint64_t)(X + (m * g.C + sc * 8));
    } else if (m < g.M) {
      const uint32_t hw = (uint32_t)(g.Ho * g.Wo), m32 = (uint32_t)m;
      const int n = (int)(m32 / hw);
      const int rem = (int)(m32 - (uint32_t)n * hw);
      const int ho = (int)((uint32_t)rem / (uint32_t)g.Wo), wo = rem - ho * g.Wo;
      const int pad = g.ks >> 1;
      const int hi0 = ho * g.st - pad, wi0 = wo * g.st - pad;
      uint32_t v = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool ok = r < g.ks && s < g.ks && (unsigned)(hi0 + r) < (unsigned)g.H &&
                          (unsigned)(wi0 + s) < (unsigned)g.W;
          v |= (ok ? 1u : 0u) << (r * g.ks + s);
        }
      ri.valid[i] = v;
      ri.addr[i] = (uint64_t)(X + ((((int64_t)n * g.H + hi0) * g.W + wi0) * g.C + sc * 8));
    }
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// EPI: 0 plain, 1 + BN statistics of y (forward), 2 the BN+ReLU (mode 1) backward reduce
// of the BN whose output was this conv's input: y is the data gradient dy of that output,
// d = (x_bn * scale + bias > 0) ? bf16(dy) : 0 is written instead, partials (sum d,
// sum d (x_bn - mean)) — mv_bn.hip's bwd_reduce_kernel<1> folded into the epilogue.
// the second launch bound asks for 2 resident workgroups (the LDS ring allows 2): the
// 8-wave BN-reduce variant otherwise grows past 128 VGPRs and runs one workgroup per CU
template <int BM, int BN, int WM, int WN, int EPI, int NS = 3, bool DG = false>
__global__ __launch_bounds__(WM * WN * 64)
__attribute__((amdgpu_waves_per_eu((NS == 2 && WM * WN == 8) ? 4 : 1))) void conv3x3_kernel(
    const __bf16* __restrict__ X, const __bf16* __restrict__ Wt, __bf16* __restrict__ Y, Geo g,
    int ntn, int64_t ntm, const float* __restrict__ shift, float* __restrict__ partial,
    const __bf16* __restrict__ bnx, const float* __restrict__ bnvec) {
  constexpr bool STATS = EPI != 0;
  constexpr int NT = WM * WN * 64;
  constexpr int A_CH = BM * 8 / NT;               // 16-byte chunks per thread per A stage
  constexpr int WTN = BN / WN, WTM = BM / WM;
  constexpr int TN = WTN / 16, TM = WTM / 16;
  constexpr int B_CH = BN * 8 / NT;
  constexpr int LPS = A_CH + B_CH;                // glds per thread per stage
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(NS == 2 || NS == 3, "LDS ring: 2 slots (1 stage in flight, 2 workgroups per "
                                     "CU) or 3 slots (2 stages in flight)");
  __shared__ __attribute__((aligned(16))) __bf16 smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int wm = wid / WN, wn = wid % WN;
  const int t = remap(blockIdx.x, gridDim.x);
  const int nt = t % ntn;
  const int64_t stream = t / ntn, nstreams = gridDim.x / ntn;
  const int n0 = nt * BN;
  const int taps = g.ks * g.ks;
  const int csteps = g.C / BK, KT = (DG ? (1 + g.ph) * (1 + g.pw) : taps) * csteps;
  // (tap, channel step) of a K tile by shift for power-of-two steps (C = 64 / 128 / 256 ..)
  const bool cpow2 = (csteps & (csteps - 1)) == 0;
  const int cshift = __builtin_ctz((unsigned)csteps);
  const int64_t wrow = (int64_t)taps * g.C;       // filter row length
  const int sc = (tid & 7) ^ ((tid >> 3) & 7);    // swizzled source chunk of this thread

  uint64_t brow[B_CH];                            // filter rows of this thread
#pragma unroll
  for (int i = 0; i < B_CH; ++i)
    brow[i] = (uint64_t)(Wt + (int64_t)(n0 + i * (NT / 8) + (tid >> 3)) * wrow + sc * 8);
  const uint64_t zaddr = (uint64_t)(g_zero + (tid & 7) * 4);

  auto issue = [&](const RowInfo<A_CH>& ri, int kt, int buf) {
    int tap = cpow2 ? kt >> cshift : kt / csteps;
    const int c0 = (kt - tap * csteps) * BK;   // wave-uniform
    int64_t offa, offb;
    if constexpr (DG) {
      // class tap t: dy row + tR, column + tS; flipped-filter tap (ph ? 2 tR : 1, pw ? 2 tS : 1)
      const int tR = g.pw ? tap >> 1 : tap, tS = g.pw ? tap & 1 : 0;
      const int rr = g.ph ? 2 * tR : 1, ss = g.pw ? 2 * tS : 1;
      offa = (((int64_t)tR * g.Wo + tS) * g.C + c0) * 2;
      offb = ((int64_t)(rr * 3 + ss) * g.C + c0) * 2;
      tap = 2 * tR + tS;                     // validity bit
    } else {
      const int r = g.ks == 3 ? (tap * 11) >> 5 : tap / g.ks;     // tap < 9: (11 t) >> 5 = t / 3
      const int s = tap - r * g.ks;
      offa = (((int64_t)r * g.W + s) * g.C + c0) * 2;
      offb = ((int64_t)tap * g.C + c0) * 2;
    }
    __bf16* As = smem + buf * STAGE;
    __bf16* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const uint64_t a = ((ri.valid[i] >> tap) & 1u) ? ri.addr[i] + offa : zaddr;
      glds16((const void*)a, As + (i * NT + wid * 64) * 8);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) glds16((const void*)(brow[i] + offb), Bs + (i * NT + wid * 64) * 8);
  };

  const int gq = lane >> 4, rl = lane & 15;
  // EPI 2 reads its per-channel (mean, scale, bias) in the epilogue from the cache: held
  // in registers across the K loop they pushed the kernel past 2 waves per SIMD
  float sh[EPI == 1 ? TN : 1][4], s1[TN][4], s2[TN][4];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = n0 + wn * WTN + a * 16 + 4 * gq + r;
      if constexpr (EPI == 1) sh[a][r] = shift ? shift[col] : 0.f;
      s1[a][r] = 0.f;
      s2[a][r] = 0.f;
    }
  f32x4v acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};

  // Step j computes from ring slot j % NS while the loads of steps j+1 and j+2 are
  // in flight; one raw barrier per step, after a COUNTED vmcnt wait that retires only
  // step j's loads (loads retire in order, so "<= LPS outstanding" with step j+2's
  // LPS loads issued last means step j's — and j+1's predecessors — landed; epilogue
  // stores in between do not disturb the count), so the in-flight loads survive it.
  // Tiles are the outer loop so the accumulators stay in AGPRs through the K loop.
  int64_t mt = stream;
  if (mt < ntm) {
    RowInfo<A_CH> iri;
    row_info<A_CH, NT, DG>(g, X, mt * BM, tid, sc, iri);
    int64_t imt = mt;          // (tile, step) of the last issued stage
    int ikt = 0;
    int islot = 0;
    issue(iri, 0, 0);
    auto issue_next = [&]() -> bool {
      int k2 = ikt + 1;
      int64_t m2 = imt;
      if (k2 == KT) { k2 = 0; m2 += nstreams; }
      if (m2 >= ntm) return false;
      if (m2 != imt) row_info<A_CH, NT, DG>(g, X, m2 * BM, tid, sc, iri);
      islot = islot + 1 == NS ? 0 : islot + 1;
      issue(iri, k2, islot);
      imt = m2;
      ikt = k2;
      return true;
    };
    bool ahead = NS == 3 ? issue_next() : false;   // 3 slots: stage of step 1 in flight
    int slot = 0;
    while (true) {
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
      for (int kt = 0; kt < KT; ++kt) {
        if (NS == 3 && ahead) wait_vm<LPS>(); else wait_vm<0>();
        raw_barrier();          // this step's stage is visible to all; the oldest slot is free
        ahead = issue_next();
        const __bf16* As = smem + slot * STAGE;
        const __bf16* Bs = As + BM * BK;
#pragma unroll
        for (int kk = 0; kk < BK / 32; ++kk) {
          const int ch = kk * 4 + gq;
          bf16x8 wf[TN], af[TM];
#pragma unroll
          for (int a = 0; a < TN; ++a)
            wf[a] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * WTN + a * 16 + rl, ch));
#pragma unroll
          for (int b = 0; b < TM; ++b)
            af[b] = *reinterpret_cast<const bf16x8*>(As + swz(wm * WTM + b * 16 + rl, ch));
#pragma unroll
          for (int a = 0; a < TN; ++a)
#pragma unroll
            for (int b = 0; b < TM; ++b) acc[a][b] = mfma(wf[a], af[b], acc[a][b]);
        }
        slot = slot + 1 == NS ? 0 : slot + 1;
      }
      // tile done: store (+ statistics) while the next tile's first loads fly
      const int64_t m0 = mt * BM;
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        int64_t row = m0 + wm * WTM + b * 16 + rl;
        if (row < g.M) {
          if constexpr (DG) {          // class row -> dx pixel (n, 2 ci + ph, 2 cj + pw)
            const uint32_t hw = (uint32_t)(g.Ho * g.Wo), r32 = (uint32_t)row;
            const uint32_t n = r32 / hw, rem = r32 - n * hw;
            const uint32_t ci = rem / (uint32_t)g.Wo, cj = rem - ci * (uint32_t)g.Wo;
            row = ((int64_t)n * g.H + 2 * ci + g.ph) * g.W + 2 * cj + g.pw;
          }
#pragma unroll
          for (int a = 0; a < TN; ++a) {
            const f32x4v v = acc[a][b];
            const int col = n0 + wn * WTN + a * 16 + 4 * gq;
            if constexpr (EPI == 2) {
              const u32x2 xw = *reinterpret_cast<const u32x2*>(bnx + row * g.K + col);
              const float xv[4] = {__uint_as_float(xw[0] << 16), __uint_as_float(xw[0] & 0xffff0000u),
                                   __uint_as_float(xw[1] << 16), __uint_as_float(xw[1] & 0xffff0000u)};
              const float4 mu = *reinterpret_cast<const float4*>(bnvec + col);
              const float4 sc4 = *reinterpret_cast<const float4*>(bnvec + 2 * g.K + col);
              const float4 bi4 = *reinterpret_cast<const float4*>(bnvec + 3 * g.K + col);
              const float mus[4] = {mu.x, mu.y, mu.z, mu.w};
              const float scs[4] = {sc4.x, sc4.y, sc4.z, sc4.w};
              const float bis[4] = {bi4.x, bi4.y, bi4.z, bi4.w};
              float dv[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float d =
                    __builtin_fmaf(xv[r], scs[r], bis[r]) > 0.f ? round_bf16(v[r]) : 0.f;
                dv[r] = d;
                s1[a][r] += d;
                s2[a][r] += d * (xv[r] - mus[r]);
              }
              *reinterpret_cast<u32x2*>(Y + row * g.K + col) =
                  u32x2{cvt_pk_bf16(dv[0], dv[1]), cvt_pk_bf16(dv[2], dv[3])};
            } else {
              *reinterpret_cast<u32x2*>(Y + row * g.K + col) =
                  u32x2{cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3])};
            }
            if (EPI == 1) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float d = round_bf16(v[r]) - sh[a][r];
                s1[a][r] += d;
                s2[a][r] += d * d;
              }
            }
          }
        }
      }
      mt += nstreams;
      if (mt >= ntm) break;
    }
    wait_vm<0>();
    __syncthreads();
  }
  if (!STATS) return;
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[a][r] += __shfl_xor(s1[a][r], o, kWave);
        s2[a][r] += __shfl_xor(s2[a][r], o, kWave);
      }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);      // [2][WM][BN]
  if (rl == 0) {
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wn * WTN + a * 16 + 4 * gq + r;
        red[(0 * WM + wm) * BN + c] = s1[a][r];
        red[(1 * WM + wm) * BN + c] = s2[a][r];
      }
  }
  __syncthreads();
  if (stream >= ntm) return;
  for (int v = tid; v < 2 * BN; v += NT) {
    const int k = v / BN, c = v - k * BN;
    float acc_s = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) acc_s += red[(k * WM + w) * BN + c];
    partial[(stream * 2 + k) * g.K + n0 + c] = acc_s;
  }
}

// tile configs (8 waves): BN = 128 -> 256 x 128 (4 x 2 waves of 64 x 64); BN = 64 -> 256 x 64
// (4 x 2 waves of 64 x 32)
template <int BN, bool STATS>
struct Cfg;
template <bool STATS>
struct Cfg<128, STATS> {
  static constexpr int BM = 128, WM = 2, WN = 2, NS = 2;    // 64 KB: 2 workgroups per CU
};
template <bool STATS>
struct Cfg<64, STATS> {
  static constexpr int BM = 256, WM = 4, WN = 2, NS = 2;    // 80 KB: 2 workgroups per CU
};

template <int BN, bool STATS, int EPI = STATS ? 1 : 0>
static const void* kernel_ptr() {
  using C = Cfg<BN, STATS>;
  return (const void*)&conv3x3_kernel<C::BM, BN, C::WM, C::WN, EPI, C::NS>;
}

template <int BN, bool STATS>
static int64_t streams_for(int64_t ntm, int ntn) {
  static int per = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &v, kernel_ptr<BN, STATS>(), Cfg<BN, STATS>::WM * Cfg<BN, STATS>::WN * 64, 0) !=
            hipSuccess || v < 1)
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
  int64_t s = (int64_t)cus * per / ntn;
  const char* e = std::getenv("MIVOD_CONV_WAVES");   // tiles in flight per CU (A/B knob)
  if (e && std::atoi(e) > 0) s = (int64_t)cus * std::atoi(e) / ntn;
  s = std::max<int64_t>(1, std::min(s, ntm));
  return s;
}

}  // namespace conv
}  // namespace mv

static int conv_bn_of(int K) { return K % 128 == 0 ? 128 : 64; }

// Cout % 256 == 0 (ResNet-50 layers 3-4): the 256 x 256 glds pipeline (mv_gemm256.hip,
// AMODE 3) — decided by K alone so that mv_conv3x3_partials(M, K) matches the launch
static bool conv256_route(int K) {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_CONV256");
    return !(e && e[0] == '0');
  }();
  return on && K % 256 == 0 && K <= 2048;
}

int64_t mv_conv3x3_partials(int64_t M, int K) {
  using namespace mv::conv;
  if (conv256_route(K)) return mv_gemm256_partials(M, K);
  if (conv_bn_of(K) == 128)
    return streams_for<128, true>((M + Cfg<128, true>::BM - 1) / Cfg<128, true>::BM, K / 128);
  return streams_for<64, true>((M + Cfg<64, true>::BM - 1) / Cfg<64, true>::BM, K / 64);
}

bool mv_conv3x3(const void* x, const void* w, void* y, int N, int H, int W, int C, int K,
                int stride, const float* shift, float* partial, hipStream_t st,
                const void* bn_x, const float* bn_vec) {
  return mv_conv_nhwc(x, w, y, N, H, W, C, K, 3, stride, shift, partial, st, bn_x, bn_vec);
}

bool mv_conv_nhwc(const void* x, const void* w, void* y, int N, int H, int W, int C, int K, int ks,
                  int stride, const float* shift, float* partial, hipStream_t st,
                  const void* bn_x, const float* bn_vec, const float* in_scale,
                  const float* in_bias) {
  using namespace mv::conv;
  if (C % 64 != 0 || K % 64 != 0 || (stride != 1 && stride != 2) || (ks != 1 && ks != 3))
    return false;
  // row_info's 32-bit pixel divisions need N * H * W < 2^31
  if ((int64_t)N * H * W >= (int64_t(1) << 31)) return false;
  const bool bna = in_scale != nullptr;
  // 64 -> 64 channel 3x3 stride 1 (ResNet-50 layer1): the row-patch kernel (mv_conv64.hip)
  static const bool c64 = [] {
    const char* e = std::getenv("MIVOD_CONV64");
    return !(e && e[0] == '0');
  }();
  if (c64 && mv_conv64_supported(N, H, W, C, K, ks, stride)) {
    const int64_t M = (int64_t)N * H * W;
    int grid = partial ? (int)mv_conv3x3_partials(M, K) : 0;
    if (!partial) {
      int dev = 0, cus = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          cus < 1)
        cus = 256;
      grid = cus;
    }
    return mv_conv64(x, w, y, N, H, W, shift, partial, grid, st, bn_x, bn_vec, in_scale,
                     in_bias);
  }
  if (bna) return false;          // the input BN apply: the row-patch kernel only
  if (conv256_route(K))      // (a shape it cannot take is an error: the partial rows differ)
    return mv_conv256(x, w, y, N, H, W, C, K, ks, stride, shift, partial, bn_x, bn_vec, st);
  Geo g;
  g.ks = ks;
  g.H = H;
  g.W = W;
  g.C = C;
  g.K = K;
  g.st = stride;
  g.Ho = (H - 1) / stride + 1;   // (H + 2 (ks / 2) - ks) / stride + 1 for ks = 1, 3
  g.Wo = (W - 1) / stride + 1;
  g.M = (int64_t)N * g.Ho * g.Wo;
  const __bf16* X = (const __bf16*)x;
  const __bf16* Wt = (const __bf16*)w;
  __bf16* Y = (__bf16*)y;
  const __bf16* BX = (const __bf16*)bn_x;
  if (bn_x && !partial) return false;
#define MV_LAUNCH(BNV, ST)                                                                     \
  {                                                                                            \
    constexpr int BMV = Cfg<BNV, ST>::BM, WMV = Cfg<BNV, ST>::WM, WNV = Cfg<BNV, ST>::WN;      \
    constexpr int NSV = Cfg<BNV, ST>::NS;                                                      \
    const int64_t ntm = (g.M + BMV - 1) / BMV;                                                 \
    const int ntn = K / BNV;                                                                   \
    const int64_t ns = streams_for<BNV, ST>(ntm, ntn);                                         \
    if (BX)                                                                                    \
      hipLaunchKernelGGL((conv3x3_kernel<BMV, BNV, WMV, WNV, 2, NSV>), dim3((unsigned)(ns * ntn)),\
                         dim3(WMV * WNV * 64), 0, st, X, Wt, Y, g, ntn, ntm, shift, partial, BX, \
                         bn_vec);                                                              \
    else                                                                                       \
      hipLaunchKernelGGL((conv3x3_kernel<BMV, BNV, WMV, WNV, ST ? 1 : 0, NSV>),                  \
                         dim3((unsigned)(ns * ntn)), dim3(WMV * WNV * 64), 0, st, X, Wt, Y, g,   \
                         ntn, ntm, shift, partial, BX, bn_vec);                                \
  }
  if (conv_bn_of(K) == 128) {
    if (partial) MV_LAUNCH(128, true) else MV_LAUNCH(128, false)
  } else {
    if (partial) MV_LAUNCH(64, true) else MV_LAUNCH(64, false)
  }
#undef MV_LAUNCH
  return true;
}

// Data-gradient filters of many convs in ONE launch: each w [K][ks][ks][C] (a channels_last
// [K, C, ks, ks] filter) -> wt [C][ks][ks][K] with the taps rotated 180 degrees (the
// channels_last [C, K, ks, ks] filter of dX = conv(dY, wt); for ks = 1 plain W^T).  A block
// transposes one 64 (k) x 64 (c) tile of one tap through LDS (both sides coalesced); the
// block table (tensor, tap, k0, c0) is built on the host.  Replaces a flip + layout copy
// (or a transpose copy) per conv per step: ~55 small PyTorch launches at ResNet-50.
namespace mv {
namespace conv {
struct TfTensor {
  const __bf16* src;
  __bf16* dst;
  int K, C, ks;
};
struct TfBlock {
  int t, tap, k0, c0;
};
__global__ __launch_bounds__(256) void transpose_filters_kernel(const TfTensor* __restrict__ ts,
                                                                const TfBlock* __restrict__ bl) {
  __shared__ __bf16 tile[64][66];
  const TfBlock b = bl[blockIdx.x];
  const TfTensor tt = ts[b.t];
  const int ks = tt.ks, taps = ks * ks;
  const int r = b.tap / ks, s = b.tap - r * ks;
  const int ftap = (ks - 1 - r) * ks + (ks - 1 - s);   // source tap (rotated)
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {                   // read rows k, c contiguous
    const int k = b.k0 + i, c = b.c0 + tx;
    tile[i][tx] = (k < tt.K && c < tt.C) ? tt.src[((int64_t)k * taps + ftap) * tt.C + c]
                                         : (__bf16)0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {                   // write rows c, k contiguous
    const int c = b.c0 + i, k = b.k0 + tx;
    if (c < tt.C && k < tt.K) tt.dst[((int64_t)c * taps + b.tap) * tt.K + k] = tile[tx][i];
  }
}
}  // namespace conv
}  // namespace mv

int64_t mv_transpose_filters_blocks(const int* K, const int* C, const int* ks, int n) {
  int64_t nb = 0;
  for (int i = 0; i < n; ++i)
    nb += (int64_t)ks[i] * ks[i] * ((K[i] + 63) / 64) * ((C[i] + 63) / 64);
  return nb;
}

// table: device memory of n TfTensor (32 bytes each) followed by the block list (16 bytes
// each), written by the caller from mv_transpose_filters_table's host image
void mv_transpose_filters_table(const void* const* src, void* const* dst, const int* K,
                                const int* C, const int* ks, int n, void* host_image) {
  using namespace mv::conv;
  TfTensor* ts = reinterpret_cast<TfTensor*>(host_image);
  TfBlock* bl = reinterpret_cast<TfBlock*>(ts + n);
  int64_t j = 0;
  for (int i = 0; i < n; ++i) {
    ts[i] = TfTensor{(const __bf16*)src[i], (__bf16*)dst[i], K[i], C[i], ks[i]};
    for (int tap = 0; tap < ks[i] * ks[i]; ++tap)
      for (int k0 = 0; k0 < K[i]; k0 += 64)
        for (int c0 = 0; c0 < C[i]; c0 += 64) bl[j++] = TfBlock{i, tap, k0, c0};
  }
}

int64_t mv_transpose_filters_table_bytes(int n, int64_t blocks) {
  return (int64_t)n * (int64_t)sizeof(mv::conv::TfTensor) + blocks * (int64_t)sizeof(mv::conv::TfBlock);
}

void mv_transpose_filters(const void* table, int n, int64_t blocks, hipStream_t st) {
  using namespace mv::conv;
  const TfTensor* ts = reinterpret_cast<const TfTensor*>(table);
  const TfBlock* bl = reinterpret_cast<const TfBlock*>(ts + n);
  hipLaunchKernelGGL(transpose_filters_kernel, dim3((unsigned)blocks), dim3(256), 0, st, ts, bl);
}

// Stride-2 3x3 (pad 1) data gradient: dx [Nb, H, W, C] from dy [Nb, H/2, W/2, K] and the
// transposed flipped filter wt [C][3][3][K]; four parity-class launches (DG), every dx pixel
// written once.  C % 256 == 0 goes to mv_gemm256.hip's AMODE 4, else conv3x3_kernel.
bool mv_conv3x3_s2_dgrad_supported(int Nb, int H, int W, int C, int K) {
  if (mv_dgrad256_s2_supported(Nb, H, W, C, K)) return true;
  return Nb > 0 && H >= 2 && W >= 2 && !(H & 1) && !(W & 1) && C % 64 == 0 && K % 64 == 0 &&
         C > 0 && K > 0 && (int64_t)Nb * H * W * std::max(C, K) < (int64_t(1) << 40) &&
         (int64_t)Nb * H * W < (int64_t(1) << 31);
}

bool mv_conv3x3_s2_dgrad(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int C,
                         int K, hipStream_t st) {
  using namespace mv::conv;
  if (mv_dgrad256_s2_supported(Nb, H, W, C, K))
    return mv_dgrad256_s2(dy, wt, dx, Nb, H, W, C, K, st);
  if (!mv_conv3x3_s2_dgrad_supported(Nb, H, W, C, K)) return false;
  Geo g;
  g.ks = 3;
  g.st = 2;
  g.H = H;
  g.W = W;
  g.C = K;             // gathered (dy) channels
  g.K = C;             // output (dx) channels
  g.Ho = H / 2;
  g.Wo = W / 2;
  g.M = (int64_t)Nb * g.Ho * g.Wo;
  const __bf16* X = (const __bf16*)dy;
  const __bf16* Wt = (const __bf16*)wt;
  __bf16* Y = (__bf16*)dx;
#define MV_LAUNCH_DG(BNV)                                                                      \
  {                                                                                            \
    constexpr int BMV = Cfg<BNV, false>::BM, WMV = Cfg<BNV, false>::WM;                        \
    constexpr int WNV = Cfg<BNV, false>::WN, NSV = Cfg<BNV, false>::NS;                        \
    const int64_t ntm = (g.M + BMV - 1) / BMV;                                                 \
    const int ntn = C / BNV;                                                                   \
    const int64_t ns = streams_for<BNV, false>(ntm, ntn);                                      \
    hipLaunchKernelGGL((conv3x3_kernel<BMV, BNV, WMV, WNV, 0, NSV, true>),                      \
                       dim3((unsigned)(ns * ntn)), dim3(WMV * WNV * 64), 0, st, X, Wt, Y, g, ntn, \
                       ntm, nullptr, nullptr, nullptr, nullptr);                               \
  }
  for (int c = 3; c >= 0; --c) {      // the 4-tap class first
    g.ph = c >> 1;
    g.pw = c & 1;
    if (conv_bn_of(C) == 128) MV_LAUNCH_DG(128) else MV_LAUNCH_DG(64)
  }
#undef MV_LAUNCH_DG
  return true;
}

// ===========================================================================
// 3x3 weight gradient (pad 1, stride 1 / 2):
//   dW[k][tap][c] = sum_m dy[m][k] . X[pixel(m) + tap][c]   (filter in [K][3][3][C] order)
// A GEMM with the reduction over the output pixels m (N*Ho*Wo rows): a workgroup owns
// one 64(k) x 64(c) block for ALL 9 taps (accumulators resident for the whole kernel)
// and a contiguous range of 32-row m chunks; per chunk it stages the dy tile and the 9
// tap-shifted X tiles (gathered rows, zero page at the image border) with
// global_load_lds into a 2-slot ring (two workgroups per CU).  Both MFMA operands
// are k(=m)-major, so they are read with gfx950's transposed LDS read
// (ds_read_b64_tr_b16).  Each workgroup writes an fp32 partial [9][64][64] block; a
// fixed-order reduce kernel sums the m splits and writes the bf16 filter gradient.
// ===========================================================================
namespace mv {
namespace conv {

typedef short s16x4 __attribute__((ext_vector_type(4)));

// [32][64] bf16 stage tiles (128-B rows) with a row-dependent 16-byte-chunk XOR: slot
// (r, ch) holds chunk ch ^ wswz(r).  A transposed read touches 4 rows per 16-lane group
// and rows 8 apart in the other group of its 32-lane half; rows 2 apart share a bank
// window on 128-B rows, so {r, r+2, r+8, r+10} get chunk offsets {0, 2, 4, 6} (XOR by
// even values keeps a 32-byte column pair together): conflict-free instead of 4-way.
__device__ __forceinline__ int wswz(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ s16x4 tr4(const __bf16* base, int r0, int col0, int c) {
  const int r = r0 + (c >> 2), e = col0 + 4 * (c & 3);
  const __bf16* p = base + r * 64 + (((e >> 3) ^ wswz(r)) << 3) + (e & 7);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}
// lane c of each 16-lane group: rows ra..ra+3, rb..rb+3 of column col0 + c
__device__ __forceinline__ bf16x8 tr8(const __bf16* base, int ra, int rb, int col0, int c) {
  const s16x4 a = tr4(base, ra, col0, c);
  const s16x4 b = tr4(base, rb, col0, c);
  bf16x8 o;
  short* q = reinterpret_cast<short*>(&o);
  q[0] = a[0]; q[1] = a[1]; q[2] = a[2]; q[3] = a[3];
  q[4] = b[0]; q[5] = b[1]; q[6] = b[2]; q[7] = b[3];
  return o;
}

constexpr int WG_NT = 256;                 // 4 waves, wave w = c tile w, all 4 k tiles
constexpr int WG_ROWS = 32;                // m rows per stage (one MFMA k step)
constexpr int WG_TILE = WG_ROWS * 64;      // elements of one [32][64] tile
constexpr int WG_STAGE = 10 * WG_TILE;     // dy + 9 taps
constexpr int WG_NS = 2;                   // 80 KB of LDS: two workgroups (8 waves) per CU
constexpr int WG_LPS = 10 * 256 / WG_NT;   // glds per thread per stage (10)

__global__ __launch_bounds__(WG_NT) void wgrad3x3_kernel(const __bf16* __restrict__ X,
                                                          const __bf16* __restrict__ DY,
                                                          float* __restrict__ partial, Geo g,
                                                          int nkc, int msplit, int64_t nchunks) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[WG_NS * WG_STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = remap(blockIdx.x, gridDim.x);
  const int kc = t % nkc, ms = t / nkc;
  const int cblocks = g.C / 64;
  const int k0 = (kc / cblocks) * 64, c0 = (kc % cblocks) * 64;
  const int64_t per = (nchunks + msplit - 1) / msplit;
  const int64_t ch0 = ms * per;
  const int64_t ch1 = ch0 + per < nchunks ? ch0 + per : nchunks;

  // staging role: row tid >> 3, 16-byte chunk tid & 7 of all 10 tiles of a stage.  The
  // row's output pixel advances by 32 per stage: (n, ho, wo) is carried incrementally
  // (no per-stage division)
  const int srow = tid >> 3, sch = (tid & 7) ^ wswz(tid >> 3);   // swizzled source chunk
  const uint64_t zaddr = (uint64_t)(g_zero + (tid & 7) * 4);
  int64_t pm = ch0 * WG_ROWS + srow;           // this thread's row of the next issued stage
  int pn = 0, pho = 0, pwo = 0;
  {
    const int64_t hw = (int64_t)g.Ho * g.Wo;
    const int64_t mm = pm < g.M ? pm : 0;
    pn = (int)(mm / hw);
    const int rem = (int)(mm - (int64_t)pn * hw);
    pho = rem / g.Wo;
    pwo = rem - pho * g.Wo;
  }
  auto issue = [&](int slot) {
    const bool in = pm < g.M;
    const int hi0 = pho * g.st - 1, wi0 = pwo * g.st - 1;
    const int64_t xrow = (((int64_t)pn * g.H + hi0) * g.W + wi0) * g.C + c0 + sch * 8;
    __bf16* st = smem + slot * WG_STAGE;
    glds16(in ? (const void*)(DY + pm * g.K + k0 + sch * 8) : (const void*)zaddr,
           st + (wid * 64) * 8);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap % 3;
      const bool ok = in && (unsigned)(hi0 + r) < (unsigned)g.H && (unsigned)(wi0 + s) < (unsigned)g.W;
      const uint64_t a = ok ? (uint64_t)(X + xrow + ((int64_t)r * g.W + s) * g.C) : zaddr;
      glds16((const void*)a, st + ((1 + tap) * WG_NT + wid * 64) * 8);
    }
    // advance this thread's row by one stage (32 pixels)
    pm += WG_ROWS;
    pwo += WG_ROWS;
    while (pwo >= g.Wo) {
      pwo -= g.Wo;
      if (++pho == g.Ho) {
        pho = 0;
        ++pn;
      }
    }
  };

  const int ct = wid;
  const int gq = lane >> 4, cl = lane & 15;
  f32x4v acc[9][4];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[tp][u] = f32x4v{0.f, 0.f, 0.f, 0.f};

  if (ch0 < ch1) {
    // 2-slot ring: stage j+1 is issued right after the barrier that retires stage j
    // (and frees slot (j+1) % 2) and lands while stage j is multiplied
    issue(0);
    int slot = 0;
    for (int64_t chk = ch0; chk < ch1; ++chk) {
      wait_vm<0>();
      raw_barrier();
      if (chk + 1 < ch1) issue(slot ^ 1);
      const __bf16* st = smem + slot * WG_STAGE;
      bf16x8 af[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) af[u] = tr8(st, 8 * gq, 8 * gq + 4, 16 * u, cl);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const bf16x8 bfr = tr8(st + (1 + tp) * WG_TILE, 8 * gq, 8 * gq + 4, 16 * ct, cl);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[tp][u] = mfma(af[u], bfr, acc[tp][u]);
      }
      slot ^= 1;
    }
    wait_vm<0>();
  }
  // partial[ms][tap][k][c] (fp32, this block's 64 x 64 window); every block writes its
  // window even with no chunks (zeros) so the reduce never reads garbage
  float* pb = partial + (int64_t)ms * 9 * g.K * g.C;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + 16 * u + 4 * gq + r, c = c0 + 16 * ct + cl;
        pb[((int64_t)tp * g.K + k) * g.C + c] = acc[tp][u][r];
      }
}

// dw[k][tap][c] (bf16) = sum over the m splits, fixed order
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ partial,
                                                            __bf16* __restrict__ dw, int K, int C,
                                                            int msplit) {
  const int64_t n = (int64_t)9 * K * C;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;    // index in [tap][k][c]
  if (i >= n) return;
  float s = 0.f;
  for (int p = 0; p < msplit; ++p) s += partial[(int64_t)p * n + i];
  const int c = (int)(i % C);
  const int64_t tk = i / C;
  const int k = (int)(tk % K), tap = (int)(tk / K);
  dw[((int64_t)k * 9 + tap) * C + c] = (__bf16)s;
}

}  // namespace conv
}  // namespace mv

namespace mv {
namespace conv {
template <int PS, typename TO>
__global__ void wgrad1x1_reduce_kernel(const float* __restrict__ partial, TO* __restrict__ dw,
                                       int64_t E, int P);
}  // namespace conv
}  // namespace mv

static int wgrad_msplit(int64_t nchunks, int nkc) {
  const char* e = std::getenv("MIVOD_WGRAD_BLOCKS");       // workgroups per launch (A/B)
  const int64_t target = e && std::atoi(e) > 0 ? std::atoi(e) : 512;
  int64_t ms = target / nkc;
  if (ms < 1) ms = 1;
  if (ms > nchunks) ms = nchunks;
  return (int)ms;
}

// C, K % 256 == 0 (ResNet-50 layers 3-4): the 256 x 256 pipeline (mv_gemm256.hip
// wgrad256_kernel<9>: one tap's 256 x 256 (k, c) block per tile, X rows gathered)
static bool w256_3x3_on() {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_WGRAD256_3X3");
    return !(e && e[0] == '0');
  }();
  return on;
}

int64_t mv_wgrad3x3_workspace(int64_t M, int K, int C) {
  const int nkc = (K / 64) * (C / 64);
  const int64_t nchunks = (M + 31) / 32;
  int64_t n = (int64_t)wgrad_msplit(nchunks, nkc) * 9 * K * C;
  if (C % 256 == 0 && K % 256 == 0) {
    const int64_t n256 = mv_wgrad256_splits(M, 9 * C, K) * 9 * K * C;
    n = n256 > n ? n256 : n;
  }
  return n;
}

bool mv_wgrad3x3(const void* x, const void* dy, void* dw, float* work, int N, int H, int W, int C,
                 int K, int stride, hipStream_t st, const float* in_scale, const float* in_bias) {
  using namespace mv::conv;
  if (C % 64 != 0 || K % 64 != 0 || (stride != 1 && stride != 2)) return false;
  const bool bna = in_scale != nullptr;
  if (bna && !mv_wgrad64_supported(N, H, W, C, K, stride)) return false;
  Geo g;
  g.H = H;
  g.W = W;
  g.C = C;
  g.K = K;
  g.st = stride;
  g.Ho = (H - 1) / stride + 1;
  g.Wo = (W - 1) / stride + 1;
  g.M = (int64_t)N * g.Ho * g.Wo;
  const int nkc = (K / 64) * (C / 64);
  const int64_t nchunks = (g.M + 31) / 32;
  const int ms = wgrad_msplit(nchunks, nkc);
  if (!bna && w256_3x3_on() && mv_wgrad256_3x3_supported(N, H, W, C, K, stride) &&
      mv_wgrad256_3x3(x, dy, work, N, H, W, C, K, stride, st)) {
    const int P = (int)mv_wgrad256_3x3_splits(N, H, W, C, K, stride);
    const int64_t E = (int64_t)9 * K * C;       // [K][9][C] = the channels_last filter
    hipLaunchKernelGGL((wgrad1x1_reduce_kernel<16, __bf16>),
                       dim3((unsigned)((E / 4 + 256 / 16 - 1) / (256 / 16))), dim3(256), 0, st,
                       (const float*)work, (__bf16*)dw, E, P);
    return true;
  }
  static const bool w64 = [] {
    const char* e = std::getenv("MIVOD_WGRAD64");
    return !(e && e[0] == '0');
  }();
  if ((w64 || bna) && mv_wgrad64_supported(N, H, W, C, K, stride)) {
    // 64 -> 64 stride 1: the row-patch kernel (mv_conv64.hip), one persistent 136-KB-LDS
    // workgroup per CU (<= ms partial rows, so the workspace above is large enough)
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
          n < 1)
        n = 256;
      return n;
    }();
    const int grid = ms < cus ? ms : cus;
    mv_wgrad64(x, dy, work, grid, N, H, W, st, in_scale, in_bias);
    const int64_t n = (int64_t)9 * K * C;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       (const float*)work, (__bf16*)dw, K, C, grid);
    return true;
  }
  hipLaunchKernelGGL(wgrad3x3_kernel, dim3((unsigned)(nkc * ms)), dim3(WG_NT), 0, st,
                     (const __bf16*)x, (const __bf16*)dy, work, g, nkc, ms, nchunks);
  const int64_t n = (int64_t)9 * K * C;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (const float*)work, (__bf16*)dw, K, C, ms);
  return true;
}

// ===========================================================================
// 1x1 weight gradient (pad 0, stride 1 / 2):  dW[k][c] = sum_m dy[m][k] . X[pix(m)][c]
// (pix(m) = m at stride 1; the strided input pixel of output pixel m at stride 2).
// A dy^T . X GEMM reduced over the N*Ho*Wo output pixels: each wave owns a 64(k) x
// 64(c) accumulator block; a workgroup's 4 waves are laid out WK x WC over a
// (64 WK) x (64 WC) output tile and WS ways over the m rows of a stage (WS > 1 only for
// the 64-channel tiles, so every workgroup still runs 4 waves), and a workgroup walks
// a contiguous range of stages.  Staging as wgrad3x3: per stage WS x (WK + WC) [32][64]
// row-major sub-tiles via global_load_lds (one 16-B load per thread per sub-tile,
// XOR-swizzled chunk), an NS-slot ring with counted vmcnt waits, both operands read
// with ds_read_b64_tr_b16.  fp32 partials [msplit * WS][K][C] + a fixed-order reduce.
// ===========================================================================
namespace mv {
namespace conv {

template <int WK, int WC, int WS, int ST, int NS, int FK = 1>
__global__ __launch_bounds__(WK * WC * WS * 64)
__attribute__((amdgpu_waves_per_eu(FK == 2 ? 2 : 1))) void wgrad1x1_kernel(
    const __bf16* __restrict__ X, const __bf16* __restrict__ DY, float* __restrict__ partial,
    Geo g, int nkc, int msplit, int64_t nchunks) {
  constexpr int NW = WK * WC * WS;
  static_assert(NW == 4 || NW == 8, "four or eight waves per workgroup");
  constexpr int KS = FK * WK;                  // dy sub-tiles (64 k each) per m slice
  constexpr int SUB = KS + WC;                 // sub-tiles per m slice
  constexpr int NSUB = WS * SUB;               // [32][64] sub-tiles per stage
  constexpr int HPW = NW / 4;                  // 256-thread groups (one sub-tile each)
  static_assert(NSUB % HPW == 0, "sub-tiles split evenly over the thread groups");
  constexpr int LPS = NSUB / HPW;              // glds per thread per stage
  constexpr int ROWS = 32 * WS;                // m rows per stage
  constexpr int STAGE = NSUB * WG_TILE;
  __shared__ __attribute__((aligned(16))) __bf16 smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int t = remap(blockIdx.x, gridDim.x);
  const int kc = t % nkc, ms = t / nkc;
  const int cblocks = g.C / (64 * WC);
  const int k0 = (kc / cblocks) * (64 * KS), c0 = (kc % cblocks) * (64 * WC);
  const int64_t per = (nchunks + msplit - 1) / msplit;
  const int64_t ch0 = ms * per;
  const int64_t ch1 = ch0 + per < nchunks ? ch0 + per : nchunks;

  // staging role: thread group h = tid >> 8 loads sub-tiles h, h + HPW, ...; within a
  // sub-tile, row l >> 3 and (swizzled) 16-byte chunk of l = tid & 255
  const int hg = HPW == 1 ? 0 : tid >> 8, l = tid & 255;
  const int srow = l >> 3, sch = (l & 7) ^ wswz(l >> 3);
  const uint64_t zaddr = (uint64_t)(g_zero + (l & 7) * 4);
  const uint32_t hw = (uint32_t)(g.Ho * g.Wo);
  auto issue = [&](int64_t chk, int slot) {
    __bf16* stg = smem + slot * STAGE + (l - lane) * 8;     // + this wave's 1 KB of a sub-tile
    int64_t mrow[WS], xrow[WS];
#pragma unroll
    for (int ws = 0; ws < WS; ++ws) {
      const int64_t m = chk * ROWS + ws * 32 + srow;
      mrow[ws] = m;
      xrow[ws] = m;
      if (ST == 2 && m < g.M) {
        const uint32_t mm = (uint32_t)m, n = mm / hw, rem = mm - n * hw;
        const uint32_t ho = rem / (uint32_t)g.Wo, wo = rem - ho * (uint32_t)g.Wo;
        xrow[ws] = ((int64_t)n * g.H + 2 * ho) * g.W + 2 * wo;
      }
    }
#pragma unroll
    for (int i = 0; i < LPS; ++i) {
      const int j = i * HPW + hg;                 // sub-tile (thread-group uniform)
      const int ws = WS == 1 ? 0 : j / SUB, r = j % SUB;
      const bool in = mrow[ws] < g.M;
      const int kk = k0 + r * 64;                 // sub-tile uniform: one source per sub-tile
      const void* src =
          r >= KS ? (const void*)(X + xrow[ws] * g.C + c0 + (r - KS) * 64 + sch * 8)
          : kk < g.k1 ? (const void*)(DY + mrow[ws] * g.k1 + kk + sch * 8)
                      : (const void*)(g.dy2 + (g.dy2x ? xrow[ws] : mrow[ws]) * (g.K - g.k1) +
                                      (kk - g.k1) + sch * 8);
      glds16(in ? src : (const void*)zaddr, stg + j * WG_TILE);
    }
  };

  // wave role: m slice wsw, k block wkw, c block wcw
  const int wcw = wid % WC, wkw = (wid / WC) % WK, wsw = wid / (WC * WK);
  const int gq = lane >> 4, cl = lane & 15;
  f32x4v acc[4 * FK][4];
#pragma unroll
  for (int u = 0; u < 4 * FK; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) acc[u][v] = f32x4v{0.f, 0.f, 0.f, 0.f};

  if (ch0 < ch1) {
    // lookahead NS - 1 stages: stage chk + NS - 1 is issued right after the barrier that
    // retires stage chk - 1 (the slot it reuses)
#pragma unroll
    for (int p = 0; p < NS - 1; ++p)
      if (ch0 + p < ch1) issue(ch0 + p, p);
    int slot = 0;
    for (int64_t chk = ch0; chk < ch1; ++chk) {
      if (NS == 3 && chk + 1 < ch1)
        wait_vm<LPS>();
      else
        wait_vm<0>();
      raw_barrier();
      if (chk + NS - 1 < ch1) issue(chk + NS - 1, slot == 0 ? NS - 1 : slot - 1);
      const __bf16* st = smem + slot * STAGE;
      const __bf16* ta = st + (wsw * SUB + wkw * FK) * WG_TILE;
      const __bf16* tb = st + (wsw * SUB + KS + wcw) * WG_TILE;
      bf16x8 af[4 * FK], bfr[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) bfr[v] = tr8(tb, 8 * gq, 8 * gq + 4, 16 * v, cl);
#pragma unroll
      for (int u = 0; u < 4 * FK; ++u)
        af[u] = tr8(ta + (u >> 2) * WG_TILE, 8 * gq, 8 * gq + 4, 16 * (u & 3), cl);
#pragma unroll
      for (int u = 0; u < 4 * FK; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = mfma(af[u], bfr[v], acc[u][v]);
      slot = slot == NS - 1 ? 0 : slot + 1;
    }
    wait_vm<0>();
  }
  // partial[ms * WS + wsw][k][c]; written even with no chunks (zeros)
  float* pb = partial + ((int64_t)ms * WS + wsw) * g.K * g.C;
#pragma unroll
  for (int u = 0; u < 4 * FK; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = k0 + wkw * FK * 64 + 16 * u + 4 * gq + r, c = c0 + wcw * 64 + 16 * v + cl;
        pb[(int64_t)k * g.C + c] = acc[u][v][r];
      }
}

// dw[e] (bf16) = sum_p partial[p][e], fixed order: PS lanes split the P slices, then one
// lane sums the PS lane totals in lane order
template <int PS, typename TO>
__global__ __launch_bounds__(256) void wgrad1x1_reduce_kernel(const float* __restrict__ partial,
                                                               TO* __restrict__ dw, int64_t E,
                                                               int P) {
  constexpr int COLS = 256 / PS;
  __shared__ float4 red[PS][COLS];
  const int q = threadIdx.x % COLS, p = threadIdx.x / COLS;
  const int64_t i4 = (int64_t)blockIdx.x * COLS + q;
  const bool ok = i4 * 4 < E;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok)
    for (int pp = p; pp < P; pp += PS) {
      const float4 v = reinterpret_cast<const float4*>(partial + (int64_t)pp * E)[i4];
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
  red[p][q] = s;
  __syncthreads();
  if (p == 0 && ok) {
    float4 a = red[0][q];
    for (int j = 1; j < PS; ++j) {
      const float4 b = red[j][q];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
    }
    TO* o = dw + i4 * 4;
    o[0] = (TO)a.x;
    o[1] = (TO)a.y;
    o[2] = (TO)a.z;
    o[3] = (TO)a.w;
  }
}

}  // namespace conv
}  // namespace mv

namespace {
struct W1Cfg {
  int wk, wc, ws, ns, fk = 1;
};
// tile layout per shape (scripts/micro_wgrad1x1.py sweeps): 128x128 tiles on a 2-slot ring
// (4 workgroups per CU) once there are >= 8 tiles, else a 3-slot ring (3 per CU) — fewer
// tiles mean more m splits and the 64 MB of partials of a full grid start to show;
// 64-channel shapes split the m rows of a stage over the waves
W1Cfg w1_cfg(int K, int C) {
  const char* fk = std::getenv("MIVOD_WGRAD1_FK");
  if (fk && std::atoi(fk) == 2 && K % 256 == 0 && C % 128 == 0) return {2, 2, 1, 3, 2};
  const char* wv = std::getenv("MIVOD_WGRAD1_WAVES");
  if (wv && std::atoi(wv) == 8) {
    if (K % 256 == 0 && C % 128 == 0) return {4, 2, 1, 3};
    if (K % 128 == 0 && C % 256 == 0) return {2, 4, 1, 3};
  }
  if (K % 128 == 0 && C % 128 == 0) {
    const char* e = std::getenv("MIVOD_WGRAD1_NS");     // ring depth A/B for the 128x128 tile
    const int ntiles = (K / 128) * (C / 128);
    const int ns = e && std::atoi(e) > 0 ? std::atoi(e) : (ntiles >= 8 ? 2 : 3);
    return {2, 2, 1, ns == 2 ? 2 : 3};
  }
  if (K % 128 == 0) return {2, 1, 2, 2};
  if (C % 128 == 0) return {1, 2, 2, 2};
  return {1, 1, 4, 2};
}
int w1_msplit(int64_t nchunks, int ntiles, const W1Cfg& c) {
  const char* e = std::getenv("MIVOD_WGRAD1_BLOCKS");
  const int nw = c.wk * c.wc * c.ws;
  const int64_t target = e && std::atoi(e) > 0 ? std::atoi(e)
                         : (nw == 8 || c.fk == 2) ? 512
                         : (c.ns == 3 ? 768 : (c.wk == 2 && c.wc == 2 ? 1024 : 512));
  int64_t ms = target / ntiles;
  if (ms < 1) ms = 1;
  if (ms > nchunks) ms = nchunks;
  return (int)ms;
}
}  // namespace

// stride-1 shapes with C, K (and the dual split k1) multiples of 256 run on the 256 x 256
// pipeline (mv_gemm256.hip wgrad256_kernel)
static bool w256_on(int64_t M, int C, int K, int k1, int stride) {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_WGRAD256");
    return !(e && e[0] == '0');
  }();
  return on && stride == 1 && mv_wgrad256_supported(M, C, K, k1);
}

int64_t mv_wgrad1x1_workspace(int64_t M, int K, int C) {
  if (w256_on(M, C, K, K, 1)) {
    // the dual (k1 < K) call shares the shape test; size for whichever runs
    const int64_t w256 = mv_wgrad256_splits(M, C, K) * (int64_t)K * C;
    const W1Cfg c = w1_cfg(K, C);
    const int nt = (K / (64 * c.wk * c.fk)) * (C / (64 * c.wc));
    const int64_t old = (int64_t)w1_msplit((M + 32 * c.ws - 1) / (32 * c.ws), nt, c) * c.ws * K * C;
    return w256 > old ? w256 : old;
  }
  const W1Cfg c = w1_cfg(K, C);
  const int ntiles = (K / (64 * c.wk * c.fk)) * (C / (64 * c.wc));
  const int64_t nchunks = (M + 32 * c.ws - 1) / (32 * c.ws);
  return (int64_t)w1_msplit(nchunks, ntiles, c) * c.ws * K * C;
}

bool mv_wgrad1x1(const void* x, const void* dy, void* dw, float* work, int N, int H, int W, int C,
                 int K, int stride, hipStream_t st, bool dw_fp32, const void* dy2, int k1,
                 bool dy2_gather) {
  using namespace mv::conv;
  if (C % 64 != 0 || K % 64 != 0 || (stride != 1 && stride != 2)) return false;
  if (dy2_gather && (!dy2 || stride == 1)) return false;
  Geo g;
  g.dy2 = (const __bf16*)dy2;
  g.k1 = dy2 ? k1 : K;
  g.dy2x = dy2_gather ? 1 : 0;
  if (dy2) {     // each staged k block must come from one source
    const W1Cfg c = w1_cfg(K, C);
    if (k1 <= 0 || k1 >= K || k1 % (64 * c.wk * c.fk) != 0) return false;
  }
  g.H = H;
  g.W = W;
  g.C = C;
  g.K = K;
  g.st = stride;
  g.ks = 1;
  g.Ho = (H - 1) / stride + 1;
  g.Wo = (W - 1) / stride + 1;
  g.M = (int64_t)N * g.Ho * g.Wo;
  if (stride == 2 && g.M >= (int64_t(1) << 32)) return false;
  const W1Cfg c = w1_cfg(K, C);
  const int ntiles = (K / (64 * c.wk * c.fk)) * (C / (64 * c.wc));
  const int64_t nchunks = (g.M + 32 * c.ws - 1) / (32 * c.ws);
  int ms = w1_msplit(nchunks, ntiles, c);
  const dim3 grid((unsigned)(ntiles * ms)), blk((unsigned)(64 * c.wk * c.wc * c.ws));
  bool w256 = false;
  if (w256_on(g.M, C, K, g.k1, stride)) {
    w256 = mv_wgrad256(x, dy, dy2, work, g.M, C, K, g.k1, st);
    if (w256) ms = (int)mv_wgrad256_splits(g.M, C, K);
  }
  const __bf16 *xp = (const __bf16*)x, *dp = (const __bf16*)dy;
#define MV_W1F(WKV, WCV, WSV, NSV, FKV)                                                       \
  if (stride == 1)                                                                           \
    hipLaunchKernelGGL((wgrad1x1_kernel<WKV, WCV, WSV, 1, NSV, FKV>), grid, blk, 0, st, xp, dp,  \
                       work, g, ntiles, ms, nchunks);                                        \
  else                                                                                       \
    hipLaunchKernelGGL((wgrad1x1_kernel<WKV, WCV, WSV, 2, NSV, FKV>), grid, blk, 0, st, xp, dp,  \
                       work, g, ntiles, ms, nchunks);
#define MV_W1(WKV, WCV, WSV, NSV) MV_W1F(WKV, WCV, WSV, NSV, 1)
  if (w256) {
  } else if (c.fk == 2) {
    MV_W1F(2, 2, 1, 3, 2)
  } else if (c.wk == 4) {
    MV_W1(4, 2, 1, 3)
  } else if (c.wc == 4) {
    MV_W1(2, 4, 1, 3)
  } else if (c.wk == 2 && c.wc == 2) {
    if (c.ns == 3) {
      MV_W1(2, 2, 1, 3)
    } else {
      MV_W1(2, 2, 1, 2)
    }
  } else if (c.wk == 2) {
    MV_W1(2, 1, 2, 2)
  } else if (c.wc == 2) {
    MV_W1(1, 2, 2, 2)
  } else {
    MV_W1(1, 1, 4, 2)
  }
#undef MV_W1
#undef MV_W1F
  const int P = w256 ? ms : ms * c.ws;
  const int64_t E = (int64_t)K * C;
  const float* wk = work;
#define MV_W1R(PSV, TO)                                                                        \
  hipLaunchKernelGGL((wgrad1x1_reduce_kernel<PSV, TO>),                                        \
                     dim3((unsigned)((E / 4 + 256 / PSV - 1) / (256 / PSV))), dim3(256), 0, st, wk, \
                     (TO*)dw, E, P)
  if (dw_fp32) {
    if (P >= 64)
      MV_W1R(64, float);
    else if (P >= 16)
      MV_W1R(16, float);
    else
      MV_W1R(4, float);
  } else {
    if (P >= 64)
      MV_W1R(64, __bf16);
    else if (P >= 16)
      MV_W1R(16, __bf16);
    else
      MV_W1R(4, __bf16);
  }
#undef MV_W1R
  return true;
}
