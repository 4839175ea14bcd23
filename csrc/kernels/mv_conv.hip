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
};

// per-thread state of the A rows it stages (A_CH rows, fixed source chunk): the byte
// address of tap (0, 0) and a 9-bit mask of the taps that fall inside the image —
// per K step only a wave-uniform offset is added (keeps the issue path a few VALU ops)
template <int A_CH>
struct RowInfo {
  uint64_t addr[A_CH];
  uint32_t valid[A_CH];
};

template <int A_CH, int NT>
__device__ __forceinline__ void row_info(const Geo& g, const __bf16* X, int64_t m0, int tid,
                                         int sc, RowInfo<A_CH>& ri) {
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int64_t m = m0 + i * (NT / 8) + (tid >> 3);
    ri.valid[i] = 0;
    ri.addr[i] = 0;
    if (m < g.M) {
      const int64_t hw = (int64_t)g.Ho * g.Wo;
      const int n = (int)(m / hw);
      const int rem = (int)(m - (int64_t)n * hw);
      const int ho = rem / g.Wo, wo = rem - ho * g.Wo;
      const int hi0 = ho * g.st - 1, wi0 = wo * g.st - 1;
      uint32_t v = 0;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool ok = (unsigned)(hi0 + r) < (unsigned)g.H && (unsigned)(wi0 + s) < (unsigned)g.W;
          v |= (ok ? 1u : 0u) << (r * 3 + s);
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
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(WM * WN * 64) void conv3x3_kernel(
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
  constexpr int NS = 3;                           // LDS ring: 2 stages in flight
  __shared__ __attribute__((aligned(16))) __bf16 smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
  const int wm = wid / WN, wn = wid % WN;
  const int t = remap(blockIdx.x, gridDim.x);
  const int nt = t % ntn;
  const int64_t stream = t / ntn, nstreams = gridDim.x / ntn;
  const int n0 = nt * BN;
  const int csteps = g.C / BK, KT = 9 * csteps;
  const int64_t wrow = (int64_t)9 * g.C;          // filter row length
  const int sc = (tid & 7) ^ ((tid >> 3) & 7);    // swizzled source chunk of this thread

  uint64_t brow[B_CH];                            // filter rows of this thread
#pragma unroll
  for (int i = 0; i < B_CH; ++i)
    brow[i] = (uint64_t)(Wt + (int64_t)(n0 + i * (NT / 8) + (tid >> 3)) * wrow + sc * 8);
  const uint64_t zaddr = (uint64_t)(g_zero + (tid & 7) * 4);

  auto issue = [&](const RowInfo<A_CH>& ri, int kt, int buf) {
    const int tap = kt / csteps, c0 = (kt - tap * csteps) * BK;   // wave-uniform
    const int r = tap / 3, s = tap - r * 3;
    const int64_t offa = (((int64_t)r * g.W + s) * g.C + c0) * 2;
    const int64_t offb = ((int64_t)tap * g.C + c0) * 2;
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
  float sh[TN][4], s1[TN][4], s2[TN][4];
  float bsc[EPI == 2 ? TN : 1][4], bbi[EPI == 2 ? TN : 1][4];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int col = n0 + wn * WTN + a * 16 + 4 * gq + r;
      sh[a][r] = (EPI == 1 && shift) ? shift[col] : 0.f;
      if constexpr (EPI == 2) {
        sh[a][r] = bnvec[col];                   // saved mean
        bsc[a][r] = bnvec[2 * g.K + col];        // scale = gamma * invstd
        bbi[a][r] = bnvec[3 * g.K + col];        // bias = beta - mean * scale
      }
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
    row_info<A_CH, NT>(g, X, mt * BM, tid, sc, iri);
    int64_t imt = mt;          // (tile, step) of the last issued stage
    int ikt = 0;
    int islot = 0;
    issue(iri, 0, 0);
    auto issue_next = [&]() -> bool {
      int k2 = ikt + 1;
      int64_t m2 = imt;
      if (k2 == KT) { k2 = 0; m2 += nstreams; }
      if (m2 >= ntm) return false;
      if (m2 != imt) row_info<A_CH, NT>(g, X, m2 * BM, tid, sc, iri);
      islot = islot + 1 == NS ? 0 : islot + 1;
      issue(iri, k2, islot);
      imt = m2;
      ikt = k2;
      return true;
    };
    bool ahead = issue_next();      // stage of step 1 in flight
    int slot = 0;
    while (true) {
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
      for (int kt = 0; kt < KT; ++kt) {
        if (ahead) wait_vm<LPS>(); else wait_vm<0>();
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
        const int64_t row = m0 + wm * WTM + b * 16 + rl;
        if (row < g.M) {
#pragma unroll
          for (int a = 0; a < TN; ++a) {
            const f32x4v v = acc[a][b];
            const int col = n0 + wn * WTN + a * 16 + 4 * gq;
            if constexpr (EPI == 2) {
              const u32x2 xw = *reinterpret_cast<const u32x2*>(bnx + row * g.K + col);
              const float xv[4] = {__uint_as_float(xw[0] << 16), __uint_as_float(xw[0] & 0xffff0000u),
                                   __uint_as_float(xw[1] << 16), __uint_as_float(xw[1] & 0xffff0000u)};
              float dv[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float d =
                    __builtin_fmaf(xv[r], bsc[a][r], bbi[a][r]) > 0.f ? round_bf16(v[r]) : 0.f;
                dv[r] = d;
                s1[a][r] += d;
                s2[a][r] += d * (xv[r] - sh[a][r]);
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
  static constexpr int BM = 256, WM = 4, WN = 2;
};
template <bool STATS>
struct Cfg<64, STATS> {
  static constexpr int BM = 256, WM = 4, WN = 2;
};

template <int BN, bool STATS, int EPI = STATS ? 1 : 0>
static const void* kernel_ptr() {
  using C = Cfg<BN, STATS>;
  return (const void*)&conv3x3_kernel<C::BM, BN, C::WM, C::WN, EPI>;
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

int64_t mv_conv3x3_partials(int64_t M, int K) {
  using namespace mv::conv;
  if (conv_bn_of(K) == 128)
    return streams_for<128, true>((M + Cfg<128, true>::BM - 1) / Cfg<128, true>::BM, K / 128);
  return streams_for<64, true>((M + Cfg<64, true>::BM - 1) / Cfg<64, true>::BM, K / 64);
}

bool mv_conv3x3(const void* x, const void* w, void* y, int N, int H, int W, int C, int K,
                int stride, const float* shift, float* partial, hipStream_t st,
                const void* bn_x, const float* bn_vec) {
  using namespace mv::conv;
  if (C % 64 != 0 || K % 64 != 0 || (stride != 1 && stride != 2)) return false;
  Geo g;
  g.H = H;
  g.W = W;
  g.C = C;
  g.K = K;
  g.st = stride;
  g.Ho = (H - 1) / stride + 1;
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
    const int64_t ntm = (g.M + BMV - 1) / BMV;                                                 \
    const int ntn = K / BNV;                                                                   \
    const int64_t ns = streams_for<BNV, ST>(ntm, ntn);                                         \
    if (BX)                                                                                    \
      hipLaunchKernelGGL((conv3x3_kernel<BMV, BNV, WMV, WNV, 2>), dim3((unsigned)(ns * ntn)),     \
                         dim3(WMV * WNV * 64), 0, st, X, Wt, Y, g, ntn, ntm, shift, partial, BX, \
                         bn_vec);                                                              \
    else                                                                                       \
      hipLaunchKernelGGL((conv3x3_kernel<BMV, BNV, WMV, WNV, ST ? 1 : 0>),                       \
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
