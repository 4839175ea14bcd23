// NT GEMM on gfx950 MFMA for NHWC 1x1 convolutions, with fused epilogues.
//
//   C[M, N] (bf16) = A[M, K] (bf16, row-major: NHWC activations) . B[N, K]^T (bf16,
//   row-major: a channels_last [Cout, Cin, 1, 1] filter; for the data gradient the
//   channel-transposed filter)                              fp32 accumulation
//
// Epilogue STATS (the following BatchNorm's statistics pass, fused): per output
// channel n, over this workgroup's rows, s1 = sum(c - shift[n]), s2 = sum((c -
// shift[n])^2) of the bf16-ROUNDED outputs, written as partial[blockM][2][N] in a
// fixed order — the exact layout the BN finalize kernel (mv_bn.hip) reduces, so
// the statistics are deterministic and bit-identical on every rank, and the
// separate full read of C by the statistics pass disappears.
//
// MFMA mapping (v_mfma_f32_16x16x32_bf16): the FILTER tile is the A operand and the
// activation tile the B operand, so D = W . A^T = C^T and each lane's 4 accumulator
// registers are 4 CONSECUTIVE output channels of one output row — an 8-byte store
// per 16x16 tile, and the per-channel statistics reduce across the 16 lanes of a
// lane group with 4 xor-shuffles.
//
// Staging: global -> registers (16-byte loads) -> LDS double buffer with a 16-byte
// chunk XOR swizzle (row r's chunk c lives at c ^ (r & 7)), one barrier per
// 64-deep K step.  Grid: 1-D, tiles remapped so the N tiles of one row block are
// consecutive on one XCD (they share the activation rows through that XCD's L2).
#include "mv_common.h"
#include "mv_gemm.h"

#include <cstdlib>

namespace mv {
namespace gemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int BK = 64;
constexpr int KC = BK / 8;          // 16-byte chunks per staged row

__device__ __forceinline__ f32x4v mfma(const bf16x8& a, const bf16x8& b, const f32x4v& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int swz(int row, int ch) { return row * BK + ((ch ^ (row & 7)) << 3); }

__device__ __forceinline__ float round_bf16(float x) { return (float)(__bf16)x; }

// bijective XCD-aware remap of the 1-D workgroup id (8 XCDs, round-robin dispatch)
__device__ __forceinline__ int remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

template <int BM, int BN, int WM, int WN, bool STATS>
__global__ __launch_bounds__(WM * WN * 64) void gemm_nt_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
    int64_t M, int N, int K, int ntn, const float* __restrict__ shift,
    float* __restrict__ partial) {
  constexpr int NT = WM * WN * 64;
  constexpr int A_CH = BM * KC / NT;
  constexpr int B_CH = BN * KC / NT;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(BM * KC % NT == 0 && BN * KC % NT == 0, "tile / thread mismatch");
  static_assert(WTM % 16 == 0 && WTN % 16 == 0, "wave tile");
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int t = remap(blockIdx.x, gridDim.x);
  const int mt = t / ntn, nt = t - mt * ntn;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;

  u32x4 ra[A_CH], rb[B_CH];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + i * NT, row = q / KC, ch = q % KC;
      int64_t gm = m0 + row;
      gm = gm < M ? gm : M - 1;                 // rows past M: read a valid row, never stored
      ra[i] = *reinterpret_cast<const u32x4*>(A + gm * K + k0 + ch * 8);
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + i * NT, row = q / KC, ch = q % KC;
      rb[i] = *reinterpret_cast<const u32x4*>(B + (int64_t)(n0 + row) * K + k0 + ch * 8);
    }
  };
  auto sstore = [&](int buf) {
    __bf16* As = smem + buf * STAGE;
    __bf16* Bs = As + BM * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + i * NT, row = q / KC, ch = q % KC;
      *reinterpret_cast<u32x4*>(As + swz(row, ch)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int q = tid + i * NT, row = q / KC, ch = q % KC;
      *reinterpret_cast<u32x4*>(Bs + swz(row, ch)) = rb[i];
    }
  };

  f32x4v acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};

  const int KT = K / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + 1 < KT) gload((kt + 1) * BK);
    const __bf16* As = smem + (kt & 1) * STAGE;
    const __bf16* Bs = As + BM * BK;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 wf[TN], af[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a)
        wf[a] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * WTN + a * 16 + (lane & 15), ch));
#pragma unroll
      for (int b = 0; b < TM; ++b)
        af[b] = *reinterpret_cast<const bf16x8*>(As + swz(wm * WTM + b * 16 + (lane & 15), ch));
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mfma(wf[a], af[b], acc[a][b]);
    }
    if (kt + 1 < KT) sstore((kt + 1) & 1);
    __syncthreads();
  }

  // ---- epilogue: lane holds C[row][col .. col+3] for every (a, b) tile ----
  const int g = lane >> 4, rl = lane & 15;
  float s1[TN][4], s2[TN][4];
#pragma unroll
  for (int a = 0; a < TN; ++a) {
    const int col = n0 + wn * WTN + a * 16 + 4 * g;
    float sh[4] = {0.f, 0.f, 0.f, 0.f};
    if (STATS && shift) {
#pragma unroll
      for (int r = 0; r < 4; ++r) sh[r] = shift[col + r];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[a][r] = 0.f; s2[a][r] = 0.f; }
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int64_t row = m0 + wm * WTM + b * 16 + rl;
      if (row < M) {
        const f32x4v v = acc[a][b];
        u32x2 o = {cvt_pk_bf16(v[0], v[1]), cvt_pk_bf16(v[2], v[3])};
        *reinterpret_cast<u32x2*>(C + row * N + col) = o;
        if (STATS) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = round_bf16(v[r]) - sh[r];
            s1[a][r] += d;
            s2[a][r] += d * d;
          }
        }
      }
    }
  }
  if (!STATS) return;
  // reduce over the 16 lanes (rows) of each lane group: fixed xor tree
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[a][r] += __shfl_xor(s1[a][r], o, kWave);
        s2[a][r] += __shfl_xor(s2[a][r], o, kWave);
      }
    }
  // combine the WM waves of a column in a fixed order through LDS (reuses the stage)
  float* red = reinterpret_cast<float*>(smem);      // [2][WM][BN]
  if (rl == 0) {
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wn * WTN + a * 16 + 4 * g + r;
        red[(0 * WM + wm) * BN + c] = s1[a][r];
        red[(1 * WM + wm) * BN + c] = s2[a][r];
      }
  }
  __syncthreads();
  for (int v = tid; v < 2 * BN; v += NT) {
    const int k = v / BN, c = v - k * BN;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < WM; ++w) s += red[(k * WM + w) * BN + c];
    partial[((int64_t)mt * 2 + k) * N + n0 + c] = s;
  }
}

// ---------------------------------------------------------------------------
// Weight-stationary streaming variant for small K (64 / 128 / 256): the skinny,
// HBM-bound 1x1 convs of ResNet's early stages.  A persistent workgroup keeps its
// [BN, K] filter slice in LDS for the whole kernel and streams 64-row tiles of A:
// the next tile's 16-byte global loads are in flight (in registers) while the
// current tile is multiplied and stored, and the fused epilogue's per-channel
// sums accumulate in registers across ALL the tiles a workgroup processes — one
// cross-lane reduction and one [2][BN] partial row per workgroup at the end.
// The 4 waves split the BN columns, 64 rows x WTN columns per wave per tile.
//
// Column permutation: MFMA tile a's output row i (a filter row) is physical column
// TN*4*(i >> 2) + 4a + (i & 3) of the wave's slice, so each lane ends up holding
// 4*TN CONSECUTIVE channels of one output row: 16-byte stores, and 16-byte loads
// for the epilogue operands.
//
// Epilogues (EPI):
//   0  C = A . B^T
//   1  + BN statistics of the bf16-rounded C around shift (forward, fused stats pass)
//   2  BN+add+ReLU BACKWARD reduce fused into the data-gradient GEMM that produces
//      the BN output's gradient dy: d = relu_mask ? bf16(dy) + dy2 : 0 is written
//      (dz, the residual branch's gradient) instead of dy, and the partials are
//      (sum d, sum d * (x - mean)) — exactly mv_bn.hip's bwd_reduce_kernel<3>
//      (x = the BN input, mask = the forward's bitmask, dy2 = the shortcut gradient).
// ---------------------------------------------------------------------------
struct BwdEpi {
  const __bf16* dy2;      // [M, N] second gradient stream (shortcut), may be null
  const uint8_t* mask;    // [M, N/8] bitmask of the forward output > 0
  const __bf16* x;        // [M, N] BN input; null: only sum dz (second partial 0)
  const float* mean;      // [N] saved mean
  // ds > 1: dy2 lives on the stride-ds grid of the [*, H, W] rows (the input gradient
  // of a strided 1x1 shortcut conv, ops/bn.py downsample_tap): row (n, h, w) adds
  // dy2[n, h/ds, w/ds] when h and w are multiples of ds
  int ds, H, W;
  // EPI 3 (BN apply): y = relu(c * sc + bi + dy2) with dy2 = the residual, bitmask of y > 0
  // -> mo ([M, N/8], mv_bn.hip's mode-3 layout)
  const float* sc;
  const float* bi;
  uint8_t* mo;
  // EPI 4 (the BN3 fold's data gradient with BN2's ReLU backward reduce): A's columns
  // [K1, K) come from a2 ([M, K - K1]); badd [N] is added before rounding; the mask is
  // fma(x, sc, bi) > 0 (x = the BN's input) and the partials are (sum d, sum d (x - mean))
  const __bf16* a2;
  const float* badd;
  // EPI 5 = EPI 3 with an affine residual: the residual operand is the shortcut BN's input
  // and bf16(fma(r, rsc, rbi)) is added (the shortcut BN's apply, bit-identical)
  const float* rsc;
  const float* rbi;
  // EPI 7 = EPI 5 with the residual operand itself recomputed: r = bf16(a2 . b2^T) (the
  // stride-1 projection shortcut conv; a2 [M, K], b2 [N, K]) — it is never written
  const __bf16* b2;
};

// raw 16-/8-byte loads of NC consecutive bf16 (issued early, unpacked in the epilogue)
template <int NC>
__device__ __forceinline__ void ld_raw(const __bf16* p, uint32_t (&r)[NC / 2]) {
  if constexpr (NC == 4) {
    const u32x2 w = *reinterpret_cast<const u32x2*>(p);
    r[0] = w[0];
    r[1] = w[1];
  } else {
#pragma unroll
    for (int h = 0; h < NC / 8; ++h) {
      const u32x4 w = *reinterpret_cast<const u32x4*>(p + 8 * h);
#pragma unroll
      for (int j = 0; j < 4; ++j) r[4 * h + j] = w[j];
    }
  }
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

template <int K, int BN, int EPI, int BM = 64, int K1 = K>
__global__ __launch_bounds__(256) void gemm_stream_kernel(
    const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
    int64_t M, int N, int ntn, int64_t ntm, const float* __restrict__ shift,
    float* __restrict__ partial, BwdEpi be) {
  constexpr int KCH = K / 8;                 // 16-byte chunks per row
  constexpr int A_CH = BM * KCH / 256;       // A chunks per thread per tile
  constexpr int W_CH = BN * KCH / 256;
  constexpr int WTN = BN / 4;                // columns per wave
  constexpr int TN = WTN / 16, TM = BM / 16;
  constexpr int NC = 4 * TN;                 // consecutive channels per lane
  constexpr bool DUAL = EPI == 7;             // second GEMM (a2 . b2^T) in the same tile loop
  __shared__ __attribute__((aligned(16))) __bf16 smem[(BN + BM) * K * (DUAL ? 2 : 1)];
  __bf16* Ws = smem;
  __bf16* As = smem + BN * K;
  __bf16* Ws2 = smem + (BN + BM) * K;        // DUAL only
  __bf16* As2 = Ws2 + BN * K;
  auto sw = [](int row, int ch) { return row * K + ((ch ^ (row & 7)) << 3); };

  const int tid = threadIdx.x, lane = tid & 63, wn = tid >> 6;
  const int g = lane >> 4, rl = lane & 15;
  const int t = remap(blockIdx.x, gridDim.x);
  const int nt = t % ntn;
  const int64_t stream = t / ntn, nstreams = gridDim.x / ntn;
  const int n0 = nt * BN;
  const int cbase = n0 + wn * WTN + NC * g;  // this lane's first output channel

  // filter slice -> LDS (once)
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    const int q = tid + i * 256, row = q / KCH, ch = q % KCH;
    *reinterpret_cast<u32x4*>(Ws + sw(row, ch)) =
        *reinterpret_cast<const u32x4*>(B + (int64_t)(n0 + row) * K + ch * 8);
    if constexpr (DUAL)
      *reinterpret_cast<u32x4*>(Ws2 + sw(row, ch)) =
          *reinterpret_cast<const u32x4*>(be.b2 + (int64_t)(n0 + row) * K + ch * 8);
  }
  u32x4 ra[A_CH], ra2[DUAL ? A_CH : 1];
  auto gload = [&](int64_t mt) {
    const int64_t m0 = mt * BM;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + i * 256, row = q / KCH, ch = q % KCH;
      int64_t gm = m0 + row;
      gm = gm < M ? gm : M - 1;
      if constexpr (K1 == K) {
        ra[i] = *reinterpret_cast<const u32x4*>(A + gm * K + ch * 8);
        if constexpr (DUAL) ra2[i] = *reinterpret_cast<const u32x4*>(be.a2 + gm * K + ch * 8);
      } else {       // two row-major sources side by side along K
        const __bf16* p = ch < K1 / 8 ? A + gm * K1 + ch * 8
                                      : be.a2 + gm * (K - K1) + (ch - K1 / 8) * 8;
        ra[i] = *reinterpret_cast<const u32x4*>(p);
      }
    }
  };
  float sh[NC], s1[NC], s2[NC];
  constexpr bool APPLY = EPI == 3 || EPI == 5 || EPI == 7;
  constexpr bool RAFF = EPI == 5 || EPI == 7;
  // EPI 6: EPI 4's dual-source GEMM + badd with a plain store (no mask, no partials)
  constexpr bool BADD = EPI == 4 || EPI == 6;
  float apl_sc[EPI >= 3 ? NC : 1], apl_bi[EPI >= 3 ? NC : 1], add[BADD ? NC : 1];
  float res_sc[RAFF ? NC : 1], res_bi[RAFF ? NC : 1];
  if constexpr (RAFF) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      res_sc[j] = be.rsc[cbase + j];
      res_bi[j] = be.rbi[cbase + j];
    }
  }
  if constexpr (EPI == 4) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      apl_sc[j] = be.sc[cbase + j];
      apl_bi[j] = be.bi[cbase + j];
    }
  }
  if constexpr (BADD) {
#pragma unroll
    for (int j = 0; j < NC; ++j) add[j] = be.badd[cbase + j];
  }
  if constexpr (APPLY) {
    static_assert(NC == 8 || NC == 16, "EPI 3 writes whole mask bytes");
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      apl_sc[j] = be.sc[cbase + j];
      apl_bi[j] = be.bi[cbase + j];
    }
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    sh[j] = 0.f;
    if (EPI == 1 && shift) sh[j] = shift[cbase + j];
    if (EPI == 2 || EPI == 4) sh[j] = be.mean[cbase + j];
    s1[j] = 0.f;
    s2[j] = 0.f;
  }
  int64_t mt = stream;
  if (mt < ntm) gload(mt);
  for (; mt < ntm; mt += nstreams) {
    // EPI 2 / 3: this tile's epilogue operands, in flight during the MFMA work
    uint32_t e2[EPI == 2 || APPLY ? TM : 1][NC / 2], ex[EPI == 2 || EPI == 4 ? TM : 1][NC / 2];
    uint32_t em[EPI == 2 ? TM : 1];
    if constexpr (APPLY && !DUAL) {
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        int64_t row = mt * BM + b * 16 + rl;
        row = row < M ? row : M - 1;
        ld_raw<NC>(be.dy2 + row * N + cbase, e2[b]);
      }
    }
    if constexpr (EPI == 4) {
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        int64_t row = mt * BM + b * 16 + rl;
        row = row < M ? row : M - 1;
        ld_raw<NC>(be.x + row * N + cbase, ex[b]);
      }
    }
    if constexpr (EPI == 2) {
#pragma unroll
      for (int b = 0; b < TM; ++b) {
        int64_t row = mt * BM + b * 16 + rl;
        row = row < M ? row : M - 1;
        if (be.dy2) {
          int64_t r2 = row;
          bool has = true;
          if (be.ds > 1) {     // rows < 2^31 (checked by the binding)
            const uint32_t m = (uint32_t)row, hw = (uint32_t)(be.H * be.W);
            const uint32_t n = m / hw, rem = m - n * hw;
            const uint32_t h = rem / (uint32_t)be.W, w = rem - h * (uint32_t)be.W;
            const uint32_t hs = ((uint32_t)be.H + be.ds - 1) / be.ds;
            const uint32_t ws = ((uint32_t)be.W + be.ds - 1) / be.ds;
            has = h % be.ds == 0 && w % be.ds == 0;
            r2 = ((int64_t)n * hs + h / be.ds) * ws + w / be.ds;
          }
          if (has) {
            ld_raw<NC>(be.dy2 + r2 * N + cbase, e2[b]);
          } else {
#pragma unroll
            for (int j = 0; j < NC / 2; ++j) e2[b][j] = 0u;
          }
        }
        if (be.x) {
          ld_raw<NC>(be.x + row * N + cbase, ex[b]);
        } else {
#pragma unroll
          for (int j = 0; j < NC / 2; ++j) ex[b][j] = 0u;
        }
        const uint8_t* mp = be.mask + row * (N / 8) + cbase / 8;
        if constexpr (NC == 4) em[b] = (uint32_t)mp[0] >> (cbase & 7);
        else if constexpr (NC == 8) em[b] = mp[0];
        else em[b] = *reinterpret_cast<const uint16_t*>(mp);
      }
    }
    __syncthreads();                                   // previous tile's LDS reads done
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int q = tid + i * 256, row = q / KCH, ch = q % KCH;
      *reinterpret_cast<u32x4*>(As + sw(row, ch)) = ra[i];
      if constexpr (DUAL) *reinterpret_cast<u32x4*>(As2 + sw(row, ch)) = ra2[i];
    }
    __syncthreads();
    if (mt + nstreams < ntm) gload(mt + nstreams);     // in flight during compute + stores
    f32x4v acc[TN][TM];
#pragma unroll
    for (int a = 0; a < TN; ++a)
#pragma unroll
      for (int b = 0; b < TM; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
    if constexpr (DUAL) {
      // the shortcut GEMM first: its bf16-rounded result becomes this tile's residual
      // operand (packed like a prefetched residual row), then the main GEMM
      f32x4v acc2[TN][TM];
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc2[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < K / 32; ++kk) {
        const int ch = kk * 4 + g;
        bf16x8 wf[TN], af[TM];
#pragma unroll
        for (int a = 0; a < TN; ++a)
          wf[a] = *reinterpret_cast<const bf16x8*>(
              Ws2 + sw(wn * WTN + NC * (rl >> 2) + 4 * a + (rl & 3), ch));
#pragma unroll
        for (int b = 0; b < TM; ++b)
          af[b] = *reinterpret_cast<const bf16x8*>(As2 + sw(b * 16 + rl, ch));
#pragma unroll
        for (int a = 0; a < TN; ++a)
#pragma unroll
          for (int b = 0; b < TM; ++b) acc2[a][b] = mfma(wf[a], af[b], acc2[a][b]);
      }
#pragma unroll
      for (int b = 0; b < TM; ++b)
#pragma unroll
        for (int a = 0; a < TN; ++a) {
          e2[b][2 * a] = cvt_pk_bf16(acc2[a][b][0], acc2[a][b][1]);
          e2[b][2 * a + 1] = cvt_pk_bf16(acc2[a][b][2], acc2[a][b][3]);
        }
    }
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) {
      const int ch = kk * 4 + g;
      bf16x8 wf[TN], af[TM];
#pragma unroll
      for (int a = 0; a < TN; ++a)
        wf[a] = *reinterpret_cast<const bf16x8*>(
            Ws + sw(wn * WTN + NC * (rl >> 2) + 4 * a + (rl & 3), ch));
#pragma unroll
      for (int b = 0; b < TM; ++b)
        af[b] = *reinterpret_cast<const bf16x8*>(As + sw(b * 16 + rl, ch));
#pragma unroll
      for (int a = 0; a < TN; ++a)
#pragma unroll
        for (int b = 0; b < TM; ++b) acc[a][b] = mfma(wf[a], af[b], acc[a][b]);
    }
    const int64_t m0 = mt * BM;
#pragma unroll
    for (int b = 0; b < TM; ++b) {
      const int64_t row = m0 + b * 16 + rl;
      if (row >= M) continue;
      uint32_t pk[2 * TN];
#pragma unroll
      for (int a = 0; a < TN; ++a) {
        if constexpr (BADD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[a][b][r] += add[4 * a + r];
        }
        pk[2 * a] = cvt_pk_bf16(acc[a][b][0], acc[a][b][1]);
        pk[2 * a + 1] = cvt_pk_bf16(acc[a][b][2], acc[a][b][3]);
      }
      float v[NC];
#pragma unroll
      for (int j = 0; j < NC / 2; ++j) {
        v[2 * j] = __uint_as_float(pk[j] << 16);
        v[2 * j + 1] = __uint_as_float(pk[j] & 0xffff0000u);
      }
      if (EPI == 1) {
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const float d = v[j] - sh[j];
          s1[j] += d;
          s2[j] += d * d;
        }
      }
      if constexpr (EPI == 2) {
        if (be.dy2) {
#pragma unroll
          for (int j = 0; j < NC / 2; ++j) {
            v[2 * j] += bf_lo(e2[b][j]);
            v[2 * j + 1] += bf_hi(e2[b][j]);
          }
        }
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const float xv = (j & 1) ? bf_hi(ex[b][j >> 1]) : bf_lo(ex[b][j >> 1]);
          const float d = ((em[b] >> j) & 1u) ? v[j] : 0.f;
          v[j] = d;
          s1[j] += d;
          s2[j] += be.x ? d * (xv - sh[j]) : 0.f;      // x == null: second partial 0
        }
#pragma unroll
        for (int j = 0; j < NC / 2; ++j) pk[j] = cvt_pk_bf16(v[2 * j], v[2 * j + 1]);
      }
      if constexpr (EPI == 4) {
        // mv_bn.hip bwd_reduce_kernel<1>: d = relu'(bn(x)) * dx on the bf16-rounded dx
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const float xv = (j & 1) ? bf_hi(ex[b][j >> 1]) : bf_lo(ex[b][j >> 1]);
          const float d = __builtin_fmaf(xv, apl_sc[j], apl_bi[j]) > 0.f ? v[j] : 0.f;
          v[j] = d;
          s1[j] += d;
          s2[j] += d * (xv - sh[j]);
        }
#pragma unroll
        for (int j = 0; j < NC / 2; ++j) pk[j] = cvt_pk_bf16(v[2 * j], v[2 * j + 1]);
      }
      if constexpr (APPLY) {
        // mv_bn.hip apply_kernel's arithmetic on the bf16-rounded z: bit-identical y
        uint32_t bits = 0;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          float r = (j & 1) ? bf_hi(e2[b][j >> 1]) : bf_lo(e2[b][j >> 1]);
          if constexpr (RAFF) r = round_bf16(__builtin_fmaf(r, res_sc[j], res_bi[j]));
          float a = __builtin_fmaf(v[j], apl_sc[j], apl_bi[j]);
          a += r;
          a = fmaxf(a, 0.f);
          v[j] = a;
          bits |= (a > 0.f ? 1u : 0u) << j;
        }
#pragma unroll
        for (int j = 0; j < NC / 2; ++j) pk[j] = cvt_pk_bf16(v[2 * j], v[2 * j + 1]);
        uint8_t* mp = be.mo + row * (N / 8) + cbase / 8;
        if constexpr (NC == 8) *mp = (uint8_t)bits;
        else *reinterpret_cast<uint16_t*>(mp) = (uint16_t)bits;
      }
      if (EPI == 1 && C == nullptr) continue;      // statistics only (the recompute pass)
      __bf16* cp = C + row * N + cbase;
      if constexpr (NC == 4) {
        *reinterpret_cast<u32x2*>(cp) = u32x2{pk[0], pk[1]};
      } else {
#pragma unroll
        for (int h = 0; h < NC / 8; ++h)
          *reinterpret_cast<u32x4*>(cp + 8 * h) =
              u32x4{pk[4 * h], pk[4 * h + 1], pk[4 * h + 2], pk[4 * h + 3]};
      }
    }
  }
  if (EPI == 0 || EPI == 6 || APPLY) return;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1[j] += __shfl_xor(s1[j], o, kWave);
      s2[j] += __shfl_xor(s2[j], o, kWave);
    }
  }
  if (rl == 0 && stream < ntm) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      partial[(stream * 2 + 0) * N + cbase + j] = s1[j];
      partial[(stream * 2 + 1) * N + cbase + j] = s2[j];
    }
  }
}

template <int BM, int BN, int WM, int WN>
static void launch(const __bf16* A, const __bf16* B, __bf16* C, int64_t M, int N, int K,
                   const float* shift, float* partial, hipStream_t st) {
  const int ntn = N / BN;
  const int64_t ntm = (M + BM - 1) / BM;
  const dim3 grid((unsigned)(ntm * ntn));
  if (partial)
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, true>), grid, dim3(WM * WN * 64), 0, st, A,
                       B, C, M, N, K, ntn, shift, partial);
  else
    hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, false>), grid, dim3(WM * WN * 64), 0, st,
                       A, B, C, M, N, K, ntn, shift, partial);
}

}  // namespace gemm
}  // namespace mv

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

// streaming variant: the BN it uses for (K, N), or false for the tiled kernel
static bool stream_cfg(int K, int N, int* bn) {
  const char* e = std::getenv("MIVOD_GEMM_STREAM");
  if (e && e[0] == '0') return false;
  if (K == 64 || K == 128) { *bn = N % 256 == 0 ? 256 : (N % 128 == 0 ? 128 : 64); return true; }
  if (K == 256) { *bn = N % 128 == 0 ? 128 : 64; return true; }
  return false;
}

// rows per streamed tile: the K = 256 backward-reduce variant streams 32-row tiles so two
// workgroups fit a CU (its 64 KB filter slice + 16 KB A tile) — its epilogue reads three
// [M, N] operands, so resident waves matter more than MFMA tile depth
// (the K = 256 apply epilogues likewise: one 96 KB workgroup per CU at 64 rows)
template <int K, int EPI>
constexpr int stream_bm() { return (K == 256 && (EPI == 2 || EPI == 3 || EPI == 5)) ? 32 : 64; }

template <int K, int BN, int EPI>
static int64_t streams_for(int64_t M, int N) {
  constexpr int BMV = stream_bm<K, EPI>();
  static int per = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &v, (const void*)&mv::gemm::gemm_stream_kernel<K, BN, EPI, BMV>, 256, 0) != hipSuccess ||
        v < 1)
      v = 1;
    return v;
  }();
  const int ntn = N / BN;
  const int64_t ntm = (M + BMV - 1) / BMV;
  int64_t streams = (int64_t)num_cus() * per / ntn;
  if (streams < 1) streams = 1;
  if (streams > ntm) streams = ntm;
  return streams;
}

template <int K, int BN>
static void launch_stream(const __bf16* a, const __bf16* b, __bf16* c, int64_t M, int N,
                          const float* shift, float* partial, const mv::gemm::BwdEpi* be,
                          hipStream_t st) {
  using namespace mv::gemm;
  const int ntn = N / BN;
  BwdEpi e{};
  if (be) {
    e = *be;
    constexpr int BMV = stream_bm<K, 2>();
    const int64_t ntm = (M + BMV - 1) / BMV;
    const dim3 grid((unsigned)(streams_for<K, BN, 2>(M, N) * ntn));
    hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 2, BMV>), grid, dim3(256), 0, st, a, b, c, M, N,
                       ntn, ntm, shift, partial, e);
  } else if (partial) {
    const int64_t ntm = (M + 63) / 64;
    const dim3 grid((unsigned)(streams_for<K, BN, 1>(M, N) * ntn));
    hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 1>), grid, dim3(256), 0, st, a, b, c, M, N,
                       ntn, ntm, shift, partial, e);
  } else {
    const int64_t ntm = (M + 63) / 64;
    const dim3 grid((unsigned)(streams_for<K, BN, 0>(M, N) * ntn));
    hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 0>), grid, dim3(256), 0, st, a, b, c, M, N,
                       ntn, ntm, shift, partial, e);
  }
}

// EPI 3 for the streamed (K, BN): BN >= 128, so a lane's NC channels fill whole mask bytes
template <int K, int BN>
static void launch_apply(const __bf16* a, const __bf16* b, __bf16* y, int64_t M, int N,
                         const mv::gemm::BwdEpi& e, hipStream_t st) {
  using namespace mv::gemm;
  if constexpr (BN >= 128) {
    const int ntn = N / BN;
    const int64_t ntm = (M + 63) / 64;
    if (e.b2) {
      if constexpr (K == 64) {       // the stride-1 shortcut's K equals conv3's (layer1)
        const dim3 grid((unsigned)(streams_for<K, BN, 7>(M, N) * ntn));
        hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 7>), grid, dim3(256), 0, st, a, b, y, M, N,
                           ntn, ntm, nullptr, nullptr, e);
      }
    } else if (e.rsc) {
      constexpr int BMV = stream_bm<K, 5>();
      const dim3 grid((unsigned)(streams_for<K, BN, 5>(M, N) * ntn));
      hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 5, BMV>), grid, dim3(256), 0, st, a, b, y, M,
                         N, ntn, (M + BMV - 1) / BMV, nullptr, nullptr, e);
    } else {
      constexpr int BMV = stream_bm<K, 3>();
      const dim3 grid((unsigned)(streams_for<K, BN, 3>(M, N) * ntn));
      hipLaunchKernelGGL((gemm_stream_kernel<K, BN, 3, BMV>), grid, dim3(256), 0, st, a, b, y, M,
                         N, ntn, (M + BMV - 1) / BMV, nullptr, nullptr, e);
    }
  }
}

// EPI 4 (dual-source A: K = K1 + K2, weight-stationary, 64-column tiles)
template <int K, int K1, int EPI = 4>
static bool launch_fold_dx(const __bf16* a, const __bf16* b, __bf16* d, int64_t M, int N,
                           const mv::gemm::BwdEpi& e, float* partial, int64_t* P, hipStream_t st) {
  using namespace mv::gemm;
  constexpr int BN = 64;
  static int per = [] {
    int v = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &v, (const void*)&gemm_stream_kernel<K, BN, EPI, 64, K1>, 256, 0) != hipSuccess || v < 1)
      v = 1;
    return v;
  }();
  const int ntn = N / BN;
  const int64_t ntm = (M + 63) / 64;
  int64_t streams = (int64_t)num_cus() * per / ntn;
  if (streams < 1) streams = 1;
  if (streams > ntm) streams = ntm;
  *P = streams;
  if (EPI == 4 ? !partial : !a) return true;
  hipLaunchKernelGGL((gemm_stream_kernel<K, BN, EPI, 64, K1>), dim3((unsigned)(streams * ntn)),
                     dim3(256), 0, st, a, b, d, M, N, ntn, ntm, nullptr, partial, e);
  return true;
}

#define MV_STREAM_CASES(X) \
  X(64, 256) X(64, 128) X(64, 64) X(128, 256) X(128, 128) X(128, 64) X(256, 128) X(256, 64)

// the 256 x 256 kernel (mv_gemm256.hip) for the tiled (K >= 512) shapes with N % 256 == 0
static bool gemm256_on() {
  static const bool on = [] {
    const char* e = std::getenv("MIVOD_GEMM256");
    return !(e && e[0] == '0');
  }();
  return on;
}

// shapes the 256 x 256 kernel takes before the streaming kernel (plain / statistics /
// statistics-only): K = 256 -> N >= 1024 (ResNet-50 layer3 conv3, scripts/micro_gemm256.py:
// 348 us vs 371 us at bs2048)
static bool g256_first(int64_t M, int N, int K) {
  return gemm256_on() && K == 256 && N % 256 == 0 && N >= 1024 && N <= 8192 &&
         mv_gemm256_supported(M, N, K);
}

// number of [2][N] statistics partial rows gemm_nt writes for this problem
int64_t mv_gemm_partials(int64_t M, int N, int K) {
  int bn;
  if (g256_first(M, N, K)) return mv_gemm256_partials(M, N);
  if (stream_cfg(K, N, &bn)) {
#define MV_P(KK, BB) \
    if (K == KK && bn == BB) return streams_for<KK, BB, 1>(M, N);
    MV_STREAM_CASES(MV_P)
#undef MV_P
  }
  if (gemm256_on() && mv_gemm256_supported(M, N, K)) return mv_gemm256_partials(M, N);
  const int bm = N % 128 == 0 ? 128 : 256;
  return (M + bm - 1) / bm;
}

void mv_gemm_nt(const void* A, const void* B, void* C, int64_t M, int N, int K,
                const float* shift, float* partial, hipStream_t st) {
  using namespace mv::gemm;
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  __bf16* c = (__bf16*)C;
  int bn;
  if (g256_first(M, N, K) && mv_gemm256_nt(A, B, C, M, N, K, shift, partial, st)) return;
  if (stream_cfg(K, N, &bn)) {
#define MV_L(KK, BB) \
    if (K == KK && bn == BB) { launch_stream<KK, BB>(a, b, c, M, N, shift, partial, nullptr, st); return; }
    MV_STREAM_CASES(MV_L)
#undef MV_L
  }
  if (gemm256_on() && mv_gemm256_nt(A, B, C, M, N, K, shift, partial, st)) return;
  if (N % 256 == 0)
    launch<128, 256, 2, 2>(a, b, c, M, N, K, shift, partial, st);
  else if (N % 128 == 0)
    launch<128, 128, 2, 2>(a, b, c, M, N, K, shift, partial, st);
  else
    launch<256, 64, 4, 1>(a, b, c, M, N, K, shift, partial, st);
}

// column-tile width of the EPI 2 kernel (req > 0 forces one).  The widest tile wins
// despite 1 wave/SIMD: its epilogue operands are prefetched a whole tile ahead, and the
// A operand is read once (scripts/micro_gemm1x1.py bwd sweep: K64N256 bn256 1878 us vs
// bn128 2245 / bn64 3415; K256N1024 bn128 751 vs bn64 1090)
static bool bwd_cfg(int K, int N, int req, int* bn) {
  if (K != 64 && K != 128 && K != 256) return false;
  int b = req > 0 ? req : (K == 256 ? 128 : 256);
  if (K == 256 && b > 128) b = 128;
  while (b > 64 && N % b) b >>= 1;
  if (b != 64 && b != 128 && b != 256) return false;
  if (N % b) return false;
  *bn = b;
  return true;
}

// number of partial rows of mv_gemm_nt_bn_bwd (the EPI 2 kernel's persistent grid)
int64_t mv_gemm_bwd_partials(int64_t M, int N, int K, int req_bn) {
  int bn;
  if (!bwd_cfg(K, N, req_bn, &bn)) return -1;
#define MV_PB(KK, BB) \
  if (K == KK && bn == BB) return streams_for<KK, BB, 2>(M, N);
  MV_STREAM_CASES(MV_PB)
#undef MV_PB
  return -1;
}

bool mv_gemm_nt_bn_bwd(const void* A, const void* B, void* DZ, int64_t M, int N, int K,
                       const void* dy2, const void* mask, const void* x, const float* mean,
                       float* partial, int req_bn, hipStream_t st, int dy2_stride, int H, int W) {
  using namespace mv::gemm;
  int bn;
  if (!bwd_cfg(K, N, req_bn, &bn)) return false;
  BwdEpi e{(const __bf16*)dy2, (const uint8_t*)mask, (const __bf16*)x, mean,
           dy2_stride > 1 ? dy2_stride : 1, H, W};
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  __bf16* c = (__bf16*)DZ;
#define MV_LB(KK, BB) \
  if (K == KK && bn == BB) { launch_stream<KK, BB>(a, b, c, M, N, nullptr, partial, &e, st); return true; }
  MV_STREAM_CASES(MV_LB)
#undef MV_LB
  return false;
}

bool mv_gemm_apply_supported(int N, int K) {
  int bn;
  return K % 64 == 0 && N % 64 == 0 && stream_cfg(K, N, &bn) && bn >= 128;
}

bool mv_gemm_nt_apply(const void* A, const void* B, void* Y, int64_t M, int N, int K,
                      const void* res, const float* scale, const float* bias, void* mask,
                      hipStream_t st, const float* rscale, const float* rbias) {
  using namespace mv::gemm;
  int bn;
  if (!mv_gemm_apply_supported(N, K) || !stream_cfg(K, N, &bn)) return false;
  BwdEpi e{};
  e.dy2 = (const __bf16*)res;
  e.ds = 1;
  e.sc = scale;
  e.bi = bias;
  e.mo = (uint8_t*)mask;
  e.rsc = rscale;
  e.rbi = rscale ? rbias : nullptr;
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  __bf16* y = (__bf16*)Y;
#define MV_LA(KK, BB) \
  if (K == KK && bn == BB && BB >= 128) { launch_apply<KK, BB>(a, b, y, M, N, e, st); return true; }
  MV_STREAM_CASES(MV_LA)
#undef MV_LA
  return false;
}

// (K1, K2) = (cout, cin) of the folded conv: 256 + 64 (layer1), 512 + 128 (layer2)
static bool fold_dx_dispatch(int K1, int K2, const __bf16* a, const __bf16* b, __bf16* d,
                             int64_t M, int N, const mv::gemm::BwdEpi& e, float* partial,
                             int64_t* P, hipStream_t st) {
  if (N % 64 || N != K2) return false;
  if (K1 == 256 && K2 == 64) return launch_fold_dx<320, 256>(a, b, d, M, N, e, partial, P, st);
  if (K1 == 512 && K2 == 128) return launch_fold_dx<640, 512>(a, b, d, M, N, e, partial, P, st);
  return false;
}

// the 256 x 256 dual-source kernel for the fold data gradients the streaming kernel does
// not cover (ResNet-50 layers 3-4: (K1, K2) = (1024, 256), (2048, 512))
static bool fold_dx_g256(int64_t M, int K1, int K2) {
  return gemm256_on() && K1 % 64 == 0 && mv_gemm256_supported(M, K2, K1 + K2) && 4 * K2 <= 8192;
}

int64_t mv_gemm_fold_dx_partials(int64_t M, int K1, int K2) {
  int64_t P = -1;
  mv::gemm::BwdEpi e{};
  if (!fold_dx_dispatch(K1, K2, nullptr, nullptr, nullptr, M, K2, e, nullptr, &P, nullptr))
    return fold_dx_g256(M, K1, K2) ? mv_gemm256_partials(M, K2) : -1;
  return P;
}

bool mv_gemm_fold_dx(const void* A1, const void* A2, const void* B, const float* badd,
                     void* D, int64_t M, int K1, int K2, const void* x, const float* mean,
                     const float* scale, const float* bias, float* partial, hipStream_t st) {
  mv::gemm::BwdEpi e{};
  e.x = (const __bf16*)x;
  e.mean = mean;
  e.sc = scale;
  e.bi = bias;
  e.a2 = (const __bf16*)A2;
  e.badd = badd;
  e.ds = 1;
  int64_t P = 0;
  if (fold_dx_dispatch(K1, K2, nullptr, nullptr, nullptr, M, K2, e, nullptr, &P, nullptr))
    return fold_dx_dispatch(K1, K2, (const __bf16*)A1, (const __bf16*)B, (__bf16*)D, M, K2, e,
                            partial, &P, st);
  return fold_dx_g256(M, K1, K2) &&
         mv_gemm256_dual(A1, A2, B, badd, D, M, K1, K2, K2, x, mean, scale, bias, partial, st);
}

// (256, 64) on the streaming kernel; K2 % 256 == 0 on the 256 x 256 kernel
bool mv_gemm_dual_supported(int K1, int K2) {
  return (K1 == 256 && K2 == 64) || (gemm256_on() && K1 % 64 == 0 && K2 % 256 == 0);
}

bool mv_gemm_dual_bias(const void* A1, const void* A2, const void* B, const float* badd, void* D,
                       int64_t M, int K1, int K2, hipStream_t st) {
  if (!mv_gemm_dual_supported(K1, K2)) return false;
  if (K2 % 256 == 0)
    return mv_gemm256_dual(A1, A2, B, badd, D, M, K1, K2, K2, nullptr, nullptr, nullptr, nullptr,
                           nullptr, st);
  mv::gemm::BwdEpi e{};
  e.a2 = (const __bf16*)A2;
  e.badd = badd;
  e.ds = 1;
  int64_t P = 0;
  return launch_fold_dx<320, 256, 6>((const __bf16*)A1, (const __bf16*)B, (__bf16*)D, M, K2, e,
                                     nullptr, &P, st);
}

bool mv_gemm_apply_dual_supported(int N, int K) {
  int bn;
  return K == 64 && mv_gemm_apply_supported(N, K) && stream_cfg(K, N, &bn) && bn >= 128;
}

bool mv_gemm_nt_apply_dual(const void* A, const void* B, const void* A2, const void* B2, void* Y,
                           int64_t M, int N, int K, const float* scale, const float* bias,
                           const float* rscale, const float* rbias, void* mask, hipStream_t st) {
  if (!mv_gemm_apply_dual_supported(N, K) || !rscale || !rbias) return false;
  using namespace mv::gemm;
  int bn;
  stream_cfg(K, N, &bn);
  BwdEpi e{};
  e.ds = 1;
  e.sc = scale;
  e.bi = bias;
  e.mo = (uint8_t*)mask;
  e.rsc = rscale;
  e.rbi = rbias;
  e.a2 = (const __bf16*)A2;
  e.b2 = (const __bf16*)B2;
  const __bf16* a = (const __bf16*)A;
  const __bf16* b = (const __bf16*)B;
  __bf16* y = (__bf16*)Y;
  // 128-column tiles: the 256-wide tile's two accumulator sets leave 1 wave per SIMD
  // (200 VGPRs + 116 AGPRs), the 128-wide one keeps 2 (MIVOD_GEMM_DUAL_BN=256 for A/B)
  static const int want = [] {
    const char* v = std::getenv("MIVOD_GEMM_DUAL_BN");
    return v && std::atoi(v) == 256 ? 256 : 128;
  }();
  if (bn == 256 && want == 256) { launch_apply<64, 256>(a, b, y, M, N, e, st); return true; }
  launch_apply<64, 128>(a, b, y, M, N, e, st);
  return true;
}
