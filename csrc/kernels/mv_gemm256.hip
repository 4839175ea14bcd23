// 256 x 256 NT GEMM for the compute-bound 1x1 convolutions (ResNet-50 layers 3-4:
// K = 256..2048, N = 256..2048), with the BN-statistics epilogue of mv_gemm.hip.
//
//   C[M, N] (bf16) = A[M, K] . B[N, K]^T, fp32 accumulation; N % 256 == 0, K % 64 == 0
//
// Why a second tiled kernel: mv_gemm.hip's 128 x 128 register-staged loop (two barriers
// per 64-deep K step, ~1 block per SIMD pair) tops out near 550-620 TFLOP/s on these
// shapes, below the vendor convolutions.  This one is built around the CDNA4 MFMA
// pipeline instead:
//   * 256 x 256 tile, 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave (32 MFMA
//     accumulators = 128 VGPRs): 128 FLOP per staged byte, one workgroup per CU.
//   * Operands staged with global_load_lds (16 B per lane, LDS image lane-linear, the
//     16-B chunk XOR swizzle applied to the SOURCE address and undone on the read).
//     LDS = 2 K-tile buffers x 4 half-tiles (A rows of quadrant row 0 / 1, B columns
//     of quadrant column 0 / 1) x 16 KB = 128 KB.
//   * Each K tile runs as 4 phases, one per 64 x 32 output quadrant of the wave
//     (16 MFMAs): the phase reads its operand half-tiles from LDS (A half 0 + B half 0,
//     B half 1, A half 1, nothing), issues one half-tile of the NEXT K tile into the
//     other buffer, and waits (counted vmcnt, never 0 in the steady state) for the
//     half-tile the next phase reads.
//   * Persistent (one workgroup per CU): one stream of K tiles runs over all of a
//     workgroup's output tiles, so the next tile's first K tile is staged during the
//     current tile's last one and its epilogue (short-K shapes: K = 256 is 4 K tiles).
//   * The two wave groups (wm = 0 / 1, one wave of each per SIMD) run one barrier apart:
//     while one group's phase is in its MFMA cluster (s_setprio 1), the other group is
//     reading fragments and issuing loads, so each SIMD's matrix pipe always has a wave
//     with MFMAs ready.  Reads of a staged half-tile always come one phase after the
//     wait that retired it, which under the one-barrier stagger still orders every
//     wave's DMA before any wave's read.
// Output mapping as mv_gemm.hip: the filter tile is the MFMA A operand, so a lane's
// 4 accumulators are 4 consecutive channels of one output row and the per-channel
// statistics reduce over the 16 lanes of a lane group; C leaves as 16-byte stores after
// a v_permlane16_swap exchange between n-tile pairs.
#include "mv_common.h"
#include "mv_gemm.h"

#include <cstdlib>

namespace mv {
namespace g256 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int HALF = 128 * BK;            // elements per half-tile (16 KB)
constexpr int BUF = 4 * HALF;             // one K tile: A0, A1, B0, B1

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
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Kernel arguments.  A modes: 0 plain A[M, K]; 1 strided gather (a stride-ds 1x1 conv:
// A is the [*, H, W, K] input, output row (n, ho, wo) reads input row (n, ho ds, wo ds));
// 2 dual source (A columns [0, K1) from A [M, K1], [K1, K) from A2 [M, K - K1]);
// 3 implicit ks x ks convolution (pad ks / 2, stride ds, ks = 1 or 3): A = im2col of the
// [*, H, W, Cin] input, never materialised — K tile kt is channels [c0, c0 + 64) of filter
// tap kt / (Cin / 64); each staged row carries its tap-(0, 0) address and a 9-bit mask of
// the taps inside the image (padding taps read a zero page); B = the [N][ks][ks][Cin]
// filter, already K-contiguous.
// 4 stride-2 3x3 (pad 1) DATA gradient, one output parity class (ph, pw) per launch: dx
// pixel (n, 2i + ph, 2j + pw) only receives the taps r' = 1 (ph = 0) or r' in {0, 2}
// (ph = 1) of the flipped filter (columns likewise), reading dy (n, i + r'/2, j + s'/2) —
// a gather GEMM over the class's 1, 2 or 4 taps (K = taps x Cin, dy channels) with no
// structurally-zero products and no zero-filled dx (every dx pixel is in one class).
// A = dy [*, Ho, Wo, Cin]; B = the transposed, flipped filter [N][3][3][Cin] (row Kb =
// 9 Cin); M = Nb Ho Wo class rows, stored at dx row (n, 2i + ph, 2j + pw) of [*, H, W, N].
// Epilogues: 0 plain; 1 + BN statistics of the bf16 C around shift; 4 the BN fold's data
// gradient (mv_gemm.hip EPI 4): C + badd (badd may be null: the 3x3 data gradient with the
// producing BN+ReLU's backward reduce, mv_conv.hip EPI 2), d = fma(xb, sc, bi) > 0 ? bf16 : 0
// is stored, partials (sum d, sum d (xb - mean)); 6 C + badd, plain store.
struct Args {
  const __bf16* A;
  const __bf16* A2;
  const __bf16* B;
  __bf16* C;
  int64_t M;
  int N, K, K1, ntn;
  int64_t ntiles;
  int ds, H, W, Ho, Wo;
  int Cin, ks;                    // AMODE 3
  int ph, pw, Kb;                 // AMODE 4: parity class, filter row length (9 Cin)
  const float* shift;
  float* partial;
  const float* badd;
  const __bf16* xb;
  const float* mean;
  const float* sc;
  const float* bi;
};

template <int EPI>
constexpr int nvec() { return EPI == 1 ? 1 : EPI == 4 ? 4 : EPI == 6 ? 1 : 0; }
constexpr int kVecFloats = 8192;          // LDS for the per-channel epilogue vectors (32 KB)

// zero page: padding taps (AMODE 3) and rows past M (the weight gradient)
__device__ __attribute__((aligned(16))) uint32_t g_w256_zero[64];

// MT: m tiles (16 rows) per wave group — 8 (BM = 256) or 7 (BM = 224: ResNet-50's
// M = 2048 x 196 / x 49 split into 1792 / 448 row blocks, a whole number of rounds over 256
// CUs for every N tile count, where 256-row blocks leave a 1/8- to 1/2-full last round).
// With MT = 7 the second A half-tile holds 48 live rows (the other 16 re-stage live rows,
// never read).
template <int EPI, int AMODE, int MT>
__global__ __launch_bounds__(NT, 1) void gemm256_kernel(Args p) {
  constexpr int BMv = MT * 32;
  constexpr int MH1 = MT - 4;               // m tiles in A half 1
  constexpr int NV = nvec<EPI>();
  constexpr bool STATS = EPI == 1 || EPI == 4;
  constexpr bool BADD = EPI == 4 || EPI == 6;
  // 2 K-tile buffers + the epilogue's per-channel vectors: ONE LDS object (a second one
  // makes hipcc drain the in-flight LDS DMA before every fragment read)
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF + (NV ? 2 * kVecFloats : 0)];
  // [NV][256]: this workgroup's column tile of the per-channel vectors, then (STATS) the
  // statistics accumulators [2 wave groups][2][256] summed over all of its output tiles
  float* vecs = reinterpret_cast<float*>(smem + 2 * BUF);
  float* stacc = vecs + 4 * BN;
  const int N = p.N;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;
  const int G = gridDim.x;
  // persistent: workgroups of one XCD take consecutive tiles (the N tiles of an M block
  // share its A rows through that XCD's L2)
  int64_t tile = remap(blockIdx.x, G);
  if (tile >= p.ntiles) return;
  // G % ntn == 0 (g256_launch): a workgroup's tiles tile, tile + G, ... share one column
  // tile, so its statistics accumulate on chip and leave as ONE partial row per wave group
  // (row group tile0 / ntn) — 2 G / ntn partial rows instead of 2 per row block
  const int64_t tile0 = tile;
  const int nw0 = (int)(tile0 % p.ntn) * BN;

  // ---- staging roles: glds instruction i (0, 1) of a half-tile lands at half row
  // r = (2 w + i) * 8 + lane / 8, LDS chunk lane % 8, which holds source chunk
  // (lane % 8) ^ (r & 7).  Half h of A = tile rows {128 q + 64 h + j}, of B = tile
  // columns {64 q + 32 h + j}.  Byte offsets at K offset 0 (the host checks < 4 GB).
  // (dual source: the A row index instead, both sources' offsets formed at issue)
  uint32_t offa[2][2], offb[2][2];
  uint32_t offa2[2][2];            // AMODE 2: A2's row (the strided input row when ds > 1)
  uint32_t abase[2][2];            // AMODE 3: tap-(0, 0) byte offset of the row's chunk in
                                   // A (mod 2^32: negative at the top-left padding, only
                                   // used with a tap that lands inside the image)
  uint32_t avalid[2];              // AMODE 3: taps inside the image, row i at bit 16 i
  const uint32_t scb = (uint32_t)(((lane & 7) ^ ((lane >> 3) & 7)) * 16);   // = sc * 16 bytes
  const int KT = p.K / BK, KT1 = AMODE == 2 ? p.K1 / BK : KT;
  const int csteps = (AMODE == 3 || AMODE == 4) ? p.Cin / BK : 1;
  // K tile -> (tap, channel step) by shift when csteps is a power of two (Cin = 256 / 512 /
  // ..: always on ResNet shapes) — two scalar divisions per issued K tile otherwise
  const bool cpow2 = (csteps & (csteps - 1)) == 0;
  const int cshift = __builtin_ctz((unsigned)csteps);
  auto set_src = [&](int64_t tl) {
    const int64_t mt = tl / p.ntn;
    const int nt = (int)(tl - mt * p.ntn);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (2 * w + i) * 8 + (lane >> 3);
      const int sc = (lane & 7) ^ (r & 7);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int rr = (r & 63);
        int64_t row = mt * BMv + (r >> 6) * (MT * 16) + h * 64 +
                      ((h == 1 && rr >= 16 * MH1) ? rr - 16 * MH1 : rr);
        row = row < p.M ? row : p.M - 1;           // rows past M: a valid row, never stored
        if constexpr (AMODE == 1) {          // rows < 2^31: 32-bit unsigned divisions
          const uint32_t hw = (uint32_t)(p.Ho * p.Wo), r32 = (uint32_t)row;
          const int64_t n = r32 / hw;
          const int rem = (int)(r32 - (uint32_t)n * hw);
          const int ho = (int)((uint32_t)rem / (uint32_t)p.Wo), wo = rem - ho * p.Wo;
          row = (n * p.H + (int64_t)ho * p.ds) * p.W + (int64_t)wo * p.ds;
        }
        if constexpr (AMODE == 3) {          // rows < 2^31: 32-bit unsigned divisions
          const uint32_t hw = (uint32_t)(p.Ho * p.Wo), r32 = (uint32_t)row;
          const int64_t n = r32 / hw;
          const int rem = (int)(r32 - (uint32_t)n * hw);
          const int ho = (int)((uint32_t)rem / (uint32_t)p.Wo), wo = rem - ho * p.Wo;
          const int pad = p.ks >> 1;
          const int hi0 = ho * p.ds - pad, wi0 = wo * p.ds - pad;
          uint32_t v = 0;
#pragma unroll
          for (int tr = 0; tr < 3; ++tr)
#pragma unroll
            for (int ts = 0; ts < 3; ++ts) {
              const bool ok = tr < p.ks && ts < p.ks && (unsigned)(hi0 + tr) < (unsigned)p.H &&
                              (unsigned)(wi0 + ts) < (unsigned)p.W;
              v |= (ok ? 1u : 0u) << (tr * p.ks + ts);
            }
          if (i == 0) avalid[h] = v;
          else avalid[h] |= v << 16;
          abase[h][i] =
              (uint32_t)(((((int64_t)n * p.H + hi0) * p.W + wi0) * p.Cin + sc * 8) * 2);
        }
        if constexpr (AMODE == 4) {
          // class row (n, ci, cj) reads dy (n, ci + di, cj + dj), di, dj in {0, 1}: bit
          // 2 di + dj set when that pixel is inside dy
          const uint32_t hw = (uint32_t)(p.Ho * p.Wo);
          const int rem = (int)((uint32_t)row % hw);
          const int ci = (int)((uint32_t)rem / (uint32_t)p.Wo), cj = rem - ci * p.Wo;
          const bool r1 = ci + 1 < p.Ho, c1 = cj + 1 < p.Wo;
          const uint32_t v = 1u | (c1 ? 2u : 0u) | (r1 ? 4u : 0u) | (r1 && c1 ? 8u : 0u);
          if (i == 0) avalid[h] = v;
          else avalid[h] |= v << 16;
          abase[h][i] = (uint32_t)((row * p.Cin + sc * 8) * 2);
        }
        if constexpr (AMODE == 2) {
          offa[h][i] = (uint32_t)row;
          int64_t row2 = row;
          if (p.ds > 1) {          // A2 = x [*, H, W, K2] read at the output row's stride pixel
            const uint32_t hw = (uint32_t)(p.Ho * p.Wo), r32 = (uint32_t)row;
            const int64_t n = r32 / hw;
            const int rem = (int)(r32 - (uint32_t)n * hw);
            const int ho = (int)((uint32_t)rem / (uint32_t)p.Wo), wo = rem - ho * p.Wo;
            row2 = (n * p.H + (int64_t)ho * p.ds) * p.W + (int64_t)wo * p.ds;
          }
          offa2[h][i] = (uint32_t)row2;
        } else {
          offa[h][i] = (uint32_t)((row * p.K + sc * 8) * 2);
        }
        const int col = nt * BN + (r >> 5) * 64 + h * 32 + (r & 31);
        offb[h][i] = (uint32_t)(((int64_t)col * (AMODE == 4 ? p.Kb : p.K) + sc * 8) * 2);
      }
    }
  };
  auto issue = [&](int slot, int buf, int kt) {
    // AMODE 3: the K tile's filter tap and channel block (wave-uniform)
    uint32_t toff = 0, boff = kt * (BK * 2);
    int tap = 0;
    if constexpr (AMODE == 3) {
      tap = cpow2 ? kt >> cshift : kt / csteps;
      const int c0 = (kt - tap * csteps) * BK;
      const int tr = p.ks == 3 ? (tap * 11) >> 5 : tap / p.ks;     // tap < 9: (11 t) >> 5 = t / 3
      const int ts = tap - tr * p.ks;
      toff = (uint32_t)(((tr * p.W + ts) * p.Cin + c0) * 2);
    }
    if constexpr (AMODE == 4) {
      // class tap t: row tap r' = ph ? 2 tR : 1 (dy row + tR), column s' = pw ? 2 tS : 1
      const int t = cpow2 ? kt >> cshift : kt / csteps;
      const int c0 = (kt - t * csteps) * BK;
      const int tR = p.pw ? t >> 1 : t, tS = p.pw ? t & 1 : 0;
      const int rr = p.ph ? 2 * tR : 1, ss = p.pw ? 2 * tS : 1;
      tap = 2 * tR + tS;                                   // the validity bit of (di, dj)
      toff = (uint32_t)(((tR * p.Wo + tS) * p.Cin + c0) * 2);
      boff = (uint32_t)(((rr * 3 + ss) * p.Cin + c0) * 2);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const char* src;
      if (slot >= 2) {
        src = reinterpret_cast<const char*>(p.B) + offb[slot - 2][i] + boff;
      } else if (AMODE == 3 || AMODE == 4) {
        // (padding taps: every lane reads the same zero chunk — the DMA writes lane * 16)
        src = ((avalid[slot] >> (tap + 16 * i)) & 1u)
                  ? reinterpret_cast<const char*>(p.A) + (uint32_t)(abase[slot][i] + toff)
                  : reinterpret_cast<const char*>(g_w256_zero);
      } else if (AMODE == 2) {
        src = kt < KT1 ? reinterpret_cast<const char*>(p.A) + offa[slot][i] * (uint32_t)(p.K1 * 2) +
                             scb + kt * (BK * 2)
                       : reinterpret_cast<const char*>(p.A2) +
                             (uint64_t)offa2[slot][i] * (uint32_t)((p.K - p.K1) * 2) + scb +
                             (kt - KT1) * (BK * 2);
      } else {
        src = reinterpret_cast<const char*>(p.A) + offa[slot][i] + kt * (BK * 2);
      }
      glds16(src, smem + buf * BUF + slot * HALF + (2 * w + i) * 512);
    }
  };

  f32x4v acc[4][8];                // [n tile][m tile]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2][2];   // A half frags [m tile][kk]; B [half][n tile][kk]
  const int rl = lane & 15, g = lane >> 4;

  auto read_a = [&](int buf, int h) {
    const __bf16* base = smem + buf * BUF + h * HALF;
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (h == 0 || b < MH1)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          af[b][kk] = *reinterpret_cast<const bf16x8*>(base + swz(wm * 64 + b * 16 + rl, kk * 4 + g));
  };
  auto read_b = [&](int buf, int h) {
    const __bf16* base = smem + buf * BUF + (2 + h) * HALF;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bfr[h][a][kk] = *reinterpret_cast<const bf16x8*>(base + swz(wn * 32 + a * 16 + rl, kk * 4 + g));
  };
  auto mma = [&](int qm, int qn) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (qm == 0 || b < MH1)
            acc[qn * 2 + a][qm * 4 + b] = mfma(bfr[qn][a][kk], af[b][kk], acc[qn * 2 + a][qm * 4 + b]);
    __builtin_amdgcn_s_setprio(0);
  };
  // C rows of this tile (+ the epilogue's statistics partial row (mt, wm)); no barrier:
  // wave group 0 runs it while group 1 (one barrier behind) is still in its last MFMA
  // phase, and the next tile's first K tile has already landed (waited before it: the
  // counted waits never have to account for the epilogue's own loads and stores).
  // 16-byte stores: v_permlane16_swap pairs n tiles (2q, 2q + 1) so that lane group g
  // holds 8 consecutive channels of its row — g = 0 / 2: tile 2q columns 0-7 / 8-15,
  // g = 1 / 3: tile 2q + 1 columns 0-7 / 8-15 (half the store instructions of the
  // fragment layout's 8-byte stores, 64-B row segments instead of 32-B).
  // C / xb row of GEMM row `row` (AMODE 4: the class pixel (n, 2i + ph, 2j + pw) of dx)
  auto out_row = [&](int64_t row) -> int64_t {
    if constexpr (AMODE != 4) {
      return row;
    } else {
      const uint32_t hw = (uint32_t)(p.Ho * p.Wo), r32 = (uint32_t)row;
      const uint32_t n = r32 / hw, rem = r32 - n * hw;
      const uint32_t ci = rem / (uint32_t)p.Wo, cj = rem - ci * (uint32_t)p.Wo;
      return ((int64_t)n * p.H + 2 * ci + p.ph) * p.W + 2 * cj + p.pw;
    }
  };
  auto epilogue = [&](int64_t tl) {
    const int64_t mt = tl / p.ntn;
    const int n0 = (int)(tl - mt * p.ntn) * BN;
    const int64_t m0 = mt * BMv;
    float s1[2][8], s2[2][8];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[q][j] = 0.f;
        s2[q][j] = 0.f;
      }
    // EPI 4: every BN-input row of the tile is loaded before the first store (the stores
    // may alias xb for the compiler: loads issued inside the loop each wait out a full
    // memory latency behind the previous store — ~100 us per 3x3 data gradient)
    // (in batches of 2 row blocks: 16 VGPRs — 4 blocks already spill at 256 VGPRs)
    uint4 xr[2][2];
#pragma unroll
    for (int b = 0; b < MT; ++b) {
      if (EPI == 4 && (b & 1) == 0) {
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
          const int64_t row = m0 + wm * (MT * 16) + (b + bb) * 16 + rl;
          const int64_t orow = out_row(row);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int c0 = n0 + wn * 64 + q * 32 + (g & 1) * 16 + (g >> 1) * 8;
            xr[bb][q] = (b + bb < MT && row < p.M) ? *reinterpret_cast<const uint4*>(p.xb + orow * N + c0)
                                  : uint4{0u, 0u, 0u, 0u};
          }
        }
      }
      const int64_t row = m0 + wm * (MT * 16) + b * 16 + rl;
      const bool in = row < p.M;
      const int64_t orow = out_row(row);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        f32x4v u = acc[2 * q][b], v = acc[2 * q + 1][b];
        if constexpr (BADD) {
          const int cu = n0 + wn * 64 + 2 * q * 16 + 4 * g;
          const f32x4v bu = *reinterpret_cast<const f32x4v*>(vecs + (cu - n0));
          const f32x4v bv = *reinterpret_cast<const f32x4v*>(vecs + (cu - n0) + 16);
          u += bu;
          v += bv;
        }
        uint32_t x0 = cvt_pk_bf16(u[0], u[1]), x1 = cvt_pk_bf16(u[2], u[3]);
        uint32_t y0 = cvt_pk_bf16(v[0], v[1]), y1 = cvt_pk_bf16(v[2], v[3]);
        const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        uint32_t o[4] = {r0[0], r1[0], r0[1], r1[1]};        // 8 consecutive channels
        const int c0 = n0 + wn * 64 + q * 32 + (g & 1) * 16 + (g >> 1) * 8;
        if constexpr (EPI == 1) {
          if (in) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float f = (j & 1) ? __uint_as_float(o[j >> 1] & 0xffff0000u)
                                      : __uint_as_float(o[j >> 1] << 16);
              const float d = f - vecs[c0 - n0 + j];
              s1[q][j] += d;
              s2[q][j] += d * d;
            }
          }
        }
        if constexpr (EPI == 4) {
          if (in) {
            const uint32_t xw[4] = {xr[b & 1][q].x, xr[b & 1][q].y, xr[b & 1][q].z, xr[b & 1][q].w};
            const float* mean = vecs + BN - n0;      // indexed by the global column c0 + j
            const float* scv = vecs + 2 * BN - n0;
            const float* biv = vecs + 3 * BN - n0;
            float dv[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float f = (j & 1) ? __uint_as_float(o[j >> 1] & 0xffff0000u)
                                      : __uint_as_float(o[j >> 1] << 16);
              const float xv = (j & 1) ? __uint_as_float(xw[j >> 1] & 0xffff0000u)
                                       : __uint_as_float(xw[j >> 1] << 16);
              const float d = __builtin_fmaf(xv, scv[c0 + j], biv[c0 + j]) > 0.f ? f : 0.f;
              dv[j] = d;
              s1[q][j] += d;
              s2[q][j] += d * (xv - mean[c0 + j]);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = cvt_pk_bf16(dv[2 * j], dv[2 * j + 1]);
          }
        }
        if (in && (EPI != 1 || p.C))        // EPI 1 with C == null: statistics only
          *reinterpret_cast<uint4*>(p.C + orow * N + c0) = uint4{o[0], o[1], o[2], o[3]};
      }
    }
    if constexpr (STATS) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            s1[q][j] += __shfl_xor(s1[q][j], o, kWave);
            s2[q][j] += __shfl_xor(s2[q][j], o, kWave);
          }
      // each (wave, lane group) owns its 16 columns of the accumulator: no other wave
      // touches them, so no barrier (fixed order: the workgroup's tiles in sequence)
      if (rl == 0) {
        float* ac = stacc + wm * 2 * BN;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int cl = wn * 64 + q * 32 + (g & 1) * 16 + (g >> 1) * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            ac[cl + j] += s1[q][j];
            ac[BN + cl + j] += s2[q][j];
          }
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
  };

  // this column tile's per-channel epilogue vectors -> LDS (EPI 1: shift; 4: badd, mean,
  // sc, bi; 6: badd); zeroed statistics accumulators
  if constexpr (NV > 0) {
    for (int c = tid; c < BN; c += NT) {
      const int gc = nw0 + c;
      if constexpr (EPI == 1) vecs[c] = p.shift ? p.shift[gc] : 0.f;
      if constexpr (BADD) vecs[c] = p.badd ? p.badd[gc] : 0.f;
      if constexpr (EPI == 4) {
        vecs[BN + c] = p.mean[gc];
        vecs[2 * BN + c] = p.sc[gc];
        vecs[3 * BN + c] = p.bi[gc];
      }
    }
    if constexpr (STATS)
      for (int c = tid; c < 4 * BN; c += NT) stacc[c] = 0.f;
  }
  // prologue: this workgroup's first tile, K tile 0, in the consumption order A0, B0,
  // B1, A1; A0 + B0 retired
  set_src(tile);
  issue(0, 0, 0);
  issue(2, 0, 0);
  issue(3, 0, 0);
  issue(1, 0, 0);
  wait_vm<4>();
  barrier();
  if (wm == 1) barrier();          // the one-barrier stagger of wave group 1

  // one stream of K tiles over all of this workgroup's output tiles: the next tile's
  // first K tile is staged during the current tile's last one (and its epilogue)
  int kt = 0, buf = 0;
  bool after = false;              // an epilogue ran since the last wait: nothing to retire
  int64_t ntile = tile + G;
  for (;;) {
    const bool last_k = kt + 1 == KT;
    const bool more = !last_k || ntile < p.ntiles;
    const int nkt = last_k ? 0 : kt + 1;
    const int nb = buf ^ 1;
    if (last_k && more) set_src(ntile);
    // Steady state: phase q issues one half-tile of the next K tile (A0', B0', B1', A1')
    // and retires, by a counted wait, the half-tile phase q + 1 reads.  Before a tile's
    // epilogue (last_k && more) the next tile's four half-tiles go out in phases 0-1 and
    // are all retired in phase 3 — the epilogue's stores are then never inside a count.
    // phase 0: quadrant (0, 0) — reads A0 + B0, retires B1
    read_a(buf, 0);
    read_b(buf, 0);
    if (!more) {
      wait_vm<2>();
    } else if (last_k) {
      issue(0, nb, nkt);
      issue(2, nb, nkt);
      wait_vm<4>();
    } else {
      issue(0, nb, nkt);
      if (!after) wait_vm<4>();
    }
    barrier();
    mma(0, 0);
    barrier();
    // phase 1: quadrant (0, 1) — reads B1, retires A1
    read_b(buf, 1);
    if (!more) {
      wait_vm<0>();
    } else if (last_k) {
      issue(3, nb, nkt);
      issue(1, nb, nkt);
      wait_vm<8>();
    } else {
      issue(2, nb, nkt);
      if (!after) wait_vm<4>();
    }
    barrier();
    mma(0, 1);
    barrier();
    // phase 2: quadrant (1, 1) — reads A1
    read_a(buf, 1);
    if (more && !last_k) issue(3, nb, nkt);
    barrier();
    mma(1, 1);
    barrier();
    // phase 3: quadrant (1, 0) — no reads (B0 kept in registers); retires A0' + B0'
    if (more) {
      if (last_k) {
        wait_vm<0>();
      } else {
        issue(1, nb, nkt);
        wait_vm<4>();
      }
    }
    barrier();
    mma(1, 0);
    barrier();
    buf = nb;
    after = last_k;
    if (last_k) {
      epilogue(tile);
      if (!more) break;
      tile = ntile;
      ntile += G;
      kt = 0;
    } else {
      ++kt;
    }
  }
  if (wm == 0) barrier();          // close the stagger: equal barrier counts
  if constexpr (STATS) {
    // partial row (tile0 / ntn) * 2 + wm: this wave's 64 columns of the column tile
    __syncthreads();
    float* pr = p.partial + ((tile0 / p.ntn) * 2 + wm) * 2 * N + nw0;
    const float* ac = stacc + wm * 2 * BN;
    pr[wn * 64 + lane] = ac[wn * 64 + lane];
    pr[N + wn * 64 + lane] = ac[BN + wn * 64 + lane];
  }
}

// ===========================================================================
// 1x1 weight gradient on the same pipeline:  dW[k][c] = sum_m DY[m][k] . X[m][c]
// (stride 1; C % 256 == 0, K % 256 == 0; DY's channels [k1, K) from DY2 when k1 < K —
// the BN fold's [dz | x]^T x Gram pass).  One workgroup = one 256 (c) x 256 (k) output
// tile over one contiguous pixel range (the reduction), fp32 partial [split][K][C] rows
// reduced in a fixed order by mv_conv.hip's wgrad1x1 reduce.  The reduction dimension is
// the pixel, the OUTER index of both NHWC operands, so the LDS images are pixel-major
// [64 px][128 ch] half-tiles (256-B rows) and both MFMA operands come from gfx950's
// transposed LDS reads (ds_read_b64_tr_b16: 4 consecutive pixels per read).  The 16-B
// chunk XOR (row & 3) | (row >> 3 & 1) << 2 (in 32-B pairs) spreads the rows one
// 32-lane half reads ({r..r+3, r+8..r+11}) over the 8 distinct 32-B bank windows.
// MFMA A = X^T (c rows), B = DY (k columns): a lane's accumulators are 4 consecutive
// c of one k — 16-byte partial stores.  Waves 2 (c) x 4 (k), 128 c x 64 k per wave, the
// 4-phase / one-barrier-stagger K loop of gemm256_kernel.
// ===========================================================================

struct WArgs {
  const __bf16* X;
  const __bf16* DY;
  const __bf16* DY2;
  float* partial;
  int64_t M;
  int C, K, k1, ntc, ntiles, ms;
  int64_t per;                  // 64-pixel chunks per split
  // TAPS = 9 (3x3, pad 1, stride ds): the output columns are (tap, c) — C = 9 Cx, a 256-
  // column tile is 256 channels of ONE tap (Cx % 256 == 0) — and X rows are gathered:
  // output pixel (n, ho, wo) reads input pixel (n, ho ds - 1 + r, wo ds - 1 + s)
  int Cx, H, W, Ho, Wo, ds;
  // magic multipliers ceil(2^32 / d) for d = Ho Wo and Wo (0: divide): q = umulhi(n, mg) is
  // exact for n d < 2^32 (the host checks M Ho Wo < 2^32) — the two per-row divisions were
  // ~2 VALU instructions per MFMA
  uint32_t mg_hw, mg_wo;
};

__device__ __forceinline__ int wf(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }

// The transposed reads are inline asm: hipcc treats the ds_read_tr builtin as aliasing
// the in-flight LDS DMA and drains vmcnt(0) before every one (the whole prefetch).  The
// consumer waits lgkmcnt(0) itself (mma_wait), ahead of the MFMAs.
typedef short s16x4w __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4w tr_asm(const __bf16* p) {
  s16x4w v;
  asm volatile("ds_read_b64_tr_b16 %0, %1"
               : "=v"(v)
               : "v"((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p));
  return v;
}
__device__ __forceinline__ bf16x8 trp(const __bf16* pa, const __bf16* pb) {
  const s16x4w a = tr_asm(pa);
  const s16x4w b = tr_asm(pb);
  typedef short s16x8w __attribute__((ext_vector_type(8)));
  const s16x8w o = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, o);
}

template <int TAPS>
__global__ __launch_bounds__(NT, 1) void wgrad256_kernel(WArgs p) {
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = w >> 2, wk = w & 3;
  // workgroups of one XCD share a pixel split (consecutive ids: same rows, other tiles)
  const int t = remap(blockIdx.x, gridDim.x);
  const int split = t / p.ntiles, tl = t - split * p.ntiles;
  const int c0 = (tl % p.ntc) * 256, k0 = (tl / p.ntc) * 256;
  // TAPS = 9: this tile's filter tap and its channel block in X
  const int tap = TAPS == 9 ? c0 / p.Cx : 0;
  const int xc0 = TAPS == 9 ? c0 - tap * p.Cx : c0;
  const int tr = tap / 3, ts = tap - 3 * (tap / 3);
  const int64_t mb = (int64_t)split * p.per * BK;
  int64_t me = mb + p.per * BK;
  me = me < p.M ? me : p.M;
  const int KT = me > mb ? (int)((me - mb + BK - 1) / BK) : 0;

  // staging: glds instruction i of a half-tile = pixel rows (2 w + i) * 4 + lane / 16 of
  // the 64-pixel chunk, LDS chunk lane % 16, holding logical chunk (lane % 16) ^ wf(row)
  const __bf16* srcb[4];         // per slot: channel base of instruction i = 0 / 1 (i adds 0)
  int choff[4][2];
  const bool dual = p.k1 < p.K && k0 >= p.k1;
  const __bf16* dyb = dual ? p.DY2 : p.DY;
  const int ldy = dual ? p.K - p.k1 : p.k1;
  const int kb = dual ? k0 - p.k1 : k0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (2 * w + i) * 4 + (lane >> 4);
    const int lc = (lane & 15) ^ wf(r);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      choff[h][i] = xc0 + 128 * (lc >> 3) + 64 * h + 8 * (lc & 7);         // X half h
      choff[2 + h][i] = kb + 64 * (lc >> 2) + 32 * h + 8 * (lc & 3);       // DY half h
    }
  }
  srcb[0] = srcb[1] = p.X;
  srcb[2] = srcb[3] = dyb;
  // TAPS = 9: the gathered X pixel of each staged row (-1: padding or past M), formed at
  // the K tile's first X half (slot 0) and reused by the second (slot 1)
  int64_t xpix[2] = {-1, -1};
  auto issue = [&](int slot, int buf, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int64_t row = mb + (int64_t)kt * BK + (2 * w + i) * 4 + (lane >> 4);
      const void* src;
      if (TAPS == 9 && slot < 2) {
        if (slot == 0) {
          xpix[i] = -1;
          if (row < me) {            // (M < 2^31: 32-bit unsigned divisions)
            const uint32_t r32 = (uint32_t)row, hw = (uint32_t)(p.Ho * p.Wo);
            const uint32_t n = p.mg_hw ? __umulhi(r32, p.mg_hw) : r32 / hw;
            const uint32_t rem = r32 - n * hw;
            const uint32_t ho = p.mg_wo ? __umulhi(rem, p.mg_wo) : rem / (uint32_t)p.Wo;
            const uint32_t wo = rem - ho * (uint32_t)p.Wo;
            const int hi = (int)ho * p.ds - 1 + tr, wi = (int)wo * p.ds - 1 + ts;
            if ((unsigned)hi < (unsigned)p.H && (unsigned)wi < (unsigned)p.W)
              xpix[i] = ((int64_t)n * p.H + hi) * p.W + wi;
          }
        }
        src = xpix[i] >= 0 ? (const void*)(p.X + xpix[i] * p.Cx + choff[slot][i])
                           : (const void*)(g_w256_zero + (lane & 15) * 4);
      } else {
        const int ld = slot < 2 ? p.C : ldy;
        src = row < me ? (const void*)(srcb[slot] + row * ld + choff[slot][i])
                       : (const void*)(g_w256_zero + (lane & 15) * 4);
      }
      glds16(src, smem + buf * BUF + slot * HALF + (2 * w + i) * 512);
    }
  };

  f32x4v acc[4][8];                // [k tile][c tile]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4v{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bfr[2][2][2];
  const int rl = lane & 15, g = lane >> 4;
  // transposed-read element offset of (pixel row r, half-local channel e)
  auto toff = [&](int r, int e) { return r * 128 + (((e >> 3) ^ wf(r)) << 3) + (e & 7); };
  auto read_a = [&](int buf, int h) {          // X^T fragments: c tiles of half h
    const __bf16* base = smem + buf * BUF + h * HALF;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r = 32 * kk + 8 * g + (rl >> 2), e = 64 * wc + 16 * b + 4 * (rl & 3);
        af[b][kk] = trp(base + toff(r, e), base + toff(r + 4, e));
      }
  };
  auto read_b = [&](int buf, int h) {          // DY fragments: k tiles of half h
    const __bf16* base = smem + buf * BUF + (2 + h) * HALF;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int r = 32 * kk + 8 * g + (rl >> 2), e = 32 * wk + 16 * a + 4 * (rl & 3);
        bfr[h][a][kk] = trp(base + toff(r, e), base + toff(r + 4, e));
      }
  };
  auto mma = [&](int qc, int qk) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // this phase's asm reads
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[qk * 2 + a][qc * 4 + b] = mfma(af[b][kk], bfr[qk][a][kk], acc[qk * 2 + a][qc * 4 + b]);
    __builtin_amdgcn_s_setprio(0);
  };

  if (KT > 0) {
    issue(0, 0, 0);
    issue(2, 0, 0);
    issue(3, 0, 0);
    issue(1, 0, 0);
    wait_vm<4>();
    barrier();
    if (wc == 1) barrier();
    for (int kt = 0; kt < KT; ++kt) {
      const int buf = kt & 1, nb = buf ^ 1;
      const bool more = kt + 1 < KT;
      read_a(buf, 0);
      read_b(buf, 0);
      if (more) {
        issue(0, nb, kt + 1);
        wait_vm<4>();
      } else {
        wait_vm<2>();
      }
      barrier();
      mma(0, 0);
      barrier();
      read_b(buf, 1);
      if (more) {
        issue(2, nb, kt + 1);
        wait_vm<4>();
      } else {
        wait_vm<0>();
      }
      barrier();
      mma(0, 1);
      barrier();
      read_a(buf, 1);
      if (more) issue(3, nb, kt + 1);
      barrier();
      mma(1, 1);
      barrier();
      if (more) {
        issue(1, nb, kt + 1);
        wait_vm<4>();
      }
      barrier();
      mma(1, 0);
      barrier();
    }
    if (wc == 0) barrier();
  }
  // partial[split][k][c .. c + 3] (zeros for an empty split)
  float* pp = p.partial + (int64_t)split * p.K * p.C;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const int k = k0 + 64 * wk + 16 * a + rl, c = c0 + 128 * wc + 16 * b + 4 * g;
      *reinterpret_cast<f32x4v*>(pp + (int64_t)k * p.C + c) = acc[a][b];
    }
}

}  // namespace g256
}  // namespace mv

static int g256_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v < 1)
      v = 256;
    return v;
  }();
  return n;
}

// 224-row blocks when they tile M exactly and there is one column tile (N = 256: ResNet-50
// layer 3's 1024 -> 256 1x1 convs, 251 -> 238 us; with 2+ column tiles 256 rows measured
// faster, and the 3x3 convs' long K leaves them level) — see gemm256_kernel's MT;
// MIVOD_G256_BM=256 forces 256
static int g256_bm(int64_t M, int N) {
  static const bool allow224 = [] {
    const char* e = std::getenv("MIVOD_G256_BM");
    return !(e && std::atoi(e) == 256);
  }();
  return allow224 && N == 256 && M % 224 == 0 ? 224 : 256;
}

bool mv_gemm256_supported(int64_t M, int N, int K) {
  return M > 0 && N % 256 == 0 && K % 64 == 0 && K >= 64 &&
         (M + 255) / 256 * (N / 256) < (int64_t(1) << 31) && M * K * 2 < (int64_t(1) << 32) &&
         (int64_t)N * K * 2 < (int64_t(1) << 32);
}

// persistent grid: one workgroup per CU, a multiple of the column-tile count so that every
// workgroup keeps one column tile (its statistics accumulate on chip)
static int64_t g256_grid(int64_t M, int N) {
  const int64_t ntn = N / mv::g256::BN, bm = g256_bm(M, N);
  const int64_t ntiles = (M + bm - 1) / bm * ntn, cus = g256_cus();
  const int64_t g = (ntiles < cus ? ntiles : cus) / ntn * ntn;
  return g > ntn ? g : ntn;
}

// two statistics rows (one per M wave group) per row group of G / ntn workgroups
int64_t mv_gemm256_partials(int64_t M, int N) {
  return 2 * (g256_grid(M, N) / (N / mv::g256::BN));
}

template <int EPI, int AMODE>
static void g256_launch(mv::g256::Args a, hipStream_t st) {
  using namespace mv::g256;
  const int bm = g256_bm(a.M, a.N);
  a.ntn = a.N / BN;
  a.ntiles = (a.M + bm - 1) / bm * a.ntn;
  const dim3 grid((unsigned)g256_grid(a.M, a.N));
  if (bm == 224)
    hipLaunchKernelGGL((gemm256_kernel<EPI, AMODE, 7>), grid, dim3(NT), 0, st, a);
  else
    hipLaunchKernelGGL((gemm256_kernel<EPI, AMODE, 8>), grid, dim3(NT), 0, st, a);
}

bool mv_gemm256_nt(const void* A, const void* B, void* C, int64_t M, int N, int K,
                   const float* shift, float* partial, hipStream_t st) {
  using namespace mv::g256;
  if (!mv_gemm256_supported(M, N, K) || (partial && N > kVecFloats) || (!C && !partial))
    return false;
  Args a{};
  a.A = (const __bf16*)A;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.shift = shift;
  a.partial = partial;
  if (partial) g256_launch<1, 0>(a, st);
  else g256_launch<0, 0>(a, st);
  return true;
}

bool mv_gemm256_strided(const void* X, const void* B, void* C, int Nb, int H, int W, int K, int N,
                        int ds, const float* shift, float* partial, hipStream_t st) {
  using namespace mv::g256;
  const int Ho = (H - 1) / ds + 1, Wo = (W - 1) / ds + 1;
  const int64_t M = (int64_t)Nb * Ho * Wo;
  if (ds < 1 || !mv_gemm256_supported(M, N, K) || (partial && N > kVecFloats) ||
      (int64_t)Nb * H * W * K * 2 >= (int64_t(1) << 32))
    return false;
  Args a{};
  a.A = (const __bf16*)X;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.ds = ds;
  a.H = H;
  a.W = W;
  a.Ho = Ho;
  a.Wo = Wo;
  a.shift = shift;
  a.partial = partial;
  if (partial) g256_launch<1, 1>(a, st);
  else g256_launch<0, 1>(a, st);
  return true;
}

bool mv_gemm256_dual(const void* A1, const void* A2, const void* B, const float* badd, void* D,
                     int64_t M, int K1, int K2, int N, const void* xb, const float* mean,
                     const float* scale, const float* bias, float* partial, hipStream_t st,
                     int ds, int H, int W) {
  using namespace mv::g256;
  const int K = K1 + K2;
  if (K1 % 64 || K2 % 64 || !mv_gemm256_supported(M, N, K) || 4 * N > kVecFloats) return false;
  Args a{};
  if (ds > 1) {       // A2 = [Nb, H, W, K2] read at the stride grid (M = Nb Ho Wo rows)
    a.Ho = (H - 1) / ds + 1;
    a.Wo = (W - 1) / ds + 1;
    const int64_t hw = (int64_t)a.Ho * a.Wo;
    if (H < 1 || W < 1 || M % hw != 0 || (M / hw) * H * W * (int64_t)K2 * 2 >= (int64_t(1) << 32))
      return false;
    a.ds = ds;
    a.H = H;
    a.W = W;
  }
  a.A = (const __bf16*)A1;
  a.A2 = (const __bf16*)A2;
  a.B = (const __bf16*)B;
  a.C = (__bf16*)D;
  a.M = M;
  a.N = N;
  a.K = K;
  a.K1 = K1;
  a.badd = badd;
  a.xb = (const __bf16*)xb;
  a.mean = mean;
  a.sc = scale;
  a.bi = bias;
  a.partial = partial;
  if (partial) g256_launch<4, 2>(a, st);
  else g256_launch<6, 2>(a, st);
  return true;
}

// ---------------------------------------------------------------- implicit ks x ks conv
bool mv_conv256_supported(int N, int H, int W, int Cin, int Cout, int ks, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t M = (int64_t)N * Ho * Wo;
  // (A rows are 32-bit byte offsets: the input must stay below 4 GB)
  return (ks == 1 || ks == 3) && stride >= 1 && stride <= 2 && Cin % 64 == 0 && Cin > 0 &&
         (int64_t)N * H * W * Cin * 2 < (int64_t(1) << 32) &&
         Cout % 256 == 0 && Cout <= mv::g256::kVecFloats / 4 && M > 0 &&
         (M + 255) / 256 * (Cout / 256) < (int64_t(1) << 31) &&
         (int64_t)Cout * ks * ks * Cin * 2 < (int64_t(1) << 32);
}

bool mv_conv256(const void* X, const void* Wt, void* Y, int Nb, int H, int W, int Cin, int Cout,
                int ks, int stride, const float* shift, float* partial, const void* bn_x,
                const float* bn_vec, hipStream_t st) {
  using namespace mv::g256;
  if (!mv_conv256_supported(Nb, H, W, Cin, Cout, ks, stride) || (bn_x && !partial)) return false;
  Args a{};
  a.A = (const __bf16*)X;
  a.B = (const __bf16*)Wt;
  a.C = (__bf16*)Y;
  a.Ho = (H - 1) / stride + 1;
  a.Wo = (W - 1) / stride + 1;
  a.M = (int64_t)Nb * a.Ho * a.Wo;
  a.N = Cout;
  a.K = ks * ks * Cin;
  a.ds = stride;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.ks = ks;
  a.shift = shift;
  a.partial = partial;
  if (bn_x) {         // data gradient + the producing BN+ReLU's backward reduce ([4][Cout] vec)
    a.xb = (const __bf16*)bn_x;
    a.mean = bn_vec;
    a.sc = bn_vec + 2 * Cout;
    a.bi = bn_vec + 3 * Cout;
    g256_launch<4, 3>(a, st);
  } else if (partial) {
    g256_launch<1, 3>(a, st);
  } else {
    g256_launch<0, 3>(a, st);
  }
  return true;
}

// ---------------------------------------------------------------- stride-2 3x3 data gradient
// (AMODE 4): four launches, one per output parity class, each a gather GEMM over that
// class's taps.  Cin = dx channels (the GEMM's N), Cout = dy channels.
bool mv_dgrad256_s2_supported(int Nb, int H, int W, int Cin, int Cout) {
  if (Nb < 1 || H < 2 || W < 2 || (H & 1) || (W & 1)) return false;
  const int64_t M = (int64_t)Nb * (H / 2) * (W / 2);
  return Cin % 256 == 0 && Cin <= mv::g256::kVecFloats / 4 && Cout % 64 == 0 && Cout > 0 &&
         M * Cout * 2 < (int64_t(1) << 32) && (M + 255) / 256 * (Cin / 256) < (int64_t(1) << 31) &&
         (int64_t)Cin * 9 * Cout * 2 < (int64_t(1) << 32) && M * 4 < (int64_t(1) << 31);
}

bool mv_dgrad256_s2(const void* dy, const void* wt, void* dx, int Nb, int H, int W, int Cin,
                    int Cout, hipStream_t st) {
  using namespace mv::g256;
  if (!mv_dgrad256_s2_supported(Nb, H, W, Cin, Cout)) return false;
  Args a{};
  a.A = (const __bf16*)dy;
  a.B = (const __bf16*)wt;
  a.C = (__bf16*)dx;
  a.H = H;
  a.W = W;
  a.Ho = H / 2;
  a.Wo = W / 2;
  a.M = (int64_t)Nb * a.Ho * a.Wo;
  a.N = Cin;
  a.Cin = Cout;
  a.Kb = 9 * Cout;
  a.ds = 2;
  // the 4-tap class first: the later, shorter launches fill in behind it.  (A BN-reduce
  // epilogue here measured slower than the separate reduce pass: the BN-input reads of the
  // scattered class rows are latency-bound, 683 -> 1081 us for ResNet-50's layer3 shape.)
  for (int c = 3; c >= 0; --c) {
    a.ph = c >> 1;
    a.pw = c & 1;
    a.K = (1 + a.ph) * (1 + a.pw) * Cout;
    g256_launch<0, 4>(a, st);
  }
  return true;
}

// ---------------------------------------------------------------- 1x1 weight gradient
bool mv_wgrad256_supported(int64_t M, int C, int K, int k1) {
  return M > 0 && C % 256 == 0 && K % 256 == 0 && k1 > 0 && k1 <= K && k1 % 256 == 0 &&
         M < (int64_t(1) << 31);
}

static void w256_split(int64_t M, int C, int K, int* ms, int64_t* per) {
  const int ntiles = (C / 256) * (K / 256);
  const int64_t chunks = (M + 63) / 64;
  int m = g256_cus() / ntiles;
  if (m < 1) m = 1;
  if (m > chunks) m = (int)chunks;
  *per = (chunks + m - 1) / m;
  *ms = (int)((chunks + *per - 1) / *per);
}

int64_t mv_wgrad256_splits(int64_t M, int C, int K) {
  int ms;
  int64_t per;
  w256_split(M, C, K, &ms, &per);
  return ms;
}

bool mv_wgrad256(const void* X, const void* DY, const void* DY2, float* partial, int64_t M, int C,
                 int K, int k1, hipStream_t st) {
  using namespace mv::g256;
  if (!mv_wgrad256_supported(M, C, K, k1) || (k1 < K && !DY2)) return false;
  WArgs a{};
  a.X = (const __bf16*)X;
  a.DY = (const __bf16*)DY;
  a.DY2 = (const __bf16*)DY2;
  a.partial = partial;
  a.M = M;
  a.C = C;
  a.K = K;
  a.k1 = k1;
  a.ntc = C / 256;
  a.ntiles = (C / 256) * (K / 256);
  w256_split(M, C, K, &a.ms, &a.per);
  hipLaunchKernelGGL(wgrad256_kernel<1>, dim3((unsigned)(a.ntiles * a.ms)), dim3(NT), 0, st, a);
  return true;
}

// ---------------------------------------------------------------- 3x3 weight gradient
bool mv_wgrad256_3x3_supported(int N, int H, int W, int C, int K, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  return N > 0 && (stride == 1 || stride == 2) && C % 256 == 0 && K % 256 == 0 &&
         mv_wgrad256_supported((int64_t)N * Ho * Wo, 9 * C, K, K);
}

int64_t mv_wgrad256_3x3_splits(int N, int H, int W, int C, int K, int stride) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  return mv_wgrad256_splits((int64_t)N * Ho * Wo, 9 * C, K);
}

bool mv_wgrad256_3x3(const void* X, const void* DY, float* partial, int N, int H, int W, int C,
                     int K, int stride, hipStream_t st) {
  using namespace mv::g256;
  if (!mv_wgrad256_3x3_supported(N, H, W, C, K, stride)) return false;
  WArgs a{};
  a.X = (const __bf16*)X;
  a.DY = (const __bf16*)DY;
  a.partial = partial;
  a.Ho = (H - 1) / stride + 1;
  a.Wo = (W - 1) / stride + 1;
  a.M = (int64_t)N * a.Ho * a.Wo;
  a.C = 9 * C;
  a.K = K;
  a.k1 = K;
  a.Cx = C;
  a.H = H;
  a.W = W;
  a.ds = stride;
  a.ntc = a.C / 256;
  a.ntiles = (a.C / 256) * (K / 256);
  {
    const uint64_t hw = (uint64_t)a.Ho * a.Wo;
    auto magic = [](uint64_t d) { return (uint32_t)(((uint64_t(1) << 32) + d - 1) / d); };
    if (hw >= 2 && a.Wo >= 2 && (uint64_t)a.M * hw < (uint64_t(1) << 32)) {
      a.mg_hw = magic(hw);
      a.mg_wo = magic((uint64_t)a.Wo);
    }
  }
  w256_split(a.M, a.C, K, &a.ms, &a.per);
  hipLaunchKernelGGL(wgrad256_kernel<9>, dim3((unsigned)(a.ntiles * a.ms)), dim3(NT), 0, st, a);
  return true;
}
