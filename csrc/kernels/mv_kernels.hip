// mivod hand-written CDNA4 (gfx950) kernels for the data-parallel gradient path.
//
// Replaces, MI355X-first, what the reference's engine (horovod 0.18.1, used by
// /root/reference/mnist_keras.py:87 and tensorflow2_keras_mnist.py:58) does with
// per-tensor cudaMemcpyAsync + TF elementwise ops + NCCL-side scaling:
//   K1/K2  mv_mt_copy        multi-tensor fusion-buffer pack / unpack, fused cast
//                            (fp32/bf16/fp16 compression) and pre/post scale
//   K4/K5  mv_flat_cast      flat compress / decompress / scale of a bucket
//   K6     mv_{sgd,adam,adadelta}_flat, mv_lars_*  fused optimizer steps that
//                            run directly on a reduced flat gradient bucket,
//                            fp32 master weights + bf16 model copy written in
//                            the same pass (grad read once)
//   K8     mv_seg_dot3 / mv_adasum_combine  Adasum per-tensor Gram terms and
//                            the (1-d/2|a|^2)a + (1-d/2|b|^2)b merge
// See SURVEY.md §2.5.b for the inventory.  All kernels are HBM-bound: the design
// goal is 16-byte lanes, >=1k workgroups per launch and a single pass over
// every byte (no separate scale / cast / unscale passes).
#include "mv_common.h"
#include "mv_kernels.h"

namespace mv {

// -------------------------------------------------------------------------
// K1/K2: multi-tensor pack / unpack.
// The tensor table travels in the kernel arguments (no H2D copy, graph-capture
// safe).  Workgroup b finds its tensor by a uniform binary search over the
// chunk prefix sums (scalar loads from the kernarg segment).
// -------------------------------------------------------------------------
template <typename TS, typename TD>
__device__ __forceinline__ void copy_range(const TS* __restrict__ s, TD* __restrict__ d,
                                           int64_t n, float scale, int* found_nonfinite) {
  bool bad = false;
  if (aligned16(s) && aligned16(d)) {
    const int64_t nv = n / kVec;
    for (int64_t i = threadIdx.x; i < nv; i += kBlock) {
      float v[8];
      load8(s + i * kVec, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] *= scale;
        if (found_nonfinite) bad |= !__builtin_isfinite(v[j]);
      }
      store8(d + i * kVec, v);
    }
    for (int64_t i = nv * kVec + threadIdx.x; i < n; i += kBlock) {
      float x = ld1(s + i) * scale;
      if (found_nonfinite) bad |= !__builtin_isfinite(x);
      st1(d + i, x);
    }
  } else {
    for (int64_t i = threadIdx.x; i < n; i += kBlock) {
      float x = ld1(s + i) * scale;
      if (found_nonfinite) bad |= !__builtin_isfinite(x);
      st1(d + i, x);
    }
  }
  if (found_nonfinite && __any(bad) && (threadIdx.x & 63) == 0) atomicOr(found_nonfinite, 1);
}

template <typename TT, typename TF, bool TO_FLAT>
__global__ __launch_bounds__(kBlock) void mt_copy_kernel(MtArgs args, TF* __restrict__ flat,
                                                          float scale, int* found_nonfinite) {
  const int b = blockIdx.x;
  // uniform binary search: largest t with chunk_start[t] <= b
  int lo = 0, hi = args.ntensors - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (args.chunk_start[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  const int64_t c = b - args.chunk_start[t];
  const int64_t begin = c * kChunk;
  const int64_t numel = args.numel[t];
  const int64_t n = (numel - begin < kChunk) ? (numel - begin) : kChunk;
  if (n <= 0) return;
  TT* tp = reinterpret_cast<TT*>(args.ptr[t]) + begin;
  TF* fp = flat + args.flat_off[t] + begin;
  if constexpr (TO_FLAT) copy_range<TT, TF>(tp, fp, n, scale, found_nonfinite);
  else copy_range<TF, TT>(fp, tp, n, scale, found_nonfinite);
}

template <typename TT, typename TF>
static void launch_mt(const MtArgs& a, void* flat, bool to_flat, float scale, int* nf,
                      hipStream_t st) {
  const int nblocks = a.chunk_start[a.ntensors];
  if (nblocks <= 0) return;
  if (to_flat)
    hipLaunchKernelGGL((mt_copy_kernel<TT, TF, true>), dim3(nblocks), dim3(kBlock), 0, st, a,
                       reinterpret_cast<TF*>(flat), scale, nf);
  else
    hipLaunchKernelGGL((mt_copy_kernel<TT, TF, false>), dim3(nblocks), dim3(kBlock), 0, st, a,
                       reinterpret_cast<TF*>(flat), scale, nf);
}

template <typename TT>
static void dispatch_flat(const MtArgs& a, void* flat, int flat_dtype, bool to_flat, float scale,
                          int* nf, hipStream_t st) {
  switch (flat_dtype) {
    case F32: launch_mt<TT, float>(a, flat, to_flat, scale, nf, st); break;
    case BF16: launch_mt<TT, __bf16>(a, flat, to_flat, scale, nf, st); break;
    case F16: launch_mt<TT, _Float16>(a, flat, to_flat, scale, nf, st); break;
  }
}

}  // namespace mv

using namespace mv;

void mv_launch_mt_copy(const MtArgs& a, int tensor_dtype, void* flat, int flat_dtype,
                       bool to_flat, float scale, int* found_nonfinite, hipStream_t st) {
  switch (tensor_dtype) {
    case F32: dispatch_flat<float>(a, flat, flat_dtype, to_flat, scale, found_nonfinite, st); break;
    case BF16: dispatch_flat<__bf16>(a, flat, flat_dtype, to_flat, scale, found_nonfinite, st); break;
    case F16: dispatch_flat<_Float16>(a, flat, flat_dtype, to_flat, scale, found_nonfinite, st); break;
  }
}

// -------------------------------------------------------------------------
// K4/K5: flat cast + scale (compress / decompress / average in place)
// -------------------------------------------------------------------------
namespace mv {
template <typename TS, typename TD>
__global__ __launch_bounds__(kBlock) void flat_cast_kernel(const TS* __restrict__ s,
                                                            TD* __restrict__ d, int64_t n,
                                                            float scale, int* nf) {
  const int64_t begin = (int64_t)blockIdx.x * kChunk;
  const int64_t cnt = (n - begin < kChunk) ? (n - begin) : kChunk;
  copy_range<TS, TD>(s + begin, d + begin, cnt, scale, nf);
}
template <typename TS>
static void flat_cast_d(const void* s, void* d, int dd, int64_t n, float scale, int* nf,
                        hipStream_t st) {
  const int nb = (int)((n + kChunk - 1) / kChunk);
  if (nb <= 0) return;
  const TS* sp = reinterpret_cast<const TS*>(s);
  switch (dd) {
    case F32: hipLaunchKernelGGL((flat_cast_kernel<TS, float>), dim3(nb), dim3(kBlock), 0, st, sp, (float*)d, n, scale, nf); break;
    case BF16: hipLaunchKernelGGL((flat_cast_kernel<TS, __bf16>), dim3(nb), dim3(kBlock), 0, st, sp, (__bf16*)d, n, scale, nf); break;
    case F16: hipLaunchKernelGGL((flat_cast_kernel<TS, _Float16>), dim3(nb), dim3(kBlock), 0, st, sp, (_Float16*)d, n, scale, nf); break;
  }
}
}  // namespace mv

void mv_launch_flat_cast(const void* src, int sd, void* dst, int dd, int64_t n, float scale,
                         int* found_nonfinite, hipStream_t st) {
  switch (sd) {
    case F32: flat_cast_d<float>(src, dst, dd, n, scale, found_nonfinite, st); break;
    case BF16: flat_cast_d<__bf16>(src, dst, dd, n, scale, found_nonfinite, st); break;
    case F16: flat_cast_d<_Float16>(src, dst, dd, n, scale, found_nonfinite, st); break;
  }
}

// -------------------------------------------------------------------------
// Overflow guard: read-only non-finite scan of a REDUCED bucket.  A non-finite
// contribution of any rank (or an overflow inside the reduction) propagates
// into the reduced sum, and every rank holds the same reduced bits, so every
// rank sets the same flag without another collective.
// -------------------------------------------------------------------------
namespace mv {
template <typename T>
__global__ __launch_bounds__(kBlock) void nonfinite_scan_kernel(const T* __restrict__ x, int64_t n,
                                                                 int* __restrict__ flag) {
  const int64_t begin = (int64_t)blockIdx.x * kChunk;
  const int64_t cnt = (n - begin < kChunk) ? (n - begin) : kChunk;
  const T* s = x + begin;
  bool bad = false;
  if (aligned16(s)) {
    const int64_t nv = cnt / kVec;
    for (int64_t i = threadIdx.x; i < nv; i += kBlock) {
      float v[8];
      load8(s + i * kVec, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) bad |= !__builtin_isfinite(v[j]);
    }
    for (int64_t i = nv * kVec + threadIdx.x; i < cnt; i += kBlock) bad |= !__builtin_isfinite(ld1(s + i));
  } else {
    for (int64_t i = threadIdx.x; i < cnt; i += kBlock) bad |= !__builtin_isfinite(ld1(s + i));
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}
}  // namespace mv

void mv_launch_nonfinite_scan(const void* x, int dt, int64_t n, int* flag, hipStream_t st) {
  const int nb = (int)((n + kChunk - 1) / kChunk);
  if (nb <= 0) return;
  switch (dt) {
    case F32: hipLaunchKernelGGL((nonfinite_scan_kernel<float>), dim3(nb), dim3(kBlock), 0, st, (const float*)x, n, flag); break;
    case BF16: hipLaunchKernelGGL((nonfinite_scan_kernel<__bf16>), dim3(nb), dim3(kBlock), 0, st, (const __bf16*)x, n, flag); break;
    case F16: hipLaunchKernelGGL((nonfinite_scan_kernel<_Float16>), dim3(nb), dim3(kBlock), 0, st, (const _Float16*)x, n, flag); break;
  }
}

// -------------------------------------------------------------------------
// K6: fused optimizers on flat buckets.
// grad (TG: the wire / bucket dtype), fp32 master + fp32 state, and an optional
// low-precision model copy (TP) written in the same pass.  Arena segments are
// 64-element aligned, so the vector path covers everything but a final tail.
// -------------------------------------------------------------------------
namespace mv {

struct SgdHp { float lr, momentum, dampening, wd, gscale; int nesterov, first; };
// Graph-replayable hyperparameters: when ``dyn`` is non-null the kernel reads the
// per-step values from device memory instead of its by-value launch arguments,
// so a captured HIP graph keeps following LR schedules and step counters:
// dyn = [lr, first (0/1), bias_correction1, bias_correction2] (fp32, 16 bytes),
// refreshed on the stream before every replay (mivod/torch/graphs.py).
struct AdamHp { float lr, b1, b2, eps, wd, gscale, bc1, bc2; int adamw, keras_eps; };
struct AdadeltaHp { float lr, rho, eps, wd, gscale; };

template <typename TP>
__device__ __forceinline__ void store_model(TP* p, const float (&v)[8]) { store8(p, v); }

template <typename TG, typename TP>
__global__ __launch_bounds__(kBlock) void sgd_flat_kernel(const TG* __restrict__ g,
                                                           float* __restrict__ w,
                                                           float* __restrict__ mom,
                                                           TP* __restrict__ model, int64_t n,
                                                           SgdHp hp,
                                                           const float* __restrict__ dyn,
                                                           const int* __restrict__ skip) {
  if (skip && *skip) return;   // overflow guard: every rank skips this step identically
  if (dyn) { hp.lr = dyn[0]; hp.first = dyn[1] != 0.f; }
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  for (int64_t i = base + threadIdx.x * kVec; i < base + kChunk; i += kBlock * kVec) {
    if (i + kVec <= n) {
      float gv[8], wv[8], mv_[8];
      load8(g + i, gv);
      load8(w + i, wv);
      if (mom) load8(mom + i, mv_);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = gv[j] * hp.gscale + hp.wd * wv[j];
        if (mom) {
          float b = hp.first ? d : hp.momentum * mv_[j] + (1.f - hp.dampening) * d;
          mv_[j] = b;
          d = hp.nesterov ? d + hp.momentum * b : b;
        }
        wv[j] -= hp.lr * d;
      }
      store8(w + i, wv);
      if (mom) store8(mom + i, mv_);
      if (model) store_model(model + i, wv);
    } else {
      for (int64_t k = i; k < n && k < i + kVec; ++k) {
        float wk = w[k];
        float d = ld1(g + k) * hp.gscale + hp.wd * wk;
        if (mom) {
          float b = hp.first ? d : hp.momentum * mom[k] + (1.f - hp.dampening) * d;
          mom[k] = b;
          d = hp.nesterov ? d + hp.momentum * b : b;
        }
        wk -= hp.lr * d;
        w[k] = wk;
        if (model) st1(model + k, wk);
      }
    }
  }
}

template <typename TG, typename TP>
__global__ __launch_bounds__(kBlock) void adam_flat_kernel(const TG* __restrict__ g,
                                                            float* __restrict__ w,
                                                            float* __restrict__ m,
                                                            float* __restrict__ v,
                                                            TP* __restrict__ model, int64_t n,
                                                            AdamHp hp,
                                                            const float* __restrict__ dyn,
                                                            const int* __restrict__ skip) {
  if (skip && *skip) return;
  if (dyn) { hp.lr = dyn[0]; hp.bc1 = dyn[2]; hp.bc2 = dyn[3]; }
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  const float step = hp.lr / hp.bc1;
  const float rbc2 = 1.f / sqrtf(hp.bc2);
  for (int64_t i = base + threadIdx.x * kVec; i < base + kChunk; i += kBlock * kVec) {
    const int cnt = (i + kVec <= n) ? kVec : (i < n ? (int)(n - i) : 0);
    if (cnt == 0) break;
    float gv[8], wv[8], mv_[8], vv[8];
    if (cnt == kVec) {
      load8(g + i, gv); load8(w + i, wv); load8(m + i, mv_); load8(v + i, vv);
    } else {
      for (int j = 0; j < kVec; ++j) {
        gv[j] = j < cnt ? ld1(g + i + j) : 0.f; wv[j] = j < cnt ? w[i + j] : 0.f;
        mv_[j] = j < cnt ? m[i + j] : 0.f; vv[j] = j < cnt ? v[i + j] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gr = gv[j] * hp.gscale;
      if (!hp.adamw) gr += hp.wd * wv[j];
      mv_[j] = hp.b1 * mv_[j] + (1.f - hp.b1) * gr;
      vv[j] = hp.b2 * vv[j] + (1.f - hp.b2) * gr * gr;
      if (hp.adamw) wv[j] *= (1.f - hp.lr * hp.wd);
      // torch: m_hat / (sqrt(v_hat) + eps); Keras/TF: lr*sqrt(bc2)/bc1 * m / (sqrt(v) + eps)
      float denom = hp.keras_eps ? (sqrtf(vv[j]) + hp.eps) * rbc2 : sqrtf(vv[j]) * rbc2 + hp.eps;
      wv[j] -= step * mv_[j] / denom;
    }
    if (cnt == kVec) {
      store8(w + i, wv); store8(m + i, mv_); store8(v + i, vv);
      if (model) store_model(model + i, wv);
    } else {
      for (int j = 0; j < cnt; ++j) {
        w[i + j] = wv[j]; m[i + j] = mv_[j]; v[i + j] = vv[j];
        if (model) st1(model + i + j, wv[j]);
      }
    }
  }
}

template <typename TG, typename TP>
__global__ __launch_bounds__(kBlock) void adadelta_flat_kernel(const TG* __restrict__ g,
                                                                float* __restrict__ w,
                                                                float* __restrict__ sq,
                                                                float* __restrict__ acc,
                                                                TP* __restrict__ model, int64_t n,
                                                                AdadeltaHp hp,
                                                                const float* __restrict__ dyn,
                                                                const int* __restrict__ skip) {
  if (skip && *skip) return;
  if (dyn) hp.lr = dyn[0];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  for (int64_t i = base + threadIdx.x * kVec; i < base + kChunk; i += kBlock * kVec) {
    const int cnt = (i + kVec <= n) ? kVec : (i < n ? (int)(n - i) : 0);
    if (cnt == 0) break;
    float gv[8], wv[8], sv[8], av[8];
    if (cnt == kVec) {
      load8(g + i, gv); load8(w + i, wv); load8(sq + i, sv); load8(acc + i, av);
    } else {
      for (int j = 0; j < kVec; ++j) {
        gv[j] = j < cnt ? ld1(g + i + j) : 0.f; wv[j] = j < cnt ? w[i + j] : 0.f;
        sv[j] = j < cnt ? sq[i + j] : 0.f; av[j] = j < cnt ? acc[i + j] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gr = gv[j] * hp.gscale + hp.wd * wv[j];
      sv[j] = hp.rho * sv[j] + (1.f - hp.rho) * gr * gr;
      float delta = sqrtf(av[j] + hp.eps) / sqrtf(sv[j] + hp.eps) * gr;
      av[j] = hp.rho * av[j] + (1.f - hp.rho) * delta * delta;
      wv[j] -= hp.lr * delta;
    }
    if (cnt == kVec) {
      store8(w + i, wv); store8(sq + i, sv); store8(acc + i, av);
      if (model) store_model(model + i, wv);
    } else {
      for (int j = 0; j < cnt; ++j) {
        w[i + j] = wv[j]; sq[i + j] = sv[j]; acc[i + j] = av[j];
        if (model) st1(model + i + j, wv[j]);
      }
    }
  }
}

// ---- segmented reductions (LARS norms, Adasum Gram terms) ----
// Chunk table (static per bucket layout): chunk c covers [begin[c], begin[c]+len[c])
// of segment seg[c]; chunks never straddle segments.  Pass 1 writes one partial
// per chunk (block-level, fixed-order => deterministic, so every rank computes
// bit-identical coefficients); pass 2 sums a segment's partials in chunk order.
template <typename TA, typename TB, int MODE>  // MODE 0: (a.a, b.b)  MODE 1: (a.b, a.a, b.b)
__global__ __launch_bounds__(kBlock) void seg_partial_kernel(const TA* __restrict__ a,
                                                              const TB* __restrict__ b,
                                                              const int64_t* __restrict__ cbeg,
                                                              const int32_t* __restrict__ clen,
                                                              float* __restrict__ partial,
                                                              float bscale) {
  constexpr int NV = MODE == 0 ? 2 : 3;
  const int c = blockIdx.x;
  const int64_t beg = cbeg[c];
  const int len = clen[c];
  float s[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) s[k] = 0.f;
  const TA* ap = a + beg;
  const TB* bp = b + beg;
  const bool vec = aligned16(ap) && aligned16(bp) && (len % kVec) == 0;
  if (vec) {
    for (int i = threadIdx.x * kVec; i < len; i += kBlock * kVec) {
      float av[8], bv[8];
      load8(ap + i, av);
      load8(bp + i, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = av[j], y = bv[j] * bscale;
        if (MODE == 0) { s[0] += x * x; s[1] += y * y; }
        else { s[0] += x * y; s[1] += x * x; s[2] += y * y; }
      }
    }
  } else {
    for (int i = threadIdx.x; i < len; i += kBlock) {
      float x = ld1(ap + i), y = ld1(bp + i) * bscale;
      if (MODE == 0) { s[0] += x * x; s[1] += y * y; }
      else { s[0] += x * y; s[1] += x * x; s[2] += y * y; }
    }
  }
  block_sum<NV>(s);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; ++k) partial[(int64_t)c * NV + k] = s[k];
  }
}

template <int NV>
__global__ __launch_bounds__(kWave) void seg_reduce_kernel(const float* __restrict__ partial,
                                                            const int32_t* __restrict__ seg_c0,
                                                            const int32_t* __restrict__ seg_nc,
                                                            float* __restrict__ out) {
  const int s = blockIdx.x;
  const int c0 = seg_c0[s], nc = seg_nc[s];
  float v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.f;
  for (int c = threadIdx.x; c < nc; c += kWave) {
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += partial[(int64_t)(c0 + c) * NV + k];
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    v[k] = wave_sum(v[k]);
    if (threadIdx.x == 0) out[s * NV + k] = v[k];
  }
}

struct LarsHp { float lr, momentum, wd, eta, gscale, eps; int first; };

// LARS: per-segment trust ratio eta*|w| / (|g| + wd*|w|); segments flagged
// (bit0) skip both adaptation and weight decay (BN / bias convention).
template <typename TG, typename TP>
__global__ __launch_bounds__(kBlock) void lars_flat_kernel(const TG* __restrict__ g,
                                                            float* __restrict__ w,
                                                            float* __restrict__ mom,
                                                            TP* __restrict__ model,
                                                            const int64_t* __restrict__ cbeg,
                                                            const int32_t* __restrict__ clen,
                                                            const int32_t* __restrict__ cseg,
                                                            const int32_t* __restrict__ sflag,
                                                            const float* __restrict__ norms,
                                                            LarsHp hp,
                                                            const float* __restrict__ dyn,
                                                            const int* __restrict__ skip) {
  if (skip && *skip) return;
  if (dyn) { hp.lr = dyn[0]; hp.first = dyn[1] != 0.f; }
  const int c = blockIdx.x;
  const int64_t beg = cbeg[c];
  const int len = clen[c];
  const int s = cseg[c];
  const bool skip_seg = sflag[s] & 1;
  const float wn = sqrtf(norms[2 * s]);
  const float gn = sqrtf(norms[2 * s + 1]);
  const float wd = skip_seg ? 0.f : hp.wd;
  float trust = 1.f;
  if (!skip_seg && wn > 0.f && gn > 0.f) trust = hp.eta * wn / (gn + wd * wn + hp.eps);
  const float slr = hp.lr * trust;
  // 8-wide vector body over the 16-byte-aligned prefix (arena segments are
  // 64-element aligned and chunks start on 4096-element boundaries), scalar tail
  const int nvec = (aligned16(g + beg) && aligned16(w + beg) && aligned16(mom + beg) &&
                    (!model || aligned16(model + beg))) ? (len / kVec) * kVec : 0;
  for (int i = threadIdx.x * kVec; i < nvec; i += kBlock * kVec) {
    const int64_t k = beg + i;
    float gv[8], wv[8], mv_[8];
    load8(g + k, gv);
    load8(w + k, wv);
    load8(mom + k, mv_);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float d = gv[j] * hp.gscale + wd * wv[j];
      float b = hp.first ? slr * d : hp.momentum * mv_[j] + slr * d;
      mv_[j] = b;
      wv[j] -= b;
    }
    store8(w + k, wv);
    store8(mom + k, mv_);
    if (model) store_model(model + k, wv);
  }
  for (int i = nvec + threadIdx.x; i < len; i += kBlock) {
    const int64_t k = beg + i;
    float wk = w[k];
    float d = ld1(g + k) * hp.gscale + wd * wk;
    float b = hp.first ? slr * d : hp.momentum * mom[k] + slr * d;
    mom[k] = b;
    wk -= b;
    w[k] = wk;
    if (model) st1(model + k, wk);
  }
}

// Adasum merge: a <- ca*a + cb*b with ca = 1 - a.b/(2|a|^2), cb = 1 - a.b/(2|b|^2)
template <typename T>
__global__ __launch_bounds__(kBlock) void adasum_combine_kernel(T* __restrict__ a,
                                                                 const T* __restrict__ b,
                                                                 const int64_t* __restrict__ cbeg,
                                                                 const int32_t* __restrict__ clen,
                                                                 const int32_t* __restrict__ cseg,
                                                                 const float* __restrict__ dots) {
  const int c = blockIdx.x;
  const int64_t beg = cbeg[c];
  const int len = clen[c];
  const int s = cseg[c];
  const float dot = dots[3 * s], na = dots[3 * s + 1], nb = dots[3 * s + 2];
  const float ca = na >= 1e-8f ? 1.f - dot / (2.f * na) : 1.f;
  const float cb = nb >= 1e-8f ? 1.f - dot / (2.f * nb) : 1.f;
  T* ap = a + beg;
  const T* bp = b + beg;
  if (aligned16(ap) && aligned16(bp) && (len % kVec) == 0) {
    for (int i = threadIdx.x * kVec; i < len; i += kBlock * kVec) {
      float av[8], bv[8];
      load8(ap + i, av);
      load8(bp + i, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) av[j] = ca * av[j] + cb * bv[j];
      store8(ap + i, av);
    }
  } else {
    for (int i = threadIdx.x; i < len; i += kBlock) st1(ap + i, ca * ld1(ap + i) + cb * ld1(bp + i));
  }
}

// Vector-halving Adasum merge on the fp32 running sum f (the wire copy r may be
// fp16/bf16: only the wire is compressed, the merge stays fp32).
// swap == 0: f is the lower group's vector a, r is b;  swap == 1: f is b, r is a.
template <typename TB>
__global__ __launch_bounds__(kBlock) void adasum_fcombine_kernel(float* __restrict__ f,
                                                                  const TB* __restrict__ r,
                                                                  const int64_t* __restrict__ cbeg,
                                                                  const int32_t* __restrict__ clen,
                                                                  const int32_t* __restrict__ cseg,
                                                                  const float* __restrict__ dots,
                                                                  int swap) {
  const int c = blockIdx.x;
  const int64_t beg = cbeg[c];
  const int len = clen[c];
  const int s = cseg[c];
  const float dot = dots[3 * s], na = dots[3 * s + 1], nb = dots[3 * s + 2];
  const float ca = na >= 1e-8f ? 1.f - dot / (2.f * na) : 1.f;
  const float cb = nb >= 1e-8f ? 1.f - dot / (2.f * nb) : 1.f;
  const float cf = swap ? cb : ca;
  const float cr = swap ? ca : cb;
  float* fp = f + beg;
  const TB* rp = r + beg;
  if (aligned16(fp) && aligned16(rp) && (len % kVec) == 0) {
    for (int i = threadIdx.x * kVec; i < len; i += kBlock * kVec) {
      float fv[8], rv[8];
      load8(fp + i, fv);
      load8(rp + i, rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) fv[j] = cf * fv[j] + cr * rv[j];
      store8(fp + i, fv);
    }
  } else {
    for (int i = threadIdx.x; i < len; i += kBlock) fp[i] = cf * fp[i] + cr * ld1(rp + i);
  }
}

}  // namespace mv

// ---------------- host launchers ----------------
#define MV_GRID(n) dim3((unsigned)(((n) + kChunk - 1) / kChunk))

#define DISPATCH_GP(gd, md, MACRO)                                  \
  do {                                                              \
    if (md == F32) {                                                \
      using TP = float;                                             \
      if (gd == F32) { using TG = float; MACRO; }                   \
      else if (gd == BF16) { using TG = __bf16; MACRO; }            \
      else { using TG = _Float16; MACRO; }                          \
    } else if (md == BF16) {                                        \
      using TP = __bf16;                                            \
      if (gd == F32) { using TG = float; MACRO; }                   \
      else if (gd == BF16) { using TG = __bf16; MACRO; }            \
      else { using TG = _Float16; MACRO; }                          \
    } else {                                                        \
      using TP = _Float16;                                          \
      if (gd == F32) { using TG = float; MACRO; }                   \
      else if (gd == BF16) { using TG = __bf16; MACRO; }            \
      else { using TG = _Float16; MACRO; }                          \
    }                                                               \
  } while (0)

void mv_launch_sgd(const void* g, int gd, float* w, float* mom, void* model, int md, int64_t n,
                   float lr, float momentum, float dampening, float wd, float gscale, int nesterov,
                   int first, const float* dyn, const int* skip, hipStream_t st) {
  if (n <= 0) return;
  SgdHp hp{lr, momentum, dampening, wd, gscale, nesterov, first};
  DISPATCH_GP(gd, md, hipLaunchKernelGGL((sgd_flat_kernel<TG, TP>), MV_GRID(n), dim3(kBlock), 0,
                                         st, (const TG*)g, w, mom, (TP*)model, n, hp, dyn, skip));
}

void mv_launch_adam(const void* g, int gd, float* w, float* m, float* v, void* model, int md,
                    int64_t n, float lr, float b1, float b2, float eps, float wd, float gscale,
                    float bc1, float bc2, int adamw, int keras_eps, const float* dyn,
                    const int* skip, hipStream_t st) {
  if (n <= 0) return;
  AdamHp hp{lr, b1, b2, eps, wd, gscale, bc1, bc2, adamw, keras_eps};
  DISPATCH_GP(gd, md, hipLaunchKernelGGL((adam_flat_kernel<TG, TP>), MV_GRID(n), dim3(kBlock), 0,
                                         st, (const TG*)g, w, m, v, (TP*)model, n, hp, dyn, skip));
}

void mv_launch_adadelta(const void* g, int gd, float* w, float* sq, float* acc, void* model,
                        int md, int64_t n, float lr, float rho, float eps, float wd, float gscale,
                        const float* dyn, const int* skip, hipStream_t st) {
  if (n <= 0) return;
  AdadeltaHp hp{lr, rho, eps, wd, gscale};
  DISPATCH_GP(gd, md, hipLaunchKernelGGL((adadelta_flat_kernel<TG, TP>), MV_GRID(n), dim3(kBlock),
                                         0, st, (const TG*)g, w, sq, acc, (TP*)model, n, hp, dyn,
                                         skip));
}

void mv_launch_lars(const void* g, int gd, float* w, float* mom, void* model, int md,
                    const ChunkTable& ct, const int32_t* sflag, float* partial, float* norms,
                    float lr, float momentum, float wd, float eta, float gscale, float eps,
                    int first, const float* dyn, const int* skip, hipStream_t st) {
  if (ct.nchunks <= 0) return;
  // pass 1: per-chunk (|w|^2, |g|^2)
  switch (gd) {
    case F32: hipLaunchKernelGGL((seg_partial_kernel<float, float, 0>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const float*)w, (const float*)g, ct.begin, ct.len, partial, gscale); break;
    case BF16: hipLaunchKernelGGL((seg_partial_kernel<float, __bf16, 0>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const float*)w, (const __bf16*)g, ct.begin, ct.len, partial, gscale); break;
    case F16: hipLaunchKernelGGL((seg_partial_kernel<float, _Float16, 0>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const float*)w, (const _Float16*)g, ct.begin, ct.len, partial, gscale); break;
  }
  hipLaunchKernelGGL((seg_reduce_kernel<2>), dim3(ct.nseg), dim3(kWave), 0, st, partial, ct.seg_c0,
                     ct.seg_nc, norms);
  // norms[2s+1] already includes gscale (bscale in pass 1)
  LarsHp hp{lr, momentum, wd, eta, gscale, eps, first};
  DISPATCH_GP(gd, md, hipLaunchKernelGGL((lars_flat_kernel<TG, TP>), dim3(ct.nchunks), dim3(kBlock),
                                         0, st, (const TG*)g, w, mom, (TP*)model, ct.begin, ct.len,
                                         ct.seg, sflag, norms, hp, dyn, skip));
}

void mv_launch_seg_dot3(const void* a, const void* b, int dt, const ChunkTable& ct, float* partial,
                        float* out, hipStream_t st) {
  if (ct.nchunks <= 0) return;
  switch (dt) {
    case F32: hipLaunchKernelGGL((seg_partial_kernel<float, float, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const float*)a, (const float*)b, ct.begin, ct.len, partial, 1.f); break;
    case BF16: hipLaunchKernelGGL((seg_partial_kernel<__bf16, __bf16, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const __bf16*)a, (const __bf16*)b, ct.begin, ct.len, partial, 1.f); break;
    case F16: hipLaunchKernelGGL((seg_partial_kernel<_Float16, _Float16, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, (const _Float16*)a, (const _Float16*)b, ct.begin, ct.len, partial, 1.f); break;
  }
  hipLaunchKernelGGL((seg_reduce_kernel<3>), dim3(ct.nseg), dim3(kWave), 0, st, partial, ct.seg_c0,
                     ct.seg_nc, out);
}

void mv_launch_seg_dot3_f(const float* a, const void* b, int bdt, const ChunkTable& ct,
                          float* partial, float* out, hipStream_t st) {
  if (ct.nchunks <= 0) return;
  switch (bdt) {
    case F32: hipLaunchKernelGGL((seg_partial_kernel<float, float, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, a, (const float*)b, ct.begin, ct.len, partial, 1.f); break;
    case BF16: hipLaunchKernelGGL((seg_partial_kernel<float, __bf16, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, a, (const __bf16*)b, ct.begin, ct.len, partial, 1.f); break;
    case F16: hipLaunchKernelGGL((seg_partial_kernel<float, _Float16, 1>), dim3(ct.nchunks), dim3(kBlock), 0, st, a, (const _Float16*)b, ct.begin, ct.len, partial, 1.f); break;
  }
  hipLaunchKernelGGL((seg_reduce_kernel<3>), dim3(ct.nseg), dim3(kWave), 0, st, partial, ct.seg_c0,
                     ct.seg_nc, out);
}

void mv_launch_adasum_fcombine(float* f, const void* r, int rdt, const ChunkTable& ct,
                               const float* dots, int swap, hipStream_t st) {
  if (ct.nchunks <= 0) return;
  switch (rdt) {
    case F32: hipLaunchKernelGGL((adasum_fcombine_kernel<float>), dim3(ct.nchunks), dim3(kBlock), 0, st, f, (const float*)r, ct.begin, ct.len, ct.seg, dots, swap); break;
    case BF16: hipLaunchKernelGGL((adasum_fcombine_kernel<__bf16>), dim3(ct.nchunks), dim3(kBlock), 0, st, f, (const __bf16*)r, ct.begin, ct.len, ct.seg, dots, swap); break;
    case F16: hipLaunchKernelGGL((adasum_fcombine_kernel<_Float16>), dim3(ct.nchunks), dim3(kBlock), 0, st, f, (const _Float16*)r, ct.begin, ct.len, ct.seg, dots, swap); break;
  }
}

void mv_launch_adasum_combine(void* a, const void* b, int dt, const ChunkTable& ct,
                              const float* dots, hipStream_t st) {
  if (ct.nchunks <= 0) return;
  switch (dt) {
    case F32: hipLaunchKernelGGL((adasum_combine_kernel<float>), dim3(ct.nchunks), dim3(kBlock), 0, st, (float*)a, (const float*)b, ct.begin, ct.len, ct.seg, dots); break;
    case BF16: hipLaunchKernelGGL((adasum_combine_kernel<__bf16>), dim3(ct.nchunks), dim3(kBlock), 0, st, (__bf16*)a, (const __bf16*)b, ct.begin, ct.len, ct.seg, dots); break;
    case F16: hipLaunchKernelGGL((adasum_combine_kernel<_Float16>), dim3(ct.nchunks), dim3(kBlock), 0, st, (_Float16*)a, (const _Float16*)b, ct.begin, ct.len, ct.seg, dots); break;
  }
}
