// PyTorch bindings for the mivod gfx950 kernels (module mivod._mvk).
// Every entry point validates shapes / dtypes / devices on the host before a
// launch: a kernel is never started on operands that disagree with the grid
// it assumes.  All launches go to the caller's current HIP stream.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>

#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "mv_attn.h"
#include "mv_bert.h"
#include "mv_bn.h"
#include "mv_gemm.h"
#include "mv_fold.h"
#include "mv_stem.h"
#include "mv_conv.h"
#include "mv_kernels.h"
#include "mv_pool.h"

namespace {

constexpr int64_t kChunk = 4096;

int dtype_code(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return 0;
    case at::kBFloat16: return 1;
    case at::kHalf: return 2;
    default: TORCH_CHECK(false, "mivod kernels: unsupported dtype ", t.scalar_type());
  }
  return -1;
}

void check_dev(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), "mivod kernels: ", what, " must be a GPU tensor");
  TORCH_CHECK(t.is_non_overlapping_and_dense(), "mivod kernels: ", what,
              " must be dense and non-overlapping");
}

void check_flat(const at::Tensor& t, const char* what) {
  check_dev(t, what);
  TORCH_CHECK(t.is_contiguous(), "mivod kernels: ", what, " must be contiguous");
}

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

int* nf_ptr(const c10::optional<at::Tensor>& nf) {
  if (!nf.has_value()) return nullptr;
  TORCH_CHECK(nf->is_cuda() && nf->scalar_type() == at::kInt && nf->numel() >= 1,
              "nonfinite flag must be an int32 GPU tensor");
  return nf->data_ptr<int>();
}

// K1/K2: pack (to_flat) or unpack tensors <-> flat[offsets[i] : offsets[i]+numel]
void mt_copy(const std::vector<at::Tensor>& tensors, at::Tensor flat,
             const std::vector<int64_t>& offsets, bool to_flat, double scale,
             c10::optional<at::Tensor> nonfinite) {
  TORCH_CHECK(tensors.size() == offsets.size(), "mt_copy: tensors/offsets length mismatch");
  if (tensors.empty()) return;
  check_flat(flat, "flat");
  c10::DeviceGuard guard(flat.device());
  const int tdt = dtype_code(tensors[0]);
  const int fdt = dtype_code(flat);
  const int64_t fnumel = flat.numel();
  int* nf = nf_ptr(nonfinite);
  hipStream_t st = cur_stream();
  MtArgs a;
  a.ntensors = 0;
  a.chunk_start[0] = 0;
  auto flush = [&]() {
    if (a.ntensors == 0) return;
    mv_launch_mt_copy(a, tdt, flat.data_ptr(), fdt, to_flat, (float)scale, nf, st);
    a.ntensors = 0;
    a.chunk_start[0] = 0;
  };
  for (size_t i = 0; i < tensors.size(); ++i) {
    const at::Tensor& t = tensors[i];
    check_dev(t, "tensor");
    TORCH_CHECK(t.device() == flat.device(), "mt_copy: tensor on a different device");
    TORCH_CHECK(dtype_code(t) == tdt, "mt_copy: mixed tensor dtypes in one call");
    const int64_t n = t.numel();
    TORCH_CHECK(offsets[i] >= 0 && offsets[i] + n <= fnumel, "mt_copy: tensor ", i,
                " [", offsets[i], ", +", n, ") exceeds flat buffer of ", fnumel);
    if (n == 0) continue;
    const int64_t chunks = (n + kChunk - 1) / kChunk;
    TORCH_CHECK(chunks < (1 << 30), "mt_copy: tensor too large");
    if (a.ntensors == kMvMaxTensors ||
        (int64_t)a.chunk_start[a.ntensors] + chunks > (int64_t)(1u << 30))
      flush();
    const int k = a.ntensors++;
    a.ptr[k] = t.data_ptr();
    a.numel[k] = n;
    a.flat_off[k] = offsets[i];
    a.chunk_start[k + 1] = a.chunk_start[k] + (int32_t)chunks;
  }
  flush();
}

void flat_cast(at::Tensor src, at::Tensor dst, double scale, c10::optional<at::Tensor> nonfinite) {
  check_flat(src, "src");
  check_flat(dst, "dst");
  TORCH_CHECK(src.numel() == dst.numel(), "flat_cast: numel mismatch");
  c10::DeviceGuard guard(src.device());
  mv_launch_flat_cast(src.data_ptr(), dtype_code(src), dst.data_ptr(), dtype_code(dst), src.numel(),
                      (float)scale, nf_ptr(nonfinite), cur_stream());
}

void nonfinite_scan(at::Tensor x, at::Tensor flag) {
  check_flat(x, "x");
  TORCH_CHECK(flag.is_cuda() && flag.scalar_type() == at::kInt && flag.numel() >= 1 &&
                  flag.device() == x.device() && flag.is_contiguous(),
              "nonfinite_scan: flag must be an int32 GPU tensor on x's device");
  c10::DeviceGuard guard(x.device());
  mv_launch_nonfinite_scan(x.data_ptr(), dtype_code(x), x.numel(), flag.data_ptr<int>(),
                           cur_stream());
}

void check_master(const at::Tensor& g, const at::Tensor& t, const char* what) {
  check_flat(t, what);
  TORCH_CHECK(t.scalar_type() == at::kFloat, what, " must be fp32");
  TORCH_CHECK(t.numel() == g.numel(), what, " numel ", t.numel(), " != grad numel ", g.numel());
  TORCH_CHECK(t.device() == g.device(), what, " on a different device");
}

void* model_ptr(const c10::optional<at::Tensor>& model, const at::Tensor& g, int* md) {
  *md = 0;
  if (!model.has_value()) return nullptr;
  check_flat(*model, "model");
  TORCH_CHECK(model->numel() == g.numel(), "model numel mismatch");
  *md = dtype_code(*model);
  return model->data_ptr();
}

// optional device int32 skip flag (fp16-wire overflow guard)
const int* skip_ptr(const c10::optional<at::Tensor>& skip, const at::Tensor& g) {
  if (!skip.has_value()) return nullptr;
  TORCH_CHECK(skip->is_cuda() && skip->scalar_type() == at::kInt && skip->numel() >= 1 &&
                  skip->device() == g.device(),
              "skip must be an int32 GPU tensor on the grad's device");
  return skip->data_ptr<int>();
}

// optional device hyperparameter block [lr, first, bc1, bc2] (HIP-graph replays)
const float* dyn_ptr(const c10::optional<at::Tensor>& dyn, const at::Tensor& g) {
  if (!dyn.has_value()) return nullptr;
  TORCH_CHECK(dyn->is_cuda() && dyn->scalar_type() == at::kFloat && dyn->is_contiguous() &&
                  dyn->numel() >= 4 && dyn->device() == g.device(),
              "dyn must be a contiguous fp32 [4] tensor on the grad's device");
  return dyn->data_ptr<float>();
}

void sgd_step(at::Tensor g, at::Tensor w, c10::optional<at::Tensor> mom,
              c10::optional<at::Tensor> model, double lr, double momentum, double dampening,
              double wd, double gscale, bool nesterov, bool first, c10::optional<at::Tensor> dyn,
              c10::optional<at::Tensor> skip) {
  check_flat(g, "grad");
  check_master(g, w, "master");
  if (mom.has_value()) check_master(g, *mom, "momentum");
  int md;
  void* mp = model_ptr(model, g, &md);
  const float* dp = dyn_ptr(dyn, g);
  c10::DeviceGuard guard(g.device());
  mv_launch_sgd(g.data_ptr(), dtype_code(g), w.data_ptr<float>(),
                mom.has_value() ? mom->data_ptr<float>() : nullptr, mp, md, g.numel(), (float)lr,
                (float)momentum, (float)dampening, (float)wd, (float)gscale, nesterov, first, dp,
                skip_ptr(skip, g), cur_stream());
}

void adam_step(at::Tensor g, at::Tensor w, at::Tensor m, at::Tensor v,
               c10::optional<at::Tensor> model, double lr, double b1, double b2, double eps,
               double wd, double gscale, int64_t step, bool adamw, bool keras_eps,
               c10::optional<at::Tensor> dyn, c10::optional<at::Tensor> skip) {
  check_flat(g, "grad");
  check_master(g, w, "master");
  check_master(g, m, "exp_avg");
  check_master(g, v, "exp_avg_sq");
  TORCH_CHECK(step >= 1, "adam_step: step must be >= 1");
  int md;
  void* mp = model_ptr(model, g, &md);
  const double bc1 = 1.0 - std::pow(b1, (double)step);
  const double bc2 = 1.0 - std::pow(b2, (double)step);
  c10::DeviceGuard guard(g.device());
  mv_launch_adam(g.data_ptr(), dtype_code(g), w.data_ptr<float>(), m.data_ptr<float>(),
                 v.data_ptr<float>(), mp, md, g.numel(), (float)lr, (float)b1, (float)b2,
                 (float)eps, (float)wd, (float)gscale, (float)bc1, (float)bc2, adamw, keras_eps,
                 dyn_ptr(dyn, g), skip_ptr(skip, g), cur_stream());
}

void adadelta_step(at::Tensor g, at::Tensor w, at::Tensor sq, at::Tensor acc,
                   c10::optional<at::Tensor> model, double lr, double rho, double eps, double wd,
                   double gscale, c10::optional<at::Tensor> dyn, c10::optional<at::Tensor> skip) {
  check_flat(g, "grad");
  check_master(g, w, "master");
  check_master(g, sq, "square_avg");
  check_master(g, acc, "acc_delta");
  int md;
  void* mp = model_ptr(model, g, &md);
  c10::DeviceGuard guard(g.device());
  mv_launch_adadelta(g.data_ptr(), dtype_code(g), w.data_ptr<float>(), sq.data_ptr<float>(),
                     acc.data_ptr<float>(), mp, md, g.numel(), (float)lr, (float)rho, (float)eps,
                     (float)wd, (float)gscale, dyn_ptr(dyn, g), skip_ptr(skip, g), cur_stream());
}

ChunkTable make_table(const at::Tensor& begin, const at::Tensor& len, const at::Tensor& seg,
                      const at::Tensor& seg_c0, const at::Tensor& seg_nc, int64_t total) {
  TORCH_CHECK(begin.is_cuda() && begin.scalar_type() == at::kLong && begin.is_contiguous(),
              "chunk begin must be contiguous int64 on GPU");
  for (const at::Tensor* t : {&len, &seg, &seg_c0, &seg_nc})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->is_contiguous(),
                "chunk tables must be contiguous int32 on GPU");
  TORCH_CHECK(len.numel() == begin.numel() && seg.numel() == begin.numel(),
              "chunk table length mismatch");
  TORCH_CHECK(seg_c0.numel() == seg_nc.numel(), "segment table length mismatch");
  (void)total;
  ChunkTable ct;
  ct.begin = begin.data_ptr<int64_t>();
  ct.len = len.data_ptr<int32_t>();
  ct.seg = seg.data_ptr<int32_t>();
  ct.seg_c0 = seg_c0.data_ptr<int32_t>();
  ct.seg_nc = seg_nc.data_ptr<int32_t>();
  ct.nchunks = (int32_t)begin.numel();
  ct.nseg = (int32_t)seg_c0.numel();
  return ct;
}

void lars_step(at::Tensor g, at::Tensor w, at::Tensor mom, c10::optional<at::Tensor> model,
               at::Tensor cbeg, at::Tensor clen, at::Tensor cseg, at::Tensor seg_c0,
               at::Tensor seg_nc, at::Tensor sflag, at::Tensor partial, at::Tensor norms, double lr,
               double momentum, double wd, double eta, double gscale, double eps, bool first,
               c10::optional<at::Tensor> dyn, c10::optional<at::Tensor> skip) {
  check_flat(g, "grad");
  check_master(g, w, "master");
  check_master(g, mom, "momentum");
  int md;
  void* mp = model_ptr(model, g, &md);
  ChunkTable ct = make_table(cbeg, clen, cseg, seg_c0, seg_nc, g.numel());
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.numel() >= 2 * ct.nchunks,
              "lars: partial buffer too small");
  TORCH_CHECK(norms.scalar_type() == at::kFloat && norms.numel() >= 2 * ct.nseg,
              "lars: norms buffer too small");
  TORCH_CHECK(sflag.scalar_type() == at::kInt && sflag.numel() >= ct.nseg, "lars: flags");
  c10::DeviceGuard guard(g.device());
  mv_launch_lars(g.data_ptr(), dtype_code(g), w.data_ptr<float>(), mom.data_ptr<float>(), mp, md,
                 ct, sflag.data_ptr<int32_t>(), partial.data_ptr<float>(), norms.data_ptr<float>(),
                 (float)lr, (float)momentum, (float)wd, (float)eta, (float)gscale, (float)eps, first,
                 dyn_ptr(dyn, g), skip_ptr(skip, g), cur_stream());
}

void seg_dot3(at::Tensor a, at::Tensor b, at::Tensor cbeg, at::Tensor clen, at::Tensor cseg,
              at::Tensor seg_c0, at::Tensor seg_nc, at::Tensor partial, at::Tensor out) {
  check_flat(a, "a");
  check_flat(b, "b");
  TORCH_CHECK(a.numel() == b.numel(), "seg_dot3: a/b numel mismatch");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() || a.scalar_type() == at::kFloat,
              "seg_dot3: a must match b or be fp32");
  ChunkTable ct = make_table(cbeg, clen, cseg, seg_c0, seg_nc, a.numel());
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.numel() >= 3 * ct.nchunks,
              "seg_dot3: partial buffer too small");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 3 * ct.nseg, "seg_dot3: out too small");
  c10::DeviceGuard guard(a.device());
  if (a.scalar_type() == b.scalar_type())
    mv_launch_seg_dot3(a.data_ptr(), b.data_ptr(), dtype_code(a), ct, partial.data_ptr<float>(),
                       out.data_ptr<float>(), cur_stream());
  else
    mv_launch_seg_dot3_f(a.data_ptr<float>(), b.data_ptr(), dtype_code(b), ct,
                         partial.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
}

void adasum_combine(at::Tensor a, at::Tensor b, at::Tensor cbeg, at::Tensor clen, at::Tensor cseg,
                    at::Tensor seg_c0, at::Tensor seg_nc, at::Tensor dots) {
  check_flat(a, "a");
  check_flat(b, "b");
  TORCH_CHECK(a.numel() == b.numel() && a.scalar_type() == b.scalar_type(),
              "adasum_combine: a/b mismatch");
  ChunkTable ct = make_table(cbeg, clen, cseg, seg_c0, seg_nc, a.numel());
  TORCH_CHECK(dots.scalar_type() == at::kFloat && dots.numel() >= 3 * ct.nseg, "adasum: dots");
  c10::DeviceGuard guard(a.device());
  mv_launch_adasum_combine(a.data_ptr(), b.data_ptr(), dtype_code(a), ct, dots.data_ptr<float>(),
                           cur_stream());
}

void adasum_fcombine(at::Tensor f, at::Tensor r, at::Tensor cbeg, at::Tensor clen, at::Tensor cseg,
                     at::Tensor seg_c0, at::Tensor seg_nc, at::Tensor dots, bool swap) {
  check_flat(f, "f");
  check_flat(r, "r");
  TORCH_CHECK(f.scalar_type() == at::kFloat, "adasum_fcombine: running merge must be fp32");
  TORCH_CHECK(f.numel() == r.numel(), "adasum_fcombine: f/r numel mismatch");
  ChunkTable ct = make_table(cbeg, clen, cseg, seg_c0, seg_nc, f.numel());
  TORCH_CHECK(dots.scalar_type() == at::kFloat && dots.is_contiguous() && dots.numel() >= 3 * ct.nseg,
              "adasum: dots");
  c10::DeviceGuard guard(f.device());
  mv_launch_adasum_fcombine(f.data_ptr<float>(), r.data_ptr(), dtype_code(r), ct,
                            dots.data_ptr<float>(), swap ? 1 : 0, cur_stream());
}

// ---------------------------------------------------------------------------
// Fused NHWC BatchNorm (+ residual add) (+ ReLU), bf16 activations, fp32 params
// ---------------------------------------------------------------------------
int64_t bn_check_act(const at::Tensor& t, const char* what, int64_t* C) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, "bn: ", what,
              " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() >= 2, "bn: ", what, " must have a channel dim");
  const bool ok = (t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast)) ||
                  (t.dim() == 2 && t.is_contiguous());
  TORCH_CHECK(ok, "bn: ", what, " must be channels_last 4-D or contiguous 2-D");
  *C = t.size(1);
  TORCH_CHECK(*C % 8 == 0, "bn: channel count must be a multiple of 8");
  return t.numel() / *C;
}

const float* opt_f32(const c10::optional<at::Tensor>& t, int64_t C, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
              t->numel() == C, "bn: ", what, " must be a contiguous fp32 [C] GPU tensor");
  return t->data_ptr<float>();
}

// want_mask (relu + residual only): also return the [M, C/8] uint8 bitmask of y > 0 that
// backward mode 3 reads instead of y
std::vector<at::Tensor> bn_fwd_train_impl(at::Tensor x, c10::optional<at::Tensor> gamma,
                                          c10::optional<at::Tensor> beta,
                                          c10::optional<at::Tensor> running_mean,
                                          c10::optional<at::Tensor> running_var, double momentum,
                                          double eps, bool relu,
                                          c10::optional<at::Tensor> residual, bool want_mask,
                                          c10::optional<at::Tensor> stats = c10::nullopt) {
  int64_t C;
  const int64_t M = bn_check_act(x, "x", &C);
  TORCH_CHECK(M > 0, "bn: empty input");
  c10::DeviceGuard guard(x.device());
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    int64_t C2;
    bn_check_act(*residual, "residual", &C2);
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->strides() == x.strides(),
                "bn: residual must match x in shape and layout");
    rp = residual->data_ptr();
  }
  auto fo = x.options().dtype(at::kFloat);
  const int P = mv_bn_partials(M, (int)C);
  at::Tensor partial = stats.has_value() ? at::Tensor() : at::empty({(int64_t)P * 2 * C}, fo);
  at::Tensor vec = at::empty({4, C}, fo);   // save_mean, save_invstd, scale, bias
  at::Tensor y = at::empty_like(x);
  at::Tensor mask;
  if (want_mask) {
    TORCH_CHECK(relu && rp != nullptr, "bn: the output bitmask needs relu and a residual");
    mask = at::empty({M, C / 8}, x.options().dtype(at::kByte));
  }
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "bn: running_mean/var must both be given");
  if (stats.has_value()) {
    // statistics from the producing conv's epilogue: [P, 2, C] partials around rm
    TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kFloat && stats->is_contiguous() &&
                    stats->dim() == 3 && stats->size(1) == 2 && stats->size(2) == C &&
                    stats->size(0) > 0,
                "bn: stats must be fp32 [P, 2, C] partials");
    mv_bn_fwd_from_partials(x.data_ptr(), rp, y.data_ptr(), M, (int)C, rm, rv,
                            opt_f32(gamma, C, "weight"), opt_f32(beta, C, "bias"),
                            (float)momentum, (float)eps, relu, stats->data_ptr<float>(),
                            (int)stats->size(0), vec[0].data_ptr<float>(),
                            vec[1].data_ptr<float>(), vec[2].data_ptr<float>(),
                            vec[3].data_ptr<float>(), cur_stream(),
                            want_mask ? mask.data_ptr() : nullptr);
  } else {
    mv_bn_fwd_train(x.data_ptr(), rp, y.data_ptr(), M, (int)C, rm, rv, opt_f32(gamma, C, "weight"),
                    opt_f32(beta, C, "bias"), (float)momentum, (float)eps, relu,
                    partial.data_ptr<float>(), P, vec[0].data_ptr<float>(),
                    vec[1].data_ptr<float>(), vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                    cur_stream(), want_mask ? mask.data_ptr() : nullptr);
  }
  if (want_mask) return {y, vec, mask};
  return {y, vec};
}

std::vector<at::Tensor> bn_fwd_train(at::Tensor x, c10::optional<at::Tensor> gamma,
                                     c10::optional<at::Tensor> beta,
                                     c10::optional<at::Tensor> running_mean,
                                     c10::optional<at::Tensor> running_var, double momentum,
                                     double eps, bool relu, c10::optional<at::Tensor> residual) {
  return bn_fwd_train_impl(x, gamma, beta, running_mean, running_var, momentum, eps, relu,
                           residual, false);
}

// forward with statistics partials from the conv GEMM epilogue ({y, vec} or {y, vec, mask})
std::vector<at::Tensor> bn_fwd_train_stats(at::Tensor x, at::Tensor stats,
                                           c10::optional<at::Tensor> gamma,
                                           c10::optional<at::Tensor> beta,
                                           c10::optional<at::Tensor> running_mean,
                                           c10::optional<at::Tensor> running_var, double momentum,
                                           double eps, bool relu,
                                           c10::optional<at::Tensor> residual, bool want_mask) {
  return bn_fwd_train_impl(x, gamma, beta, running_mean, running_var, momentum, eps, relu,
                           residual, want_mask, stats);
}

// {y, vec, mask}: add+ReLU forward that also records the backward bitmask (mode 3)
std::vector<at::Tensor> bn_fwd_train_mask(at::Tensor x, c10::optional<at::Tensor> gamma,
                                          c10::optional<at::Tensor> beta,
                                          c10::optional<at::Tensor> running_mean,
                                          c10::optional<at::Tensor> running_var, double momentum,
                                          double eps, at::Tensor residual) {
  return bn_fwd_train_impl(x, gamma, beta, running_mean, running_var, momentum, eps, true,
                           residual, true);
}

at::Tensor bn_apply(at::Tensor x, at::Tensor scale, at::Tensor bias, bool relu,
                    c10::optional<at::Tensor> residual) {
  int64_t C;
  const int64_t M = bn_check_act(x, "x", &C);
  c10::DeviceGuard guard(x.device());
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    TORCH_CHECK(residual->sizes() == x.sizes() && residual->strides() == x.strides() &&
                residual->scalar_type() == at::kBFloat16, "bn: residual must match x");
    rp = residual->data_ptr();
  }
  at::Tensor y = at::empty_like(x);
  mv_bn_apply(x.data_ptr(), rp, y.data_ptr(), M, (int)C, opt_f32(scale, C, "scale"),
              opt_f32(bias, C, "bias"), relu, cur_stream());
  return y;
}

// {y, partial}: y = relu(x * scale + bias) and [P, C] column-sum partials of y
std::vector<at::Tensor> bn_apply_colsum(at::Tensor x, at::Tensor scale, at::Tensor bias) {
  int64_t C;
  const int64_t M = bn_check_act(x, "x", &C);
  TORCH_CHECK(M > 0, "bn: empty input");
  c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty_like(x);
  at::Tensor partial = at::empty({(int64_t)mv_bn_partials(M, (int)C), C},
                                 x.options().dtype(at::kFloat));
  const int P = mv_bn_apply_colsum(x.data_ptr(), y.data_ptr(), M, (int)C,
                                   opt_f32(scale, C, "scale"), opt_f32(bias, C, "bias"),
                                   partial.data_ptr<float>(), cur_stream());
  return {y, partial.narrow(0, 0, P)};
}

// statistics only: running-stat update + saved {mean, invstd, scale, bias}; no apply pass
at::Tensor bn_stats(at::Tensor x, c10::optional<at::Tensor> gamma, c10::optional<at::Tensor> beta,
                    c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                    double momentum, double eps) {
  int64_t C;
  const int64_t M = bn_check_act(x, "x", &C);
  TORCH_CHECK(M > 0, "bn: empty input");
  c10::DeviceGuard guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  const int P = mv_bn_partials(M, (int)C);
  at::Tensor partial = at::empty({(int64_t)P * 2 * C}, fo);
  at::Tensor vec = at::empty({4, C}, fo);
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "bn: running_mean/var must both be given");
  mv_bn_fwd_train(x.data_ptr(), nullptr, nullptr, M, (int)C, rm, rv, opt_f32(gamma, C, "weight"),
                  opt_f32(beta, C, "bias"), (float)momentum, (float)eps, false,
                  partial.data_ptr<float>(), P, vec[0].data_ptr<float>(),
                  vec[1].data_ptr<float>(), vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                  cur_stream());
  return vec;
}

// statistics of x[:, :, ::s, ::s] without the strided copy -> [4, C] {mean, invstd, ...}
at::Tensor bn_stats_strided(at::Tensor x, int64_t stride) {
  int64_t C;
  bn_check_act(x, "x", &C);
  TORCH_CHECK(stride >= 1 && stride < 65536 && x.size(2) < 65536 && x.size(3) < 65536,
              "bn_stats_strided: bad stride / size");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t M = N * ((H - 1) / stride + 1) * ((W - 1) / stride + 1);
  TORCH_CHECK(M > 0 && M < (int64_t(1) << 32), "bn_stats_strided: empty or too large");
  c10::DeviceGuard guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  const int P = mv_bn_partials(M, (int)C);
  at::Tensor partial = at::empty({(int64_t)P * 2 * C}, fo);
  at::Tensor vec = at::empty({4, C}, fo);
  mv_bn_stats_strided(x.data_ptr(), (int)N, (int)H, (int)W, (int)C, (int)stride,
                      partial.data_ptr<float>(), P, vec[0].data_ptr<float>(),
                      vec[1].data_ptr<float>(), vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                      cur_stream());
  return vec;
}

// returns {dx, dgamma, dbeta, dz}; dz defined only for modes 2 and 3 (residual branch grad)
std::vector<at::Tensor> bn_bwd(int64_t mode, at::Tensor dy, at::Tensor x,
                               c10::optional<at::Tensor> y, at::Tensor vec,
                               c10::optional<at::Tensor> gamma, bool need_affine_grad,
                               c10::optional<at::Tensor> dy2, int64_t dy2_stride) {
  int64_t C, C2;
  const int64_t M = bn_check_act(x, "x", &C);
  bn_check_act(dy, "grad", &C2);
  TORCH_CHECK(dy.sizes() == x.sizes() && dy.strides() == x.strides(), "bn: grad layout mismatch");
  TORCH_CHECK(mode >= 0 && mode <= 3, "bn: bad mode");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
              vec.numel() == 4 * C, "bn: saved stats must be fp32 [4, C]");
  const void* yp = nullptr;
  if (mode == 2) {
    TORCH_CHECK(y.has_value() && y->defined() && y->sizes() == x.sizes() &&
                y->strides() == x.strides() && y->scalar_type() == at::kBFloat16,
                "bn: mode 2 needs the saved output");
    yp = y->data_ptr();
  } else if (mode == 3) {
    TORCH_CHECK(y.has_value() && y->defined() && y->is_cuda() && y->is_contiguous() &&
                y->scalar_type() == at::kByte && y->dim() == 2 && y->size(0) == M &&
                y->size(1) == C / 8, "bn: mode 3 needs the forward's [M, C/8] uint8 bitmask");
    yp = y->data_ptr();
  }
  const void* dy2p = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    TORCH_CHECK(mode >= 2, "bn: a second gradient stream is supported for modes 2 and 3 only");
    TORCH_CHECK(dy2_stride >= 1, "bn: bad dy2 stride");
    if (dy2_stride == 1) {
      TORCH_CHECK(dy2->sizes() == x.sizes() && dy2->strides() == x.strides() &&
                  dy2->scalar_type() == at::kBFloat16 && dy2->is_cuda(),
                  "bn: dy2 must match x in shape, layout and dtype");
    } else {
      const int64_t s = dy2_stride;
      TORCH_CHECK(M < (int64_t(1) << 32), "bn: strided dy2 needs fewer than 2^32 rows");
      TORCH_CHECK(x.dim() == 4 && dy2->dim() == 4 && dy2->size(0) == x.size(0) &&
                  dy2->size(1) == x.size(1) && dy2->size(2) == (x.size(2) + s - 1) / s &&
                  dy2->size(3) == (x.size(3) + s - 1) / s &&
                  dy2->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                  dy2->scalar_type() == at::kBFloat16 && dy2->is_cuda(),
                  "bn: strided dy2 must be channels_last bf16 [N, C, ceil(H/s), ceil(W/s)]");
    }
    dy2p = dy2->data_ptr();
  }
  c10::DeviceGuard guard(x.device());
  auto fo = x.options().dtype(at::kFloat);
  const int P = mv_bn_partials(M, (int)C);
  at::Tensor partial = at::empty({(int64_t)P * 2 * C}, fo);
  at::Tensor work = at::empty({5, C}, fo);  // dgamma, dbeta, a, b, c
  at::Tensor dx = at::empty_like(x);
  at::Tensor dz;
  if (mode >= 2) dz = at::empty_like(x);
  mv_bn_bwd((int)mode, dy.data_ptr(), dy2p, x.data_ptr(), yp, mode >= 2 ? dz.data_ptr() : nullptr,
            dx.data_ptr(), M, (int)C, vec[0].data_ptr<float>(), vec[1].data_ptr<float>(),
            opt_f32(gamma, C, "weight"), vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
            work[0].data_ptr<float>(), work[1].data_ptr<float>(), partial.data_ptr<float>(), P,
            work[2].data_ptr<float>(), work[3].data_ptr<float>(), work[4].data_ptr<float>(),
            dy2p ? (int)dy2_stride : 1, x.dim() == 4 ? (int)x.size(2) : 1,
            x.dim() == 4 ? (int)x.size(3) : 1, cur_stream());
  at::Tensor dg, db;
  if (need_affine_grad) {
    dg = work[0];
    db = work[1];
  }
  return {dx, dg, db, dz};
}

// ---------------------------------------------------------------------------
// Fused MFMA attention (head dim 64)
// ---------------------------------------------------------------------------
AttnParams attn_params(const at::Tensor& qkv, const c10::optional<at::Tensor>& mask,
                       double p_drop, int64_t seed) {
  TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.is_contiguous(),
              "attn: qkv must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(qkv.dim() == 5 && qkv.size(2) == 3 && qkv.size(4) == 64,
              "attn: qkv must be [b, s, 3, h, 64]");
  AttnParams p{};
  p.qkv = qkv.data_ptr();
  p.b = (int)qkv.size(0);
  p.s = (int)qkv.size(1);
  p.h = (int)qkv.size(3);
  p.scale_log2 = (float)(1.4426950408889634 / 8.0);
  p.mask = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kFloat && mask->is_contiguous() &&
                mask->numel() == (int64_t)p.b * p.s, "attn: mask must be fp32 [b, s]");
    p.mask = mask->data_ptr<float>();
  }
  TORCH_CHECK(p_drop >= 0.0 && p_drop < 1.0, "attn: dropout must be in [0, 1)");
  p.p_drop = (float)p_drop;
  p.seed = (uint32_t)seed;
  p.thresh = (uint32_t)std::min(4294967295.0, p_drop * 4294967296.0);
  return p;
}

std::vector<at::Tensor> attn_fwd(at::Tensor qkv, c10::optional<at::Tensor> mask, double p_drop,
                                 int64_t seed) {
  c10::DeviceGuard guard(qkv.device());
  AttnParams p = attn_params(qkv, mask, p_drop, seed);
  at::Tensor out = at::empty({p.b, p.s, p.h, 64}, qkv.options());
  at::Tensor lse = at::empty({p.b, p.h, p.s}, qkv.options().dtype(at::kFloat));
  p.out = out.data_ptr();
  p.lse = lse.data_ptr<float>();
  mv_attn_fwd(p, cur_stream());
  return {out, lse};
}

at::Tensor attn_bwd(at::Tensor qkv, at::Tensor out, at::Tensor dout, at::Tensor lse,
                    c10::optional<at::Tensor> mask, double p_drop, int64_t seed) {
  c10::DeviceGuard guard(qkv.device());
  AttnParams p = attn_params(qkv, mask, p_drop, seed);
  TORCH_CHECK(out.is_contiguous() && dout.is_contiguous() && out.sizes() == dout.sizes() &&
              out.numel() == (int64_t)p.b * p.s * p.h * 64 &&
              dout.scalar_type() == at::kBFloat16, "attn_bwd: out/dout must be bf16 [b,s,h,64]");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)p.b * p.h * p.s, "attn_bwd: lse");
  TORCH_CHECK((int64_t)p.b * p.s * p.h < (int64_t(1) << 32), "attn_bwd: b*s*h must be < 2^32");
  p.lse = lse.data_ptr<float>();
  auto fo = qkv.options().dtype(at::kFloat);
  const int nkb = (p.s + 63) / 64;
  // s <= 128 runs the single-workgroup-per-(b, h) kernel: no delta / dQ partials
  const bool short_seq = p.s <= 128;
  at::Tensor delta = at::empty({short_seq ? 1 : (int64_t)p.b * p.h * p.s}, fo);
  at::Tensor dq_part = at::empty({short_seq ? 1 : (int64_t)nkb * p.b * p.s * p.h * 64}, fo);
  at::Tensor dqkv = at::empty_like(qkv);
  mv_attn_bwd(p, out.data_ptr(), dout.data_ptr(), delta.data_ptr<float>(),
              dq_part.data_ptr<float>(), dqkv.data_ptr(), cur_stream());
  return dqkv;
}

at::Tensor attn_dropout_mask(int64_t b, int64_t h, int64_t s, double p_drop, int64_t seed,
                             at::Device device) {
  c10::DeviceGuard guard(device);
  at::Tensor keep = at::empty({b, h, s, s}, at::TensorOptions().dtype(at::kByte).device(device));
  const uint32_t th = (uint32_t)std::min(4294967295.0, p_drop * 4294967296.0);
  mv_attn_dropout_mask((int)b, (int)h, (int)s, (uint32_t)seed, th, keep.data_ptr<uint8_t>(),
                       cur_stream());
  return keep;
}

// ---------------------------------------------------------------------------
// Fused transformer elementwise ops (bias+GELU, bias+dropout+residual+LayerNorm)
// ---------------------------------------------------------------------------
void check_rows(const at::Tensor& t, int64_t M, int64_t N, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(),
              "tx: ", what, " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(t.numel() == M * N, "tx: ", what, " has ", t.numel(), " elements, expected ",
              M * N);
}
uint32_t drop_thresh(double p) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "tx: dropout must be in [0, 1)");
  return (uint32_t)std::min(4294967295.0, p * 4294967296.0);
}

at::Tensor bias_gelu_fwd(at::Tensor x, at::Tensor b) {
  c10::DeviceGuard guard(x.device());
  const int64_t N = b.numel(), M = N ? x.numel() / N : 0;
  TORCH_CHECK(N % 8 == 0 && x.size(-1) == N, "bias_gelu: last dim must equal bias size (%8)");
  check_rows(x, M, N, "x");
  check_rows(b, 1, N, "bias");
  at::Tensor y = at::empty_like(x);
  if (M) mv_bias_gelu_fwd(x.data_ptr(), b.data_ptr(), y.data_ptr(), M, (int)N, cur_stream());
  return y;
}

std::vector<at::Tensor> bias_gelu_bwd(at::Tensor dy, at::Tensor x, at::Tensor b) {
  c10::DeviceGuard guard(x.device());
  const int64_t N = b.numel(), M = N ? x.numel() / N : 0;
  TORCH_CHECK(N % 8 == 0 && x.size(-1) == N, "bias_gelu: last dim must equal bias size (%8)");
  check_rows(x, M, N, "x");
  check_rows(dy, M, N, "dy");
  check_rows(b, 1, N, "bias");
  at::Tensor dx = at::empty_like(x);
  at::Tensor db = M ? at::empty_like(b) : at::zeros_like(b);
  if (M) {
    at::Tensor partial =
        at::empty({mv_bias_gelu_partials(M, (int)N), N}, x.options().dtype(at::kFloat));
    mv_bias_gelu_bwd(dy.data_ptr(), x.data_ptr(), b.data_ptr(), dx.data_ptr(),
                     partial.data_ptr<float>(), db.data_ptr(), M, (int)N, cur_stream());
  }
  return {dx, db};
}

std::vector<at::Tensor> ln_fwd(at::Tensor z, c10::optional<at::Tensor> bias,
                               c10::optional<at::Tensor> res, at::Tensor gamma, at::Tensor beta,
                               double eps, double p_drop, int64_t seed, bool save_v) {
  c10::DeviceGuard guard(z.device());
  const int64_t H = gamma.numel(), M = H ? z.numel() / H : 0;
  TORCH_CHECK(H % 8 == 0 && H <= 4096 && z.size(-1) == H,
              "ln: hidden size must be a multiple of 8, <= 4096, and match the last dim");
  check_rows(z, M, H, "z");
  check_rows(gamma, 1, H, "gamma");
  check_rows(beta, 1, H, "beta");
  LnFwdParams p{};
  p.z = z.data_ptr();
  if (bias.has_value() && bias->defined()) {
    check_rows(*bias, 1, H, "bias");
    p.bias = bias->data_ptr();
  }
  if (res.has_value() && res->defined()) {
    check_rows(*res, M, H, "residual");
    p.res = res->data_ptr();
  }
  p.gamma = gamma.data_ptr();
  p.beta = beta.data_ptr();
  at::Tensor y = at::empty_like(z);
  at::Tensor v;
  // without dropout/bias/residual the pre-LN value is z itself
  const bool v_is_z = !p.bias && !p.res && p_drop == 0.0;
  if (save_v) v = v_is_z ? z : at::empty_like(z);
  auto fo = z.options().dtype(at::kFloat);
  at::Tensor mean = at::empty({M}, fo), rstd = at::empty({M}, fo);
  p.v = (save_v && !v_is_z) ? v.data_ptr() : nullptr;
  p.y = y.data_ptr();
  p.mean = mean.data_ptr<float>();
  p.rstd = rstd.data_ptr<float>();
  p.M = M;
  p.H = (int)H;
  p.eps = (float)eps;
  p.p_drop = (float)p_drop;
  p.seed = (uint32_t)seed;
  p.thresh = drop_thresh(p_drop);
  if (M) mv_ln_fwd(p, cur_stream());
  return {y, v, mean, rstd};
}

// -> {dv, dz (undefined when p_drop == 0: equals dv), dgamma, dbeta, dbias}
std::vector<at::Tensor> ln_bwd(at::Tensor dy, at::Tensor v, at::Tensor mean, at::Tensor rstd,
                               at::Tensor gamma, double p_drop, int64_t seed, bool need_dbias,
                               c10::optional<at::Tensor> dy2) {
  c10::DeviceGuard guard(dy.device());
  const int64_t H = gamma.numel(), M = H ? dy.numel() / H : 0;
  TORCH_CHECK(H % 8 == 0 && H <= 4096, "ln: hidden size must be a multiple of 8, <= 4096");
  check_rows(dy, M, H, "dy");
  if (dy2.has_value()) check_rows(*dy2, M, H, "dy2");
  check_rows(v, M, H, "v");
  check_rows(gamma, 1, H, "gamma");
  TORCH_CHECK(mean.numel() == M && rstd.numel() == M && mean.scalar_type() == at::kFloat &&
              rstd.scalar_type() == at::kFloat, "ln_bwd: mean/rstd must be fp32 [M]");
  at::Tensor dv = at::empty_like(dy);
  at::Tensor dz = p_drop > 0.0 ? at::empty_like(dy) : at::Tensor();
  // every column sum is written by the finalize kernel when M > 0
  auto alloc = [&]() { return M ? at::empty_like(gamma) : at::zeros_like(gamma); };
  at::Tensor dg = alloc(), db = alloc();
  at::Tensor dbias = need_dbias ? alloc() : at::Tensor();
  if (M) {
    at::Tensor partial = at::empty({mv_ln_partials(M), 3, H}, dy.options().dtype(at::kFloat));
    LnBwdParams p{};
    p.dy = dy.data_ptr();
    p.v = v.data_ptr();
    p.mean = mean.data_ptr<float>();
    p.rstd = rstd.data_ptr<float>();
    p.gamma = gamma.data_ptr();
    p.dv = dv.data_ptr();
    p.dz = dz.defined() ? dz.data_ptr() : nullptr;
    p.partial = partial.data_ptr<float>();
    p.M = M;
    p.H = (int)H;
    p.p_drop = (float)p_drop;
    p.seed = (uint32_t)seed;
    p.thresh = drop_thresh(p_drop);
    p.dy2 = dy2.has_value() ? dy2->data_ptr() : nullptr;
    mv_ln_bwd(p, dg.data_ptr(), db.data_ptr(), need_dbias ? dbias.data_ptr() : nullptr,
              cur_stream());
  }
  return {dv, dz, dg, db, dbias};
}

// ---------------------------------------------------------------------------
// NHWC pooling
// ---------------------------------------------------------------------------
void check_nhwc(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 4 &&
              t.is_contiguous(at::MemoryFormat::ChannelsLast) && t.size(1) % 8 == 0,
              "pool: ", what, " must be a channels_last bf16 GPU tensor with C % 8 == 0");
}

std::vector<at::Tensor> maxpool_fwd(at::Tensor x, c10::optional<at::Tensor> scale,
                                    c10::optional<at::Tensor> bias, bool relu, int64_t k,
                                    int64_t s, int64_t p) {
  check_nhwc(x, "x");
  TORCH_CHECK(k >= 1 && k * k <= 255 && s >= 1 && p >= 0 && 2 * p <= k, "maxpool: bad window");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 * p - k) / s + 1, OW = (W + 2 * p - k) / s + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "maxpool: empty output");
  TORCH_CHECK(N * OH * OW * (C / 8) < (int64_t(1) << 32),
              "maxpool: the kernel indexes N*OH*OW*C/8 lanes in 32 bits");
  const float* sp = nullptr;
  const float* bp = nullptr;
  if (scale.has_value() && scale->defined()) {
    TORCH_CHECK(bias.has_value() && bias->defined(), "maxpool: scale needs bias");
    sp = opt_f32(scale, C, "scale");
    bp = opt_f32(bias, C, "bias");
  }
  c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor idx = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  mv_maxpool_fwd(x.data_ptr(), sp, bp, relu, y.data_ptr(), idx.data_ptr<uint8_t>(), (int)N,
                 (int)H, (int)W, (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p, cur_stream());
  return {y, idx};
}

at::Tensor maxpool_bwd(at::Tensor dy, c10::optional<at::Tensor> dy2, at::Tensor idx, int64_t H,
                       int64_t W, int64_t k, int64_t s, int64_t p) {
  check_nhwc(dy, "dy");
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  TORCH_CHECK(OH == (H + 2 * p - k) / s + 1 && OW == (W + 2 * p - k) / s + 1,
              "maxpool_bwd: output size does not match the window");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() &&
              idx.numel() == dy.numel(), "maxpool_bwd: idx must be uint8 [N, OH, OW, C]");
  TORCH_CHECK(N * H * W * (C / 8) < (int64_t(1) << 32),
              "maxpool_bwd: the kernel indexes N*H*W*C/8 lanes in 32 bits");
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    check_nhwc(*dy2, "dy2");
    TORCH_CHECK(dy2->sizes() == dy.sizes(), "maxpool_bwd: dy2 shape");
    d2 = dy2->data_ptr();
  }
  c10::DeviceGuard guard(dy.device());
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  mv_maxpool_bwd(dy.data_ptr(), d2, idx.data_ptr<uint8_t>(), dx.data_ptr(), (int)N, (int)H, (int)W,
                 (int)C, (int)OH, (int)OW, (int)k, (int)s, (int)p, cur_stream());
  return dx;
}

// [5, C] fp32 {dgamma, dbeta, ca, cb, cc} of the BN+ReLU in front of a maxpool, from a reduce
// over the pooled tensors (dy, dy2, the pooled output y); M = the BN's element rows
static at::Tensor pool_bn_coefs(const at::Tensor& dy, const void* d2, const at::Tensor& y,
                                const at::Tensor& vec, const c10::optional<at::Tensor>& gamma,
                                int64_t M) {
  const int64_t C = dy.size(1);
  auto fo = dy.options().dtype(at::kFloat);
  at::Tensor part = at::empty({(int64_t)mv_pool_bn_partials(), 2, C}, fo);
  mv_pool_bn_reduce(dy.data_ptr(), d2, y.data_ptr(), vec[0].data_ptr<float>(),
                    vec[2].data_ptr<float>(), vec[3].data_ptr<float>(), part.data_ptr<float>(),
                    dy.numel() / C, (int)C, cur_stream());
  at::Tensor work = at::empty({5, C}, fo);
  mv_bn_bwd_from_partials(nullptr, nullptr, nullptr, M, (int)C, vec[0].data_ptr<float>(),
                          vec[1].data_ptr<float>(), opt_f32(gamma, C, "weight"),
                          vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                          work[0].data_ptr<float>(), work[1].data_ptr<float>(),
                          part.data_ptr<float>(), (int)part.size(0), work[2].data_ptr<float>(),
                          work[3].data_ptr<float>(), work[4].data_ptr<float>(), cur_stream());
  return work;
}

// {dx, dgamma, dbeta}: maxpool(3, 2, 1) backward fused with the backward of the BN+ReLU that
// produced its input z (ResNet stem): y = the pooled output, vec = the BN's saved [4, C]
std::vector<at::Tensor> maxpool_bn_bwd(at::Tensor dy, c10::optional<at::Tensor> dy2,
                                       at::Tensor idx, at::Tensor y, at::Tensor z, at::Tensor vec,
                                       c10::optional<at::Tensor> gamma) {
  check_nhwc(dy, "dy");
  check_nhwc(y, "y");
  check_nhwc(z, "z");
  const int64_t N = dy.size(0), C = dy.size(1), OH = dy.size(2), OW = dy.size(3);
  const int64_t H = z.size(2), W = z.size(3);
  TORCH_CHECK(y.sizes() == dy.sizes() && z.size(0) == N && z.size(1) == C && H % 2 == 0 &&
                  W % 2 == 0 && OH == H / 2 && OW == W / 2 && C % 8 == 0 && C <= 256,
              "maxpool_bn_bwd: needs a 3x3 / 2 / pad-1 pool of an even-sized input, C % 8 == 0, C <= 256");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.is_contiguous() &&
              idx.numel() == dy.numel(), "maxpool_bn_bwd: idx must be uint8 [N, OH, OW, C]");
  TORCH_CHECK(N * H * W * (C / 8) < (int64_t(1) << 32), "maxpool_bn_bwd: too large");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
                  vec.numel() == 4 * C, "maxpool_bn_bwd: saved stats must be fp32 [4, C]");
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    check_nhwc(*dy2, "dy2");
    TORCH_CHECK(dy2->sizes() == dy.sizes(), "maxpool_bn_bwd: dy2 shape");
    d2 = dy2->data_ptr();
  }
  c10::DeviceGuard guard(dy.device());
  at::Tensor work = pool_bn_coefs(dy, d2, y, vec, gamma, N * H * W);
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  TORCH_CHECK(mv_maxpool_bn_bwd(dy.data_ptr(), d2, idx.data_ptr<uint8_t>(), z.data_ptr(),
                                vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                                work[2].data_ptr<float>(), work[3].data_ptr<float>(),
                                work[4].data_ptr<float>(), dx.data_ptr(), (int)N, (int)H, (int)W,
                                (int)C, (int)OH, (int)OW, cur_stream()),
              "maxpool_bn_bwd: launch failed");
  return {dx, work[0], work[1]};
}

at::Tensor gap_fwd(at::Tensor x) {
  check_nhwc(x, "x");
  c10::DeviceGuard guard(x.device());
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  at::Tensor y = at::empty({N, C}, x.options());
  mv_gap_fwd(x.data_ptr(), y.data_ptr(), (int)N, (int)HW, (int)C, cur_stream());
  return y;
}

at::Tensor gap_bwd(at::Tensor dy, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 &&
              dy.is_contiguous() && dy.size(1) % 8 == 0, "gap_bwd: dy must be bf16 [N, C]");
  c10::DeviceGuard guard(dy.device());
  const int64_t N = dy.size(0), C = dy.size(1);
  TORCH_CHECK(N * H * W * (C / 8) < (int64_t(1) << 32),
              "gap_bwd: the kernel indexes N*H*W*C/8 lanes in 32 bits");
  at::Tensor dx = at::empty({N, C, H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
  mv_gap_bwd(dy.data_ptr(), dx.data_ptr(), (int)N, (int)(H * W), (int)C, cur_stream());
  return dx;
}

at::Tensor pad_channels(at::Tensor x, int64_t cout) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
              x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "pad_channels: x must be a channels_last bf16 GPU tensor");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(C >= 1 && C <= 8 && cout >= C && cout <= 8, "pad_channels: need C <= cout <= 8");
  c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty({N, cout, H, W},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  mv_pad_channels(x.data_ptr(), y.data_ptr(), N * H * W, (int)C, (int)cout, cur_stream());
  return y;
}

// ---------------------------------------------------------------------------
// NT GEMM for NHWC 1x1 convolutions (+ fused BN statistics epilogue)
// ---------------------------------------------------------------------------
int64_t gemm_partials(int64_t M, int64_t N, int64_t K) {
  return mv_gemm_partials(M, (int)N, (int)K);
}

void gemm_nt(at::Tensor a, at::Tensor b, c10::optional<at::Tensor> co,
             c10::optional<at::Tensor> shift, c10::optional<at::Tensor> partial) {
  // c = None: statistics only (C is not written) — the recompute pass of ops.bn's fold
  const bool has_c = co.has_value() && co->defined();
  at::Tensor c = has_c ? *co : at::Tensor();
  for (const at::Tensor* t : {&a, &b})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2,
                "gemm_nt: A, B, C must be contiguous 2-D bf16 GPU tensors");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  if (has_c) {
    TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kBFloat16 && c.is_contiguous() && c.dim() == 2,
                "gemm_nt: C must be a contiguous 2-D bf16 GPU tensor");
    TORCH_CHECK(c.size(0) == M && c.size(1) == N && a.device() == c.device(),
                "gemm_nt: C shape/device mismatch");
  } else {
    TORCH_CHECK(partial.has_value() && mv_gemm_apply_supported((int)N, (int)K),
                "gemm_nt: C may be omitted only for a statistics pass on a streamed shape");
  }
  TORCH_CHECK(b.size(1) == K, "gemm_nt: shape mismatch");
  TORCH_CHECK(K % 64 == 0 && N % 64 == 0 && K > 0 && N > 0 && M > 0,
              "gemm_nt: K and N must be positive multiples of 64");
  TORCH_CHECK(a.device() == b.device(), "gemm_nt: devices differ");
  TORCH_CHECK(M * K < (int64_t(1) << 40) && M * N < (int64_t(1) << 40), "gemm_nt: too large");
  TORCH_CHECK((M + 63) / 64 * (N / 64) < (int64_t(1) << 31), "gemm_nt: grid too large");
  float* pp = nullptr;
  const float* sp = nullptr;
  if (partial.has_value()) {
    TORCH_CHECK(partial->is_cuda() && partial->scalar_type() == at::kFloat &&
                    partial->is_contiguous() && partial->numel() >= gemm_partials(M, N, K) * 2 * N,
                "gemm_nt: partial must be fp32 [P, 2, N] with P = gemm_partials(M, N)");
    pp = partial->data_ptr<float>();
    if (shift.has_value()) {
      TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->numel() == N,
                  "gemm_nt: shift must be fp32 [N]");
      sp = shift->data_ptr<float>();
    }
  }
  c10::DeviceGuard guard(a.device());
  mv_gemm_nt(a.data_ptr(), b.data_ptr(), has_c ? c.data_ptr() : nullptr, M, (int)N, (int)K, sp,
             pp, cur_stream());
}

// the 256 x 256 kernel alone (A/B against gemm_nt's routing; plain C, no statistics)
void gemm256_nt(at::Tensor a, at::Tensor b, at::Tensor c) {
  for (const at::Tensor* t : {&a, &b, &c})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->device() == a.device(),
                "gemm256_nt: A, B, C must be contiguous 2-D bf16 tensors on one GPU");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && c.size(0) == M && c.size(1) == N, "gemm256_nt: shape mismatch");
  TORCH_CHECK(mv_gemm256_supported(M, (int)N, (int)K),
              "gemm256_nt: needs N % 256 == 0 and K % 64 == 0");
  c10::DeviceGuard guard(a.device());
  mv_gemm256_nt(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, (int)N, (int)K, nullptr, nullptr,
                cur_stream());
}

// strided 1x1 conv forward on the 256 x 256 kernel: y[Nb, Ho, Wo, N] (NHWC, returned as
// channels_last NCHW) = conv1x1(x, w, stride ds), + BN statistics partials when shift is
// given; None when the shape is not covered
c10::optional<std::vector<at::Tensor>> conv1x1_strided_stats(at::Tensor x, at::Tensor w, int64_t ds,
                                                             c10::optional<at::Tensor> shift) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv1x1_strided_stats: x must be a channels_last bf16 GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 1 &&
                  w.size(3) == 1 && w.size(1) == x.size(1) && w.device() == x.device(),
              "conv1x1_strided_stats: w must be a bf16 [N, C, 1, 1] filter");
  TORCH_CHECK(ds >= 1, "conv1x1_strided_stats: stride >= 1");
  const int64_t Nb = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), N = w.size(0);
  const int64_t Ho = (H - 1) / ds + 1, Wo = (W - 1) / ds + 1, M = Nb * Ho * Wo;
  if (!mv_gemm256_supported(M, (int)N, (int)C) || (shift.has_value() && N > 8192))
    return c10::nullopt;
  c10::DeviceGuard guard(x.device());
  at::Tensor w2 = w.reshape({N, C}).contiguous();
  at::Tensor y = at::empty({Nb, N, Ho, Wo}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor part;
  float* pp = nullptr;
  const float* sp = nullptr;
  if (shift.has_value()) {
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->numel() == N,
                "conv1x1_strided_stats: shift must be fp32 [N]");
    part = at::empty({mv_gemm256_partials(M, (int)N), 2, N}, x.options().dtype(at::kFloat));
    pp = part.data_ptr<float>();
    sp = shift->data_ptr<float>();
  }
  if (!mv_gemm256_strided(x.data_ptr(), w2.data_ptr(), y.data_ptr(), (int)Nb, (int)H, (int)W,
                          (int)C, (int)N, (int)ds, sp, pp, cur_stream()))
    return c10::nullopt;
  std::vector<at::Tensor> out{y};
  if (pp) out.push_back(part);
  return out;
}

int64_t gemm_fold_dx_partials(int64_t M, int64_t K1, int64_t K2) {
  return mv_gemm_fold_dx_partials(M, (int)K1, (int)K2);
}

// The BN3 fold's data gradient with BN2's ReLU backward reduce: d = relu'(bn2(xb)) *
// ([a1 | a2] . b^T + badd) -> d (bf16 [M, K2]); returns the [P, 2, K2] partials
at::Tensor gemm_fold_dx(at::Tensor a1, at::Tensor a2, at::Tensor b, at::Tensor badd, at::Tensor d,
                        at::Tensor xb, at::Tensor vec) {
  for (const at::Tensor* t : {&a1, &a2, &b, &d, &xb})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->device() == a1.device(),
                "gemm_fold_dx: A1, A2, B, D, xb must be contiguous 2-D bf16 tensors on one GPU");
  const int64_t M = a1.size(0), K1 = a1.size(1), K2 = a2.size(1);
  TORCH_CHECK(M > 0 && a2.size(0) == M && b.size(0) == K2 && b.size(1) == K1 + K2 &&
                  d.size(0) == M && d.size(1) == K2 && xb.size(0) == M && xb.size(1) == K2,
              "gemm_fold_dx: shape mismatch");
  TORCH_CHECK(M * (K1 + K2) < (int64_t(1) << 40), "gemm_fold_dx: too large");
  TORCH_CHECK(badd.is_cuda() && badd.scalar_type() == at::kFloat && badd.is_contiguous() &&
                  badd.numel() == K2 && badd.device() == a1.device(),
              "gemm_fold_dx: badd must be fp32 [K2]");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
                  vec.numel() == 4 * K2 && vec.device() == a1.device(),
              "gemm_fold_dx: saved stats must be fp32 [4, K2]");
  const int64_t P = mv_gemm_fold_dx_partials(M, (int)K1, (int)K2);
  TORCH_CHECK(P > 0, "gemm_fold_dx: unsupported (K1, K2)");
  c10::DeviceGuard guard(a1.device());
  at::Tensor partial = at::empty({P, 2, K2}, a1.options().dtype(at::kFloat));
  TORCH_CHECK(mv_gemm_fold_dx(a1.data_ptr(), a2.data_ptr(), b.data_ptr(), badd.data_ptr<float>(),
                              d.data_ptr(), M, (int)K1, (int)K2, xb.data_ptr(),
                              vec[0].data_ptr<float>(), vec[2].data_ptr<float>(),
                              vec[3].data_ptr<float>(), partial.data_ptr<float>(), cur_stream()),
              "gemm_fold_dx: launch failed");
  return partial;
}

bool gemm_dual_supported(int64_t K1, int64_t K2) { return mv_gemm_dual_supported((int)K1, (int)K2); }

// D [M, N] = [A1 | x[:, :, ::s, ::s]] . B^T + badd on the 256 x 256 pipeline with the second
// source gathered from the channels_last x [Nb, K2, H, W] (no strided copy); false when the
// shape is not covered (N % 256 or the K splits)
bool gemm_dual_bias_strided(at::Tensor a1, at::Tensor x, int64_t stride, at::Tensor b,
                            at::Tensor badd, at::Tensor d) {
  for (const at::Tensor* t : {&a1, &b, &d})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 2 &&
                    t->is_contiguous() && t->device() == a1.device(),
                "gemm_dual_bias_strided: A1, B, D must be contiguous 2-D bf16 tensors on one GPU");
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.device() == a1.device(),
              "gemm_dual_bias_strided: x must be a channels_last bf16 [Nb, K2, H, W] tensor");
  TORCH_CHECK(stride >= 1 && stride < 65536 && x.size(2) < 65536 && x.size(3) < 65536,
              "gemm_dual_bias_strided: bad stride / size");
  const int64_t M = a1.size(0), K1 = a1.size(1), K2 = x.size(1), N = b.size(0);
  const int64_t H = x.size(2), W = x.size(3);
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(M == x.size(0) * Ho * Wo && b.size(1) == K1 + K2 && d.size(0) == M &&
                  d.size(1) == N, "gemm_dual_bias_strided: shape mismatch");
  TORCH_CHECK(badd.is_cuda() && badd.scalar_type() == at::kFloat && badd.is_contiguous() &&
                  badd.numel() == N && badd.device() == a1.device(),
              "gemm_dual_bias_strided: badd must be fp32 [N]");
  c10::DeviceGuard guard(a1.device());
  return mv_gemm256_dual(a1.data_ptr(), x.data_ptr(), b.data_ptr(), badd.data_ptr<float>(),
                         d.data_ptr(), M, (int)K1, (int)K2, (int)N, nullptr, nullptr, nullptr,
                         nullptr, nullptr, cur_stream(), (int)stride, (int)H, (int)W);
}

// d = [a1 | a2] . b^T + badd (bf16 [M, K2])
void gemm_dual_bias(at::Tensor a1, at::Tensor a2, at::Tensor b, at::Tensor badd, at::Tensor d) {
  for (const at::Tensor* t : {&a1, &a2, &b, &d})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->device() == a1.device(),
                "gemm_dual_bias: A1, A2, B, D must be contiguous 2-D bf16 tensors on one GPU");
  const int64_t M = a1.size(0), K1 = a1.size(1), K2 = a2.size(1);
  TORCH_CHECK(M > 0 && a2.size(0) == M && b.size(0) == K2 && b.size(1) == K1 + K2 &&
                  d.size(0) == M && d.size(1) == K2 && M * (K1 + K2) < (int64_t(1) << 40),
              "gemm_dual_bias: shape mismatch");
  TORCH_CHECK(badd.is_cuda() && badd.scalar_type() == at::kFloat && badd.is_contiguous() &&
                  badd.numel() == K2 && badd.device() == a1.device(),
              "gemm_dual_bias: badd must be fp32 [K2]");
  TORCH_CHECK(mv_gemm_dual_supported((int)K1, (int)K2), "gemm_dual_bias: unsupported (K1, K2)");
  c10::DeviceGuard guard(a1.device());
  TORCH_CHECK(mv_gemm_dual_bias(a1.data_ptr(), a2.data_ptr(), b.data_ptr(), badd.data_ptr<float>(),
                                d.data_ptr(), M, (int)K1, (int)K2, cur_stream()),
              "gemm_dual_bias: launch failed");
}

static void fold_check_f32(const at::Tensor& t, int64_t n, const at::Device& d, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n &&
                  t.device() == d, "fold: ", what, " must be a contiguous fp32 tensor of ", n,
              " elements on the GPU");
}

// {co [5, cout], xsum [cin]}: the BN fold's per-channel coefficients from the consumer's
// reduce partials part [P, 2, cout], W [cout, cin] (bf16), g = dz^T x [cout, cin] (fp32),
// the BN's saved vec [4, cout] and gamma; xsum from colsum partials [P2, cin] (or zeros
// when colsum is None — the caller supplies it)
// [1, 2, cout] BN statistics partials of z = x W^T around shift from the Gram matrix
// gram = x^T x ([cin, cin] fp32) and xsum = colsum(x) [cin] (mv_fold.hip gram_stats_kernel)
at::Tensor gram_stats(at::Tensor w, at::Tensor gram, at::Tensor xsum,
                      c10::optional<at::Tensor> shift, int64_t m) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() &&
                  w.dim() == 2, "gram_stats: W must be contiguous bf16 [cout, cin]");
  const int64_t cout = w.size(0), cin = w.size(1);
  TORCH_CHECK(gram.device() == w.device() && gram.scalar_type() == at::kFloat &&
                  gram.is_contiguous() && gram.numel() == cin * cin,
              "gram_stats: gram must be contiguous fp32 [cin, cin]");
  TORCH_CHECK(xsum.device() == w.device() && xsum.scalar_type() == at::kFloat &&
                  xsum.is_contiguous() && xsum.numel() == cin,
              "gram_stats: xsum must be contiguous fp32 [cin]");
  TORCH_CHECK(m > 0, "gram_stats: m must be positive");
  const float* sh = opt_f32(shift, cout, "shift");
  c10::DeviceGuard guard(w.device());
  at::Tensor part = at::empty({1, 2, cout}, gram.options());
  TORCH_CHECK(mv_gram_stats(w.data_ptr(), gram.data_ptr<float>(), xsum.data_ptr<float>(), sh, m,
                            (int)cout, (int)cin, part.data_ptr<float>(), cur_stream()),
              "gram_stats: needs cout % 16 == 0 and cin <= 1024");
  return part;
}

std::vector<at::Tensor> fold_coeffs(at::Tensor part, at::Tensor w, at::Tensor g, at::Tensor vec,
                                    c10::optional<at::Tensor> gamma, int64_t M,
                                    c10::optional<at::Tensor> colsum) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2,
              "fold_coeffs: W must be contiguous bf16 [cout, cin]");
  const int64_t cout = w.size(0), cin = w.size(1);
  const auto d = w.device();
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.dim() == 3 && part.size(1) == 2 && part.size(2) == cout &&
                  part.size(0) > 0 && part.device() == d,
              "fold_coeffs: part must be fp32 [P, 2, cout]");
  fold_check_f32(g, cout * cin, d, "g");
  fold_check_f32(vec, 4 * cout, d, "vec");
  const float* gp = nullptr;
  if (gamma.has_value() && gamma->defined()) {
    fold_check_f32(*gamma, cout, d, "gamma");
    gp = gamma->data_ptr<float>();
  }
  const float* cs = nullptr;
  int P2 = 0;
  if (colsum.has_value() && colsum->defined()) {
    TORCH_CHECK(colsum->is_cuda() && colsum->scalar_type() == at::kFloat && colsum->dim() == 2 &&
                    colsum->size(1) == cin && colsum->stride(1) == 1 && colsum->stride(0) == cin &&
                    colsum->device() == d,
                "fold_coeffs: colsum must be fp32 [P2, cin] row-contiguous");
    cs = colsum->data_ptr<float>();
    P2 = (int)colsum->size(0);
  }
  TORCH_CHECK(M > 0, "fold_coeffs: M must be positive");
  c10::DeviceGuard guard(d);
  at::Tensor co = at::empty({5, cout}, part.options());
  at::Tensor xsum = cs ? at::empty({cin}, part.options()) : at::zeros({cin}, part.options());
  mv_fold_coeffs(part.data_ptr<float>(), (int)part.size(0), w.data_ptr(), g.data_ptr<float>(),
                 vec.data_ptr<float>(), gp, M, (int)cout, (int)cin, cs, P2, co.data_ptr<float>(),
                 xsum.data_ptr<float>(), cur_stream());
  return {co, xsum};
}

// {dW bf16 [cout, cin] (undefined if not need_w), bcat bf16 [cin, cout + cin], badd fp32 [cin]}
std::vector<at::Tensor> fold_products(at::Tensor w, at::Tensor g, c10::optional<at::Tensor> gram,
                                      at::Tensor co, at::Tensor xsum, bool need_w) {
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2,
              "fold_products: W must be contiguous bf16 [cout, cin]");
  const int64_t cout = w.size(0), cin = w.size(1);
  TORCH_CHECK(cout % 64 == 0 && cin % 64 == 0 && cout > 0 && cin > 0,
              "fold_products: channels must be positive multiples of 64 (64x64 tiles)");
  const auto d = w.device();
  fold_check_f32(g, cout * cin, d, "g");
  fold_check_f32(co, 5 * cout, d, "co");
  fold_check_f32(xsum, cin, d, "xsum");
  const float* gr = nullptr;
  if (need_w) {
    TORCH_CHECK(gram.has_value() && gram->defined(), "fold_products: need_w needs the Gram matrix");
    fold_check_f32(*gram, cin * cin, d, "gram");
    gr = gram->data_ptr<float>();
  }
  c10::DeviceGuard guard(d);
  at::Tensor dw = need_w ? at::empty({cout, cin}, w.options()) : at::Tensor();
  at::Tensor bcat = at::empty({cin, cout + cin}, w.options());
  at::Tensor badd = at::empty({cin}, co.options());
  mv_fold_products(w.data_ptr(), g.data_ptr<float>(), gr, co.data_ptr<float>(),
                   xsum.data_ptr<float>(), (int)cout, (int)cin, need_w ? dw.data_ptr() : nullptr,
                   bcat.data_ptr(), badd.data_ptr<float>(), cur_stream());
  return {dw, bcat, badd};
}

// {z [N, 64, 112, 112] channels_last bf16, partial [P, 2, 64]}: the ResNet stem conv
// (7x7 / 2 / pad 3 on a 4-channel 224x224 NHWC image) with BN statistics around shift
std::vector<at::Tensor> stem_fwd(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> shift,
                                 int64_t grid) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  (x.size(1) == 4 || x.size(1) == 3) && x.size(2) == 224 && x.size(3) == 224 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_fwd: x must be a channels_last bf16 [N, 3 or 4, 224, 224] GPU tensor");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == 64 &&
                  w.size(1) == 4 && w.size(2) == 7 && w.size(3) == 7 &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.device() == x.device(),
              "stem_fwd: w must be a channels_last bf16 [64, 4, 7, 7] tensor on x's device");
  const int64_t N = x.size(0);
  TORCH_CHECK(N > 0 && N * 112 < (int64_t(1) << 31), "stem_fwd: bad batch");
  const float* sp = nullptr;
  if (shift.has_value() && shift->defined()) {
    TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->is_contiguous() &&
                    shift->numel() == 64 && shift->device() == x.device(),
                "stem_fwd: shift must be fp32 [64]");
    sp = shift->data_ptr<float>();
  }
  c10::DeviceGuard guard(x.device());
  at::Tensor z = at::empty({N, 64, 112, 112},
                           x.options().memory_format(at::MemoryFormat::ChannelsLast));
  // grid > 0: a non-default persistent grid (tests); any size >= 1 is valid — the
  // kernel's row loop and the partial rows follow the grid
  TORCH_CHECK(grid >= 0 && grid <= (int64_t(1) << 20), "stem_fwd: bad grid");
  const int g = grid > 0 ? (int)grid : mv_stem_partials((int)N);
  at::Tensor part = at::empty({(int64_t)g, 2, 64}, x.options().dtype(at::kFloat));
  mv_stem_fwd(x.data_ptr(), w.data_ptr(), z.data_ptr(), sp, part.data_ptr<float>(), (int)N,
              cur_stream(), g, (int)x.size(1));
  return {z, part};
}

// dw [64, 4, 7, 7] channels_last bf16: the stem conv's weight gradient (mv_stem.hip)
at::Tensor stem_wgrad(at::Tensor x, at::Tensor dz) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  (x.size(1) == 4 || x.size(1) == 3) && x.size(2) == 224 && x.size(3) == 224 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_wgrad: x must be a channels_last bf16 [N, 3 or 4, 224, 224] GPU tensor");
  const int64_t N = x.size(0);
  TORCH_CHECK(dz.is_cuda() && dz.scalar_type() == at::kBFloat16 && dz.dim() == 4 &&
                  dz.size(0) == N && dz.size(1) == 64 && dz.size(2) == 112 && dz.size(3) == 112 &&
                  dz.is_contiguous(at::MemoryFormat::ChannelsLast) && dz.device() == x.device(),
              "stem_wgrad: dz must be a channels_last bf16 [N, 64, 112, 112] tensor on x's device");
  TORCH_CHECK(N > 0 && N * 112 < (int64_t(1) << 31), "stem_wgrad: bad batch");
  c10::DeviceGuard guard(x.device());
  at::Tensor work = at::empty({(int64_t)mv_stem_wgrad_blocks((int)N) * 64 * 224},
                              x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({64, 4, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  mv_stem_wgrad(x.data_ptr(), dz.data_ptr(), dw.data_ptr(), work.data_ptr<float>(), (int)N,
                cur_stream(), (int)x.size(1));
  return dw;
}

// {dw, dgamma, dbeta}: the ResNet stem's maxpool + BN+ReLU backward and its conv's weight
// gradient in one pass over the rows (mv_stem.hip, MvStemPoolBwd): the full-resolution dz is
// never written.  x: the stem input, z: the conv output, y / idx: the pooled output and its
// window argmax, vec: the BN's saved [4, 64]; dy (+ dy2): the pooled gradients.
std::vector<at::Tensor> stem_wgrad_pool_bn(at::Tensor x, at::Tensor dy,
                                           c10::optional<at::Tensor> dy2, at::Tensor idx,
                                           at::Tensor y, at::Tensor z, at::Tensor vec,
                                           c10::optional<at::Tensor> gamma) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  (x.size(1) == 4 || x.size(1) == 3) && x.size(2) == 224 && x.size(3) == 224 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "stem_wgrad_pool_bn: x must be a channels_last bf16 [N, 3 or 4, 224, 224] GPU tensor");
  const int64_t N = x.size(0);
  check_nhwc(z, "z");
  check_nhwc(dy, "dy");
  check_nhwc(y, "y");
  TORCH_CHECK(z.sizes() == at::IntArrayRef({N, 64, 112, 112}) && z.device() == x.device(),
              "stem_wgrad_pool_bn: z must be [N, 64, 112, 112] on x's device");
  TORCH_CHECK(dy.sizes() == at::IntArrayRef({N, 64, 56, 56}) && y.sizes() == dy.sizes() &&
                  dy.device() == x.device() && y.device() == x.device(),
              "stem_wgrad_pool_bn: dy / y must be [N, 64, 56, 56] on x's device");
  TORCH_CHECK(idx.device() == x.device() && idx.scalar_type() == at::kByte &&
                  idx.is_contiguous() && idx.numel() == dy.numel(),
              "stem_wgrad_pool_bn: idx must be uint8 [N, 56, 56, 64]");
  TORCH_CHECK(vec.device() == x.device() && vec.scalar_type() == at::kFloat &&
                  vec.is_contiguous() && vec.numel() == 4 * 64,
              "stem_wgrad_pool_bn: saved stats must be fp32 [4, 64]");
  TORCH_CHECK(N > 0 && N * 112 < (int64_t(1) << 31), "stem_wgrad_pool_bn: bad batch");
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    check_nhwc(*dy2, "dy2");
    TORCH_CHECK(dy2->sizes() == dy.sizes() && dy2->device() == x.device(),
                "stem_wgrad_pool_bn: dy2 shape");
    d2 = dy2->data_ptr();
  }
  c10::DeviceGuard guard(x.device());
  at::Tensor coef = pool_bn_coefs(dy, d2, y, vec, gamma, N * 112 * 112);
  at::Tensor work = at::empty({(int64_t)mv_stem_wgrad_blocks((int)N) * 64 * 224},
                              x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({64, 4, 7, 7}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  MvStemPoolBwd pb{z.data_ptr(), dy.data_ptr(), d2, idx.data_ptr<uint8_t>(),
                   vec[2].data_ptr<float>(), vec[3].data_ptr<float>(), coef[2].data_ptr<float>(),
                   coef[3].data_ptr<float>(), coef[4].data_ptr<float>()};
  mv_stem_wgrad_pool_bn(x.data_ptr(), pb, dw.data_ptr(), work.data_ptr<float>(), (int)N,
                        cur_stream(), (int)x.size(1));
  return {dw, coef[0], coef[1]};
}

bool gemm_apply_supported(int64_t N, int64_t K) { return mv_gemm_apply_supported((int)N, (int)K); }

// {y, mask}: y = relu(bf16(a . b^T) * scale + bias + res) and its [M, N/8] bitmask (the
// GEMM recomputed with the BN+add+ReLU apply in its epilogue)
std::vector<at::Tensor> gemm_nt_apply(at::Tensor a, at::Tensor b, at::Tensor res, at::Tensor scale,
                                      at::Tensor bias, c10::optional<at::Tensor> rscale,
                                      c10::optional<at::Tensor> rbias) {
  for (const at::Tensor* t : {&a, &b, &res})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->device() == a.device(),
                "gemm_nt_apply: A, B, res must be contiguous 2-D bf16 tensors on one GPU");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(M > 0 && b.size(1) == K && res.size(0) == M && res.size(1) == N,
              "gemm_nt_apply: shape mismatch");
  TORCH_CHECK(mv_gemm_apply_supported((int)N, (int)K), "gemm_nt_apply: unsupported (K, N)");
  TORCH_CHECK(M * K < (int64_t(1) << 40) && M * N < (int64_t(1) << 40), "gemm_nt_apply: too large");
  for (const at::Tensor* t : {&scale, &bias})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == N && t->device() == a.device(),
                "gemm_nt_apply: scale/bias must be contiguous fp32 [N]");
  const bool raff = rscale.has_value() && rscale->defined();
  TORCH_CHECK(raff == (rbias.has_value() && rbias->defined()),
              "gemm_nt_apply: rscale and rbias go together");
  if (raff)
    for (const at::Tensor* t : {&*rscale, &*rbias})
      TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                      t->numel() == N && t->device() == a.device(),
                  "gemm_nt_apply: rscale/rbias must be contiguous fp32 [N]");
  c10::DeviceGuard guard(a.device());
  at::Tensor y = at::empty({M, N}, res.options());
  at::Tensor mask = at::empty({M, N / 8}, res.options().dtype(at::kByte));
  TORCH_CHECK(mv_gemm_nt_apply(a.data_ptr(), b.data_ptr(), y.data_ptr(), M, (int)N, (int)K,
                               res.data_ptr(), scale.data_ptr<float>(), bias.data_ptr<float>(),
                               mask.data_ptr(), cur_stream(),
                               raff ? rscale->data_ptr<float>() : nullptr,
                               raff ? rbias->data_ptr<float>() : nullptr),
              "gemm_nt_apply: launch failed");
  return {y, mask};
}

bool gemm_apply_dual_supported(int64_t N, int64_t K) {
  return mv_gemm_apply_dual_supported((int)N, (int)K);
}

// {y, mask}: relu(bf16(a . b^T) * scale + bias + bf16(bf16(a2 . b2^T) * rscale + rbias))
std::vector<at::Tensor> gemm_nt_apply_dual(at::Tensor a, at::Tensor b, at::Tensor a2,
                                           at::Tensor b2, at::Tensor scale, at::Tensor bias,
                                           at::Tensor rscale, at::Tensor rbias) {
  for (const at::Tensor* t : {&a, &b, &a2, &b2})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->device() == a.device(),
                "gemm_nt_apply_dual: A, B, A2, B2 must be contiguous 2-D bf16 tensors on one GPU");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(M > 0 && b.size(1) == K && a2.size(0) == M && a2.size(1) == K && b2.size(0) == N &&
                  b2.size(1) == K && M * N < (int64_t(1) << 40),
              "gemm_nt_apply_dual: shape mismatch");
  TORCH_CHECK(mv_gemm_apply_dual_supported((int)N, (int)K), "gemm_nt_apply_dual: unsupported (K, N)");
  for (const at::Tensor* t : {&scale, &bias, &rscale, &rbias})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                    t->numel() == N && t->device() == a.device(),
                "gemm_nt_apply_dual: scale/bias/rscale/rbias must be contiguous fp32 [N]");
  c10::DeviceGuard guard(a.device());
  at::Tensor y = at::empty({M, N}, a.options());
  at::Tensor mask = at::empty({M, N / 8}, a.options().dtype(at::kByte));
  TORCH_CHECK(mv_gemm_nt_apply_dual(a.data_ptr(), b.data_ptr(), a2.data_ptr(), b2.data_ptr(),
                                    y.data_ptr(), M, (int)N, (int)K, scale.data_ptr<float>(),
                                    bias.data_ptr<float>(), rscale.data_ptr<float>(),
                                    rbias.data_ptr<float>(), mask.data_ptr(), cur_stream()),
              "gemm_nt_apply_dual: launch failed");
  return {y, mask};
}

// {4, C} saved statistics (mean, invstd, scale, bias) + running-stat update from [P, 2, C]
// GEMM-epilogue partials of an M-row activation; no apply pass
at::Tensor bn_finalize(at::Tensor stats, c10::optional<at::Tensor> gamma,
                       c10::optional<at::Tensor> beta, c10::optional<at::Tensor> running_mean,
                       c10::optional<at::Tensor> running_var, double momentum, double eps,
                       int64_t M) {
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.is_contiguous() &&
                  stats.dim() == 3 && stats.size(1) == 2 && stats.size(0) > 0 && M > 0,
              "bn_finalize: stats must be fp32 [P, 2, C] partials");
  const int64_t C = stats.size(2);
  c10::DeviceGuard guard(stats.device());
  at::Tensor vec = at::empty({4, C}, stats.options());
  float* rm = const_cast<float*>(opt_f32(running_mean, C, "running_mean"));
  float* rv = const_cast<float*>(opt_f32(running_var, C, "running_var"));
  TORCH_CHECK((rm == nullptr) == (rv == nullptr), "bn: running_mean/var must both be given");
  mv_bn_fwd_from_partials(nullptr, nullptr, nullptr, M, (int)C, rm, rv, opt_f32(gamma, C, "weight"),
                          opt_f32(beta, C, "bias"), (float)momentum, (float)eps, false,
                          stats.data_ptr<float>(), (int)stats.size(0), vec[0].data_ptr<float>(),
                          vec[1].data_ptr<float>(), vec[2].data_ptr<float>(),
                          vec[3].data_ptr<float>(), cur_stream());
  return vec;
}

int64_t gemm_bwd_partials(int64_t M, int64_t N, int64_t K, int64_t bn) {
  return mv_gemm_bwd_partials(M, (int)N, (int)K, (int)bn);
}

// Data-gradient GEMM of a 1x1 conv fused with the BN+add+ReLU (mode 3) backward
// reduce of the BN that produced the conv's input: dy = a . b^T, dz = mask ? dy + dy2
// : 0 is written to dz, returns the fp32 [P, 2, N] partials (sum dz, sum dz (x - mean)).
// x = None: only sum dz (the second partial is 0; ops.bn._Conv1x1BNFold gets it from its
// weight-gradient GEMM) and the BN input is never read.
at::Tensor gemm_nt_bn_bwd(at::Tensor a, at::Tensor b, at::Tensor dz,
                          c10::optional<at::Tensor> dy2, at::Tensor mask,
                          c10::optional<at::Tensor> xo, at::Tensor vec, int64_t bn,
                          int64_t dy2_stride, int64_t H, int64_t W) {
  const bool has_x = xo.has_value() && xo->defined();
  at::Tensor x = has_x ? *xo : dz;
  for (const at::Tensor* t : {&a, &b, &dz, &x})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous(),
                "gemm_nt_bn_bwd: A, B, dz, x must be contiguous bf16 GPU tensors");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm_nt_bn_bwd: A, B must be 2-D");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && M > 0, "gemm_nt_bn_bwd: shape mismatch");
  TORCH_CHECK(dz.numel() == M * N && x.numel() == M * N, "gemm_nt_bn_bwd: dz/x must be [M, N]");
  TORCH_CHECK(M * N < (int64_t(1) << 40) && N % 64 == 0, "gemm_nt_bn_bwd: bad size");
  const int64_t P = gemm_bwd_partials(M, N, K, bn);
  TORCH_CHECK(P > 0, "gemm_nt_bn_bwd: unsupported (K, N) — K must be 64, 128 or 256");
  TORCH_CHECK(mask.is_cuda() && mask.scalar_type() == at::kByte && mask.is_contiguous() &&
                  mask.numel() == M * (N / 8),
              "gemm_nt_bn_bwd: mask must be the forward's [M, N/8] uint8 bitmask");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
                  vec.numel() == 4 * N, "gemm_nt_bn_bwd: saved stats must be fp32 [4, N]");
  const void* d2 = nullptr;
  TORCH_CHECK(dy2_stride >= 1, "gemm_nt_bn_bwd: bad dy2 stride");
  if (dy2.has_value() && dy2->defined()) {
    const bool ok_layout = dy2->dim() == 4
                               ? dy2->size(1) == N &&
                                     dy2->is_contiguous(at::MemoryFormat::ChannelsLast)
                               : dy2->is_contiguous();
    TORCH_CHECK(dy2->is_cuda() && dy2->scalar_type() == at::kBFloat16 && ok_layout,
                "gemm_nt_bn_bwd: dy2 must be bf16 [*, N] (NHWC-contiguous)");
    if (dy2_stride == 1) {
      TORCH_CHECK(dy2->numel() == M * N, "gemm_nt_bn_bwd: dy2 must be [M, N]");
    } else {
      TORCH_CHECK(H > 0 && W > 0 && M % (H * W) == 0 && M < (int64_t(1) << 31),
                  "gemm_nt_bn_bwd: strided dy2 needs M = n*H*W < 2^31");
      const int64_t s = dy2_stride, hs = (H + s - 1) / s, ws = (W + s - 1) / s;
      TORCH_CHECK(dy2->dim() == 4 && dy2->size(0) == M / (H * W) && dy2->size(2) == hs &&
                      dy2->size(3) == ws,
                  "gemm_nt_bn_bwd: strided dy2 must be [n, N, ceil(H/s), ceil(W/s)]");
    }
    d2 = dy2->data_ptr();
  }
  for (const at::Tensor* t : {&b, &dz, &x, &mask, &vec})
    TORCH_CHECK(t->device() == a.device(), "gemm_nt_bn_bwd: devices differ");
  c10::DeviceGuard guard(a.device());
  at::Tensor partial = at::empty({P, 2, N}, a.options().dtype(at::kFloat));
  TORCH_CHECK(mv_gemm_nt_bn_bwd(a.data_ptr(), b.data_ptr(), dz.data_ptr(), M, (int)N, (int)K, d2,
                                mask.data_ptr(), has_x ? x.data_ptr() : nullptr,
                                vec[0].data_ptr<float>(),
                                partial.data_ptr<float>(), (int)bn, cur_stream(), (int)dy2_stride,
                                (int)H, (int)W),
              "gemm_nt_bn_bwd: launch failed");
  return partial;
}

// [5, C] fp32 = (dgamma, dbeta, ca, cb, cc) from a GEMM-epilogue reduce's partials, with
// the BN's input gradient dx = ca * dz + cb * x + cc (per channel) left to the caller
at::Tensor bn_bwd_coeffs(at::Tensor vec, c10::optional<at::Tensor> gamma, at::Tensor partial,
                         int64_t M) {
  TORCH_CHECK(partial.is_cuda() && partial.scalar_type() == at::kFloat && partial.is_contiguous() &&
                  partial.dim() == 3 && partial.size(1) == 2 && partial.size(0) > 0 &&
                  partial.size(0) < (int64_t(1) << 31),
              "bn: partials must be fp32 [P, 2, C]");
  const int64_t C = partial.size(2);
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
              vec.numel() == 4 * C && vec.device() == partial.device(),
              "bn: saved stats must be fp32 [4, C]");
  TORCH_CHECK(M > 0, "bn: M must be positive");
  c10::DeviceGuard guard(vec.device());
  at::Tensor work = at::empty({5, C}, vec.options());
  mv_bn_bwd_from_partials(nullptr, nullptr, nullptr, M, (int)C, vec[0].data_ptr<float>(),
                          vec[1].data_ptr<float>(), opt_f32(gamma, C, "weight"),
                          vec[2].data_ptr<float>(), vec[3].data_ptr<float>(),
                          work[0].data_ptr<float>(), work[1].data_ptr<float>(),
                          partial.data_ptr<float>(), (int)partial.size(0),
                          work[2].data_ptr<float>(), work[3].data_ptr<float>(),
                          work[4].data_ptr<float>(), cur_stream());
  return work;
}

// {dx, dgamma, dbeta} from a GEMM-epilogue reduce (gemm_nt_bn_bwd)
std::vector<at::Tensor> bn_bwd_from_partials(at::Tensor dz, at::Tensor x, at::Tensor vec,
                                             c10::optional<at::Tensor> gamma,
                                             bool need_affine_grad, at::Tensor partial) {
  int64_t C, C2;
  const int64_t M = bn_check_act(x, "x", &C);
  bn_check_act(dz, "dz", &C2);
  TORCH_CHECK(dz.sizes() == x.sizes() && dz.strides() == x.strides(), "bn: dz layout mismatch");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
              vec.numel() == 4 * C, "bn: saved stats must be fp32 [4, C]");
  TORCH_CHECK(partial.is_cuda() && partial.scalar_type() == at::kFloat && partial.is_contiguous() &&
                  partial.dim() == 3 && partial.size(1) == 2 && partial.size(2) == C &&
                  partial.size(0) > 0 && partial.size(0) < (int64_t(1) << 31),
              "bn: partials must be fp32 [P, 2, C]");
  c10::DeviceGuard guard(x.device());
  at::Tensor work = at::empty({5, C}, x.options().dtype(at::kFloat));
  at::Tensor dx = at::empty_like(x);
  mv_bn_bwd_from_partials(dz.data_ptr(), x.data_ptr(), dx.data_ptr(), M, (int)C,
                          vec[0].data_ptr<float>(), vec[1].data_ptr<float>(),
                          opt_f32(gamma, C, "weight"), vec[2].data_ptr<float>(),
                          vec[3].data_ptr<float>(), work[0].data_ptr<float>(),
                          work[1].data_ptr<float>(), partial.data_ptr<float>(),
                          (int)partial.size(0), work[2].data_ptr<float>(),
                          work[3].data_ptr<float>(), work[4].data_ptr<float>(), cur_stream());
  at::Tensor dg, db;
  if (need_affine_grad) {
    dg = work[0];
    db = work[1];
  }
  return {dx, dg, db};
}

// ---------------------------------------------------------------------------
// implicit-GEMM 3x3 convolution (pad 1), channels_last bf16
// ---------------------------------------------------------------------------
int64_t conv3x3_partials(int64_t M, int64_t K) { return mv_conv3x3_partials(M, (int)K); }

// y = conv3x3(x, w, stride, pad 1) / conv1x1(x, w, stride) (+ BN statistics partials of y
// around shift)
at::Tensor conv_nhwc(at::Tensor x, at::Tensor w, int64_t stride, c10::optional<at::Tensor> shift,
                     c10::optional<at::Tensor> partial, int64_t ks,
                     c10::optional<at::Tensor> in_scale = c10::nullopt,
                     c10::optional<at::Tensor> in_bias = c10::nullopt);

// (in_scale, in_bias: x is the producing BN's input; relu(x * in_scale + in_bias) is
// convolved without being materialised — the 64 -> 64 stride-1 row-patch kernel only)
at::Tensor conv3x3(at::Tensor x, at::Tensor w, int64_t stride, c10::optional<at::Tensor> shift,
                   c10::optional<at::Tensor> partial, c10::optional<at::Tensor> in_scale,
                   c10::optional<at::Tensor> in_bias) {
  return conv_nhwc(x, w, stride, shift, partial, 3, in_scale, in_bias);
}

static const float* opt_vec(const c10::optional<at::Tensor>& t, int64_t n, const at::Tensor& like,
                            const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() &&
                  t->numel() == n && t->device() == like.device(),
              what, " must be a contiguous fp32 [", n, "] tensor on the input's device");
  return t->data_ptr<float>();
}

at::Tensor conv1x1_mfma(at::Tensor x, at::Tensor w, int64_t stride,
                        c10::optional<at::Tensor> shift, c10::optional<at::Tensor> partial) {
  return conv_nhwc(x, w, stride, shift, partial, 1);
}

at::Tensor conv_nhwc(at::Tensor x, at::Tensor w, int64_t stride, c10::optional<at::Tensor> shift,
                     c10::optional<at::Tensor> partial, int64_t ks,
                     c10::optional<at::Tensor> in_scale, c10::optional<at::Tensor> in_bias) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3: x must be a channels_last bf16 GPU tensor [N, C, H, W]");
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 &&
                  w.size(2) == ks && w.size(3) == ks && w.size(1) == x.size(1) &&
                  w.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv: w must be a channels_last bf16 [K, C, ks, ks] filter matching x");
  TORCH_CHECK(w.device() == x.device(), "conv3x3: devices differ");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0 && C > 0 && K > 0, "conv3x3: C and K must be multiples of 64");
  TORCH_CHECK(stride == 1 || stride == 2, "conv3x3: stride must be 1 or 2");
  TORCH_CHECK(N * H * W * std::max(C, K) < (int64_t(1) << 40) && H < 65536 && W < 65536,
              "conv3x3: too large");
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t M = N * Ho * Wo;
  TORCH_CHECK(M > 0, "conv3x3: empty input");
  c10::DeviceGuard guard(x.device());
  at::Tensor y = at::empty({N, K, Ho, Wo}, x.options(), at::MemoryFormat::ChannelsLast);
  float* pp = nullptr;
  const float* sp = nullptr;
  if (partial.has_value() && partial->defined()) {
    TORCH_CHECK(partial->is_cuda() && partial->scalar_type() == at::kFloat &&
                    partial->is_contiguous() && partial->numel() >= conv3x3_partials(M, K) * 2 * K &&
                    partial->device() == x.device(),
                "conv3x3: partial must be fp32 [P, 2, K] with P = conv3x3_partials(M, K)");
    pp = partial->data_ptr<float>();
    if (shift.has_value() && shift->defined()) {
      TORCH_CHECK(shift->is_cuda() && shift->scalar_type() == at::kFloat && shift->numel() == K &&
                      shift->is_contiguous(),
                  "conv3x3: shift must be fp32 [K]");
      sp = shift->data_ptr<float>();
    }
  }
  const float* isc = opt_vec(in_scale, C, x, "conv: in_scale");
  const float* ibi = opt_vec(in_bias, C, x, "conv: in_bias");
  TORCH_CHECK((isc == nullptr) == (ibi == nullptr), "conv: in_scale and in_bias go together");
  TORCH_CHECK(mv_conv_nhwc(x.data_ptr(), w.data_ptr(), y.data_ptr(), (int)N, (int)H, (int)W,
                           (int)C, (int)K, (int)ks, (int)stride, sp, pp, cur_stream(), nullptr,
                           nullptr, isc, ibi),
              "conv: unsupported shape");
  return y;
}

// data gradient of a stride-1 3x3 conv (dy . flipped filter) with the mode-1 (BN+ReLU)
// backward reduce of the BN that produced the conv's input fused into the epilogue:
// returns (d = relu'(x_bn) * dgrad, partials [P, 2, C]).  Also the stride-1 1x1 conv
// (wt [C, K, 1, 1]): the same kernel with ks = 1.
std::vector<at::Tensor> conv3x3_bn_bwd(at::Tensor dy, at::Tensor wt, at::Tensor x_bn,
                                       at::Tensor vec) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_bn_bwd: dy must be a channels_last bf16 GPU tensor");
  TORCH_CHECK(wt.is_cuda() && wt.scalar_type() == at::kBFloat16 && wt.dim() == 4 &&
                  wt.size(2) == wt.size(3) && (wt.size(2) == 3 || wt.size(2) == 1) &&
                  wt.size(1) == dy.size(1) && wt.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_bn_bwd: wt must be the channels_last [C, K, ks, ks] (ks 3 or 1) "
              "transposed filter");
  const int64_t N = dy.size(0), K = dy.size(1), H = dy.size(2), W = dy.size(3), C = wt.size(0);
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0, "conv3x3_bn_bwd: channels must be multiples of 64");
  TORCH_CHECK(x_bn.is_cuda() && x_bn.scalar_type() == at::kBFloat16 &&
                  x_bn.sizes() == at::IntArrayRef({N, C, H, W}) &&
                  x_bn.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_bn_bwd: x_bn must be the BN input [N, C, H, W], channels_last bf16");
  TORCH_CHECK(vec.is_cuda() && vec.scalar_type() == at::kFloat && vec.is_contiguous() &&
                  vec.numel() == 4 * C, "conv3x3_bn_bwd: saved stats must be fp32 [4, C]");
  for (const at::Tensor* t : {&wt, &x_bn, &vec})
    TORCH_CHECK(t->device() == dy.device(), "conv3x3_bn_bwd: devices differ");
  TORCH_CHECK(N * H * W * std::max(C, K) < (int64_t(1) << 40) && H < 65536 && W < 65536,
              "conv3x3_bn_bwd: too large");
  c10::DeviceGuard guard(dy.device());
  const int64_t M = N * H * W;
  at::Tensor d = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  at::Tensor part = at::empty({conv3x3_partials(M, C), 2, C}, dy.options().dtype(at::kFloat));
  TORCH_CHECK(mv_conv_nhwc(dy.data_ptr(), wt.data_ptr(), d.data_ptr(), (int)N, (int)H, (int)W,
                           (int)K, (int)C, (int)wt.size(2), 1, nullptr, part.data_ptr<float>(),
                           cur_stream(), x_bn.data_ptr(), vec.data_ptr<float>()),
              "conv3x3_bn_bwd: unsupported shape");
  return {d, part};
}

// data gradient of a stride-2 3x3 conv (pad 1) as four output-parity-class gather GEMMs
// (mv_conv.hip / mv_gemm256.hip): dy [N, K, H/2, W/2], wt the transposed flipped filter
// [C, K, 3, 3] -> dx [N, C, H, W].  Returns [] when the shape is not covered (the caller
// falls back).
std::vector<at::Tensor> conv3x3_s2_dgrad(at::Tensor dy, at::Tensor wt, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv3x3_s2_dgrad: dy must be a channels_last bf16 GPU tensor");
  TORCH_CHECK(wt.is_cuda() && wt.scalar_type() == at::kBFloat16 && wt.dim() == 4 &&
                  wt.size(2) == 3 && wt.size(3) == 3 && wt.size(1) == dy.size(1) &&
                  wt.is_contiguous(at::MemoryFormat::ChannelsLast) && wt.device() == dy.device(),
              "conv3x3_s2_dgrad: wt must be the channels_last [C, K, 3, 3] transposed filter");
  const int64_t N = dy.size(0), K = dy.size(1), C = wt.size(0);
  TORCH_CHECK(H > 0 && W > 0 && (H - 1) / 2 + 1 == dy.size(2) && (W - 1) / 2 + 1 == dy.size(3),
              "conv3x3_s2_dgrad: H, W do not match dy");
  if (H >= 65536 || W >= 65536 || N >= (int64_t(1) << 31) ||
      !mv_conv3x3_s2_dgrad_supported((int)N, (int)H, (int)W, (int)C, (int)K))
    return {};
  c10::DeviceGuard guard(dy.device());
  at::Tensor dx = at::empty({N, C, H, W}, dy.options(), at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(mv_conv3x3_s2_dgrad(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), (int)N, (int)H,
                                  (int)W, (int)C, (int)K, cur_stream()),
              "conv3x3_s2_dgrad: launch refused");
  return {dx};
}

// Data-gradient filters of many convs in one launch: for every channels_last bf16 w
// [K, C, ks, ks] the channels_last [C, K, ks, ks] filter with the taps rotated 180 degrees
// (w.transpose(0, 1).flip(2, 3); for 1x1 W^T).  Outputs and the device block table are
// cached per input set (the filters live in the optimizer's arena: stable pointers), so a
// step costs one kernel.
std::vector<at::Tensor> transpose_filters(std::vector<at::Tensor> ws) {
  struct Entry {
    std::vector<const void*> src;
    std::vector<at::Tensor> outs;
    at::Tensor table;
    int64_t blocks = 0;
  };
  // (heap-allocated and never destroyed: tensors must not be freed after the HIP runtime at
  // process exit)
  static std::vector<Entry>& cache = *new std::vector<Entry>();
  TORCH_CHECK(!ws.empty(), "transpose_filters: no filters");
  const int n = (int)ws.size();
  std::vector<const void*> src(n);
  std::vector<int> K(n), C(n), ks(n);
  for (int i = 0; i < n; ++i) {
    const at::Tensor& w = ws[i];
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 &&
                    w.size(2) == w.size(3) && w.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    w.device() == ws[0].device(),
                "transpose_filters: filters must be channels_last bf16 [K, C, k, k] on one GPU");
    src[i] = w.data_ptr();
    K[i] = (int)w.size(0);
    C[i] = (int)w.size(1);
    ks[i] = (int)w.size(2);
  }
  c10::DeviceGuard guard(ws[0].device());
  Entry* e = nullptr;
  for (auto& c : cache) {
    if (c.src != src || (int)c.outs.size() != n) continue;
    bool same = true;
    for (int i = 0; i < n && same; ++i)
      same = c.outs[i].size(0) == C[i] && c.outs[i].size(1) == K[i] && c.outs[i].size(2) == ks[i] &&
             c.outs[i].device() == ws[i].device();
    if (same) { e = &c; break; }
  }
  if (!e) {
    if (cache.size() >= 8) cache.erase(cache.begin());
    Entry ne;
    ne.src = src;
    std::vector<void*> dst(n);
    for (int i = 0; i < n; ++i) {
      ne.outs.push_back(at::empty({C[i], K[i], ks[i], ks[i]}, ws[i].options(),
                                  at::MemoryFormat::ChannelsLast));
      dst[i] = ne.outs[i].data_ptr();
    }
    ne.blocks = mv_transpose_filters_blocks(K.data(), C.data(), ks.data(), n);
    const int64_t bytes = mv_transpose_filters_table_bytes(n, ne.blocks);
    at::Tensor host = at::empty({bytes}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
    mv_transpose_filters_table(src.data(), dst.data(), K.data(), C.data(), ks.data(), n,
                               host.data_ptr());
    ne.table = host.to(ws[0].device(), /*non_blocking=*/false);
    cache.push_back(std::move(ne));
    e = &cache.back();
  }
  mv_transpose_filters(e->table.data_ptr(), n, e->blocks, cur_stream());
  return e->outs;
}

// weight gradient of y = conv3x3(x, w, stride, pad 1): dw [K, C, 3, 3] channels_last bf16
at::Tensor wgrad3x3(at::Tensor x, at::Tensor dy, int64_t stride,
                    c10::optional<at::Tensor> in_scale, c10::optional<at::Tensor> in_bias) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wgrad3x3: x must be a channels_last bf16 GPU tensor");
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.device() == x.device(),
              "wgrad3x3: dy must be a channels_last bf16 tensor on x's device");
  TORCH_CHECK(stride == 1 || stride == 2, "wgrad3x3: stride must be 1 or 2");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = dy.size(1);
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == Ho && dy.size(3) == Wo, "wgrad3x3: dy shape");
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0 && N * H * W * std::max(C, K) < (int64_t(1) << 40),
              "wgrad3x3: channels must be multiples of 64");
  c10::DeviceGuard guard(x.device());
  const int64_t M = N * Ho * Wo;
  at::Tensor work = at::empty({mv_wgrad3x3_workspace(M, (int)K, (int)C)},
                              x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({K, C, 3, 3}, x.options(), at::MemoryFormat::ChannelsLast);
  const float* isc = opt_vec(in_scale, C, x, "wgrad3x3: in_scale");
  const float* ibi = opt_vec(in_bias, C, x, "wgrad3x3: in_bias");
  TORCH_CHECK((isc == nullptr) == (ibi == nullptr), "wgrad3x3: in_scale and in_bias go together");
  TORCH_CHECK(mv_wgrad3x3(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), work.data_ptr<float>(),
                          (int)N, (int)H, (int)W, (int)C, (int)K, (int)stride, cur_stream(), isc,
                          ibi),
              "wgrad3x3: unsupported shape");
  return dw;
}

// weight gradient of y = conv1x1(x, w, stride, pad 0): dw [K, C, 1, 1] bf16
at::Tensor wgrad1x1(at::Tensor x, at::Tensor dy, int64_t stride, bool fp32_out,
                    c10::optional<at::Tensor> dy2) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                  x.is_contiguous(at::MemoryFormat::ChannelsLast),
              "wgrad1x1: x must be a channels_last bf16 GPU tensor");
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                  dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.device() == x.device(),
              "wgrad1x1: dy must be a channels_last bf16 tensor on x's device");
  TORCH_CHECK(stride == 1 || stride == 2, "wgrad1x1: stride must be 1 or 2");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K1 = dy.size(1);
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == Ho && dy.size(3) == Wo, "wgrad1x1: dy shape");
  // dy2: a second dy stream stacked below dy's channels (dw = [dy | dy2]^T . x)
  const bool two = dy2.has_value() && dy2->defined();
  int64_t K = K1;
  bool gather = false;
  if (two) {
    // [N, K2, Ho, Wo] at the output rows, or (stride 2) [N, K2, H, W] read at each output
    // row's strided input pixel (e.g. dy2 = x itself: the Gram pass of x[:, :, ::2, ::2])
    gather = stride > 1 && dy2->dim() == 4 && dy2->size(2) == H && dy2->size(3) == W;
    TORCH_CHECK(dy2->is_cuda() && dy2->scalar_type() == at::kBFloat16 && dy2->dim() == 4 &&
                    dy2->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dy2->device() == x.device() && dy2->size(0) == N &&
                    (gather || (dy2->size(2) == Ho && dy2->size(3) == Wo)) &&
                    dy2->size(1) % 64 == 0,
                "wgrad1x1: dy2 must be a channels_last bf16 [N, K2, Ho, Wo] (or, stride 2, "
                "[N, K2, H, W]) tensor");
    K = K1 + dy2->size(1);
  }
  TORCH_CHECK(C % 64 == 0 && K % 64 == 0 && N * H * W * std::max(C, K) < (int64_t(1) << 40),
              "wgrad1x1: channels must be multiples of 64");
  c10::DeviceGuard guard(x.device());
  const int64_t M = N * Ho * Wo;
  at::Tensor work = at::empty({mv_wgrad1x1_workspace(M, (int)K, (int)C)},
                              x.options().dtype(at::kFloat));
  at::Tensor dw = at::empty({K, C, 1, 1}, fp32_out ? x.options().dtype(at::kFloat) : x.options(),
                            at::MemoryFormat::ChannelsLast);
  TORCH_CHECK(mv_wgrad1x1(x.data_ptr(), dy.data_ptr(), dw.data_ptr(), work.data_ptr<float>(),
                          (int)N, (int)H, (int)W, (int)C, (int)K, (int)stride, cur_stream(),
                          fp32_out, two ? dy2->data_ptr() : nullptr, (int)K1, gather),
              "wgrad1x1: unsupported shape");
  return dw;
}

}  // namespace

// A tensor over device memory mivod owns elsewhere (the mesh's IPC staging
// slot): no copy, no deleter — the owner outlives every view by construction.
at::Tensor tensor_from_ptr(uintptr_t ptr, int64_t numel, at::ScalarType dtype, int64_t device) {
  TORCH_CHECK(ptr != 0 && numel >= 0, "tensor_from_ptr: bad pointer / size");
  TORCH_CHECK(ptr % 16 == 0, "tensor_from_ptr: pointer must be 16-byte aligned");
  return torch::from_blob(reinterpret_cast<void*>(ptr), {numel},
                          at::TensorOptions().dtype(dtype).device(at::kCUDA, device));
}

PYBIND11_MODULE(_mvk, m) {
  m.doc() = "mivod hand-written gfx950 (CDNA4) kernels";
  m.attr("CHUNK") = kChunk;
  m.attr("MAX_TENSORS_PER_LAUNCH") = kMvMaxTensors;
  m.def("tensor_from_ptr", &tensor_from_ptr, "tensor view of mivod-owned device memory");
  m.def("mt_copy", &mt_copy, "multi-tensor pack/unpack with fused cast+scale");
  m.def("flat_cast", &flat_cast, "flat cast + scale (compress/decompress)");
  m.def("nonfinite_scan", &nonfinite_scan, "flag |= any non-finite element (read-only)");
  m.def("sgd_step", &sgd_step, "fused flat SGD(+momentum, nesterov) step");
  m.def("adam_step", &adam_step, "fused flat Adam/AdamW step");
  m.def("adadelta_step", &adadelta_step, "fused flat Adadelta step");
  m.def("lars_step", &lars_step, "fused segmented LARS step");
  m.def("seg_dot3", &seg_dot3, "per-segment (a.b, |a|^2, |b|^2)");
  m.def("adasum_combine", &adasum_combine, "per-segment Adasum merge a <- ca*a + cb*b");
  m.def("adasum_fcombine", &adasum_fcombine,
        "vector-halving Adasum merge on the fp32 running sum f <- cf*f + cr*r");
  // roctx ranges: rocprofv3 --marker-trace shows mivod's bucket phases (pack,
  // allreduce, fused step) on the same timeline as the kernels and RCCL
  m.def("range_push", [](const std::string& s) { return roctxRangePushA(s.c_str()); });
  m.def("range_pop", []() { return roctxRangePop(); });
  m.def("mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
  m.def("attn_fwd", &attn_fwd, "fused MFMA attention forward -> (out [b,s,h,64], lse)");
  m.def("attn_bwd", &attn_bwd, "fused MFMA attention backward -> dqkv");
  m.def("attn_dropout_mask", &attn_dropout_mask, "dropout keep-mask of the fused attention");
  m.def("bias_gelu_fwd", &bias_gelu_fwd, "y = gelu(x + b) (erf form)");
  m.def("bias_gelu_bwd", &bias_gelu_bwd, "-> (dx, dbias) of y = gelu(x + b)");
  m.def("ln_fwd", &ln_fwd, "v = res + dropout(z + b); y = LN(v) -> (y, v, mean, rstd)");
  m.def("ln_bwd", &ln_bwd, "-> (dv, dz, dgamma, dbeta, dbias)");
  m.def("bn_fwd_train", &bn_fwd_train, "fused NHWC BN(+add)(+ReLU) training forward");
  m.def("bn_fwd_train_mask", &bn_fwd_train_mask,
        "fused NHWC BN+add+ReLU training forward that also returns the backward bitmask");
  m.def("bn_apply", &bn_apply, "NHWC y = act(x*scale + bias (+res))");
  m.def("bn_fwd_train_stats", &bn_fwd_train_stats,
        "fused BN(+add)(+ReLU) forward from the conv epilogue's statistics partials");
  m.def("bn_bwd", &bn_bwd, "fused NHWC BN(+add)(+ReLU) backward (+ second grad stream)");
  m.def("bn_stats", &bn_stats, "NHWC BN training statistics only -> [4, C]");
  m.def("bn_stats_strided", &bn_stats_strided,
        "statistics of x[:, :, ::s, ::s] (no strided copy) -> [4, C] {mean, invstd, ...}");
  m.def("bn_apply_colsum", &bn_apply_colsum,
        "{y, [P, C] partials}: relu(x*scale + bias) with column sums of y");
  m.def("maxpool_fwd", &maxpool_fwd, "NHWC maxpool with fused affine+ReLU prologue -> (y, idx)");
  m.def("maxpool_bwd", &maxpool_bwd, "NHWC maxpool backward (gather, + second grad stream)");
  m.def("gap_fwd", &gap_fwd, "NHWC global average pool -> [N, C]");
  m.def("gap_bwd", &gap_bwd, "NHWC global average pool backward");
  m.def("pad_channels", &pad_channels, "NHWC zero channel padding C -> cout (<= 8)");
  m.def("gemm_nt", &gemm_nt, "C = A . B^T (bf16 MFMA) with optional fused BN statistics "
        "(C = None: statistics only)");
  m.def("gemm_apply_supported", &gemm_apply_supported, "gemm_nt_apply handles (N, K)");
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd,
        "{dx, dgamma, dbeta}: maxpool(3,2,1) backward fused with its producer BN+ReLU backward");
  m.def("gram_stats", &gram_stats,
        "[1, 2, cout] BN statistics partials of x W^T from the Gram matrix x^T x and colsum(x)",
        py::arg("w"), py::arg("gram"), py::arg("xsum"), py::arg("shift") = py::none(),
        py::arg("m") = 1);
  m.def("stem_wgrad", &stem_wgrad, "ResNet stem conv weight gradient on MFMA (mv_stem.hip)");
  m.def("stem_wgrad_pool_bn", &stem_wgrad_pool_bn,
        "ResNet stem maxpool + BN+ReLU backward fused into the stem weight gradient -> [dw, dgamma, dbeta]");
  m.def("stem_fwd", &stem_fwd,
        "{z, [P, 2, 64] partials}: ResNet 7x7/2 stem conv on MFMA with BN statistics (mv_stem.hip)",
        py::arg("x"), py::arg("w"), py::arg("shift") = py::none(), py::arg("grid") = 0);
  m.def("fold_coeffs", &fold_coeffs,
        "{co [5, cout], xsum [cin]}: the BN fold's per-channel coefficients (mv_fold.hip)");
  m.def("fold_products", &fold_products,
        "{dW, bcat, badd}: the BN fold's small products (mv_fold.hip)");
  m.def("gemm_apply_dual_supported", &gemm_apply_dual_supported,
        "gemm_nt_apply_dual handles (N, K)");
  m.def("gemm_nt_apply_dual", &gemm_nt_apply_dual,
        "{y, mask}: the BN+add+ReLU apply GEMM with the shortcut conv + BN recomputed inside");
  m.def("gemm_dual_supported", &gemm_dual_supported, "gemm_dual_bias handles (K1, K2)");
  m.def("gemm_dual_bias_strided", &gemm_dual_bias_strided,
        "[A1 | x[:, :, ::s, ::s]] . B^T + badd without the strided copy; False if not covered");
  m.def("gemm_dual_bias", &gemm_dual_bias, "d = [a1 | a2] . b^T + badd (dual-source MFMA GEMM)");
  m.def("gemm_fold_dx_partials", &gemm_fold_dx_partials,
        "partial rows of gemm_fold_dx for (M, K1, K2) (-1: unsupported)");
  m.def("gemm_fold_dx", &gemm_fold_dx,
        "BN3-fold data gradient [a1|a2].b^T + badd with BN2's ReLU backward reduce -> partials");
  m.def("gemm_nt_apply", &gemm_nt_apply,
        "{y, mask}: relu(bf16(A . B^T) * scale + bias + res) from the GEMM epilogue "
        "(rscale/rbias: res = bf16(res * rscale + rbias), the shortcut BN's apply)",
        py::arg("a"), py::arg("b"), py::arg("res"), py::arg("scale"), py::arg("bias"),
        py::arg("rscale") = py::none(), py::arg("rbias") = py::none());
  m.def("bn_finalize", &bn_finalize, "BN statistics finalize from [P, 2, C] partials -> [4, C]");
  m.def("gemm_nt_bn_bwd", &gemm_nt_bn_bwd,
        "1x1-conv data-gradient GEMM with the producing BN's add+ReLU backward reduce fused",
        py::arg("a"), py::arg("b"), py::arg("dz"), py::arg("dy2"), py::arg("mask"), py::arg("x"),
        py::arg("vec"), py::arg("bn") = 0, py::arg("dy2_stride") = 1, py::arg("H") = 1,
        py::arg("W") = 1);
  m.def("gemm_bwd_partials", &gemm_bwd_partials, "partial rows of gemm_nt_bn_bwd (-1: unsupported)",
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bn") = 0);
  m.def("bn_bwd_coeffs", &bn_bwd_coeffs,
        "BN backward finalize only: [5, C] = (dgamma, dbeta, ca, cb, cc) from partials");
  m.def("bn_bwd_from_partials", &bn_bwd_from_partials,
        "BN backward finalize + dx from GEMM-epilogue partials -> (dx, dgamma, dbeta)");
  m.def("conv3x3", &conv3x3, "implicit-GEMM 3x3 conv (pad 1) with optional fused BN statistics "
        "(in_scale / in_bias: x is the producing BN's input, its BN + ReLU applied on load)",
        py::arg("x"), py::arg("w"), py::arg("stride") = 1, py::arg("shift") = py::none(),
        py::arg("partial") = py::none(), py::arg("in_scale") = py::none(),
        py::arg("in_bias") = py::none());
  m.def("conv1x1", &conv1x1_mfma, "1x1 conv (implicit-GEMM kernel) with optional fused BN statistics",
        py::arg("x"), py::arg("w"), py::arg("stride") = 1, py::arg("shift") = py::none(),
        py::arg("partial") = py::none());
  m.def("conv3x3_bn_bwd", &conv3x3_bn_bwd,
        "stride-1 3x3 data gradient with the producing BN+ReLU's backward reduce fused");
  m.def("conv3x3_s2_dgrad", &conv3x3_s2_dgrad,
        "stride-2 3x3 data gradient (parity-class gather GEMMs); [] when the shape is not "
        "covered", py::arg("dy"), py::arg("wt"), py::arg("H"), py::arg("W"));
  m.def("wgrad1x1", &wgrad1x1, "1x1 (pad 0, stride 1/2) conv weight gradient on MFMA",
        py::arg("x"), py::arg("dy"), py::arg("stride") = 1, py::arg("fp32_out") = false,
        py::arg("dy2") = py::none());
  m.def("transpose_filters", &transpose_filters,
        "data-gradient filters (transposed, taps rotated) of many convs in one launch");
  m.def("wgrad3x3", &wgrad3x3, "3x3 (pad 1) conv weight gradient on MFMA (transposed LDS reads)",
        py::arg("x"), py::arg("dy"), py::arg("stride") = 1, py::arg("in_scale") = py::none(),
        py::arg("in_bias") = py::none());
  m.def("conv3x3_partials", &conv3x3_partials, "partial rows of conv3x3's statistics epilogue");
  m.def("gemm_partials", &gemm_partials, "row tiles (statistics partial rows) of gemm_nt");
  m.def("gemm256_nt", &gemm256_nt, "C = A . B^T on the 256x256 glds-pipelined kernel alone");
  m.def("conv1x1_strided_stats", &conv1x1_strided_stats,
        "[y, (partials)] of a strided 1x1 conv on the 256x256 kernel (+ BN statistics), or None",
        py::arg("x"), py::arg("w"), py::arg("ds"), py::arg("shift") = py::none());
}
