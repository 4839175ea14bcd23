// Fused transformer elementwise kernels (bias+GELU, bias+dropout+residual+LayerNorm)
// — mv_bert.hip.  All tensors bf16 row-major [M, N] unless noted.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct LnFwdParams {
  const void* z;      // [M, H]
  const void* bias;   // [H] or nullptr
  const void* res;    // [M, H] or nullptr
  const void* gamma;  // [H]
  const void* beta;   // [H]
  void* v;            // [M, H] saved pre-LN sum (may be nullptr for inference)
  void* y;            // [M, H]
  float* mean;        // [M]
  float* rstd;        // [M]
  int64_t M;
  int H;              // multiple of 8, <= 4096
  float eps;
  float p_drop;
  uint32_t seed;
  uint32_t thresh;    // drop if hash < thresh
};

struct LnBwdParams {
  const void* dy;
  const void* v;
  const float* mean;
  const float* rstd;
  const void* gamma;
  void* dv;           // [M, H] grad of the pre-LN sum (= residual grad)
  void* dz;           // [M, H] grad of z, or nullptr
  float* partial;     // [mv_ln_partials(M)][3][H] scratch
  int64_t M;
  int H;
  float p_drop;
  uint32_t seed;
  uint32_t thresh;
  const void* dy2;    // [M, H] second gradient of y (tapped residual use), or nullptr
};

int64_t mv_bias_gelu_partials(int64_t M, int N);
void mv_bias_gelu_fwd(const void* x, const void* b, void* y, int64_t M, int N, hipStream_t st);
void mv_bias_gelu_bwd(const void* dy, const void* x, const void* b, void* dx, float* partial,
                      void* dbias, int64_t M, int N, hipStream_t st);
int64_t mv_ln_partials(int64_t M);
void mv_ln_fwd(const LnFwdParams& p, hipStream_t st);
void mv_ln_bwd(const LnBwdParams& p, void* dgamma, void* dbeta, void* dbias, hipStream_t st);
