// Fused MFMA attention (head dim 64) launchers — mv_attn.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct AttnParams {
  const void* qkv;      // bf16 [b, s, 3, h, 64]
  void* out;            // bf16 [b, s, h, 64]
  float* lse;           // [b, h, s] log2-domain log-sum-exp of the scaled scores
  const float* mask;    // [b, s] additive key bias (natural log units) or nullptr
  int b, s, h;
  float scale_log2;     // log2(e) / sqrt(64)
  float p_drop;         // attention-probability dropout
  uint32_t seed;
  uint32_t thresh;      // drop if hash < thresh  (p_drop * 2^32)
};

void mv_attn_fwd(const AttnParams& p, hipStream_t st);
void mv_attn_bwd(const AttnParams& p, const void* out, const void* dout, float* delta,
                 float* dq_part, void* dqkv, hipStream_t st);
void mv_attn_dropout_mask(int b, int h, int s, uint32_t seed, uint32_t thresh, uint8_t* keep,
                          hipStream_t st);
