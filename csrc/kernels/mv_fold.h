// Host declarations of mv_fold.hip (the BN fold's small-matrix math, ops/bn.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// co [5][cout] = (dgamma, dbeta, ca, cb, cc); xsum [cin] = column sums of the [P2][cin]
// colsum partials (colsum == null: xsum untouched)
void mv_fold_coeffs(const float* part, int P, const void* w, const float* g, const float* vec,
                    const float* gamma, int64_t M, int cout, int cin, const float* colsum, int P2,
                    float* co, float* xsum, hipStream_t st);
// dW [cout][cin] bf16 (dw == null: skipped), bcat [cin][cout + cin] bf16, badd [cin] fp32
void mv_fold_products(const void* w, const float* g, const float* gram, const float* co,
                      const float* xsum, int cout, int cin, void* dw, void* bcat, float* badd,
                      hipStream_t st);
