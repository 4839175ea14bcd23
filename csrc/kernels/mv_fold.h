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
// part [2][cout] = (sum (z - shift), sum (z - shift)^2) of z = x W^T from G = x^T x
// [cin][cin] fp32 and xsum [cin] = colsum(x); W [cout][cin] bf16, shift may be null.
// false (nothing launched): cout % 16 != 0 or cin > 1024
bool mv_gram_stats(const void* w, const float* gram, const float* xsum, const float* shift,
                   int64_t m, int cout, int cin, float* part, hipStream_t st);
