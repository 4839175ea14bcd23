// NHWC pooling kernels (mv_pool.hip): fused affine+ReLU+maxpool with uint8
// argmax, gather-form maxpool backward, global average pool fwd/bwd.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void mv_maxpool_fwd(const void* x, const float* scale, const float* bias, bool relu, void* y,
                    uint8_t* idx, int N, int H, int W, int C, int OH, int OW, int k, int s, int p,
                    hipStream_t st);
void mv_maxpool_bwd(const void* dy, const void* dy2, const uint8_t* idx, void* dx, int N, int H,
                    int W, int C, int OH, int OW, int k, int s, int p, hipStream_t st);
void mv_gap_fwd(const void* x, void* y, int N, int HW, int C, hipStream_t st);
void mv_gap_bwd(const void* dy, void* dx, int N, int HW, int C, hipStream_t st);
void mv_pad_channels(const void* x, void* y, int64_t pixels, int cin, int cout, hipStream_t st);

// ResNet stem: maxpool(3, 2, 1) backward fused with the producing BN+ReLU's backward.
// Reduce at the pooled level -> [mv_pool_bn_partials()][2][C] partials (sum d, sum d (z - mean));
// then, with (ca, cb, cc) from the finalize: dx = ca relu'(z) gsum + cb z + cc in one pass.
int mv_pool_bn_partials();
void mv_pool_bn_reduce(const void* dy, const void* dy2, const void* y, const float* mean,
                       const float* scale, const float* bias, float* partial, int64_t M, int C,
                       hipStream_t st);
bool mv_maxpool_bn_bwd(const void* dy, const void* dy2, const uint8_t* idx, const void* z,
                       const float* scale, const float* bias, const float* ca, const float* cb,
                       const float* cc, void* dx, int N, int H, int W, int C, int OH, int OW,
                       hipStream_t st);
