// rf_fusion.hip — Que2Search AttentionFusion forward (backend/layers/fusion_layers.py:35-46):
//   att = softmax(concat(x_1..x_C) @ W)            W: [C*d][C] (the Keras weight as stored)
//   out = sum_c att_c * x_c, then l2-normalised when is_norm
// One wave per example: the C logits are C dot products of length C*d (lanes stride the K axis,
// xor-shuffle reductions), the softmax and the weighted channel sum stay in registers. fp32 throughout.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {

constexpr int kMaxC = 16;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__global__ __launch_bounds__(256) void fusion_kernel(const float* __restrict__ x, int B, int C, int d, int64_t ldx,
                                                     const float* __restrict__ W, int is_norm, float* __restrict__ out,
                                                     int64_t ldo, float* __restrict__ att_out) {
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B) return;
    const float* xr = x + b * ldx;
    const int K = C * d;
    float logit[kMaxC];
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) logit[c] = 0.f;
    for (int kx = lane; kx < K; kx += 64) {
        const float xv = xr[kx];
        const float* wr = W + (int64_t)kx * C;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c)
            if (c < C) logit[c] += xv * wr[c];
    }
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
        if (c < C) {
            logit[c] = wave_sum(logit[c]);
            mx = fmaxf(mx, logit[c]);
        }
    float z = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
        if (c < C) {
            logit[c] = expf(logit[c] - mx);
            z += logit[c];
        }
#pragma unroll
    for (int c = 0; c < kMaxC; ++c)
        if (c < C) logit[c] /= z;
    if (att_out && lane < C) {
#pragma unroll
        for (int c = 0; c < kMaxC; ++c)
            if (c == lane) att_out[b * C + c] = logit[c];
    }
    // weighted channel sum (lane owns columns lane, lane + 64, ...), then the row norm
    float ss = 0.f;
    for (int j = lane; j < d; j += 64) {
        float acc = 0.f;
#pragma unroll
        for (int c = 0; c < kMaxC; ++c)
            if (c < C) acc += logit[c] * xr[(int64_t)c * d + j];
        out[b * ldo + j] = acc;
        ss += acc * acc;
    }
    if (is_norm) {
        // tf.nn.l2_normalize: x * rsqrt(max(sum(x^2), 1e-12))
        const float inv = rsqrtf(fmaxf(wave_sum(ss), 1e-12f));
        for (int j = lane; j < d; j += 64) out[b * ldo + j] *= inv;
    }
}

}  // namespace

extern "C" int rf_attention_fusion_fwd(const float* x, int32_t batch, int32_t channels, int32_t dim, int64_t ldx,
                                       const float* W, int32_t is_norm, float* out, int64_t ldo, float* att_out,
                                       void* stream) {
    RF_REQUIRE(batch >= 0 && channels >= 1 && channels <= kMaxC && dim >= 1, "rf_attention_fusion_fwd: need 1 <= channels <= 16");
    RF_REQUIRE(ldx >= (int64_t)channels * dim && ldo >= dim, "rf_attention_fusion_fwd: bad leading dimension");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(x && W && out, "rf_attention_fusion_fwd: null pointer");
    hipLaunchKernelGGL(fusion_kernel, dim3((batch + 3) / 4), dim3(256), 0, rf_stream(stream), x, batch, channels, dim, ldx,
                       W, is_norm, out, ldo, att_out);
    return rf_check_launch("rf_attention_fusion_fwd");
}
