// rf_act.h — elementwise activations of the dense epilogues (Keras: gelu(approximate=False), relu, selu).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/rf_api.h"

namespace rf_act {

// GELU, exact form 0.5 x (1 + erf(x / sqrt 2)) (Keras 'gelu', approximate=False), without branches:
// erfc(|z|) = t exp(-z^2 + P(t)), t = 1 / (1 + |z| / 2), P the Chebyshev fit of Numerical Recipes' erfcc
// (fractional error < 1.2e-7 everywhere); for z < 0 the result is x erfc(|z|) / 2 directly.
__device__ __forceinline__ float gelu_erf(float x) {
    const float z = x * 0.70710678118654752440f, a = fabsf(z);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, a, 1.0f));
    float p = fmaf(t, 0.17087277f, -0.82215223f);
    p = fmaf(t, p, 1.48851587f);
    p = fmaf(t, p, -1.13520398f);
    p = fmaf(t, p, 0.27886807f);
    p = fmaf(t, p, -0.18628806f);
    p = fmaf(t, p, 0.09678418f);
    p = fmaf(t, p, 0.37409196f);
    p = fmaf(t, p, 1.00002368f);
    p = fmaf(t, p, -1.26551223f);
    const float e = t * __expf(fmaf(-a, a, p));  // erfc(|z|)
    return z >= 0.f ? x * fmaf(-0.5f, e, 1.0f) : 0.5f * x * e;
}

struct None { __device__ __forceinline__ float operator()(float x) const { return x; } };
struct Gelu { __device__ __forceinline__ float operator()(float x) const { return gelu_erf(x); } };
struct Relu { __device__ __forceinline__ float operator()(float x) const { return x > 0.f ? x : 0.f; } };
struct Selu {
    __device__ __forceinline__ float operator()(float x) const {
        const float alpha = 1.6732632423543772848170429916717f, scale = 1.0507009873554804934193349852946f;
        const float neg = scale * alpha * (__expf(fminf(x, 0.f)) - 1.0f);  // both sides, then a select: no branch
        return x > 0.f ? scale * x : neg;
    }
};

// Runs f(Act{}) with the activation resolved once, outside the element loops f contains.
template <class F>
__device__ __forceinline__ void with_act(int act, F&& f) {
    switch (act) {
        case RF_ACT_GELU: f(Gelu{}); break;
        case RF_ACT_RELU: f(Relu{}); break;
        case RF_ACT_SELU: f(Selu{}); break;
        default: f(None{}); break;
    }
}

}  // namespace rf_act
