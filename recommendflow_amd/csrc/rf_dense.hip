// rf_dense.hip — the interaction-MLP scorer on gfx950 (create_mlp, backend/blocks/mlp.py:4-15):
//   rf_norm_fwd    LayerNormalization / BatchNormalization(inference) -> bf16 (or f32) GEMM operand
//   rf_linear_fwd  Dense: y = act(x @ W + b)
//       * bf16 x/W: v_mfma_f32_16x16x32_bf16, 128x128x64 block tile, 4 waves of 64x64, double-buffered LDS
//       * f32  x/W: v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulate), 128x128x32 tile
//       * N <= 16 or softmax heads (Dense(2, softmax), esim.py:53): one wave per row, fp32 dot + row softmax
//     bias + activation (gelu(erf) / relu / selu / softmax) fused in the epilogue.
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>
#include <cstdlib>

#include "rf_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

// GELU, exact form 0.5 x (1 + erf(x / sqrt 2)) (Keras 'gelu', approximate=False), without branches:
// erfc(|z|) = t exp(-z^2 + P(t)), t = 1 / (1 + |z| / 2), P the Chebyshev fit of Numerical Recipes' erfcc
// (fractional error < 1.2e-7 everywhere); for z < 0 the result is x erfc(|z|) / 2 directly (no 1 - (1 - e)
// cancellation). Straight-line code, so an epilogue's elements interleave instead of each taking a branch.
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

struct ActNone { __device__ __forceinline__ float operator()(float x) const { return x; } };
struct ActGelu { __device__ __forceinline__ float operator()(float x) const { return gelu_erf(x); } };
struct ActRelu { __device__ __forceinline__ float operator()(float x) const { return x > 0.f ? x : 0.f; } };
struct ActSelu {
    __device__ __forceinline__ float operator()(float x) const {
        const float alpha = 1.6732632423543772848170429916717f, scale = 1.0507009873554804934193349852946f;
        const float neg = scale * alpha * (__expf(fminf(x, 0.f)) - 1.0f);  // both sides, then a select: no branch
        return x > 0.f ? scale * x : neg;
    }
};

// Sum over each 16-lane row of the wave, result in every lane of the row, by DPP (no LDS round trips):
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror. Lane 0's value is bit-identical to
// the xor butterfly (offsets 1, 2, 4, 8): every step adds the same two partial sums, only commuted.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141>(v);  // row_half_mirror
    v += dpp_mov<0x140>(v);  // row_mirror
    return v;
}

// Sum over the whole wave, the same bits in every lane: 16-lane rows by DPP, then rows (0+1) + (2+3)
__device__ __forceinline__ float wave_sum(float v) {
    v = row16_sum(v);
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    return v;
}

// Runs f(Act{}) with the activation resolved once, outside the element loops f contains.
template <class F>
__device__ __forceinline__ void with_act(int act, F&& f) {
    switch (act) {
        case RF_ACT_GELU: f(ActGelu{}); break;
        case RF_ACT_RELU: f(ActRelu{}); break;
        case RF_ACT_SELU: f(ActSelu{}); break;
        default: f(ActNone{}); break;
    }
}

__device__ __forceinline__ float act_apply(int act, float x) {
    switch (act) {
        case RF_ACT_GELU: return gelu_erf(x);
        case RF_ACT_RELU: return ActRelu{}(x);
        case RF_ACT_SELU: return ActSelu{}(x);
        default: return x;
    }
}

// ---------------------------------------------------------------------------------------------
// row normalisation: one wave per row
// ---------------------------------------------------------------------------------------------
template <bool OUT_BF16>
__global__ __launch_bounds__(256) void norm_kernel(const float* __restrict__ x, int64_t rows, int cols, int64_t ldx,
                                                   int mode, float eps, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, const float* __restrict__ mean,
                                                   const float* __restrict__ var, void* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float* xr = x + row * ldx;
    float mu = 0.f, rstd = 1.f;
    if (mode == 0) {
        float s = 0.f;
        for (int c = lane; c < cols; c += 64) s += xr[c];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        mu = s / (float)cols;
        float v = 0.f;
        for (int c = lane; c < cols; c += 64) {
            const float dlt = xr[c] - mu;
            v += dlt * dlt;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        rstd = 1.0f / sqrtf(v / (float)cols + eps);
    }
    for (int c = lane; c < cols; c += 64) {
        float o;
        if (mode == 0)
            o = (xr[c] - mu) * rstd * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
        else
            o = (xr[c] - mean[c]) / sqrtf(var[c] + eps) * (gamma ? gamma[c] : 1.f) + (beta ? beta[c] : 0.f);
        if constexpr (OUT_BF16)
            reinterpret_cast<uint16_t*>(y)[row * ldy + c] = (uint16_t)f32_to_bf16_bits(o);
        else
            reinterpret_cast<float*>(y)[row * ldy + c] = o;
    }
}

// Vector path (cols % 4 == 0, 16-byte aligned rows, cols <= 2048): one wave per row, the row loaded
// ONCE into registers with float4 loads (NV per lane, all in flight together), mean / variance from the
// registers, 16- / 8-byte stores. The scalar kernel above re-reads the row three times with dependent
// 4-byte loads (latency-bound: 1.4 TB/s on cfg3's [4096, 1280]).
template <bool OUT_BF16, int NV>
__global__ __launch_bounds__(256) void norm_vec_kernel(const float* __restrict__ x, int64_t rows, int cols, int64_t ldx,
                                                       int mode, float eps, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, const float* __restrict__ mean,
                                                       const float* __restrict__ var, void* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
    // every load first (x, then gamma / beta at clamped columns): the stores below then wait on nothing, and
    // rows whose NV chunks are all in range store without a branch (a loaded value used inside a per-chunk
    // branch made hipcc wait for every previous store there)
    const bool full = 4 * 64 * NV == cols;
    float4 v[NV], g[NV], bb[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int c4 = lane + 64 * k;
        v[k] = full || 4 * c4 < cols ? xr[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int c4 = min(lane + 64 * k, cols / 4 - 1);
        g[k] = gamma ? reinterpret_cast<const float4*>(gamma)[c4] : make_float4(1.f, 1.f, 1.f, 1.f);
        bb[k] = beta ? reinterpret_cast<const float4*>(beta)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float mu = 0.f, rstd = 1.f;
    if (mode == 0) {
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
        s = wave_sum(s);
        mu = s / (float)cols;
        float q = 0.f;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            if (full || 4 * (lane + 64 * k) < cols) {
                const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
                q += (a * a + b * b) + (c * c + d * d);
            }
        }
        q = wave_sum(q);
        rstd = 1.0f / sqrtf(q / (float)cols + eps);
    }
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int c4 = lane + 64 * k;
        if (!full && 4 * c4 >= cols) continue;
        float o[4];
        const float xv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        const float gv[4] = {g[k].x, g[k].y, g[k].z, g[k].w}, bv[4] = {bb[k].x, bb[k].y, bb[k].z, bb[k].w};
        if (mode == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (xv[e] - mu) * rstd * gv[e] + bv[e];
        } else {
            const float4 m = reinterpret_cast<const float4*>(mean)[c4], vr = reinterpret_cast<const float4*>(var)[c4];
            const float mv[4] = {m.x, m.y, m.z, m.w}, vv[4] = {vr.x, vr.y, vr.z, vr.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = (xv[e] - mv[e]) / sqrtf(vv[e] + eps) * gv[e] + bv[e];
        }
        if constexpr (OUT_BF16) {
            const uint32_t lo = f32_to_bf16_bits(o[0]) | (f32_to_bf16_bits(o[1]) << 16);
            const uint32_t hi = f32_to_bf16_bits(o[2]) | (f32_to_bf16_bits(o[3]) << 16);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + row * ldy + 4 * c4) = make_uint2(lo, hi);
        } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + row * ldy + 4 * c4) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

// BatchNormalization at inference (mode 1) is a per-column affine map, no row reduction: each thread owns
// one float4 column chunk, computes its 4 columns' 1/sqrt(var + eps) once, and walks kRowsPerBn rows
// (coalesced across the workgroup's 256 chunks = 1024 columns of one row). Any width with cols % 4 == 0.
constexpr int kRowsPerBn = 16;

template <bool OUT_BF16>
__global__ __launch_bounds__(256) void bn_vec_kernel(const float* __restrict__ x, int64_t rows, int cols, int64_t ldx,
                                                     float eps, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, const float* __restrict__ mean,
                                                     const float* __restrict__ var, void* __restrict__ y, int64_t ldy) {
    const int ncb = (cols / 4 + 255) / 256;  // column blocks; blockIdx.x = row group * ncb + column block
    const int c4 = (int)(blockIdx.x % ncb) * 256 + threadIdx.x;
    if (4 * c4 >= cols) return;
    const float4 m = reinterpret_cast<const float4*>(mean)[c4], vr = reinterpret_cast<const float4*>(var)[c4];
    const float4 g = gamma ? reinterpret_cast<const float4*>(gamma)[c4] : make_float4(1.f, 1.f, 1.f, 1.f);
    const float4 bb = beta ? reinterpret_cast<const float4*>(beta)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    const float mv[4] = {m.x, m.y, m.z, m.w}, gv[4] = {g.x, g.y, g.z, g.w}, bv[4] = {bb.x, bb.y, bb.z, bb.w};
    const float rs[4] = {1.0f / sqrtf(vr.x + eps), 1.0f / sqrtf(vr.y + eps), 1.0f / sqrtf(vr.z + eps), 1.0f / sqrtf(vr.w + eps)};
    const int64_t r0 = (int64_t)(blockIdx.x / ncb) * kRowsPerBn;
    const int64_t r1 = r0 + kRowsPerBn < rows ? r0 + kRowsPerBn : rows;
    for (int64_t r = r0; r < r1; ++r) {
        const float4 xv4 = reinterpret_cast<const float4*>(x + r * ldx)[c4];
        const float xv[4] = {xv4.x, xv4.y, xv4.z, xv4.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (xv[e] - mv[e]) * rs[e] * gv[e] + bv[e];
        if constexpr (OUT_BF16) {
            const uint32_t lo = f32_to_bf16_bits(o[0]) | (f32_to_bf16_bits(o[1]) << 16);
            const uint32_t hi = f32_to_bf16_bits(o[2]) | (f32_to_bf16_bits(o[3]) << 16);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + r * ldy + 4 * c4) = make_uint2(lo, hi);
        } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + r * ldy + 4 * c4) = make_float4(o[0], o[1], o[2], o[3]);
        }
    }
}

// LayerNormalization of rows wider than the one-wave vector path (2048 < cols <= 32768, cols % 4 == 0):
// one 256-thread workgroup per row, the row held once in registers (NV float4 per thread), mean and
// variance (two passes over the registers) reduced through LDS.
template <bool OUT_BF16, int NV>
__global__ __launch_bounds__(256) void ln_wide_kernel(const float* __restrict__ x, int cols, int64_t ldx, float eps,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      void* __restrict__ y, int64_t ldy) {
    __shared__ float red[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t row = blockIdx.x;
    const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
    float4 v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int c4 = tid + 256 * k;
        v[k] = 4 * c4 < cols ? xr[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    auto block_sum = [&](float s) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if (lane == 0) red[wave] = s;
        __syncthreads();
        const float t = (red[0] + red[1]) + (red[2] + red[3]);
        __syncthreads();
        return t;
    };
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    const float mu = block_sum(s) / (float)cols;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        if (4 * (tid + 256 * k) < cols) {
            const float a = v[k].x - mu, b = v[k].y - mu, c = v[k].z - mu, d = v[k].w - mu;
            q += (a * a + b * b) + (c * c + d * d);
        }
    }
    const float rstd = 1.0f / sqrtf(block_sum(q) / (float)cols + eps);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int c4 = tid + 256 * k;
        if (4 * c4 >= cols) continue;
        const float4 g = gamma ? reinterpret_cast<const float4*>(gamma)[c4] : make_float4(1.f, 1.f, 1.f, 1.f);
        const float4 bb = beta ? reinterpret_cast<const float4*>(beta)[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
        const float o0 = (v[k].x - mu) * rstd * g.x + bb.x, o1 = (v[k].y - mu) * rstd * g.y + bb.y;
        const float o2 = (v[k].z - mu) * rstd * g.z + bb.z, o3 = (v[k].w - mu) * rstd * g.w + bb.w;
        if constexpr (OUT_BF16) {
            const uint32_t lo = f32_to_bf16_bits(o0) | (f32_to_bf16_bits(o1) << 16);
            const uint32_t hi = f32_to_bf16_bits(o2) | (f32_to_bf16_bits(o3) << 16);
            *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(y) + row * ldy + 4 * c4) = make_uint2(lo, hi);
        } else {
            *reinterpret_cast<float4*>(reinterpret_cast<float*>(y) + row * ldy + 4 * c4) = make_float4(o0, o1, o2, o3);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// GEMM y[M,N] = act(x[M,K] W[N,K]^T + b)
// ---------------------------------------------------------------------------------------------
// block tile BT x BT (128, or 64 when the 128-tile grid would leave CUs idle), 4 waves in 2 x 2, each
// wave BT/2 x BT/2 = FR x FR fragments of 16 x 16

// bf16: BK = 64 (128-byte rows), LDS rows padded to 72 elements (144 B): conflict-free ds_read_b128
// for the 16 rows a 16-lane group reads.
constexpr int BKH = 64, RSH = BKH + 8;
// f32: BK = 32 (128-byte rows), rows padded to 36 floats (144 B). BK = 64 measured +3 % on the K = 8704
// tower GEMM but -7 % on the cascade's K = 256 catalog scoring (139 KiB of LDS: one workgroup per CU, so
// no tile's epilogue overlaps another's main loop), so 32 it stays (profiles/r02/gemm_probe_r02f.json).
constexpr int BKF = 32, RSF = BKF + 4;

template <bool BF16, int BT>
struct GemmCfg {
    static constexpr int BK = BF16 ? BKH : BKF;
    static constexpr int RS = BF16 ? RSH : RSF;          // elements
    static constexpr int ESZ = BF16 ? 2 : 4;
    static constexpr int EPC = 16 / ESZ;                  // elements per 16-byte chunk
    static constexpr int CPR = BK / EPC;                  // chunks per tile row (8)
    static constexpr int CHUNKS = BT * CPR;               // per operand tile (1024 at BT = 128)
    static constexpr int PER_THREAD = CHUNKS / 256;       // 4 at BT = 128
    static constexpr int FR = BT / 32;                    // 16x16 fragments per wave and dimension
};

// The next k-step's tile loads are issued as inline asm: the compiler keeps volatile asm in program order,
// so they go out before the MFMAs of the current step (as plain loads of read-only memory the DAG
// scheduler places them right before their use, at the end of the step, and the latency is exposed every
// step). The compiler does not track these loads: wait_tile waits for them (vmcnt) through the registers
// themselves, so the LDS stores that consume them cannot move above the wait.
using v4u = unsigned int __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4u gload_asm(const char* p) {
    v4u r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p));
    return r;
}

// Rows past M / N read a valid row (M-1 / N-1) instead of branching: they only feed outputs that are never
// stored. Only a K tail (KTAIL: K % BK != 0) needs zeros: the chunk's mask, applied after the wait.
template <bool BF16, int BT, bool KTAIL>
__device__ __forceinline__ void load_tile(v4u (&rg)[2][(GemmCfg<BF16, BT>::PER_THREAD)], uint32_t (&msk)[(GemmCfg<BF16, BT>::PER_THREAD)],
                                          const char* __restrict__ x, const char* __restrict__ w, int64_t M, int N, int K,
                                          int64_t ldx, int64_t ldw, int64_t m0, int n0, int k0, int tid) {
    using C = GemmCfg<BF16, BT>;
#pragma unroll
    for (int i = 0; i < C::PER_THREAD; ++i) {
        const int c = tid + i * 256;
        const int r = c / C::CPR, ch = c - r * C::CPR;
        const int kk = k0 + ch * C::EPC;
        const int64_t row = m0 + r < M ? m0 + r : M - 1;
        const int64_t col = n0 + r < N ? n0 + r : N - 1;
        int kc = kk;
        if constexpr (KTAIL) {
            msk[i] = kk < K ? 0xffffffffu : 0u;
            kc = kk < K ? kk : K - C::EPC;
        }
        rg[0][i] = gload_asm(x + (row * ldx + kc) * C::ESZ);
        rg[1][i] = gload_asm(w + (col * ldw + kc) * C::ESZ);
    }
}

template <bool BF16, int BT, bool KTAIL>
__device__ __forceinline__ void wait_tile(v4u (&rg)[2][(GemmCfg<BF16, BT>::PER_THREAD)], const uint32_t (&msk)[(GemmCfg<BF16, BT>::PER_THREAD)]) {
    using C = GemmCfg<BF16, BT>;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < C::PER_THREAD; ++i) {
        asm volatile("" : "+v"(rg[0][i]), "+v"(rg[1][i]));  // the registers are defined here, after the wait
        if constexpr (KTAIL) {
            rg[0][i] &= msk[i];
            rg[1][i] &= msk[i];
        }
    }
}

template <bool BF16, int BT>
__device__ __forceinline__ void store_tile(char* __restrict__ As, char* __restrict__ Bs,
                                           const v4u (&rg)[2][(GemmCfg<BF16, BT>::PER_THREAD)], int tid) {
    using C = GemmCfg<BF16, BT>;
#pragma unroll
    for (int i = 0; i < C::PER_THREAD; ++i) {
        const int c = tid + i * 256;
        const int r = c / C::CPR, ch = c - r * C::CPR;
        *reinterpret_cast<v4u*>(As + (r * C::RS + ch * C::EPC) * C::ESZ) = rg[0][i];
        *reinterpret_cast<v4u*>(Bs + (r * C::RS + ch * C::EPC) * C::ESZ) = rg[1][i];
    }
}

// SPLIT (split-K): blockIdx.y = s takes k in [s * kspan, min(K, (s + 1) * kspan)) and stores its raw partial sums
// to y + s * M * ldy (no bias, no activation: splitk_reduce_kernel adds the partials in order s = 0, 1, ...).
template <bool BF16, int BT, bool KTAIL, bool SPLIT = false>
__global__ __launch_bounds__(256) void gemm_kernel(const void* __restrict__ xv, const void* __restrict__ wv,
                                                   const float* __restrict__ bias, float* __restrict__ y, int64_t M,
                                                   int N, int K, int64_t ldx, int64_t ldy, int act, int kspan = 0) {
    using C = GemmCfg<BF16, BT>;
    constexpr int FR = C::FR, WT = BT / 2;
    __shared__ __attribute__((aligned(16))) char smem[2][2][BT * C::RS * C::ESZ];
    const int64_t ldw = K;  // W rows are [N][K]
    const int kb = SPLIT ? (int)blockIdx.y * kspan : 0;
    const char* x = reinterpret_cast<const char*>(xv) + (int64_t)kb * C::ESZ;
    const char* w = reinterpret_cast<const char*>(wv) + (int64_t)kb * C::ESZ;
    if constexpr (SPLIT) {
        K = min(kspan, K - kb);
        y += (int64_t)blockIdx.y * M * ldy;
    }
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order (guide T1, bijective form): blocks b, b + 8, ... share an XCD and take consecutive
    // tiles, so the N-tiles of one M row-panel read that panel through ONE XCD's L2 (the DSSM towers' 142 /
    // 335 MB activations were otherwise fetched once per N-tile, from 8 different L2s)
    const int tiles_n = (N + BT - 1) / BT;
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const int64_t tid_lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int64_t m0 = (tid_lin / tiles_n) * BT;
    const int n0 = (int)(tid_lin % tiles_n) * BT;
    f4 acc[FR][FR];
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < FR; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    v4u rg[2][C::PER_THREAD];
    uint32_t msk[C::PER_THREAD];
    const int nk = (K + C::BK - 1) / C::BK;
    load_tile<BF16, BT, KTAIL>(rg, msk, x, w, M, N, K, ldx, ldw, m0, n0, 0, tid);
    wait_tile<BF16, BT, KTAIL>(rg, msk);
    store_tile<BF16, BT>(smem[0][0], smem[0][1], rg, tid);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        // the last step re-loads its own stage into the idle buffer: no branch around the loads
        load_tile<BF16, BT, KTAIL>(rg, msk, x, w, M, N, K, ldx, ldw, m0, n0, (kt + 1 < nk ? kt + 1 : kt) * C::BK, tid);
        const char* As = smem[cur][0];
        const char* Bs = smem[cur][1];
        if constexpr (BF16) {
#pragma unroll
            for (int ks = 0; ks < C::BK; ks += 32) {
                bf16x8 af[FR], bfr[FR];
#pragma unroll
                for (int i = 0; i < FR; ++i)
                    af[i] = *reinterpret_cast<const bf16x8*>(As + ((wm * WT + i * 16 + lr) * C::RS + ks + lg * 8) * 2);
#pragma unroll
                for (int j = 0; j < FR; ++j)
                    bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + ((wn * WT + j * 16 + lr) * C::RS + ks + lg * 8) * 2);
#pragma unroll
                for (int i = 0; i < FR; ++i)
#pragma unroll
                    for (int j = 0; j < FR; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
            // 16x16x4 f32: lane (lr, lg) supplies A[lr][k], B[k][lr] for k = kh + lg*8 + s at step s (the k order
            // is permuted consistently for A and B, so the dot product is over all 32 k of each half)
#pragma unroll
            for (int kh = 0; kh < C::BK; kh += 32) {
                f4 a0[FR], a1[FR], b0[FR], b1[FR];
#pragma unroll
                for (int i = 0; i < FR; ++i) {
                    const float* p = reinterpret_cast<const float*>(As) + (wm * WT + i * 16 + lr) * C::RS + kh + lg * 8;
                    a0[i] = *reinterpret_cast<const f4*>(p);
                    a1[i] = *reinterpret_cast<const f4*>(p + 4);
                }
#pragma unroll
                for (int j = 0; j < FR; ++j) {
                    const float* p = reinterpret_cast<const float*>(Bs) + (wn * WT + j * 16 + lr) * C::RS + kh + lg * 8;
                    b0[j] = *reinterpret_cast<const f4*>(p);
                    b1[j] = *reinterpret_cast<const f4*>(p + 4);
                }
#pragma unroll
                for (int s = 0; s < 8; ++s)
#pragma unroll
                    for (int i = 0; i < FR; ++i)
#pragma unroll
                        for (int j = 0; j < FR; ++j) {
                            const float av = s < 4 ? a0[i][s] : a1[i][s - 4];
                            const float bv = s < 4 ? b0[j][s] : b1[j][s - 4];
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
                        }
            }
        }
        if (kt + 1 < nk) {  // its own block: the MFMAs above stay ahead of the wait
            wait_tile<BF16, BT, KTAIL>(rg, msk);
            store_tile<BF16, BT>(smem[cur ^ 1][0], smem[cur ^ 1][1], rg, tid);
        }
        __syncthreads();
    }
    wait_tile<BF16, BT, KTAIL>(rg, msk);  // the last step's spare loads land before their registers are reused
    if constexpr (SPLIT) {  // raw partial sums
#pragma unroll
        for (int j = 0; j < FR; ++j) {
            const int col = n0 + wn * WT + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t row = m0 + wm * WT + i * 16 + lg * 4 + r;
                    if (row < M) y[row * ldy + col] = acc[i][j][r];
                }
        }
        return;
    }
    // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r. Values first, stores after (a store in a
    // per-element branch next to a loaded bias made hipcc wait for every previous store; see gemm_lds_kernel)
    const int64_t rbase = m0 + wm * WT + lg * 4;
    const int cbase = n0 + wn * WT + lr;
    float bv[FR];
#pragma unroll
    for (int j = 0; j < FR; ++j) bv[j] = bias ? bias[min(cbase + j * 16, N - 1)] : 0.f;
    with_act(act, [&](auto A) {
#pragma unroll
        for (int j = 0; j < FR; ++j)
#pragma unroll
            for (int i = 0; i < FR; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][r] = A(acc[i][j][r] + bv[j]);
    });
    if (m0 + BT <= M && n0 + BT <= N) {
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float* yr = y + (rbase + i * 16 + r) * ldy + cbase;
#pragma unroll
                for (int j = 0; j < FR; ++j) yr[j * 16] = acc[i][j][r];
            }
        return;
    }
#pragma unroll
    for (int j = 0; j < FR; ++j) {
        const int col = cbase + j * 16;
        if (col >= N) continue;
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = rbase + i * 16 + r;
                if (row < M) y[row * ldy + col] = acc[i][j][r];
            }
    }
}

// ---------------------------------------------------------------------------------------------
// bf16 GEMM on an LDS-DMA ring (K % 64 == 0): y[M,N] = act(x[M,K] W[N,K]^T + b), fp32 out.
//   * block tile BM x 128 x 64 (BM = 128: 4 waves 2 x 2 of 64 x 64; BM = 64: 4 waves 1 x 4 of 64 x 32),
//     v_mfma_f32_16x16x32_bf16 with fp32 accumulators;
//   * A and B tiles land in LDS by global_load_lds_dwordx4 (no VGPR staging, no ds_write) in a ring of
//     kLdsStages buffers: the loads of step k + kLdsStages - 1 are issued right after the barrier that opens
//     step k; each wave waits for its own copies of step k (vmcnt) and the buffer is read only after the raw
//     s_barrier that follows the wait;
//   * 128-byte tile rows, 16-byte chunk c of row r stored at chunk c ^ (r & 7): the ds_read_b128 lane
//     groups of a 16 x 32 fragment touch 16 distinct (row parity, chunk) bank quads = conflict-free.
//     LDS-DMA writes lane-linear, so the swizzle is applied on the SOURCE address (lane -> chunk);
//   * XCD-aware tile order: the workgroups of one XCD (block ids congruent mod 8) take consecutive tiles,
//     so the N-tiles sharing an A row panel share that XCD's L2.
// ---------------------------------------------------------------------------------------------
// 2 stages: the next step's tiles are in flight behind this step's MFMAs. Measured against 3- to 5-deep rings
// on MI355X (tools/gemm_lab.hip, profiles/r03/gemm_lab_r03b.txt): the smaller LDS footprint (64 / 48 KB) lets two
// or three workgroups share a CU, whose MFMAs then cover each other's load waits — 4096x1280->1024 16.2 vs
// 16.9 us (64-row tiles), 51200x1280->1024 206 vs 248 us (128-row tiles); deeper rings only add LDS.
constexpr int kLdsK = 64, kLdsBN = 128, kLdsStages = 2;

// T = uint16_t (bf16, 64 per 128-byte row) or float (fp32, 32 per row): the ring, the swizzle and the copies are
// byte-identical for both; ldw = W's row stride (elements)
// ESZ = 2 (bf16, 64 per 128-byte row) or 4 (fp32, 32 per row): the ring, the swizzle and the copies are
// byte-identical for both; ldx / ldw (W's row stride) and k0 in elements
template <int BM, int ESZ>
__device__ __forceinline__ void glds_stage(const void* __restrict__ xv, const void* __restrict__ wv, int64_t M, int N,
                                           int64_t ldx, int64_t ldw, int64_t m0, int n0, int k0, void* Asv, void* Bsv,
                                           int tid) {
    const char* x = reinterpret_cast<const char*>(xv);
    const char* w = reinterpret_cast<const char*>(wv);
    char* As = reinterpret_cast<char*>(Asv);
    char* Bs = reinterpret_cast<char*>(Bsv);
    // one wave-instruction = 8 tile rows x 8 chunks (1 KiB, lane-linear in LDS); 4 waves
    const int wave = tid >> 6, lane = tid & 63, rr = lane >> 3, pos = lane & 7;
#pragma unroll
    for (int it = 0; it < BM / 32; ++it) {
        const int g = wave + 4 * it, r = g * 8 + rr;
        const int64_t row = m0 + r < M ? m0 + r : M - 1;  // rows past M: any valid row (never stored)
        const char* src = x + (row * ldx + k0) * ESZ + ((pos ^ rr) << 4);
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(As + g * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int it = 0; it < kLdsBN / 32; ++it) {
        const int g = wave + 4 * it, r = g * 8 + rr;
        const int64_t col = n0 + r < N ? n0 + r : N - 1;
        const char* src = w + (col * ldw + k0) * ESZ + ((pos ^ rr) << 4);
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(Bs + g * 1024), 16, 0, 0);
    }
}

// Epilogue variants of gemm_lds_kernel (the LayerNorm of the next layer folded across the pair):
//   kEpiPlain  y = act(acc + b), fp32
//   kEpiStats  y = act(acc + b) stored as bf16, and for every row and 32-column slice p of it (p = column tile
//              * 4 + slice; n_p = its columns < N) the pair (S_p, M2_p) of the fp32 values: their sum and their
//              squared deviations from the slice's own mean S_p / n_p (two 16-lane shuffle reduces), written to
//              stats[row][p]; no atomics, so the reduction order (and the result) is fixed. Deviations from a
//              local mean keep the variance exact-ish for rows whose mean is large against their spread (a
//              single sum-of-squares pass loses it to cancellation)
//   kEpiLnFold y = act(rstd_r (acc - mu_r s_c) + t_c): acc = x W'^T with x the previous layer's raw bf16
//              output and W' = W diag(gamma); mu_r, rstd_r from stats over the K columns; s_c = sum_k W'[c][k],
//              t_c = W beta + b. That is LN(x) W^T + b with the normalisation applied after the product.
//              The workgroup first reduces its rows' P partials in a fixed order into LDS.
//   kEpiLnFoldStats  kEpiLnFold's y, then kEpiStats' bf16 store and slice partials of it (into ostats / oP): the
//              middle layer of an LN-folded chain whose input statistics came from its producers (cfg3: the input MLP
//              and the ESIM attention write the pooled row as bf16 + slice partials; no LayerNorm pass)
//   kEpiLnFoldHead   kEpiLnFold's y (stored only when y is given), then the per-row partial logits of a small head
//              Dense(NH) over this tile's columns: hpart[row][tile_n][h] = sum_c y[row][c] Wh[h][c], reduced over the
//              tile's waves in a fixed order (head_softmax_kernel adds the tiles in order, the bias, the softmax)
//   kEpiCompact  no output matrix: every score y[row][col] >= thr[row] is appended, in no particular order, to
//              row's candidate list (cval / cidx [row][0 .. cap), index cbase + col); ccount[row] counts every such
//              score (entries past cap are dropped: the caller sees ccount > cap). The exact-search screen of
//              FaissSearcher (rf_ip_candidates_f32): the scores are this kernel's, bit for bit, as rf_linear_fwd's
enum { kEpiPlain = 0, kEpiStats = 1, kEpiLnFold = 2, kEpiLnFoldStats = 3, kEpiLnFoldHead = 4, kEpiCompact = 5 };
// lab ablations (tools/build_variants.sh -DRF_LAB_ABL=bits; result-changing, never in the shipped build): 1 = no head
// partials / hand-off, 2 = no hand-off (partials stored), 4 = no LN-fold row statistics (loads and combine)
#ifndef RF_LAB_ABL
#define RF_LAB_ABL 0
#endif
constexpr int kHeadN = 2;  // kEpiLnFoldHead: head outputs (cfg3's Dense(2, softmax))

struct EpiArgs {
    uint16_t* yb;        // kEpiStats / kEpiLnFoldStats output
    float* stats;        // kEpiStats: written; kEpiLnFold*: read (the input row's slice partials)
    const float* fs;     // kEpiLnFold s_c
    const float* ft;     // kEpiLnFold t_c
    float eps;
    int P;               // partials per row of `stats` (4 per 128 columns)
    float* ostats;       // kEpiLnFoldStats: the output's slice partials (oP per row)
    int oP;
    const uint16_t* hw;  // kEpiLnFoldHead: head weight [kHeadN][N] bf16
    float* hpart;        // kEpiLnFoldHead: [M][tiles_n][kHeadN]
    int* hcnt;           // kEpiLnFoldHead: one counter per row block (zero between launches), or null: separate softmax
    const float* hb;     // head bias [kHeadN] or null
    int hact;            // head activation
    float* hout;         // [M][kHeadN] probabilities, row stride hldo
    int64_t hldo;
    const float* thr;    // kEpiCompact: per-row threshold [M]
    int* ccount;         // kEpiCompact: per-row candidate counts [M] (zero before the launch)
    float* cval;         // kEpiCompact: [M][cap] scores
    uint32_t* cidx;      // kEpiCompact: [M][cap] item indices
    int cap;
    int64_t cbase;       // kEpiCompact: item index of column 0
    const float* qbound; // kEpiCompact, optional: the pass test is y >= thr[row] - qbound[row] * vnorm[col] (a screen
    const float* vnorm;  //   on rounded operands with its error bound), both or neither
};

// the head's outputs of one row from its logits: softmax over the kHeadN values, or an elementwise activation
__device__ __forceinline__ void head_finish(float (&z)[kHeadN], int act, float* __restrict__ y) {
    if (act == RF_ACT_SOFTMAX) {
        float m = z[0];
#pragma unroll
        for (int h = 1; h < kHeadN; ++h) m = fmaxf(m, z[h]);
        float s = 0.f;
#pragma unroll
        for (int h = 0; h < kHeadN; ++h) {
            z[h] = expf(z[h] - m);
            s += z[h];
        }
#pragma unroll
        for (int h = 0; h < kHeadN; ++h) y[h] = z[h] / s;
    } else {
        with_act(act, [&](auto A) {
#pragma unroll
            for (int h = 0; h < kHeadN; ++h) y[h] = A(z[h]);
        });
    }
}

// Sum over aligned groups of G consecutive lanes (G = 1, 2, 4), the xor-butterfly order (offsets 1, 2) by DPP
template <int G>
__device__ __forceinline__ float lane_group_sum(float v) {
    static_assert(G == 1 || G == 2 || G == 4, "quad-local groups only");
    if constexpr (G >= 2) v += dpp_mov<0xB1>(v);  // quad_perm [1,0,3,2]: xor 1
    if constexpr (G >= 4) v += dpp_mov<0x4E>(v);  // quad_perm [2,3,0,1]: xor 2
    return v;
}

// The LN fold's per-row (mu, rstd) from the stats GEMM's P slice partials, TPR threads per row (rows whose
// partials do not fit gemm_lds_kernel's registers): Chan's combine, the same order as the register path.
template <int TPR>
__device__ __forceinline__ void ln_fold_row_stats(const float2* rs2, int P, int K, float eps, int part, int rl,
                                                  float* srow) {
    float s1 = 0.f;
    for (int p = part; p < P; p += TPR) s1 += rs2[p].x;
    s1 = lane_group_sum<TPR>(s1);
    const float m = s1 / (float)K;
    float s2 = 0.f;
    for (int p = part; p < P; p += TPR) {
        const int np = min(max(K - p * 32, 0), 32);
        if (np > 0) {
            const float2 v = rs2[p];
            const float dv = v.x - (float)np * m;
            s2 += v.y + dv * dv / (float)np;
        }
    }
    s2 = lane_group_sum<TPR>(s2);
    if (part == 0) {
        srow[2 * rl] = m;
        srow[2 * rl + 1] = 1.0f / sqrtf(s2 / (float)K + eps);
    }
}

// F32: fp32 operands (x and W both fp32) on v_mfma_f32_16x16x4f32, 32 k per 128-byte row: a lane's two 16-byte
// chunks (k = 4 lg .. 4 lg + 3 and 16 + 4 lg .. 16 + 4 lg + 3) feed 8 MFMAs, A and B in the same permuted k order.
// SPLIT (split-K, EPI plain only): blockIdx.y = s takes k in [s kspan, min(K, (s + 1) kspan)) and stores raw
// partial sums to y + s M ldy (splitk_reduce_kernel adds them in order s = 0, 1, ... with the bias / activation).
// ST: ring depth (kLdsStages by default; launch_lds_epi takes a deeper ring when the grid holds at most one tile per
// CU, where no second workgroup covers the load waits)
template <int BM, int EPI = kEpiPlain, bool F32 = false, bool SPLIT = false, int ST = kLdsStages>
__global__ __launch_bounds__(256) void gemm_lds_kernel(const void* __restrict__ xv, const void* __restrict__ wv,
                                                       const float* __restrict__ bias, float* __restrict__ y, int64_t M,
                                                       int N, int K, int64_t ldx, int64_t ldy, int act, EpiArgs ea,
                                                       int kspan = 0) {
    using T = std::conditional_t<F32, float, uint16_t>;
    constexpr int kK = 128 / (int)sizeof(T);                       // k per step (one 128-byte row)
    constexpr int SH = F32 ? 2 : 3;
    constexpr int WM = BM == 128 ? 2 : 1, WN = 4 / WM;            // wave grid
    constexpr int TM = BM / WM, TN = kLdsBN / WN;                  // wave tile
    constexpr int FM = TM / 16, FN = TN / 16;                      // fragments per wave
    constexpr int A_EL = BM * kK, B_EL = kLdsBN * kK;              // elements per stage
    constexpr int LOADS = (BM / 8 + kLdsBN / 8) / 4;               // glds per thread per stage
    static_assert(!SPLIT || EPI == kEpiPlain, "split-K: plain epilogue only");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* lds = reinterpret_cast<T*>(smem_raw);
    const int64_t ldw = K;
    const int kb = SPLIT ? (int)blockIdx.y * kspan : 0;
    const T* x = reinterpret_cast<const T*>(xv) + kb;
    const T* w = reinterpret_cast<const T*>(wv) + kb;
    if constexpr (SPLIT) {
        K = min(kspan, K - kb);
        y += (int64_t)blockIdx.y * M * ldy;
    }
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int wm = wave / WN, wn = wave % WN;
    // XCD-aware tile order (bijective): block b runs on XCD b % 8; give each XCD a contiguous tile range
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int tiles_n = (N + kLdsBN - 1) / kLdsBN;
    // kEpiCompact (a few query rows against a long item matrix): the row tiles of one item tile are consecutive, so
    // they run together on one XCD and the item tile is read from HBM once (n-fastest order re-reads it per row tile)
    const int tiles_m = (int)((M + BM - 1) / BM);
    const int64_t m0 = (int64_t)(EPI == kEpiCompact ? tile % tiles_m : tile / tiles_n) * BM;
    const int n0 = (EPI == kEpiCompact ? tile / tiles_m : tile % tiles_n) * kLdsBN;
    const int nk = K / kK;

    f4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

    auto As = [&](int s) { return lds + s * (A_EL + B_EL); };
    auto Bs = [&](int s) { return lds + s * (A_EL + B_EL) + A_EL; };
    // the ring's first ST - 1 stages. With ST >= 3 they are issued AFTER the epilogue parameter and row-statistics
    // loads below: vmcnt retires in issue order, so the loop's first wait for stage 0 with stages 1 .. ST - 2 left in
    // flight would otherwise also wait for every younger parameter load (and, in effect, for the whole prologue)
    auto ring_prologue = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p + 1 < ST; ++p)
            if (p < nk) glds_stage<BM, (int)sizeof(T)>(x, w, M, N, ldx, ldw, m0, n0, p * kK, As(p), Bs(p), tid);
    };
    if constexpr (ST < 3) ring_prologue();
    // The epilogue's per-column parameters (bias, or the LN fold's s_c / t_c) are loaded now, under the first
    // stage's copies, instead of as dependent loads after the last MFMA (one HBM round trip off the tail).
    float pb[FN], pt[FN];
    // kEpiLnFoldHead: the head weights of this lane's columns, loaded here for the same reason (0 past N)
    float hwv[EPI == kEpiLnFoldHead ? kHeadN : 1][FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        if constexpr (EPI == kEpiLnFoldHead) {
            const int c = n0 + wn * TN + j * 16 + lr;
#pragma unroll
            for (int h = 0; h < kHeadN; ++h)
                hwv[h][j] = c < N ? __uint_as_float((uint32_t)ea.hw[(int64_t)h * N + c] << 16) : 0.f;
        }
        const int col = min(n0 + wn * TN + j * 16 + lr, N - 1);
        if constexpr (EPI == kEpiLnFold || EPI == kEpiLnFoldStats || EPI == kEpiLnFoldHead) {
            pb[j] = ea.fs[col];
            pt[j] = ea.ft[col];
        } else {
            pb[j] = bias ? bias[col] : 0.f;
            pt[j] = 0.f;
        }
    }
    // kEpiCompact: this lane's row thresholds, loaded under the k-loop like the column parameters (+inf past M)
    float tv[EPI == kEpiCompact ? FM : 1][4], qv[EPI == kEpiCompact ? FM : 1][4], vv[EPI == kEpiCompact ? FN : 1];
    if constexpr (EPI == kEpiCompact) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = m0 + wm * TM + lg * 4 + i * 16 + r;
                tv[i][r] = row < M ? ea.thr[row] : INFINITY;
                qv[i][r] = ea.qbound && row < M ? ea.qbound[row] : 0.f;
            }
#pragma unroll
        for (int j = 0; j < FN; ++j) vv[j] = ea.vnorm ? ea.vnorm[min(n0 + wn * TN + j * 16 + lr, N - 1)] : 0.f;
    }
    // LN-fold row statistics (mu, rstd per tile row), in an LDS area past the ring
    float* srow = reinterpret_cast<float*>(smem_raw + (size_t)ST * (A_EL + B_EL) * sizeof(T));
    // LN fold: the tile's row statistics (complete: the previous launch wrote them) are combined in a fixed order
    // (TPR threads per row, each a strided subset, then a commutative lane combine: every lane the same bits).
    // Their loads are issued here, into registers, and the combine runs after the k-loop, so the two dependent
    // global round trips are hidden under the MFMAs instead of delaying the first one (P <= NPR * TPR, i.e.
    // K <= 2048 at BM = 64; longer rows combine before the loop)
    constexpr int TPR = 256 / BM, NPR = 16;
    const int rl = tid / TPR, part = tid % TPR;
    const float2* rs2 = nullptr;
    float2 sp[NPR];
    bool stats_late = false;
    constexpr bool LNF = EPI == kEpiLnFold || EPI == kEpiLnFoldStats || EPI == kEpiLnFoldHead;
    if constexpr (LNF) {
        const int64_t row = m0 + rl < M ? m0 + rl : M - 1;
        rs2 = reinterpret_cast<const float2*>(ea.stats) + row * ea.P;
        stats_late = ea.P <= NPR * TPR;
        if (RF_LAB_ABL & 4) {
            if (part == 0) {
                srow[2 * rl] = 0.f;
                srow[2 * rl + 1] = 1.f;
            }
            stats_late = false;
        } else if (stats_late) {
#pragma unroll
            for (int u = 0; u < NPR; ++u) {
                const int p = part + u * TPR;
                sp[u] = p < ea.P ? rs2[p] : make_float2(0.f, 0.f);
            }
        } else {
            ln_fold_row_stats<TPR>(rs2, ea.P, K, ea.eps, part, rl, srow);
            __syncthreads();  // srow visible to every wave (this also retires stage 0's copies: the loop waits for them first)
        }
    }
    if constexpr (ST >= 3) ring_prologue();
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt % ST;
        // stage kt must have landed; the stages issued after it (min(ST - 2, nk - 1 - kt)) may stay in flight
        // (vmcnt retires in issue order; the epilogue parameter loads issued after the prologue only make it wait longer)
        const int ahead = min(ST - 2, nk - 1 - kt);
        if (ST >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
        else if (ST >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage kt landed for every wave; every wave is done reading stage kt - 1
        __builtin_amdgcn_sched_barrier(0);
        if (kt + ST - 1 < nk) {
            const int s2 = (kt + ST - 1) % ST;
            glds_stage<BM, (int)sizeof(T)>(x, w, M, N, ldx, ldw, m0, n0, (kt + ST - 1) * kK, As(s2), Bs(s2), tid);
        }
        const T* A = As(s);
        const T* B = Bs(s);
        // both halves' fragments are read up front: the second half's reads run under the first half's MFMAs
        using frag = std::conditional_t<F32, f4, bf16x8>;
        frag af[2][FM], bfr[2][FN];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ch = 4 * h + lg;  // 16-byte chunk of this lane's k values
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wm * TM + i * 16 + lr;
                af[h][i] = *reinterpret_cast<const frag*>(A + r * kK + ((ch ^ (r & 7)) << SH));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int r = wn * TN + j * 16 + lr;
                bfr[h][j] = *reinterpret_cast<const frag*>(B + r * kK + ((ch ^ (r & 7)) << SH));
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep every read ahead of the MFMAs (hipcc would re-serialise them)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (F32) {
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[h][i], bfr[h][j], acc[i][j], 0, 0, 0);
            }
        }
    }
    if constexpr (LNF) {
        if (stats_late) {
            // Chan's combine of the slices: mu = sum S_p / K, M2 = sum M2_p + (S_p - n_p mu)^2 / n_p
            float s1 = 0.f;
#pragma unroll
            for (int u = 0; u < NPR; ++u) s1 += sp[u].x;  // zeros past P: the same sum as the strided loop
            s1 = lane_group_sum<TPR>(s1);
            const float m = s1 / (float)K;
            float s2 = 0.f;
#pragma unroll
            for (int u = 0; u < NPR; ++u) {
                const int p = part + u * TPR;
                const int np = min(max(K - p * 32, 0), 32);
                if (p < ea.P && np > 0) {
                    const float dv = sp[u].x - (float)np * m;
                    s2 += sp[u].y + dv * dv / (float)np;
                }
            }
            s2 = lane_group_sum<TPR>(s2);
            if (part == 0) {
                srow[2 * rl] = m;
                srow[2 * rl + 1] = 1.0f / sqrtf(s2 / (float)K + ea.eps);
            }
            __syncthreads();  // srow visible to every wave
        }
    }
    if constexpr (SPLIT) {  // raw partial sums
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row < M) y[row * ldy + col] = acc[i][j][r];
                }
        }
        return;
    }
    // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r. Values first (straight-line, in acc), stores
    // after: a store inside a per-element branch next to a use of a loaded value (bias, s_c, t_c) made hipcc put
    // an s_waitcnt vmcnt(0) in every branch block, so each store waited for the previous one to land
    // (4096x1280->1024: 20.7 vs 16.8 us with the same main loop). Interior tiles (block-uniform) store unguarded.
    const bool full = m0 + BM <= M && n0 + kLdsBN <= N;
    const int64_t rbase = m0 + wm * TM + lg * 4;
    const int cbase = n0 + wn * TN + lr;
    if constexpr (EPI == kEpiPlain) {
        with_act(act, [&](auto A) {
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i][j][r] = A(acc[i][j][r] + pb[j]);
        });
        if (full) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float* yr = y + (rbase + i * 16 + r) * ldy + cbase;
#pragma unroll
                    for (int j = 0; j < FN; ++j) yr[j * 16] = acc[i][j][r];
                }
        } else {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int col = cbase + j * 16;
                if (col >= N) continue;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t row = rbase + i * 16 + r;
                        if (row < M) y[row * ldy + col] = acc[i][j][r];
                    }
            }
        }
    } else if constexpr (EPI == kEpiCompact) {
        // per (fragment row i, accumulator row r): this lane's passing columns (4 bits, one per column fragment j), a
        // prefix count over the 16 lanes sharing the row (lane & 15) and ONE atomic add per row group and wave for
        // the group's total — every add issued before any result is used (one round trip, not 16) — then each lane
        // writes its entries at base + its exclusive prefix
        uint32_t pm[FM][4];
        int pin[FM][4], pbase[FM][4];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                uint32_t m = 0;
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    m |= (cbase + j * 16 < N && acc[i][j][r] >= tv[i][r] - qv[i][r] * vv[j]) ? (1u << j) : 0u;
                pm[i][r] = m;
                pin[i][r] = 0;
                pbase[i][r] = 0;
                // most (i, r) slices of a tile (4 rows x 64 columns) hold no candidate: one wave vote skips the count
                if (!__any(m != 0u)) continue;
                const int n = __builtin_popcount(m);
                int incl = n;
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    const int y = __shfl_up(incl, o, 16);
                    if (lr >= o) incl += y;
                }
                const int total = __shfl(incl, 15, 16);
                pin[i][r] = incl - n;
                const int64_t row = rbase + i * 16 + r;
                if (lr == 15 && total > 0) pbase[i][r] = atomicAdd(ea.ccount + row, total);
            }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (!__any(pm[i][r] != 0u)) continue;
                const int base = __shfl(pbase[i][r], 15, 16);
                const uint32_t m = pm[i][r];
                if (m) {
                    const int64_t row = rbase + i * 16 + r;
                    int off = base + pin[i][r];
                    float* cv = ea.cval + row * (int64_t)ea.cap;
                    uint32_t* ci = ea.cidx + row * (int64_t)ea.cap;
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        if (m & (1u << j)) {
                            if (off < ea.cap) {
                                cv[off] = acc[i][j][r];
                                ci[off] = (uint32_t)(ea.cbase + cbase + j * 16);
                            }
                            ++off;
                        }
                }
            }
    } else if constexpr (EPI == kEpiStats || EPI == kEpiLnFoldStats) {
        // pass 1: activation, the fp32 value kept in acc (0 past N); then the bf16 stores
        with_act(act, [&](auto A) {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const bool cok = cbase + j * 16 < N;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float v;
                        if constexpr (EPI == kEpiStats) {
                            v = A(acc[i][j][r] + pb[j]);
                        } else {
                            const int rl = wm * TM + i * 16 + lg * 4 + r;
                            v = A(srow[2 * rl + 1] * (acc[i][j][r] - srow[2 * rl] * pb[j]) + pt[j]);
                        }
                        acc[i][j][r] = cok ? v : 0.f;
                    }
            }
        });
        __bf16* yb = reinterpret_cast<__bf16*>(ea.yb);
        if (full) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    __bf16* yr = yb + (rbase + i * 16 + r) * ldy + cbase;
#pragma unroll
                    for (int j = 0; j < FN; ++j) yr[j * 16] = (__bf16)acc[i][j][r];  // v_cvt_pk_bf16_f32, RNE
                }
        } else {
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int col = cbase + j * 16;
                if (col >= N) continue;
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t row = rbase + i * 16 + r;
                        if (row < M) yb[row * ldy + col] = (__bf16)acc[i][j][r];
                    }
            }
        }
        // pass 2: per 32-column slice (fragments 2q, 2q + 1 of this wave): sum, then squared deviations from the
        // slice mean; slices past N hold (0, 0)
        constexpr int SPW = FN / 2;  // slices per wave (TN = 64: 2; TN = 32: 1)
#pragma unroll
        for (int q = 0; q < SPW; ++q) {
            const int c0 = n0 + wn * TN + q * 32;
            const int nq = min(max(N - c0, 0), 32);
            const float inv_n = nq > 0 ? 1.0f / (float)nq : 0.f;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sm = row16_sum(acc[i][2 * q][r] + acc[i][2 * q + 1][r]);
                    const float mq = sm * inv_n;
                    const float d0 = c0 + lr < N ? acc[i][2 * q][r] - mq : 0.f;
                    const float d1 = c0 + 16 + lr < N ? acc[i][2 * q + 1][r] - mq : 0.f;
                    const float m2 = row16_sum(d0 * d0 + d1 * d1);
                    const int64_t row = rbase + i * 16 + r;
                    float* so = EPI == kEpiStats ? ea.stats : ea.ostats;
                    const int sP = EPI == kEpiStats ? ea.P : ea.oP;
                    if (lr == 0 && row < M)
                        *reinterpret_cast<float2*>(so + 2 * (row * sP + (n0 / kLdsBN) * 4 + wn * SPW + q)) =
                            make_float2(sm, m2);
                }
        }
    } else {  // kEpiLnFold / kEpiLnFoldHead: the row statistics were reduced into srow before the loop
        with_act(act, [&](auto A) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rl = wm * TM + i * 16 + lg * 4 + r;
                    const float mu = srow[2 * rl], rstd = srow[2 * rl + 1];
#pragma unroll
                    for (int j = 0; j < FN; ++j) acc[i][j][r] = A(rstd * (acc[i][j][r] - mu * pb[j]) + pt[j]);
                }
        });
        if (EPI == kEpiLnFold || y) {
            if (full) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        float* yr = y + (rbase + i * 16 + r) * ldy + cbase;
#pragma unroll
                        for (int j = 0; j < FN; ++j) yr[j * 16] = acc[i][j][r];
                    }
            } else {
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int col = cbase + j * 16;
                    if (col >= N) continue;
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int64_t row = rbase + i * 16 + r;
                            if (row < M) y[row * ldy + col] = acc[i][j][r];
                        }
                }
            }
        }
        if constexpr (EPI == kEpiLnFoldHead && !(RF_LAB_ABL & 1)) {
            // this wave's TN columns of every row it holds: sum_c y[row][c] Wh[h][c], c in fragment order, then the
            // 16 lanes of a row (row16_sum); the WN waves of a row meet in LDS (the ring is free after a barrier)
            float* hred = reinterpret_cast<float*>(smem_raw);  // [WN][BM][kHeadN]
            __syncthreads();  // every wave's last fragment reads of the ring are done
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int rl = wm * TM + i * 16 + lg * 4 + r;
#pragma unroll
                    for (int h = 0; h < kHeadN; ++h) {
                        float v = 0.f;
#pragma unroll
                        for (int j = 0; j < FN; ++j) v = fmaf(acc[i][j][r], hwv[h][j], v);
                        v = row16_sum(v);
                        if (lr == 0) hred[(wn * BM + rl) * kHeadN + h] = v;
                    }
                }
            __syncthreads();
            const int tiles_n = (N + kLdsBN - 1) / kLdsBN;
            for (int t = tid; t < BM * kHeadN; t += 256) {
                const int rl = t / kHeadN, h = t % kHeadN;
                float v = 0.f;
#pragma unroll
                for (int w = 0; w < WN; ++w) v += hred[(w * BM + rl) * kHeadN + h];
                const int64_t row = m0 + rl;
                float* dst = ea.hpart + (row * tiles_n + n0 / kLdsBN) * kHeadN + h;
                if (row < M) {
                    if (ea.hcnt) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1: L2-served
                    else *dst = v;
                }
            }
            if (ea.hcnt && !(RF_LAB_ABL & 2)) {
                // the row block's last tile to finish finishes the head: MI355X_MICROARCH's hand-off table, first row,
                // in every cell: the partials are stored sc1 (relaxed agent atomic stores), every storing wave waits
                // for them (vmcnt(0)), a workgroup barrier, then ONE lane adds to the row block's counter (agent
                // scope); the workgroup whose add returned tiles_n - 1 reads every partial with sc1 loads after a
                // barrier; hipMalloc'd workspace; one workgroup per CU (the launch's 99 KB of LDS). Release / acquire
                // semantics on the add lower to an L2 write-back + L1 invalidate per workgroup and cost
                // 7.7 us of a 21 us launch (profiles/r05/scorer_gemm_ablation.txt); the sc1 form needs neither.
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                int* s_last = reinterpret_cast<int*>(smem_raw);
                if (tid == 0) {
                    const int old = __hip_atomic_fetch_add(ea.hcnt + tile / tiles_n, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_last[0] = old == tiles_n - 1;
                }
                __syncthreads();
                if (s_last[0]) {
                    if (tid == 0) __hip_atomic_store(ea.hcnt + tile / tiles_n, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    for (int rl = tid; rl < BM; rl += 256) {
                        const int64_t row = m0 + rl;
                        if (row >= M) continue;
                        float z[kHeadN];
#pragma unroll
                        for (int h = 0; h < kHeadN; ++h) {
                            float v = 0.f;
                            for (int t = 0; t < tiles_n; ++t)
                                v += __hip_atomic_load(ea.hpart + (row * tiles_n + t) * kHeadN + h, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                            z[h] = v + (ea.hb ? ea.hb[h] : 0.f);
                        }
                        head_finish(z, ea.hact, ea.hout + row * ea.hldo);
                    }
                }
            }
        }
    }
}

// cfg3's head after kEpiLnFoldHead: logits[row][h] = sum over the column tiles in order of hpart + b[h]; softmax (or
// the elementwise activation) over the kHeadN outputs; one thread per row
__global__ __launch_bounds__(256) void head_softmax_kernel(const float* __restrict__ hpart, int tiles, int64_t M,
                                                           const float* __restrict__ b, int act, float* __restrict__ y,
                                                           int64_t ldy) {
    const int64_t row = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (row >= M) return;
    float z[kHeadN];
#pragma unroll
    for (int h = 0; h < kHeadN; ++h) {
        float v = 0.f;
        for (int t = 0; t < tiles; ++t) v += hpart[(row * tiles + t) * kHeadN + h];
        z[h] = v + (b ? b[h] : 0.f);
    }
    head_finish(z, act, y + row * ldy);
}

template <int BM, int ST = kLdsStages>
constexpr size_t gemm_lds_bytes() {
    return (size_t)ST * (BM + kLdsBN) * kLdsK * 2 + (size_t)BM * 2 * sizeof(float);  // ring + LN-fold rows
}

// small-N head: one wave per row, fp32 dot products, optional row softmax (N <= 64)
template <bool BF16>
__global__ __launch_bounds__(256) void small_n_kernel(const void* __restrict__ xv, const void* __restrict__ wv,
                                                      const float* __restrict__ bias, float* __restrict__ y, int64_t M,
                                                      int N, int K, int64_t ldx, int64_t ldy, int act) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    float outv[64];
    float mx = -INFINITY;
    for (int n = 0; n < N && n < 64; ++n) {
        float s = 0.f;
        for (int k = lane; k < K; k += 64) {
            float xv_, wv_;
            if constexpr (BF16) {
                xv_ = bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(xv)[row * ldx + k]);
                wv_ = bf16_bits_to_f32(reinterpret_cast<const uint16_t*>(wv)[(int64_t)n * K + k]);
            } else {
                xv_ = reinterpret_cast<const float*>(xv)[row * ldx + k];
                wv_ = reinterpret_cast<const float*>(wv)[(int64_t)n * K + k];
            }
            s = fmaf(xv_, wv_, s);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        s += bias ? bias[n] : 0.f;
        outv[n] = act == RF_ACT_SOFTMAX ? s : act_apply(act, s);
        mx = fmaxf(mx, outv[n]);
    }
    if (act == RF_ACT_SOFTMAX) {
        float sum = 0.f;
        for (int n = 0; n < N; ++n) {
            outv[n] = expf(outv[n] - mx);
            sum += outv[n];
        }
        for (int n = 0; n < N; ++n) outv[n] /= sum;
    }
    if (lane == 0)
        for (int n = 0; n < N; ++n) y[row * ldy + n] = outv[n];
}

// small Dense head on fp32 activations (rf_dense_head_fwd): one wave per row, float4 loads of x and the
// weights' 4 matching k values per output, NMAX fp32 partial dots per lane, shuffle-reduced
template <bool WBF16, int NMAX>
__global__ __launch_bounds__(256) void dense_head_kernel(const float* __restrict__ x, int64_t M, int K, int64_t ldx,
                                                         const void* __restrict__ wv, int N, const float* __restrict__ bias,
                                                         int act, float* __restrict__ y, int64_t ldy) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= M) return;
    const float4* xr = reinterpret_cast<const float4*>(x + row * ldx);
    float acc[NMAX], bv[NMAX];
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        acc[n] = 0.f;
        bv[n] = bias ? bias[min(n, N - 1)] : 0.f;  // loaded now: not a dependent round trip after the sums
    }
    for (int k4 = lane; 4 * k4 < K; k4 += 64) {
        const float4 xv = xr[k4];
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            if (n < N) {
                float4 w;
                if constexpr (WBF16) {
                    const uint2 u = reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(wv) + (int64_t)n * K)[k4];
                    w = make_float4(bf16_bits_to_f32(u.x & 0xffffu), bf16_bits_to_f32(u.x >> 16),
                                    bf16_bits_to_f32(u.y & 0xffffu), bf16_bits_to_f32(u.y >> 16));
                } else {
                    w = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(wv) + (int64_t)n * K)[k4];
                }
                acc[n] = fmaf(xv.x, w.x, acc[n]);
                acc[n] = fmaf(xv.y, w.y, acc[n]);
                acc[n] = fmaf(xv.z, w.z, acc[n]);
                acc[n] = fmaf(xv.w, w.w, acc[n]);
            }
        }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
        if (n < N) {
            acc[n] = wave_sum(acc[n]) + bv[n];
            if (act != RF_ACT_SOFTMAX) acc[n] = act_apply(act, acc[n]);
            mx = fmaxf(mx, acc[n]);
        }
    }
    if (act == RF_ACT_SOFTMAX) {
        float sum = 0.f;
#pragma unroll
        for (int n = 0; n < NMAX; ++n)
            if (n < N) {
                acc[n] = expf(acc[n] - mx);
                sum += acc[n];
            }
#pragma unroll
        for (int n = 0; n < NMAX; ++n) acc[n] /= sum;
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
        if (n < N && lane == (n & 63)) y[row * ldy + n] = acc[n];
}

// ---------------------------------------------------------------------------------------------
// Two-layer create_mlp on a narrow input, one launch (the ESIM input_mlp: 16 -> 256 -> 512, LayerNorm,
// gelu; esim.py:45-48, mlp.py:4-15). v2 (round 3): a workgroup owns 16 rows and EVERY output column
// (grid = row blocks), 4 waves:
//   * wave 0 runs LN0 for the 16 rows (4 lanes per row) into a bf16 A tile in LDS (k zero-padded to 32);
//   * layer 0 H = act(A W0^T + b0) is split over the waves by columns (wave w: H/4 of them), so no
//     workgroup recomputes it (v1's 64-row x 128-column blocks each redid layer 0 for their column block:
//     4x the gelu work, and one wave per SIMD left it VALU-issue-bound, 4.4 K VALU per wave, 21.7 us);
//   * LN1 over the H columns: per-wave row partials (16-lane DPP sums) meet in LDS in wave order (fixed:
//     deterministic), two passes (mean, then squared deviations) -> bf16 rows in LDS;
//   * layer 1 O = act(LN1(H) W1^T + b1): wave w takes 128-column blocks w, w + 4, ...; its W1 fragments
//     (16 B per lane per MFMA) are loaded from L2 into registers at kernel start, so they land while
//     LN0 / layer 0 / LN1 run (one workgroup per CU: the register budget is the whole SIMD's).
// ---------------------------------------------------------------------------------------------
constexpr int kMlp2Rows = 16, kMlp2Cols = 128;

template <int H>
constexpr size_t mlp2_lds_bytes() {
    // xs [16][40] bf16, w0s [H][32] bf16, hs [16][H + 8] bf16, params 3 H floats, row partials [4][16] x 2
    return 2 * ((size_t)kMlp2Rows * 40 + (size_t)H * 32 + (size_t)kMlp2Rows * (H + 8)) + 4 * (3 * (size_t)H) +
           4 * 2 * 4 * kMlp2Rows;
}

// VEC0: K0 % 8 == 0 and H * K0 * 2 a multiple of 1 KiB, so W0 moves by LDS-DMA as it lies in memory.
// NB: column blocks of 128 per wave pass (O <= 512 in one pass at cfg3).
// OS: the output as bf16 (outb) plus, per row and 32-column slice, the (sum, squared deviations from the slice
// mean) pair of the fp32 values into ostats[row][op0 + slice] (oP pairs per row): the producer side of an LN-folded
// consumer GEMM (rf_linear_lnfold_*), as gemm_lds_kernel's kEpiStats
// CW: layer-1 columns per wave block (128, or 64 with gridDim.y = 2 column halves: the W1 fragments then take 128
// instead of 256 VGPRs, so two workgroups share a CU and cover each other's load and barrier waits; the two halves
// recompute layer 0 and LN1 of their 16 rows, which is cheap)
template <int H, bool VEC0, bool OS = false, int CW = kMlp2Cols>
__global__ __launch_bounds__(256, CW == 64 ? 2 : 1) void mlp2_small_kernel(const float* __restrict__ x, int64_t M, int K0, int64_t ldx, float eps,
                                                            const float* __restrict__ g0, const float* __restrict__ be0,
                                                            const uint16_t* __restrict__ W0, const float* __restrict__ b0,
                                                            const float* __restrict__ g1, const float* __restrict__ be1,
                                                            const uint16_t* __restrict__ W1, const float* __restrict__ b1,
                                                            int O, int act, float* __restrict__ out, int64_t ldo,
                                                            uint16_t* __restrict__ outb, float* __restrict__ ostats, int oP,
                                                            int op0) {
    constexpr int RS0 = 32 + 8, RSH = H + 8;  // LDS row strides (elements) of the A tiles: 16-byte row pad
    constexpr int TW = H / 64;                // layer-0 column tiles per wave (H / 4 columns)
    constexpr int KS = H / 32;                // layer-1 k steps
    constexpr int NT = CW / 16;               // layer-1 column tiles per block
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    uint16_t* xs = reinterpret_cast<uint16_t*>(smem_raw);
    uint16_t* w0s = xs + kMlp2Rows * RS0;
    uint16_t* hs = w0s + H * 32;
    float* pb0 = reinterpret_cast<float*>(hs + kMlp2Rows * RSH);
    float* pg1 = pb0 + H;
    float* pbe1 = pg1 + H;
    float* red = pbe1 + H;  // [2][4 waves][16 rows]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int64_t r0 = (int64_t)blockIdx.x * kMlp2Rows;
    const int nblk = (O + CW - 1) / CW;
    // Issue order: wave 0's LN0 inputs, W0 and the per-column parameters by LDS-DMA, then this wave's first
    // layer-1 block of W1 fragments and bias into registers (16 B per lane per MFMA, from L2): everything is
    // in flight together and lands in about one memory latency (a wave stalls issuing past 63 outstanding
    // loads, so the oldest, wave 0's x, must go first).
    float xv[8], gv[8], bv[8];
    const int xr = lane >> 2, sub = lane & 3;
    if (wave == 0) {
        const int64_t row = r0 + xr < M ? r0 + xr : M - 1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 4 * j + sub < K0 ? 4 * j + sub : K0 - 1;  // clamped: no per-element branch
            xv[j] = x[row * ldx + k];
            gv[j] = g0[k];
            bv[j] = be0[k];
        }
    }
    if (VEC0) {  // W0 as it lies in memory
        const int ni0 = H * K0 * 2 / 1024;
        for (int g = wave; g < ni0; g += 4)
            __builtin_amdgcn_global_load_lds(W0 + g * 512 + lane * 8, (__attribute__((address_space(3))) void*)(w0s + g * 512), 16, 0, 0);
    } else {  // W0 [H][K0] -> LDS [H][32], k zero-padded
        for (int i = tid; i < H * 32; i += 256) {
            const int n = i >> 5, k = i & 31;
            w0s[n * 32 + k] = k < K0 ? W0[(int64_t)n * K0 + k] : (uint16_t)0;
        }
    }
    {  // per-column parameters by LDS-DMA (one dword per lane, lane-linear; NULL: 0 / 1 by plain LDS writes)
        auto dma4 = [&](const float* src, float* dst) {
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 4, 0, 0);
        };
        if (wave * 64 < H) {
            if (b0) dma4(b0 + tid, pb0 + wave * 64); else pb0[tid] = 0.f;
            if (g1) dma4(g1 + tid, pg1 + wave * 64); else pg1[tid] = 1.f;
            if (be1) dma4(be1 + tid, pbe1 + wave * 64); else pbe1[tid] = 0.f;
        }
    }
    const int cb0 = wave + 4 * (int)blockIdx.y;  // layer-1 column blocks cb0, cb0 + 4 gridDim.y, ...
    bf16x8 wf[NT][KS];
    float bb1[NT];
    auto load_w1 = [&](int cb) __attribute__((always_inline)) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int col = min(cb * CW + nt * 16 + lr, O - 1);  // columns past O: never stored
#pragma unroll
            for (int kk = 0; kk < KS; ++kk)
                wf[nt][kk] = *reinterpret_cast<const bf16x8*>(W1 + (int64_t)col * H + kk * 32 + lg * 8);
            bb1[nt] = b1 ? b1[col] : 0.f;
        }
    };
    if (cb0 < nblk) load_w1(cb0);
    if (wave == 0) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xv[j] = 4 * j + sub < K0 ? xv[j] : 0.f;
            s += xv[j];
        }
        s = lane_group_sum<4>(s);
        const float mu = s / (float)K0;
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = 4 * j + sub < K0 ? xv[j] - mu : 0.f;
            q += d * d;
        }
        q = lane_group_sum<4>(q);
        const float rstd = 1.0f / sqrtf(q / (float)K0 + eps);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 4 * j + sub;
            xs[xr * RS0 + k] = k < K0 ? (uint16_t)f32_to_bf16_bits((xv[j] - mu) * rstd * gv[j] + bv[j]) : (uint16_t)0;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's W0 / parameter pieces (and W1 fragments) landed
    __syncthreads();
    // ---- layer 0: the 16 rows x this wave's H / 4 columns ----
    const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(xs + lr * RS0 + lg * 8);
    float hv[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
        const int n = wave * (H / 4) + t * 16 + lr;
        bf16x8 bw;
        if (VEC0) {
            const bool live = lg * 8 < K0;  // k chunk lg exists; else its A lanes are zero and B must be too
            bw = *reinterpret_cast<const bf16x8*>(w0s + n * K0 + (live ? lg * 8 : 0));
            if (!live) bw = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        } else {
            bw = *reinterpret_cast<const bf16x8*>(w0s + n * 32 + lg * 8);
        }
        const f4 c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bw, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        const float bb = pb0[n];
#pragma unroll
        for (int r = 0; r < 4; ++r) hv[t][r] = c[r] + bb;
    }
    with_act(act, [&](auto A) {
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) hv[t][r] = A(hv[t][r]);
    });
    // ---- LN1: row partials of this wave's columns (C layout: row = 4 lg + r, column lr) meet in LDS ----
    float mu[4], rstd[4];
    {
        float ps[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float t0 = 0.f;
#pragma unroll
            for (int t = 0; t < TW; ++t) t0 += hv[t][r];
            ps[r] = row16_sum(t0);
        }
        if (lr == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) red[wave * kMlp2Rows + 4 * lg + r] = ps[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * lg + r;
            mu[r] = (((red[row] + red[kMlp2Rows + row]) + red[2 * kMlp2Rows + row]) + red[3 * kMlp2Rows + row]) / (float)H;
            float t0 = 0.f;
#pragma unroll
            for (int t = 0; t < TW; ++t) t0 += (hv[t][r] - mu[r]) * (hv[t][r] - mu[r]);
            ps[r] = row16_sum(t0);
        }
        float* red2 = red + 4 * kMlp2Rows;
        if (lr == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) red2[wave * kMlp2Rows + 4 * lg + r] = ps[r];
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * lg + r;
            const float q = ((red2[row] + red2[kMlp2Rows + row]) + red2[2 * kMlp2Rows + row]) + red2[3 * kMlp2Rows + row];
            rstd[r] = 1.0f / sqrtf(q / (float)H + eps);
        }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
        const int n = wave * (H / 4) + t * 16 + lr;
        const float gg = pg1[n], bb = pbe1[n];
#pragma unroll
        for (int r = 0; r < 4; ++r)
            hs[(4 * lg + r) * RSH + n] = (uint16_t)f32_to_bf16_bits((hv[t][r] - mu[r]) * rstd[r] * gg + bb);
    }
    __syncthreads();
    // ---- layer 1: the 16 rows x this wave's 128-column blocks ----
    bf16x8 ha[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) ha[kk] = *reinterpret_cast<const bf16x8*>(hs + lr * RSH + kk * 32 + lg * 8);
    const bool rows_full = r0 + kMlp2Rows <= M;
    for (int cb = cb0; cb < nblk; cb += 4 * (int)gridDim.y) {
        if (cb != cb0) {
            load_w1(cb);
        }
        f4 c[NT];
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            c[nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < KS; ++kk) c[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha[kk], wf[nt][kk], c[nt], 0, 0, 0);
        }
        with_act(act, [&](auto A) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) c[nt][r] = A(c[nt][r] + bb1[nt]);
        });
        // values first, stores after (see gemm_lds_kernel's epilogue)
        const int c0 = cb * CW;
        if constexpr (OS) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                if (c0 + nt * 16 + lr >= O) c[nt] = f4{0.f, 0.f, 0.f, 0.f};
            if (rows_full && c0 + CW <= O) {  // interior block: unguarded stores (see gemm_lds_kernel's epilogue)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    __bf16* yr = reinterpret_cast<__bf16*>(outb) + (r0 + 4 * lg + r) * ldo + c0 + lr;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) yr[nt * 16] = (__bf16)c[nt][r];
                }
            } else {
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int n = c0 + nt * 16 + lr;
                    if (n >= O) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int64_t row = r0 + 4 * lg + r;
                        if (row < M) reinterpret_cast<__bf16*>(outb)[row * ldo + n] = (__bf16)c[nt][r];
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < NT / 2; ++q) {
                const int cq = c0 + q * 32;
                const int nq = min(max(O - cq, 0), 32);
                if (nq == 0) continue;
                const float inv_n = 1.0f / (float)nq;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float sm = row16_sum(c[2 * q][r] + c[2 * q + 1][r]);
                    const float mq = sm * inv_n;
                    const float d0 = cq + lr < O ? c[2 * q][r] - mq : 0.f;
                    const float d1 = cq + 16 + lr < O ? c[2 * q + 1][r] - mq : 0.f;
                    const float m2 = row16_sum(d0 * d0 + d1 * d1);
                    const int64_t row = r0 + 4 * lg + r;
                    if (lr == 0 && row < M)
                        *reinterpret_cast<float2*>(ostats + 2 * (row * oP + op0 + cq / 32)) = make_float2(sm, m2);
                }
            }
            continue;
        }
        if (rows_full && c0 + CW <= O) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float* yr = out + (r0 + 4 * lg + r) * ldo + c0 + lr;
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) yr[nt * 16] = c[nt][r];
            }
        } else {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = c0 + nt * 16 + lr;
                if (n >= O) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t row = r0 + 4 * lg + r;
                    if (row < M) out[row * ldo + n] = c[nt][r];
                }
            }
        }
    }
}

}  // namespace

namespace {
// the mlp2 kernel for (H, VEC0, OS) at 64-column wave blocks, and its grid: two column halves once the output has
// more than four 64-column blocks (cfg3: O = 512 -> 512 workgroups, two per CU)
using Mlp2Kern = void (*)(const float*, int64_t, int, int64_t, float, const float*, const float*, const uint16_t*,
                          const float*, const float*, const float*, const uint16_t*, const float*, int, int, float*, int64_t,
                          uint16_t*, float*, int, int);
template <bool OS>
Mlp2Kern mlp2_pick(int H, bool vec0) {
    if (H == 256) return vec0 ? mlp2_small_kernel<256, true, OS, 64> : mlp2_small_kernel<256, false, OS, 64>;
    return vec0 ? mlp2_small_kernel<128, true, OS, 64> : mlp2_small_kernel<128, false, OS, 64>;
}
dim3 mlp2_grid(int64_t M, int O) {
    const int nblk = (O + 63) / 64;
    return dim3((unsigned)((M + kMlp2Rows - 1) / kMlp2Rows), nblk > 4 ? 2u : 1u);
}
}  // namespace

extern "C" int rf_mlp2_small_fwd(const float* x, int64_t M, int32_t K0, int64_t ldx, float eps, const float* ln0_gamma,
                                 const float* ln0_beta, const void* W0, const float* b0, int32_t H, const float* ln1_gamma,
                                 const float* ln1_beta, const void* W1, const float* b1, int32_t O, int32_t act, float* out,
                                 int64_t ldo, void* stream) {
    RF_REQUIRE(K0 >= 1 && K0 <= 32, "rf_mlp2_small_fwd: input width must be 1..32 (got %d)", K0);
    RF_REQUIRE(H == 128 || H == 256, "rf_mlp2_small_fwd: hidden width must be 128 or 256 (got %d)", H);
    RF_REQUIRE(O >= 1 && M >= 0 && ldx >= K0 && ldo >= O, "rf_mlp2_small_fwd: bad shape");
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_mlp2_small_fwd: activation must be elementwise");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && W0 && W1 && out && ln0_gamma && ln0_beta, "rf_mlp2_small_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)W1 & 15) == 0 && ((uintptr_t)W0 & 15) == 0, "rf_mlp2_small_fwd: W0 / W1 must be 16-byte aligned");
    const dim3 grid = mlp2_grid(M, O);
    hipStream_t st = rf_stream(stream);
    const bool vec0 = (K0 & 7) == 0 && (H * K0 * 2) % 1024 == 0;
    auto kern = mlp2_pick<false>(H, vec0);
    const size_t lds = H == 256 ? mlp2_lds_bytes<256>() : mlp2_lds_bytes<128>();
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "mlp2_small_kernel: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, x, M, K0, ldx, eps, ln0_gamma, ln0_beta, (const uint16_t*)W0, b0,
                       ln1_gamma, ln1_beta, (const uint16_t*)W1, b1, O, act, out, ldo, nullptr, nullptr, 0, 0);
    return rf_check_launch("mlp2_small_kernel");
}

extern "C" int rf_mlp2_small_stats_fwd(const float* x, int64_t M, int32_t K0, int64_t ldx, float eps, const float* ln0_gamma,
                                       const float* ln0_beta, const void* W0, const float* b0, int32_t H,
                                       const float* ln1_gamma, const float* ln1_beta, const void* W1, const float* b1,
                                       int32_t O, int32_t act, void* out_bf16, int64_t ldo, float* stats, int32_t stats_P,
                                       int32_t stats_p0, void* stream) {
    RF_REQUIRE(K0 >= 1 && K0 <= 32, "rf_mlp2_small_stats_fwd: input width must be 1..32 (got %d)", K0);
    RF_REQUIRE(H == 128 || H == 256, "rf_mlp2_small_stats_fwd: hidden width must be 128 or 256 (got %d)", H);
    RF_REQUIRE(O >= 1 && M >= 0 && ldx >= K0 && ldo >= O, "rf_mlp2_small_stats_fwd: bad shape");
    RF_REQUIRE(stats_p0 >= 0 && stats_P >= stats_p0 + (O + 31) / 32, "rf_mlp2_small_stats_fwd: stats slots out of range");
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_mlp2_small_stats_fwd: activation must be elementwise");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && W0 && W1 && out_bf16 && stats && ln0_gamma && ln0_beta, "rf_mlp2_small_stats_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)W1 & 15) == 0 && ((uintptr_t)W0 & 15) == 0, "rf_mlp2_small_stats_fwd: W0 / W1 must be 16-byte aligned");
    const dim3 grid = mlp2_grid(M, O);
    hipStream_t st = rf_stream(stream);
    const bool vec0 = (K0 & 7) == 0 && (H * K0 * 2) % 1024 == 0;
    auto kern = mlp2_pick<true>(H, vec0);
    const size_t lds = H == 256 ? mlp2_lds_bytes<256>() : mlp2_lds_bytes<128>();
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "mlp2_small_kernel: %s", hipGetErrorString(e));
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, x, M, K0, ldx, eps, ln0_gamma, ln0_beta, (const uint16_t*)W0, b0,
                       ln1_gamma, ln1_beta, (const uint16_t*)W1, b1, O, act, nullptr, ldo, (uint16_t*)out_bf16, stats,
                       stats_P, stats_p0);
    return rf_check_launch("mlp2_small_kernel (stats)");
}

extern "C" int rf_dense_head_fwd(const float* x, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t w_dtype,
                                 int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* stream) {
    RF_REQUIRE(w_dtype == RF_DTYPE_BF16 || w_dtype == RF_DTYPE_F32, "rf_dense_head_fwd: W dtype must be BF16 or F32");
    RF_REQUIRE(act >= RF_ACT_NONE && act <= RF_ACT_SOFTMAX, "rf_dense_head_fwd: unknown activation %d", act);
    RF_REQUIRE(M >= 0 && K > 0 && K % 4 == 0 && N >= 1 && N <= 64 && ldx >= K && ldx % 4 == 0 && ldy >= N,
               "rf_dense_head_fwd: need K %% 4 == 0, 1 <= N <= 64, ldx %% 4 == 0");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && W && y, "rf_dense_head_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)W & (w_dtype == RF_DTYPE_BF16 ? 7 : 15)) == 0,
               "rf_dense_head_fwd: x must be 16-byte and W 8/16-byte aligned");
    const unsigned grid = (unsigned)((M + 3) / 4);
    hipStream_t st = rf_stream(stream);
#define RF_HEAD(WB, NM) hipLaunchKernelGGL((dense_head_kernel<WB, NM>), dim3(grid), dim3(256), 0, st, x, M, K, ldx, W, N, b, act, y, ldy)
    const bool wb = w_dtype == RF_DTYPE_BF16;
    if (N <= 2) { if (wb) RF_HEAD(true, 2); else RF_HEAD(false, 2); }
    else if (N <= 16) { if (wb) RF_HEAD(true, 16); else RF_HEAD(false, 16); }
    else { if (wb) RF_HEAD(true, 64); else RF_HEAD(false, 64); }
#undef RF_HEAD
    return rf_check_launch("dense_head_kernel");
}

extern "C" int rf_norm_fwd(const float* x, int64_t rows, int32_t cols, int64_t ldx, int32_t mode, float eps,
                           const float* gamma, const float* beta, const float* mean, const float* var, void* y,
                           int32_t y_dtype, int64_t ldy, void* stream) {
    RF_REQUIRE(mode == 0 || mode == 1, "rf_norm_fwd: mode must be 0 (LayerNorm) or 1 (BatchNorm)");
    RF_REQUIRE(y_dtype == RF_DTYPE_BF16 || y_dtype == RF_DTYPE_F32, "rf_norm_fwd: y dtype must be BF16 or F32");
    RF_REQUIRE(rows >= 0 && cols > 0 && ldx >= cols && ldy >= cols, "rf_norm_fwd: bad shape");
    RF_REQUIRE(mode == 0 || (mean && var), "rf_norm_fwd: BatchNorm needs running mean/var");
    if (rows == 0) return RF_OK;
    RF_REQUIRE(x && y, "rf_norm_fwd: null pointer");
    const unsigned grid = (unsigned)((rows + 3) / 4);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool aligned = cols % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) &&
                         ((uintptr_t)y & (y_dtype == RF_DTYPE_BF16 ? 7 : 15)) == 0 && (!gamma || al16(gamma)) &&
                         (!beta || al16(beta)) && (mode == 0 || (al16(mean) && al16(var)));
    const bool bf = y_dtype == RF_DTYPE_BF16;
    if (aligned && mode == 1) {  // BatchNorm: per-column affine, any width
        const int64_t blocks = (int64_t)((cols / 4 + 255) / 256) * ((rows + kRowsPerBn - 1) / kRowsPerBn);
        RF_REQUIRE(blocks < ((int64_t)1 << 31), "rf_norm_fwd: too many rows");
        const dim3 g((unsigned)blocks);
        if (bf) hipLaunchKernelGGL(bn_vec_kernel<true>, g, dim3(256), 0, rf_stream(stream), x, rows, cols, ldx, eps, gamma, beta, mean, var, y, ldy);
        else hipLaunchKernelGGL(bn_vec_kernel<false>, g, dim3(256), 0, rf_stream(stream), x, rows, cols, ldx, eps, gamma, beta, mean, var, y, ldy);
        return rf_check_launch("bn_vec_kernel");
    }
    if (aligned && cols > 2048 && cols <= 32768) {  // LayerNorm, wide rows: a workgroup per row
        const int nv = (cols + 1023) / 1024;
        hipStream_t st = rf_stream(stream);
        const dim3 g((unsigned)rows);
#define RF_LN_WIDE(B, N) hipLaunchKernelGGL((ln_wide_kernel<B, N>), g, dim3(256), 0, st, x, cols, ldx, eps, gamma, beta, y, ldy)
        if (bf) {
            if (nv <= 4) RF_LN_WIDE(true, 4); else if (nv <= 8) RF_LN_WIDE(true, 8);
            else if (nv <= 16) RF_LN_WIDE(true, 16); else RF_LN_WIDE(true, 32);
        } else {
            if (nv <= 4) RF_LN_WIDE(false, 4); else if (nv <= 8) RF_LN_WIDE(false, 8);
            else if (nv <= 16) RF_LN_WIDE(false, 16); else RF_LN_WIDE(false, 32);
        }
#undef RF_LN_WIDE
        return rf_check_launch("ln_wide_kernel");
    }
    const bool vec = aligned && cols <= 2048;
    if (vec) {
        const int nv = (cols + 255) / 256;
        hipStream_t st = rf_stream(stream);
#define RF_NORM_VEC(B, N)                                                                                         \
    hipLaunchKernelGGL((norm_vec_kernel<B, N>), dim3(grid), dim3(256), 0, st, x, rows, cols, ldx, mode, eps, gamma, \
                       beta, mean, var, y, ldy)
        // exact register counts for the common widths (1280 = cfg3's pooled row: 5 float4 per lane)
        if (y_dtype == RF_DTYPE_BF16) {
            if (nv <= 1) RF_NORM_VEC(true, 1); else if (nv <= 2) RF_NORM_VEC(true, 2);
            else if (nv <= 4) RF_NORM_VEC(true, 4); else if (nv == 5) RF_NORM_VEC(true, 5);
            else if (nv == 6) RF_NORM_VEC(true, 6); else RF_NORM_VEC(true, 8);
        } else {
            if (nv <= 1) RF_NORM_VEC(false, 1); else if (nv <= 2) RF_NORM_VEC(false, 2);
            else if (nv <= 4) RF_NORM_VEC(false, 4); else if (nv == 5) RF_NORM_VEC(false, 5);
            else if (nv == 6) RF_NORM_VEC(false, 6); else RF_NORM_VEC(false, 8);
        }
#undef RF_NORM_VEC
        return rf_check_launch("norm_vec_kernel");
    }
    if (y_dtype == RF_DTYPE_BF16)
        hipLaunchKernelGGL(norm_kernel<true>, dim3(grid), dim3(256), 0, rf_stream(stream), x, rows, cols, ldx, mode,
                           eps, gamma, beta, mean, var, y, ldy);
    else
        hipLaunchKernelGGL(norm_kernel<false>, dim3(grid), dim3(256), 0, rf_stream(stream), x, rows, cols, ldx, mode,
                           eps, gamma, beta, mean, var, y, ldy);
    return rf_check_launch("norm_kernel");
}

namespace {
// grids of at most this many 64-row tiles take the 4-deep ring (RF_LDS_DEEP_TILES overrides it for A/B runs; 0 = never)
int64_t lds_deep_ring_tiles() {
    static const int64_t v = [] {
        const char* e = getenv("RF_LDS_DEEP_TILES");
        return e ? (int64_t)atoll(e) : (int64_t)256;
    }();
    return v;
}

// A/B only (default 0 = never): grids of at most this many 64-row tiles (and more than lds_deep_ring_tiles) take a
// 3-deep ring (72 KB: two workgroups per CU still fit)
int64_t lds_ring3_tiles() {
    static const int64_t v = [] {
        const char* e = getenv("RF_LDS_RING3_TILES");
        return e ? (int64_t)atoll(e) : (int64_t)0;
    }();
    return v;
}

// Launches gemm_lds_kernel<BM, EPI> with the tile choice of rf_linear_fwd's LDS path.
template <int EPI>
// one_per_cu: 64-row tiles on the 4-deep ring whatever the grid (99 KB of LDS: one workgroup per CU), which the
// in-kernel head hand-off needs (MI355X_MICROARCH's sc1 hand-off row: one workgroup per CU)
int launch_lds_epi(const void* x, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t N, const float* b, int32_t act,
                   float* y, int64_t ldy, const EpiArgs& ea, hipStream_t st, const char* who, bool one_per_cu = false) {
    const int64_t t128 = ((M + 127) / 128) * ((N + kLdsBN - 1) / kLdsBN);
    const bool big = t128 >= 512 && !one_per_cu;
    const int64_t tiles = big ? t128 : ((M + 63) / 64) * ((N + kLdsBN - 1) / kLdsBN);
    RF_REQUIRE(tiles < (int64_t)1 << 31, "%s: too many tiles", who);
    if (big) {
        auto kern = gemm_lds_kernel<128, EPI>;
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<128>());
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: %s", who, hipGetErrorString(e));
        hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), gemm_lds_bytes<128>(), st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, ea, 0);
    } else if (one_per_cu || tiles <= lds_deep_ring_tiles()) {
        // at most one 64-row tile per CU (cfg3's 4096 x 1024 -> 512 output layer): nothing shares the CU, so a
        // 4-deep ring keeps three k-steps of loads in flight behind the MFMAs
        auto kern = gemm_lds_kernel<64, EPI, false, false, 4>;
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<64, 4>());
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: %s", who, hipGetErrorString(e));
        constexpr size_t deep_lds = gemm_lds_bytes<64, 4>();
        hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), deep_lds, st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, ea, 0);
    } else if (tiles <= lds_ring3_tiles()) {
        auto kern = gemm_lds_kernel<64, EPI, false, false, 3>;
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<64, 3>());
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: %s", who, hipGetErrorString(e));
        constexpr size_t r3_lds = gemm_lds_bytes<64, 3>();
        hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), r3_lds, st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, ea, 0);
    } else {
        auto kern = gemm_lds_kernel<64, EPI>;
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<64>());
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: %s", who, hipGetErrorString(e));
        hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), gemm_lds_bytes<64>(), st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, ea, 0);
    }
    return rf_check_launch(who);
}
}  // namespace

extern "C" int rf_linear_stats_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t N, const float* b,
                                   int32_t act, void* y_bf16, int64_t ldy, float* row_stats, void* stream) {
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_linear_stats_fwd: activation must be elementwise");
    RF_REQUIRE(M >= 0 && N > 0 && K >= 512 && K % 64 == 0 && ldx >= K && ldx % 8 == 0 && ldy >= N,
               "rf_linear_stats_fwd: needs K >= 512, K %% 64 == 0, ldx %% 8 == 0");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && W && y_bf16 && row_stats, "rf_linear_stats_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0, "rf_linear_stats_fwd: x/W must be 16-byte aligned");
    hipStream_t st = rf_stream(stream);
    const int P = 4 * ((N + kLdsBN - 1) / kLdsBN);  // every slot of rows < M is written by the epilogue
    EpiArgs ea{};
    ea.yb = static_cast<uint16_t*>(y_bf16);
    ea.stats = row_stats;
    ea.P = P;
    return launch_lds_epi<kEpiStats>(x, M, K, ldx, W, N, b, act, nullptr, ldy, ea, st, "rf_linear_stats_fwd");
}

extern "C" int rf_linear_lnfold_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N,
                                    const float* s, const float* t, const float* row_stats, float eps, int32_t act,
                                    float* y, int64_t ldy, void* stream) {
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_linear_lnfold_fwd: activation must be elementwise");
    RF_REQUIRE(M >= 0 && N > 0 && K >= 512 && K % 64 == 0 && ldx >= K && ldx % 8 == 0 && ldy >= N,
               "rf_linear_lnfold_fwd: needs K >= 512, K %% 64 == 0, ldx %% 8 == 0");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && Wg && s && t && row_stats && y, "rf_linear_lnfold_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)Wg & 15) == 0, "rf_linear_lnfold_fwd: x/W must be 16-byte aligned");
    EpiArgs ea{};
    ea.stats = const_cast<float*>(row_stats);
    ea.fs = s;
    ea.ft = t;
    ea.eps = eps;
    ea.P = 4 * ((K + kLdsBN - 1) / kLdsBN);  // the stats call's N is this call's K
    return launch_lds_epi<kEpiLnFold>(x, M, K, ldx, Wg, N, nullptr, act, y, ldy, ea, rf_stream(stream), "rf_linear_lnfold_fwd");
}

extern "C" int rf_linear_lnfold_stats_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N,
                                          const float* s, const float* t, const float* row_stats, float eps, int32_t act,
                                          void* y_bf16, int64_t ldy, float* out_stats, void* stream) {
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_linear_lnfold_stats_fwd: activation must be elementwise");
    RF_REQUIRE(M >= 0 && N > 0 && K >= 512 && K % 64 == 0 && ldx >= K && ldx % 8 == 0 && ldy >= N,
               "rf_linear_lnfold_stats_fwd: needs K >= 512, K %% 64 == 0, ldx %% 8 == 0");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && Wg && s && t && row_stats && y_bf16 && out_stats, "rf_linear_lnfold_stats_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)Wg & 15) == 0, "rf_linear_lnfold_stats_fwd: x/W must be 16-byte aligned");
    EpiArgs ea{};
    ea.stats = const_cast<float*>(row_stats);
    ea.fs = s;
    ea.ft = t;
    ea.eps = eps;
    ea.P = 4 * ((K + kLdsBN - 1) / kLdsBN);
    ea.yb = static_cast<uint16_t*>(y_bf16);
    ea.ostats = out_stats;
    ea.oP = 4 * ((N + kLdsBN - 1) / kLdsBN);
    return launch_lds_epi<kEpiLnFoldStats>(x, M, K, ldx, Wg, N, nullptr, act, nullptr, ldy, ea, rf_stream(stream),
                                           "rf_linear_lnfold_stats_fwd");
}

// ws = one int32 counter per 64-row block at the START of ws (the LAST tile of a row block to finish runs the
// softmax; the counters must be zero before the first launch on this ws and every launch leaves them zero), and
// the per-tile partial logits [M][tiles][kHeadN] fp32 at the END of ws (256-byte aligned down). Counters at a
// fixed offset and partials at the far end keep one zeroed ws reusable across calls of any M with the same N:
// a smaller call's partials never land on a larger call's counters (ws_bytes >= counters(M) + partials(M))
namespace {
size_t head_part_bytes(int64_t M, int32_t N) {
    return (((size_t)std::max<int64_t>(M, 1) * ((N + kLdsBN - 1) / kLdsBN) * kHeadN * sizeof(float)) + 255) & ~(size_t)255;
}
}  // namespace
extern "C" size_t rf_linear_lnfold_head_ws_bytes(int64_t M, int32_t N) {
    // counters rounded up to 256 B so that the partials, aligned down from the end, never reach them
    return head_part_bytes(M, N) + ((((size_t)((std::max<int64_t>(M, 1) + 63) / 64) * sizeof(int32_t)) + 255) & ~(size_t)255);
}

extern "C" int rf_linear_lnfold_head_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N,
                                         const float* s, const float* t, const float* row_stats, float eps, int32_t act,
                                         float* y, int64_t ldy, const void* head_w, int32_t head_n, const float* head_b,
                                         int32_t head_act, float* out, int64_t ldo, void* ws, size_t ws_bytes,
                                         void* stream) {
    RF_REQUIRE(act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX, "rf_linear_lnfold_head_fwd: activation must be elementwise");
    RF_REQUIRE(head_n == kHeadN, "rf_linear_lnfold_head_fwd: the head must have %d outputs (got %d)", kHeadN, head_n);
    RF_REQUIRE(head_act >= RF_ACT_NONE && head_act <= RF_ACT_SOFTMAX, "rf_linear_lnfold_head_fwd: unknown head activation");
    RF_REQUIRE(M >= 0 && N > 0 && K >= 512 && K % 64 == 0 && ldx >= K && ldx % 8 == 0 && (!y || ldy >= N) && ldo >= head_n,
               "rf_linear_lnfold_head_fwd: needs K >= 512, K %% 64 == 0, ldx %% 8 == 0");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && Wg && s && t && row_stats && head_w && out && ws, "rf_linear_lnfold_head_fwd: null pointer");
    RF_REQUIRE(ws_bytes >= rf_linear_lnfold_head_ws_bytes(M, N), "rf_linear_lnfold_head_fwd: workspace too small");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)Wg & 15) == 0, "rf_linear_lnfold_head_fwd: x/W must be 16-byte aligned");
    EpiArgs ea{};
    ea.stats = const_cast<float*>(row_stats);
    ea.fs = s;
    ea.ft = t;
    ea.eps = eps;
    ea.P = 4 * ((K + kLdsBN - 1) / kLdsBN);
    ea.hw = static_cast<const uint16_t*>(head_w);
    const size_t part_off = (ws_bytes - head_part_bytes(M, N)) & ~(size_t)255;
    ea.hpart = reinterpret_cast<float*>(static_cast<char*>(ws) + part_off);
    ea.hb = head_b;
    ea.hact = head_act;
    ea.hout = out;
    ea.hldo = ldo;
    hipStream_t st = rf_stream(stream);
    // the in-kernel finish needs 64-row tiles (one counter per 64 rows) and is the default; RF_HEAD_SEPARATE=1 runs
    // the softmax as its own launch (A/B)
    static const bool separate = [] {
        const char* e = getenv("RF_HEAD_SEPARATE");
        return e && e[0] == '1';
    }();
    const int64_t t128 = ((M + 127) / 128) * ((N + kLdsBN - 1) / kLdsBN);
    const bool fused = !separate && t128 < 512;  // launch_lds_epi's choice: 64-row tiles below 512 128-row tiles
    ea.hcnt = fused ? static_cast<int*>(ws) : nullptr;
    const int rc = launch_lds_epi<kEpiLnFoldHead>(x, M, K, ldx, Wg, N, nullptr, act, y, ldy, ea, st, "rf_linear_lnfold_head_fwd",
                                                  fused);
    if (rc != RF_OK || fused) return rc;
    hipLaunchKernelGGL(head_softmax_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st, (const float*)ea.hpart,
                       (N + kLdsBN - 1) / kLdsBN, M, head_b, head_act, out, ldo);
    return rf_check_launch("head_softmax_kernel");
}

extern "C" int rf_linear_fwd(const void* x, int32_t x_dtype, int64_t M, int32_t K, int64_t ldx, const void* W,
                             int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* stream);

namespace {
// y = act(sum_s part[s] + b), partials added in order s = 0 .. S-1 (fixed: replay-deterministic), float4 columns
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int64_t M, int N,
                                                            const float* __restrict__ bias, int act,
                                                            float* __restrict__ y, int64_t ldy) {
    const int n4 = N / 4;
    const int64_t total = M * n4;
    const int64_t plane = M * (int64_t)N;
    with_act(act, [&](auto A) {
        for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
            const int64_t m = e / n4;
            const int c = (int)(e - m * n4) * 4;
            float4 a = *reinterpret_cast<const float4*>(part + m * N + c);
            for (int s2 = 1; s2 < S; ++s2) {
                const float4 v = *reinterpret_cast<const float4*>(part + s2 * plane + m * N + c);
                a.x += v.x;
                a.y += v.y;
                a.z += v.z;
                a.w += v.w;
            }
            const float4 bv = bias ? *reinterpret_cast<const float4*>(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            float* d = y + m * ldy + c;
            d[0] = A(a.x + bv.x);
            d[1] = A(a.y + bv.y);
            d[2] = A(a.z + bv.z);
            d[3] = A(a.w + bv.w);
        }
    });
}

// split count for the fp32 GEMM: 128-tiles filling at most one workgroup per CU and a deep K get S splits so
// two workgroups share each CU (their MFMAs cover each other's load waits). RF_SPLITK=<S> overrides (A/B only).
int splitk_count(int32_t x_dtype, int64_t M, int32_t K, int32_t N) {
    if (x_dtype != RF_DTYPE_F32 || N % 4 != 0 || N <= 16) return 1;
    const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
    static const int force = [] {
        const char* e = getenv("RF_SPLITK");
        return e ? atoi(e) : 0;
    }();
    if (force > 0) return K >= 64 * force ? std::min(force, 8) : 1;
    if (tiles > 256 || K < 2048) return 1;
    int S = 2;
    while (S < 8 && tiles * S * 2 <= 512 && K / (S * 2) >= 1024) S *= 2;
    return S;
}

// the fp32 operand form of the LDS-DMA ring kernel (K % 32 == 0)
template <int BM, bool SPLIT>
int launch_lds_f32(const void* x, const void* W, const float* b, float* y, int64_t M, int N, int K, int64_t ldx,
                   int64_t ldy, int act, int S, int kspan, hipStream_t st) {
    auto kern = gemm_lds_kernel<BM, kEpiPlain, true, SPLIT>;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)gemm_lds_bytes<BM>());
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "gemm_lds_kernel: %s", hipGetErrorString(e));
    const int64_t tiles = ((M + BM - 1) / BM) * ((N + kLdsBN - 1) / kLdsBN);
    RF_REQUIRE(tiles < (int64_t)1 << 31, "rf_linear_fwd: too many tiles");
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles, (unsigned)S), dim3(256), gemm_lds_bytes<BM>(), st, x, W, b, y, M, N, K,
                       ldx, ldy, act, EpiArgs{}, kspan);
    return rf_check_launch("gemm_lds_kernel (fp32)");
}

// rf_ip_candidates_f32: the compaction form of the fp32 LDS-DMA GEMM (gemm_lds_kernel<128, kEpiCompact, F32>)
template <bool F32>
int launch_ip_candidates(const void* q, int64_t ldq, int64_t M, const void* items, int N, int K, const EpiArgs& ea,
                         hipStream_t st) {
    auto kern = gemm_lds_kernel<128, kEpiCompact, F32>;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)gemm_lds_bytes<128>());
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "gemm_lds_kernel (compact): %s", hipGetErrorString(e));
    const int64_t tiles = ((M + 127) / 128) * ((N + kLdsBN - 1) / kLdsBN);
    RF_REQUIRE(tiles < (int64_t)1 << 31, "rf_ip_candidates: too many tiles");
    hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), gemm_lds_bytes<128>(), st, q, items, nullptr, nullptr, M, N,
                       K, ldq, (int64_t)0, RF_ACT_NONE, ea, 0);
    return rf_check_launch("gemm_lds_kernel (compact)");
}

// ---------------------------------------------------------------------------------------------
// Query-stationary bf16 screen (rf_ip_candidates_bf16 at K = 64 / 128 / 256): the kEpiCompact test of
// gemm_lds_kernel<128, kEpiCompact, bf16> without its per-tile operand traffic. At the cascade's shapes (1024
// queries x ~1M items x 256) the 128 x 128 tile GEMM re-reads a 64 KB query panel for every 8.4 MFLOP tile and
// drains its 4-step ring at every tile: 14 % of the bf16 peak (1.29 ms). Here
//   * a workgroup owns 256 query rows (wave w: rows 64 w .. 64 w + 63) and a contiguous range of 64-item tiles;
//     each wave keeps its 64 rows x K in registers for the whole launch (A fragments, 16 K / 4 VGPRs per 16 rows);
//   * the item tiles stream through a 3-deep LDS-DMA ring (global_load_lds_dwordx4, 16-byte chunk c of row r stored
//     at chunk c ^ (r & 7): conflict-free ds_read_b128 B fragments), tile t + 2 issued when tile t opens;
//   * per tile and wave 16 accumulator tiles x K / 32 v_mfma_f32_16x16x32_bf16, then the pass test
//     y >= thr[row] - qbound[row] * vnorm[col] (kEpiCompact's) on all 64 values; one wave vote skips the tile when
//     nothing passes. At the cascade's pass rate (~0.06 %) most wave tiles (4096 pairs) still hold one or two
//     passing pairs, and an atomic round trip per tile at one wave per SIMD doubled the launch: passing pairs are
//     appended to the wave's LDS list instead (a ballot and a lane rank per slot) and the list is flushed to the
//     rows' candidate lists (one atomic add per pair on its row's counter; counts past cap are kept: the caller's
//     overflow test) when half full and at the end;
//   * block b runs on XCD b % 8: the query blocks of one item range are b, b + 8, ..., so they share that XCD's L2
//     and the items come from HBM about once.
// One workgroup per CU (the A fragments and accumulators take ~300 registers at one wave per SIMD).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lds_u32(const void* p) {  // the LDS byte address of a generic pointer into LDS
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

constexpr int kScrTN = 64, kScrStages = 3, kScrQ = 256;  // items per tile, ring depth, query rows per workgroup
constexpr int kScrList = 1024;                            // passing pairs listed per wave before a flush
// lab ablations (tools/build_variants.sh -DRF_LAB_SCR=bits; wrong results, never in the shipped build): 1 = no pass
// test / list, 2 = no MFMAs, 4 = no item copies or waits (stale LDS), 8 = the row pre-filter without the list,
// 16 = the list never flushed
#ifndef RF_LAB_SCR
#define RF_LAB_SCR 0
#endif

template <int KT>
__global__ __launch_bounds__(256) void ip_screen_bf16_kernel(const uint16_t* __restrict__ q, int64_t ldq, int M,
                                                             const uint16_t* __restrict__ items, int N, EpiArgs ea) {
    constexpr int KB = KT * 64;           // bytes per item row (K = 32 KT bf16)
    constexpr int CPR = KB / 16;          // 16-byte chunks per row
    constexpr int RPI = 1024 / KB;        // rows per 1 KiB DMA wave-instruction
    constexpr int STAGE = kScrTN * KB + 1024;  // bytes per ring stage: the items, then each wave's copy of their norms
    constexpr int DMA = kScrTN / RPI / 4; // DMA instructions per wave and stage (= KT)
    static_assert(CPR >= 8 && RPI * CPR == 64, "K = 64, 128 or 256");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int QB = (M + kScrQ - 1) / kScrQ;
    const int b = blockIdx.x, qb = (b / 8) % QB, c = (b % 8) + 8 * (b / (8 * QB));
    const int nch = gridDim.x / QB;
    const int64_t T = (N + kScrTN - 1) / kScrTN;
    const int t0 = (int)(T * c / nch), t1 = (int)(T * (c + 1) / nch);
    if (t0 >= t1) return;  // workgroup-uniform
    const int nt = t1 - t0;
    auto dma = [&](int t, int s) __attribute__((always_inline)) {
        char* dst = smem_raw + s * STAGE;
        const int64_t n0 = (int64_t)t * kScrTN;
#pragma unroll
        for (int it = 0; it < DMA; ++it) {
            const int g = wave + 4 * it, r = g * RPI + lane / CPR, p = lane % CPR;
            const int64_t item = n0 + r < N ? n0 + r : N - 1;  // rows past N: any valid row (never passes)
            const char* src = reinterpret_cast<const char*>(items) + item * KB + ((p ^ (r & 7)) << 4);
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(dst + g * 1024), 16, 0, 0);
        }
        // the tile's item norms by LDS-DMA as well (one copy per wave, so each wave's own vmcnt covers its copy): an
        // ordinary global load used while a DMA is in flight makes hipcc drain every DMA (vmcnt(0)) at that use
        const float* vsrc = ea.vnorm + (n0 + lane < N ? n0 + lane : N - 1);
        __builtin_amdgcn_global_load_lds(vsrc, (__attribute__((address_space(3))) void*)(dst + kScrTN * KB + wave * 256), 4, 0, 0);
    };
    dma(t0, 0);
    if (nt > 1) dma(t0 + 1, 1);
    // this wave's query rows: A fragments (row qrow0 + 16 i + lr, k = 32 kt + 8 lg ..) and the rows' thresholds
    const int64_t qrow0 = (int64_t)qb * kScrQ + wave * 64;
    bf16x8 a[4][KT];
    float tv[4][4], qv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t row = qrow0 + 16 * i + lr;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
            a[i][kt] = row < M ? *reinterpret_cast<const bf16x8*>(q + row * ldq + 32 * kt + 8 * lg) : bf16x8{};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t rr = qrow0 + 16 * i + 4 * lg + r;
            tv[i][r] = rr < M ? ea.thr[rr] : INFINITY;
            qv[i][r] = rr < M ? ea.qbound[rr] : 0.f;
        }
    }
    // retire these loads here and hand their registers on through empty asm: a use inside the loop of a load result
    // still pending at loop entry gets a vmcnt(0) in the loop body (every tile, draining the DMAs in flight)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) asm volatile("" : "+v"(a[i][kt]));
#pragma unroll
        for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(tv[i][r]), "+v"(qv[i][r]));
    }
    // this wave's list of passing pairs (score, column, row in the wave's 64) past the ring
    char* lbase = smem_raw + kScrStages * STAGE + wave * kScrList * 9;
    float* lv = reinterpret_cast<float*>(lbase);
    uint32_t* lc = reinterpret_cast<uint32_t*>(lbase + kScrList * 4);
    uint8_t* lrw = reinterpret_cast<uint8_t*>(lbase + kScrList * 8);
    int nb = 0;  // wave-uniform
    auto emit = [&](int rl, float v, int64_t col) __attribute__((always_inline)) {
        const int64_t row = qrow0 + rl;
        const int off = atomicAdd(ea.ccount + row, 1);
        if (off < ea.cap) {
            ea.cval[row * (int64_t)ea.cap + off] = v;
            ea.cidx[row * (int64_t)ea.cap + off] = (uint32_t)(ea.cbase + col);
        }
    };
    auto flush = [&]() __attribute__((always_inline)) {
        if (RF_LAB_SCR & 16) {  // lab: the list is dropped
            nb = 0;
            return;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the list writes of every lane (DS ops retire in order)
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < nb; e += 64) emit(lrw[e], lv[e], lc[e]);
        __builtin_amdgcn_wave_barrier();
        nb = 0;
    };
    for (int u = 0; u < nt; ++u) {
        const int t = t0 + u;
        const int64_t n0 = (int64_t)t * kScrTN;
        // tile t landed (vmcnt retires in issue order: tile t + 1's copies may stay in flight)
        if (RF_LAB_SCR & 4) {
        } else if (u + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA + 1) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's part of tile t is in; every wave is done with tile t - 1
        __builtin_amdgcn_sched_barrier(0);
        if (u + 2 < nt && !(RF_LAB_SCR & 4)) dma(t + 2, (u + 2) % kScrStages);
        // The tile's LDS reads are inline asm: hipcc cannot tell them from reads of the stage being DMA'd and would
        // put a vmcnt(0) (drain tile t + 2's copies, just issued) in front of the first use of each; their lgkmcnt
        // waits are explicit, and an empty asm on each fragment orders its use after its wait
        const uint32_t bsl = lds_u32(smem_raw + (u % kScrStages) * STAGE);
        float vv[4];  // the item norms of this lane's columns
#pragma unroll
        for (int j = 0; j < 4; ++j)
            asm volatile("ds_read_b32 %0, %1" : "=v"(vv[j]) : "v"(bsl + kScrTN * KB + wave * 256 + (16 * j + lr) * 4));
        bf16x8 bfr[2][KT];
        auto read_b = [&](int j, bf16x8(&f)[KT]) __attribute__((always_inline)) {
#pragma unroll
            for (int kt = 0; kt < KT; ++kt)
                asm volatile("ds_read_b128 %0, %1"
                             : "=v"(f[kt])
                             : "v"(bsl + (16 * j + lr) * KB + (((4 * kt + lg) ^ (lr & 7)) << 4)));
        };
        read_b(0, bfr[0]);
        f4 acc[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j < 3) {
                read_b(j + 1, bfr[(j + 1) & 1]);  // in flight under this column block's MFMAs
                asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(KT));
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)");
            }
#pragma unroll
            for (int kt = 0; kt < KT; ++kt) asm volatile("" : "+v"(bfr[j & 1][kt]));
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
                if (RF_LAB_SCR & 2) {
                    acc[i][j] = f4{(float)bfr[j & 1][i % KT][0], (float)bfr[j & 1][(i + 1) % KT][1], (float)a[i][0][0],
                                   (float)bfr[j & 1][j % KT][2]};
                } else {
#pragma unroll
                    for (int kt = 0; kt < KT; ++kt)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kt], bfr[j & 1][kt], acc[i][j], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(vv[j]));  // read before the last wait above
        // C/D layout: column n0 + 16 j + lr, row qrow0 + 16 i + 4 lg + r. A row pre-filter first: the largest of the
        // lane's four scores of a row against the row's bar at the lane's largest item norm (qbound >= 0, so no pair
        // that passes is missed; columns past N are excluded by the exact test only)
        const float vmax = fmaxf(fmaxf(vv[0], vv[1]), fmaxf(vv[2], vv[3]));
        uint32_t pm = 0;  // bit 4 i + r: row (i, r) may hold a passing pair in this lane's columns
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float m = fmaxf(fmaxf(acc[i][0][r], acc[i][1][r]), fmaxf(acc[i][2][r], acc[i][3][r]));
                pm |= m >= tv[i][r] - qv[i][r] * vmax ? 1u << (4 * i + r) : 0u;
            }
        if (RF_LAB_SCR & 1) {
            float z = 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) z += acc[i][j][0] + acc[i][j][3];
            pm = z == 12345.f;
        }
        // most wave tiles hold a pair or two that pass: they go to the wave's LDS list (a ballot and a lane rank per
        // passing slot, no global round trip here); the list is flushed to the rows' candidate lists when half full
        if (RF_LAB_SCR & 8) {
            if (__any(pm != 0u)) asm volatile("" ::"v"(pm));  // keeps the pre-filter; nb (the list) stays empty
        } else if (__any(pm != 0u)) {
            if (nb > kScrList / 2) flush();
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (!__any((pm >> (4 * i + r)) & 1u)) continue;  // wave-uniform: most rows of a tile
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const bool p = n0 + 16 * j + lr < N && acc[i][j][r] >= tv[i][r] - qv[i][r] * vv[j];
                        const uint64_t bm = __ballot(p);
                        if (bm) {
                            if (p) {
                                const int pos = nb + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
                                if (pos < kScrList) {  // (asm: see the tile reads)
                                    asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %2, %3\n\tds_write_b8 %4, %5"
                                                 :
                                                 : "v"(lds_u32(lv + pos)), "v"(acc[i][j][r]), "v"(lds_u32(lc + pos)),
                                                   "v"((uint32_t)(n0 + 16 * j + lr)), "v"(lds_u32(lrw + pos)),
                                                   "v"((uint32_t)(16 * i + 4 * lg + r))
                                                 : "memory");
                                } else {  // a tile with more passing pairs than the list holds: straight to the rows
                                    emit(16 * i + 4 * lg + r, acc[i][j][r], n0 + 16 * j + lr);
                                }
                            }
                            nb = min(nb + __popcll(bm), kScrList);
                        }
                    }
                }
        }
    }
    flush();
}

template <int KT>
int launch_ip_screen_bf16(const void* q, int64_t ldq, int M, const void* items, int N, const EpiArgs& ea, hipStream_t st) {
    auto kern = ip_screen_bf16_kernel<KT>;
    constexpr int lds = kScrStages * (kScrTN * KT * 64 + 1024) + 4 * kScrList * 9;
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "ip_screen_bf16_kernel: %s", hipGetErrorString(e));
    const int QB = (M + kScrQ - 1) / kScrQ;
    const int C8 = std::max(1, 256 / (8 * QB));  // item ranges per XCD: about one workgroup per CU in all
    const int64_t grid = 8LL * QB * C8;
    RF_REQUIRE(grid < (int64_t)1 << 31, "rf_ip_candidates_bf16: too many query rows");
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, st, (const uint16_t*)q, ldq, M, (const uint16_t*)items, N, ea);
    return rf_check_launch("ip_screen_bf16_kernel");
}

bool screen_gemm_forced() {  // RF_SCREEN_GEMM=1: the bf16 screen on gemm_lds_kernel<128, kEpiCompact> (A/B only)
    static const bool on = [] {
        const char* e = getenv("RF_SCREEN_GEMM");
        return e && e[0] == '1';
    }();
    return on;
}

bool lds_disabled() {  // RF_GEMM_LDS=0: the register-staged kernel everywhere (A/B measurement only)
    static const bool off = [] {
        const char* e = getenv("RF_GEMM_LDS");
        return e && e[0] == '0';
    }();
    return off;
}
}  // namespace

extern "C" size_t rf_linear_splitk_ws_bytes(int32_t x_dtype, int64_t M, int32_t K, int32_t N) {
    const int S = splitk_count(x_dtype, M, K, N);
    return S > 1 ? (size_t)S * (size_t)M * (size_t)N * sizeof(float) : 0;
}

extern "C" int rf_linear_splitk_fwd(const void* x, int32_t x_dtype, int64_t M, int32_t K, int64_t ldx, const void* W,
                                    int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* ws,
                                    size_t ws_bytes, void* stream) {
    const int S = splitk_count(x_dtype, M, K, N);
    if (S == 1 || !ws || ws_bytes < rf_linear_splitk_ws_bytes(x_dtype, M, K, N) || act == RF_ACT_SOFTMAX)
        return rf_linear_fwd(x, x_dtype, M, K, ldx, W, N, b, act, y, ldy, stream);
    RF_REQUIRE(M > 0 && K % 4 == 0 && ldx % 4 == 0 && ldx >= K && ldy >= N && x && W && y, "rf_linear_splitk_fwd: bad shape");
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0 && ((uintptr_t)ws & 15) == 0 && ((uintptr_t)y & 3) == 0,
               "rf_linear_splitk_fwd: alignment");
    RF_REQUIRE(!b || ((uintptr_t)b & 15) == 0, "rf_linear_splitk_fwd: bias must be 16-byte aligned");
    hipStream_t st = rf_stream(stream);
    const int kspan = ((K + S - 1) / S + BKF - 1) / BKF * BKF;
    const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
    const dim3 g((unsigned)tiles, (unsigned)S);
    const bool ktail = K % BKF != 0 || kspan % BKF != 0;
    if (!ktail && !lds_disabled()) {
        const int rc = launch_lds_f32<128, true>(x, W, nullptr, (float*)ws, M, N, K, ldx, (int64_t)N, RF_ACT_NONE, S, kspan, st);
        if (rc != RF_OK) return rc;
    } else if (ktail)
        hipLaunchKernelGGL((gemm_kernel<false, 128, true, true>), g, dim3(256), 0, st, x, W, nullptr, (float*)ws, M, N, K,
                           ldx, (int64_t)N, RF_ACT_NONE, kspan);
    else
        hipLaunchKernelGGL((gemm_kernel<false, 128, false, true>), g, dim3(256), 0, st, x, W, nullptr, (float*)ws, M, N, K,
                           ldx, (int64_t)N, RF_ACT_NONE, kspan);
    if (rf_check_launch("gemm_kernel (split-K)") != RF_OK) return RF_EHIP;
    const int64_t total = M * (N / 4);
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, st, (const float*)ws, S, M, N, b, act, y, ldy);
    return rf_check_launch("splitk_reduce_kernel");
}

extern "C" int rf_ip_candidates_f32(const float* q, int64_t ldq, int32_t M, const float* items, int32_t N, int32_t K,
                                    const float* thr, int32_t cap, int32_t* count, float* cand_val, uint32_t* cand_idx,
                                    int64_t col_base, void* stream) {
    RF_REQUIRE(M >= 0 && N >= 0 && K >= 256 && K % 32 == 0 && ldq >= K && ldq % 4 == 0 && cap >= 1,
               "rf_ip_candidates_f32: needs K >= 256, K %% 32 == 0, ldq %% 4 == 0, cap >= 1");
    RF_REQUIRE(col_base >= 0 && col_base + N <= ((int64_t)1 << 32) - 1, "rf_ip_candidates_f32: item index must fit 32 bits");
    if (M == 0 || N == 0) return RF_OK;
    RF_REQUIRE(q && items && thr && count && cand_val && cand_idx, "rf_ip_candidates_f32: null pointer");
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)items & 15) == 0, "rf_ip_candidates_f32: q / items must be 16-byte aligned");
    EpiArgs ea{};
    ea.thr = thr;
    ea.ccount = count;
    ea.cval = cand_val;
    ea.cidx = cand_idx;
    ea.cap = cap;
    ea.cbase = col_base;
    return launch_ip_candidates<true>(q, ldq, M, items, N, K, ea, rf_stream(stream));
}

extern "C" int rf_ip_candidates_bf16(const void* q, int64_t ldq, int32_t M, const void* items, int32_t N, int32_t K,
                                     const float* thr, const float* qbound, const float* vnorm, int32_t cap, int32_t* count,
                                     float* cand_val, uint32_t* cand_idx, int64_t col_base, void* stream) {
    RF_REQUIRE(M >= 0 && N >= 0 && K >= 64 && K % 64 == 0 && ldq >= K && ldq % 8 == 0 && cap >= 1,
               "rf_ip_candidates_bf16: needs K %% 64 == 0, ldq %% 8 == 0, cap >= 1");
    RF_REQUIRE(col_base >= 0 && col_base + N <= ((int64_t)1 << 32) - 1, "rf_ip_candidates_bf16: item index must fit 32 bits");
    if (M == 0 || N == 0) return RF_OK;
    RF_REQUIRE(q && items && thr && qbound && vnorm && count && cand_val && cand_idx, "rf_ip_candidates_bf16: null pointer");
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)items & 15) == 0, "rf_ip_candidates_bf16: q / items must be 16-byte aligned");
    EpiArgs ea{};
    ea.thr = thr;
    ea.qbound = qbound;
    ea.vnorm = vnorm;
    ea.ccount = count;
    ea.cval = cand_val;
    ea.cidx = cand_idx;
    ea.cap = cap;
    ea.cbase = col_base;
    if (!screen_gemm_forced()) {
        if (K == 256) return launch_ip_screen_bf16<8>(q, ldq, M, items, N, ea, rf_stream(stream));
        if (K == 128) return launch_ip_screen_bf16<4>(q, ldq, M, items, N, ea, rf_stream(stream));
        if (K == 64) return launch_ip_screen_bf16<2>(q, ldq, M, items, N, ea, rf_stream(stream));
    }
    return launch_ip_candidates<false>(q, ldq, M, items, N, K, ea, rf_stream(stream));
}

extern "C" int rf_linear_fwd(const void* x, int32_t x_dtype, int64_t M, int32_t K, int64_t ldx, const void* W,
                             int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* stream) {
    RF_REQUIRE(x_dtype == RF_DTYPE_BF16 || x_dtype == RF_DTYPE_F32, "rf_linear_fwd: x dtype must be BF16 or F32");
    RF_REQUIRE(act >= RF_ACT_NONE && act <= RF_ACT_SOFTMAX, "rf_linear_fwd: unknown activation %d", act);
    RF_REQUIRE(M >= 0 && K > 0 && N > 0 && ldx >= K && ldy >= N, "rf_linear_fwd: bad shape");
    RF_REQUIRE(act != RF_ACT_SOFTMAX || N <= 64, "rf_linear_fwd: softmax head needs N <= 64");
    const int epc = x_dtype == RF_DTYPE_BF16 ? 8 : 4;
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && W && y, "rf_linear_fwd: null pointer");
    hipStream_t st = rf_stream(stream);
    const bool bf = x_dtype == RF_DTYPE_BF16;
    if (N <= 16 || act == RF_ACT_SOFTMAX) {
        const unsigned grid = (unsigned)((M + 3) / 4);
        if (bf)
            hipLaunchKernelGGL(small_n_kernel<true>, dim3(grid), dim3(256), 0, st, x, W, b, y, M, N, K, ldx, ldy, act);
        else
            hipLaunchKernelGGL(small_n_kernel<false>, dim3(grid), dim3(256), 0, st, x, W, b, y, M, N, K, ldx, ldy, act);
        return rf_check_launch("small_n_kernel");
    }
    RF_REQUIRE(K % epc == 0 && ldx % epc == 0, "rf_linear_fwd: K and ldx must be multiples of %d (16-byte rows)", epc);
    RF_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)W & 15) == 0, "rf_linear_fwd: x/W must be 16-byte aligned");
    // 128-tiles unless that grid would give fewer than 2 workgroups per CU (256 CUs): then 64-tiles
    // (4x the workgroups; same per-element accumulation order, so identical results)
    const bool lds_off = lds_disabled();
    // fp32 operands on the LDS-DMA ring (K % 32 == 0): 128-row tiles from one per CU, else 64-row tiles
    if (!bf && !lds_off && K % 32 == 0 && K >= 256 && ((uintptr_t)y & 3) == 0) {
        const int64_t t128 = ((M + 127) / 128) * ((N + kLdsBN - 1) / kLdsBN);
        if (t128 >= 256) return launch_lds_f32<128, false>(x, W, b, y, M, N, K, ldx, ldy, act, 1, 0, st);
        return launch_lds_f32<64, false>(x, W, b, y, M, N, K, ldx, ldy, act, 1, 0, st);
    }
    // the LDS-DMA kernel where it measured faster (profiles/r02/gemm_ab.txt): deep K, at most ~4 tiles of
    // 64 x 128 per CU (its per-CU load path is the limit on long grids; short K is all pipeline fill)
    const int64_t t64 = ((M + 63) / 64) * ((N + kLdsBN - 1) / kLdsBN);
    if (bf && !lds_off && K % kLdsK == 0 && K >= 512 && t64 <= 1024) {
        const int64_t t128 = ((M + 127) / 128) * ((N + kLdsBN - 1) / kLdsBN);
        static const int force_bm = [] {  // A/B of the row tile (measurement only): RF_GEMM_BM=64|128
            const char* e = getenv("RF_GEMM_BM");
            return e ? atoi(e) : 0;
        }();
        // 128-row tiles when they give two per CU (one 98 KiB workgroup per CU), else 64-row tiles: two
        // 74 KiB workgroups share a CU
        const bool big = force_bm ? force_bm == 128 : t128 >= 512;
        const int64_t tiles = big ? t128 : ((M + 63) / 64) * ((N + kLdsBN - 1) / kLdsBN);
        RF_REQUIRE(tiles < (int64_t)1 << 31, "rf_linear_fwd: too many tiles");
        if (big) {
            auto kern = gemm_lds_kernel<128>;
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<128>());
            if (e != hipSuccess) return rf_set_error(RF_EHIP, "gemm_lds_kernel: %s", hipGetErrorString(e));
            hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), gemm_lds_bytes<128>(), st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, EpiArgs{}, 0);
        } else {
            auto kern = gemm_lds_kernel<64>;
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)gemm_lds_bytes<64>());
            if (e != hipSuccess) return rf_set_error(RF_EHIP, "gemm_lds_kernel: %s", hipGetErrorString(e));
            hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(256), gemm_lds_bytes<64>(), st, (const uint16_t*)x, (const uint16_t*)W, b, y, M, N, K, ldx, ldy, act, EpiArgs{}, 0);
        }
        return rf_check_launch("gemm_lds_kernel");
    }
    const int64_t tiles128 = ((M + 127) / 128) * ((N + 127) / 128);
    static const int force_bt = [] {  // A/B of the tile choice (measurement only): RF_GEMM_BT=64|128
        const char* e = getenv("RF_GEMM_BT");
        return e ? atoi(e) : 0;
    }();
    // bf16: 64-tiles below two 128-tiles per CU; fp32 (4x the MFMA cycles per byte staged): 128-tiles from one
    // per CU (profiles/r02/gemm_ab2.txt: 8704 -> 1024 at M = 4096, 108 -> 116 TFLOP/s)
    const bool small = force_bt ? force_bt == 64 : tiles128 < (bf ? 512 : 256);
    const int bt = small ? 64 : 128;
    const int64_t tiles = ((M + bt - 1) / bt) * ((N + bt - 1) / bt);
    RF_REQUIRE(tiles < (int64_t)1 << 31, "rf_linear_fwd: too many tiles");
    const dim3 g((unsigned)tiles);
    const bool ktail = K % (bf ? BKH : BKF) != 0;
#define RF_GEMM(BF, BT_)                                                                                              \
    do {                                                                                                             \
        if (ktail) hipLaunchKernelGGL((gemm_kernel<BF, BT_, true>), g, dim3(256), 0, st, x, W, b, y, M, N, K, ldx, ldy, act); \
        else hipLaunchKernelGGL((gemm_kernel<BF, BT_, false>), g, dim3(256), 0, st, x, W, b, y, M, N, K, ldx, ldy, act); \
    } while (0)
    if (bf && small) RF_GEMM(true, 64);
    else if (bf) RF_GEMM(true, 128);
    else if (small) RF_GEMM(false, 64);
    else RF_GEMM(false, 128);
#undef RF_GEMM
    return rf_check_launch("gemm_kernel");
}
