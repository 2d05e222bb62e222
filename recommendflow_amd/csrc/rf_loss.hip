// rf_loss.hip — the two-tower training losses of SURVEY §8f.1, forward and gradient in one call.
//
// cosent_loss (backend/losses/match_losses.py:42-56):
//   x_ij = scale * (s_i - s_j) for pairs with y_i < y_j (other pairs get -1e12, i.e. exp -> 0)
//   loss = logsumexp([0, x_ij ...]) = m + log(exp(-m) + sum_valid exp(x_ij - m)),  m = max(0, max_valid x_ij)
//   dloss/ds_i = scale * (R_i - C_i) / Z,  R_i = sum_{j: y_i<y_j} e^{x_ij - m},  C_i = sum_{j: y_j<y_i} e^{x_ji - m}
// batch_neg_sample_scaled_multi_class_ce_loss (match_losses.py:150-165, Que2Search):
//   loss = mean_i( -log(exp(s P_ii) / sum_j exp(s P_ij)) * y_i ),  P = query . doc^T (a library GEMM)
//   dloss/dP_ij = s * y_i / B * (softmax_j(s P_i.) - [i == j])
// Deterministic: fixed-order block reductions, no atomics. cosent: (i block, j chunk) tiles of 256 x 256 pairs,
// the j scores and labels staged through LDS; the tile partials are summed in tile order.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {

constexpr int kRows = 256;  // i rows per block (one per thread)

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The B x B pairs run as (i block, j chunk) tiles: grid (ceil(B / 256), ceil(B / 256)), a thread per i walking
// its tile's 256 j through LDS, so a 4096 batch fills 256 workgroups (a thread per i over every j kept 16 busy).
// pass A: per-tile max of the valid x_ij
__global__ __launch_bounds__(kRows) void cosent_max_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                                           int B, float scale, float* __restrict__ part) {
    __shared__ float sj[kRows], yj[kRows];
    __shared__ float red[kRows / 64];
    const int i = blockIdx.x * kRows + threadIdx.x;
    const float si = i < B ? s[i] : 0.f, yi = i < B ? y[i] : 0.f;
    const int j0 = blockIdx.y * kRows;
    const int j = j0 + threadIdx.x;
    sj[threadIdx.x] = j < B ? s[j] : 0.f;
    yj[threadIdx.x] = j < B ? y[j] : -INFINITY;
    __syncthreads();
    float m = -INFINITY;
    if (i < B) {
        const int n = min(kRows, B - j0);
        for (int k = 0; k < n; ++k)
            if (yi < yj[k]) m = fmaxf(m, scale * si - scale * sj[k]);
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float r = red[0];
        for (int w = 1; w < kRows / 64; ++w) r = fmaxf(r, red[w]);
        part[blockIdx.y * gridDim.x + blockIdx.x] = r;
    }
}

// pass B: per-tile partials of R_i and C_i with the global m (m = max(0, every tile maximum))
__global__ __launch_bounds__(kRows) void cosent_sums_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                                            int B, float scale, const float* __restrict__ part, int nparts,
                                                            float* __restrict__ Rp, float* __restrict__ Cp) {
    __shared__ float sj[kRows], yj[kRows];
    float m = 0.f;
    for (int p = 0; p < nparts; ++p) m = fmaxf(m, part[p]);
    const int i = blockIdx.x * kRows + threadIdx.x;
    const float si = i < B ? s[i] : 0.f, yi = i < B ? y[i] : 0.f;
    const int j0 = blockIdx.y * kRows;
    const int j = j0 + threadIdx.x;
    sj[threadIdx.x] = j < B ? s[j] : 0.f;
    yj[threadIdx.x] = j < B ? y[j] : 0.f;
    __syncthreads();
    if (i >= B) return;
    float r = 0.f, c = 0.f;
    const int n = min(kRows, B - j0);
    for (int k = 0; k < n; ++k) {
        if (yi < yj[k]) r += expf(scale * si - scale * sj[k] - m);
        if (yj[k] < yi) c += expf(scale * sj[k] - scale * si - m);
    }
    Rp[(int64_t)blockIdx.y * B + i] = r;
    Cp[(int64_t)blockIdx.y * B + i] = c;
}

// pass C (one block): R_i, C_i = the tile partials summed in tile order; Z, loss, gradient
__global__ __launch_bounds__(1024) void cosent_final_kernel(const float* __restrict__ Rp, const float* __restrict__ Cp, int B,
                                                            int nj, float scale, const float* __restrict__ part, int nparts,
                                                            float* __restrict__ loss, float* __restrict__ ds) {
    __shared__ float red[16];
    __shared__ float s_z;
    float m = 0.f;
    for (int p = 0; p < nparts; ++p) m = fmaxf(m, part[p]);
    auto rsum = [&](const float* P, int i) {
        float a = 0.f;
        for (int t = 0; t < nj; ++t) a += P[(int64_t)t * B + i];
        return a;
    };
    float acc = 0.f;
    for (int i = threadIdx.x; i < B; i += 1024) acc += rsum(Rp, i);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        float z = expf(-m);
        for (int w = 0; w < 16; ++w) z += red[w];
        s_z = z;
        *loss = m + logf(z);
    }
    __syncthreads();
    const float z = s_z;
    if (ds)
        for (int i = threadIdx.x; i < B; i += 1024) ds[i] = scale * (rsum(Rp, i) - rsum(Cp, i)) / z;
}

// in-batch CE: one block per row i (256 threads), logits row of length B
__global__ __launch_bounds__(256) void inbatch_ce_kernel(const float* __restrict__ P, int64_t ld, const float* __restrict__ y,
                                                         int B, float scale, float* __restrict__ row_loss,
                                                         float* __restrict__ dP, int64_t ldd) {
    __shared__ float red[4];
    const int i = blockIdx.x;
    const float* row = P + (int64_t)i * ld;
    float m = -INFINITY;
    for (int j = threadIdx.x; j < B; j += 256) m = fmaxf(m, scale * row[j]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    float z = 0.f;
    for (int j = threadIdx.x; j < B; j += 256) z += expf(scale * row[j] - m);
    z = wave_sum(z);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = z;
    __syncthreads();
    z = red[0] + red[1] + red[2] + red[3];
    const float yi = y[i];
    if (threadIdx.x == 0) row_loss[i] = -(scale * row[i] - m - logf(z)) * yi;  // -log(num / den) * y_i
    if (dP) {
        const float g = scale * yi / (float)B;
        float* drow = dP + (int64_t)i * ldd;
        for (int j = threadIdx.x; j < B; j += 256) drow[j] = g * (expf(scale * row[j] - m) / z - (j == i ? 1.f : 0.f));
    }
}

__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ v, int B, float* __restrict__ out) {
    __shared__ float red[16];
    float a = 0.f;
    for (int i = threadIdx.x; i < B; i += 1024) a += v[i];
    a = wave_sum(a);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        float t = 0.f;
        for (int w = 0; w < 16; ++w) t += red[w];
        *out = t / (float)B;
    }
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" size_t rf_loss_ws_bytes(int32_t batch) {
    if (batch < 0) return 0;
    const size_t nb = (size_t)(batch + kRows - 1) / kRows + 1;
    return a256(nb * nb * 4) + 2 * a256(nb * (size_t)std::max(batch, 1) * 4);
}

extern "C" int rf_cosent_loss(const float* score, const float* label, int32_t batch, float scale, float* loss, float* dscore,
                              void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(batch >= 1, "rf_cosent_loss: batch must be >= 1");
    RF_REQUIRE(score && label && loss && ws, "rf_cosent_loss: null pointer");
    RF_REQUIRE(ws_bytes >= rf_loss_ws_bytes(batch), "rf_cosent_loss: workspace too small");
    hipStream_t st = rf_stream(stream);
    const int nb = (batch + kRows - 1) / kRows;
    char* w = static_cast<char*>(ws);
    float* part = reinterpret_cast<float*>(w);
    float* Rp = reinterpret_cast<float*>(w + a256((size_t)(nb + 1) * (nb + 1) * 4));
    float* Cp = Rp + a256((size_t)(nb + 1) * batch * 4) / 4;
    const dim3 g(nb, nb);
    hipLaunchKernelGGL(cosent_max_kernel, g, dim3(kRows), 0, st, score, label, batch, scale, part);
    hipLaunchKernelGGL(cosent_sums_kernel, g, dim3(kRows), 0, st, score, label, batch, scale, part, nb * nb, Rp, Cp);
    hipLaunchKernelGGL(cosent_final_kernel, dim3(1), dim3(1024), 0, st, Rp, Cp, batch, nb, scale, part, nb * nb, loss, dscore);
    return rf_check_launch("rf_cosent_loss");
}

extern "C" int rf_inbatch_ce_loss(const float* logits, int64_t ld, const float* label, int32_t batch, float scale,
                                  float* loss, float* dlogits, int64_t ldd, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(batch >= 1 && ld >= batch && (!dlogits || ldd >= batch), "rf_inbatch_ce_loss: bad shape");
    RF_REQUIRE(logits && label && loss && ws, "rf_inbatch_ce_loss: null pointer");
    RF_REQUIRE(ws_bytes >= rf_loss_ws_bytes(batch), "rf_inbatch_ce_loss: workspace too small");
    hipStream_t st = rf_stream(stream);
    float* rows = static_cast<float*>(ws);
    hipLaunchKernelGGL(inbatch_ce_kernel, dim3(batch), dim3(256), 0, st, logits, ld, label, batch, scale, rows, dlogits, ldd);
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, st, rows, batch, loss);
    return rf_check_launch("rf_inbatch_ce_loss");
}
