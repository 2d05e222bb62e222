// rf_tower.hip — DSSM tower training stages on gfx950 (models/matching/dssm.py:25-26 create_mlp([1024, 512, 256],
// 0.3, "selu", BatchNormalization(1e-6)) trained by model.fit, example/ranking_search/train.py:96-104).
//
// Per layer: BatchNormalization in training mode (batch statistics, Keras tf.nn.moments: biased variance) is an
// affine per column, so it folds into the following Dense (W' = W diag(a), b' = b + W c with a = gamma / sqrt(var +
// eps), c = beta - mean a) and the forward GEMM runs on the raw activations (rf_linear_fwd / rf_linear_splitk_fwd,
// SELU in its epilogue); Dropout(0.3) scales the kept values by 1 / 0.7 with a counter-hash mask. Backward: the
// SELU + dropout gradient with the bias gradient's column sums, the folded weight gradient dW = G diag(a) + db c^T
// from G = dpre^T x, and the BatchNormalization backward (column sums of dz and dz * xhat, then dx).
//
// Column reductions are deterministic: a thread per column walks a fixed chunk of rows (coalesced: consecutive
// threads, consecutive columns), chunk partials land in a workspace, and a finish kernel combines them in chunk
// order. Statistics use a per-chunk pivot (the chunk's first value) and Chan's combine across chunks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "rf_common.h"

namespace {

constexpr int kColThreads = 256;
constexpr int kRowsPerChunk = 128;

__host__ __device__ inline int tower_chunks(int64_t M) { return (int)std::min<int64_t>(64, (M + kRowsPerChunk - 1) / kRowsPerChunk); }

// keep mask of Keras Dropout(rate) in training: u = top 24 bits of splitmix64(seed ^ (row * N + col)) / 2^24,
// kept when u >= rate (oracle.dropout_keep restates it)
__device__ __forceinline__ bool keep_elem(uint64_t seed, int64_t row, int64_t N, int64_t col, float rate) {
    const uint64_t h = splitmix64_dev(seed ^ (uint64_t)(row * N + col));
    return (float)(h >> 40) * (1.0f / 16777216.0f) >= rate;
}

__device__ __forceinline__ float bn_scale(const float* gamma, const float* var, float eps, int k) {
    return gamma[k] * (1.0f / sqrtf(var[k] + eps));
}

// ---- column statistics -----------------------------------------------------------------------------------
// chunk partials: (n, mean, M2) around the chunk's first value (pivot p: S = sum(x - p), Q = sum((x - p)^2),
// mean = p + S / n, M2 = Q - S^2 / n)
__global__ __launch_bounds__(kColThreads) void col_stats_partial_kernel(const float* __restrict__ x, int64_t M, int K,
                                                                        int64_t ldx, int rows_per, float* __restrict__ part) {
    const int k = blockIdx.x * kColThreads + threadIdx.x;
    if (k >= K) return;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float mean = 0.f, m2 = 0.f;
    if (r0 < r1) {
        const float p = x[r0 * ldx + k];
        float s = 0.f, q = 0.f;
        for (int64_t r = r0; r < r1; ++r) {
            const float d = x[r * ldx + k] - p;
            s += d;
            q = fmaf(d, d, q);
        }
        const float n = (float)(r1 - r0);
        mean = p + s / n;
        m2 = fmaxf(q - s * s / n, 0.f);
    }
    float* o = part + ((int64_t)blockIdx.y * K + k) * 2;
    o[0] = mean;
    o[1] = m2;
}

__global__ __launch_bounds__(kColThreads) void col_stats_finish_kernel(const float* __restrict__ part, int64_t M, int K,
                                                                       int chunks, int rows_per, float* __restrict__ mean,
                                                                       float* __restrict__ var) {
    const int k = blockIdx.x * kColThreads + threadIdx.x;
    if (k >= K) return;
    float n = 0.f, mu = 0.f, m2 = 0.f;
    for (int c = 0; c < chunks; ++c) {
        const int64_t r0 = (int64_t)c * rows_per;
        const float nb = (float)std::max<int64_t>(0, std::min<int64_t>(M, r0 + rows_per) - r0);
        if (nb <= 0.f) continue;
        const float mb = part[((int64_t)c * K + k) * 2], m2b = part[((int64_t)c * K + k) * 2 + 1];
        const float nn = n + nb, d = mb - mu;
        mu += d * (nb / nn);
        m2 += m2b + d * d * (n * nb / nn);
        n = nn;
    }
    mean[k] = mu;
    var[k] = m2 / (float)M;
}

// ---- BatchNormalization folded into the Dense that follows it ----------------------------------------------
// one workgroup per output row n: W'[n][k] = W[n][k] a_k; b'[n] = b[n] + sum_k W[n][k] c_k (fixed order: each
// thread its strided subset, then a fixed tree)
__global__ __launch_bounds__(256) void bn_fold_kernel(const float* __restrict__ W, int K, const float* __restrict__ b,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      const float* __restrict__ mean, const float* __restrict__ var,
                                                      float eps, float* __restrict__ Wo, float* __restrict__ bo) {
    __shared__ float red[256];
    const int64_t n = blockIdx.x;
    const float* w = W + n * K;
    float* wo = Wo + n * K;
    float acc = 0.f;
    for (int k = threadIdx.x; k < K; k += 256) {
        const float a = bn_scale(gamma, var, eps, k);
        const float c = beta[k] - mean[k] * a;
        const float v = w[k];
        wo[k] = v * a;
        acc = fmaf(v, c, acc);
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) bo[n] = (b ? b[n] : 0.f) + red[0];
}

// dW[n][k] = G[n][k] a_k + db[n] c_k  (grid: x = column blocks, y = rows)
__global__ __launch_bounds__(256) void bn_fold_grad_kernel(const float* __restrict__ G, int N, int K, const float* __restrict__ db,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ mean, const float* __restrict__ var,
                                                           float eps, float* __restrict__ dW) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const int64_t e = (int64_t)blockIdx.y * K + k;
    const float a = bn_scale(gamma, var, eps, k);
    const float c = beta[k] - mean[k] * a;
    dW[e] = fmaf(G[e], a, db[blockIdx.y] * c);
}

// ---- dropout ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void dropout_fwd_kernel(const float* __restrict__ x, int64_t M, int N, int64_t ldx,
                                                          float rate, uint64_t seed, float* __restrict__ y, int64_t ldy) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= N) return;
    const int64_t r = blockIdx.y;
    const float v = x[r * ldx + c];
    y[r * ldy + c] = keep_elem(seed, r, N, c, rate) ? v * (1.0f / (1.0f - rate)) : 0.f;
}

// ---- SELU + dropout backward, bias-gradient column partials ----------------------------------------------
// h = dropout(selu(pre)): for a kept element y = selu(pre) = h (1 - rate), and the gradient factor is TF's SeluGrad
// on the activations: y + scale alpha where y < 0, scale elsewhere; dropped elements get dpre = 0
__global__ __launch_bounds__(kColThreads) void selu_dropout_bwd_kernel(const float* __restrict__ dh, int64_t lddh,
                                                                       const float* __restrict__ h, int64_t ldh, int64_t M,
                                                                       int N, float rate, uint64_t seed, int rows_per,
                                                                       float* __restrict__ dpre, int64_t ldd,
                                                                       float* __restrict__ part) {
    constexpr float kScale = 1.0507009873554804934193349852946f, kAlpha = 1.6732632423543772848170429916717f;
    const int c = blockIdx.x * kColThreads + threadIdx.x;
    if (c >= N) return;
    const float s = 1.0f / (1.0f - rate), keepv = 1.0f - rate;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float acc = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        float g = 0.f;
        if (keep_elem(seed, r, N, c, rate)) {
            const float y = h[r * ldh + c] * keepv;
            const float d = y < 0.f ? y + kScale * kAlpha : kScale;
            g = dh[r * lddh + c] * s * d;
        }
        dpre[r * ldd + c] = g;
        acc += g;
    }
    part[(int64_t)blockIdx.y * N + c] = acc;
}

__global__ __launch_bounds__(kColThreads) void col_sum_finish_kernel(const float* __restrict__ part, int N, int chunks,
                                                                     float* __restrict__ out) {
    const int c = blockIdx.x * kColThreads + threadIdx.x;
    if (c >= N) return;
    float acc = 0.f;
    for (int i = 0; i < chunks; ++i) acc += part[(int64_t)i * N + c];
    out[c] = acc;
}

// ---- BatchNormalization backward -------------------------------------------------------------------------
// column partials of sum(dz) and sum(dz * xhat), xhat = (x - mean) rstd
__global__ __launch_bounds__(kColThreads) void bn_bwd_partial_kernel(const float* __restrict__ dz, int64_t lddz,
                                                                     const float* __restrict__ x, int64_t ldx, int64_t M, int K,
                                                                     const float* __restrict__ mean, const float* __restrict__ var,
                                                                     float eps, int rows_per, float* __restrict__ part) {
    const int k = blockIdx.x * kColThreads + threadIdx.x;
    if (k >= K) return;
    const float mu = mean[k], rstd = 1.0f / sqrtf(var[k] + eps);
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float s1 = 0.f, s2 = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float g = dz[r * lddz + k];
        s1 += g;
        s2 = fmaf(g, (x[r * ldx + k] - mu) * rstd, s2);
    }
    float* o = part + ((int64_t)blockIdx.y * K + k) * 2;
    o[0] = s1;
    o[1] = s2;
}

__global__ __launch_bounds__(kColThreads) void bn_bwd_finish_kernel(const float* __restrict__ part, int K, int chunks,
                                                                    float* __restrict__ dbeta, float* __restrict__ dgamma) {
    const int k = blockIdx.x * kColThreads + threadIdx.x;
    if (k >= K) return;
    float s1 = 0.f, s2 = 0.f;
    for (int c = 0; c < chunks; ++c) {
        s1 += part[((int64_t)c * K + k) * 2];
        s2 += part[((int64_t)c * K + k) * 2 + 1];
    }
    dbeta[k] = s1;
    dgamma[k] = s2;
}

// dx = gamma rstd (dz - dbeta / M - xhat dgamma / M)  (grid: x = column blocks, y = rows)
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dz, int64_t lddz, const float* __restrict__ x,
                                                           int64_t ldx, int64_t M, int K, const float* __restrict__ mean,
                                                           const float* __restrict__ var, const float* __restrict__ gamma,
                                                           float eps, const float* __restrict__ dbeta,
                                                           const float* __restrict__ dgamma, float* __restrict__ dx, int64_t lddx) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= K) return;
    const int64_t r = blockIdx.y;
    const float invM = 1.0f / (float)M;
    const float rstd = 1.0f / sqrtf(var[k] + eps);
    const float xh = (x[r * ldx + k] - mean[k]) * rstd;
    const float g = dz[r * lddz + k] - dbeta[k] * invM - xh * dgamma[k] * invM;
    dx[r * lddx + k] = gamma[k] * rstd * g;
}


}  // namespace

extern "C" size_t rf_tower_ws_bytes(int64_t M, int32_t K) {
    return (size_t)tower_chunks(M) * (size_t)std::max(K, 1) * 2 * sizeof(float);
}

extern "C" int rf_col_stats(const float* x, int64_t M, int32_t K, int64_t ldx, float* mean, float* var, void* ws,
                            size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && K > 0 && ldx >= K && x && mean && var, "rf_col_stats: bad arguments");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, K), "rf_col_stats: workspace too small");
    const int chunks = tower_chunks(M), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const dim3 g((K + kColThreads - 1) / kColThreads, chunks);
    hipLaunchKernelGGL(col_stats_partial_kernel, g, dim3(kColThreads), 0, st, x, M, K, ldx, rows_per, (float*)ws);
    hipLaunchKernelGGL(col_stats_finish_kernel, dim3(g.x), dim3(kColThreads), 0, st, (const float*)ws, M, K, chunks, rows_per,
                       mean, var);
    return rf_check_launch("rf_col_stats");
}

extern "C" int rf_bn_fold(const float* W, int32_t N, int32_t K, const float* b, const float* gamma, const float* beta,
                          const float* mean, const float* var, float eps, float* W_out, float* b_out, void* stream) {
    RF_REQUIRE(N > 0 && K > 0 && W && gamma && beta && mean && var && W_out && b_out, "rf_bn_fold: bad arguments");
    hipLaunchKernelGGL(bn_fold_kernel, dim3(N), dim3(256), 0, rf_stream(stream), W, K, b, gamma, beta, mean, var, eps, W_out,
                       b_out);
    return rf_check_launch("rf_bn_fold");
}

extern "C" int rf_bn_fold_grad(const float* G, int32_t N, int32_t K, const float* db, const float* gamma, const float* beta,
                               const float* mean, const float* var, float eps, float* dW, void* stream) {
    RF_REQUIRE(N > 0 && K > 0 && G && db && gamma && beta && mean && var && dW, "rf_bn_fold_grad: bad arguments");
    hipLaunchKernelGGL(bn_fold_grad_kernel, dim3((K + 255) / 256, N), dim3(256), 0, rf_stream(stream), G, N, K, db, gamma, beta,
                       mean, var, eps, dW);
    return rf_check_launch("rf_bn_fold_grad");
}

extern "C" int rf_dropout_fwd(const float* x, int64_t M, int32_t N, int64_t ldx, float rate, uint64_t seed, float* y,
                              int64_t ldy, void* stream) {
    RF_REQUIRE(M >= 0 && M <= 65535 && N > 0 && ldx >= N && ldy >= N && rate >= 0.f && rate < 1.f,
               "rf_dropout_fwd: bad arguments");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && y, "rf_dropout_fwd: null pointer");
    hipLaunchKernelGGL(dropout_fwd_kernel, dim3((N + 255) / 256, (unsigned)M), dim3(256), 0, rf_stream(stream), x, M, N, ldx, rate,
                       seed, y, ldy);
    return rf_check_launch("rf_dropout_fwd");
}

extern "C" int rf_selu_dropout_bwd(const float* dh, int64_t lddh, const float* h, int64_t ldh, int64_t M, int32_t N,
                                   float rate, uint64_t seed, float* dpre, int64_t ldd, float* db, void* ws,
                                   size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && N > 0 && lddh >= N && ldh >= N && ldd >= N && rate >= 0.f && rate < 1.f,
               "rf_selu_dropout_bwd: bad arguments");
    RF_REQUIRE(dh && h && dpre && db, "rf_selu_dropout_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, N), "rf_selu_dropout_bwd: workspace too small");
    const int chunks = tower_chunks(M), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const dim3 g((N + kColThreads - 1) / kColThreads, chunks);
    hipLaunchKernelGGL(selu_dropout_bwd_kernel, g, dim3(kColThreads), 0, st, dh, lddh, h, ldh, M, N, rate, seed, rows_per, dpre,
                       ldd, (float*)ws);
    hipLaunchKernelGGL(col_sum_finish_kernel, dim3(g.x), dim3(kColThreads), 0, st, (const float*)ws, N, chunks, db);
    return rf_check_launch("rf_selu_dropout_bwd");
}

extern "C" int rf_bn_bwd(const float* dz, int64_t lddz, const float* x, int64_t ldx, int64_t M, int32_t K, const float* mean,
                         const float* var, const float* gamma, float eps, float* dx, int64_t lddx, float* dgamma,
                         float* dbeta, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && M <= 65535 && K > 0 && lddz >= K && ldx >= K && lddx >= K, "rf_bn_bwd: bad arguments");
    RF_REQUIRE(dz && x && mean && var && gamma && dx && dgamma && dbeta, "rf_bn_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, K), "rf_bn_bwd: workspace too small");
    const int chunks = tower_chunks(M), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const dim3 g((K + kColThreads - 1) / kColThreads, chunks);
    hipLaunchKernelGGL(bn_bwd_partial_kernel, g, dim3(kColThreads), 0, st, dz, lddz, x, ldx, M, K, mean, var, eps, rows_per,
                       (float*)ws);
    hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3(g.x), dim3(kColThreads), 0, st, (const float*)ws, K, chunks, dbeta, dgamma);
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3((K + 255) / 256, (unsigned)M), dim3(256), 0, st, dz, lddz, x, ldx, M, K, mean, var,
                       gamma, eps, dbeta, dgamma, dx, lddx);
    return rf_check_launch("rf_bn_bwd");
}
