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
// Column reductions are deterministic: a thread per 4 columns (one float4; 1 when a row is not 16-byte aligned)
// walks a fixed chunk of rows with 4-8 rows' loads in flight (coalesced: consecutive threads, consecutive
// columns), chunk partials land in a workspace, and a finish kernel combines them in chunk order. The chunk
// count depends only on (M, K) and is sized for ~4K workgroups: at cfg2's 4096 x 256 that is 512 chunks of 8
// rows where a fixed 128-row chunk left 32 workgroups on 256 CUs. Statistics use a per-chunk pivot (the chunk's
// first value) and Chan's combine across chunks.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <utility>
#include <cmath>

#include "rf_common.h"

namespace {

constexpr int kColThreads = 256;
constexpr int kUnroll = 8;  // rows loaded ahead of the in-order accumulation

// Row chunks of a column reduction: enough chunks that the float4 launch has ~4K workgroups (a thread per 4
// columns walks its chunk's rows in order), at least 8 rows a chunk, at most 512 chunks. Depends only on
// (M, K), so a reduction is replay-deterministic whichever vector width runs it.
__host__ inline int tower_chunks(int64_t M, int K) {
    const int64_t colblocks = std::max<int64_t>(1, ((int64_t)K + 4 * kColThreads - 1) / (4 * kColThreads));
    const int64_t want = (4096 + colblocks - 1) / colblocks;
    const int64_t cap = std::min<int64_t>(512, std::max<int64_t>(1, (M + 7) / 8));
    return (int)std::max<int64_t>(1, std::min(want, cap));
}

// columns a thread owns: 4 (one float4) when every operand's rows are 16-byte aligned, else 1
__host__ inline bool vec4_ok(int K, std::initializer_list<std::pair<const void*, int64_t>> ops) {
    if (K % 4) return false;
    for (auto& o : ops)
        if (((uintptr_t)o.first & 15) || (o.second % 4)) return false;
    return true;
}

template <int V> struct vec_t;
template <> struct vec_t<1> { using T = float; };
template <> struct vec_t<4> { using T = float4; };
template <int V> __device__ __forceinline__ float& lane(typename vec_t<V>::T& v, int i);
template <> __device__ __forceinline__ float& lane<1>(float& v, int) { return v; }
template <> __device__ __forceinline__ float& lane<4>(float4& v, int i) { return (&v.x)[i]; }
template <int V> __device__ __forceinline__ typename vec_t<V>::T ld(const float* p) {
    return *reinterpret_cast<const typename vec_t<V>::T*>(p);
}
template <int V> __device__ __forceinline__ void st(float* p, const typename vec_t<V>::T& v) {
    *reinterpret_cast<typename vec_t<V>::T*>(p) = v;
}

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
// chunk partials: (mean, M2) around the chunk's first value (pivot p: S = sum(x - p), Q = sum((x - p)^2),
// mean = p + S / n, M2 = Q - S^2 / n)
template <int V>
__global__ __launch_bounds__(kColThreads) void col_stats_partial_kernel(const float* __restrict__ x, int64_t M, int K,
                                                                        int64_t ldx, int rows_per, float* __restrict__ part) {
    const int k0 = (blockIdx.x * kColThreads + threadIdx.x) * V;
    if (k0 >= K) return;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float mean[V], m2[V];
    for (int i = 0; i < V; ++i) mean[i] = m2[i] = 0.f;
    if (r0 < r1) {
        typename vec_t<V>::T p = ld<V>(x + r0 * ldx + k0);
        float s[V], q[V];
        for (int i = 0; i < V; ++i) s[i] = q[i] = 0.f;
        int64_t r = r0;
        for (; r + kUnroll <= r1; r += kUnroll) {
            typename vec_t<V>::T v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = ld<V>(x + (r + u) * ldx + k0);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u)
#pragma unroll
                for (int i = 0; i < V; ++i) {
                    const float d = lane<V>(v[u], i) - lane<V>(p, i);
                    s[i] += d;
                    q[i] = fmaf(d, d, q[i]);
                }
        }
        for (; r < r1; ++r) {
            typename vec_t<V>::T v = ld<V>(x + r * ldx + k0);
#pragma unroll
            for (int i = 0; i < V; ++i) {
                const float d = lane<V>(v, i) - lane<V>(p, i);
                s[i] += d;
                q[i] = fmaf(d, d, q[i]);
            }
        }
        const float n = (float)(r1 - r0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            mean[i] = lane<V>(p, i) + s[i] / n;
            m2[i] = fmaxf(q[i] - s[i] * s[i] / n, 0.f);
        }
    }
    // layout [chunk][2][K]: the finish kernel reads both planes coalesced
    float* o = part + (int64_t)blockIdx.y * 2 * K + k0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        o[i] = mean[i];
        o[K + i] = m2[i];
    }
}

// ---- chunk-partial finish ---------------------------------------------------------------------------------
// A workgroup per 32 columns: 8 groups of 32 lanes each combine a contiguous run of chunks (8 loads in flight per
// lane), then group 0 combines the 8 group results in group order. A fixed tree, so replay-deterministic; a
// thread walking all (up to 512) chunks alone was latency-bound at 120-230 us a launch.
constexpr int kFinCols = 32, kFinGroups = 8;

// sums of P planes: part[c][p][K] (P = 1 or 2)
template <int P>
__device__ __forceinline__ void finish_sums(const float* __restrict__ part, int K, int chunks, float (&out)[P]) {
    __shared__ float red[kFinGroups][P][kFinCols];
    const int cl = threadIdx.x % kFinCols, grp = threadIdx.x / kFinCols;
    const int k = blockIdx.x * kFinCols + cl;
    const int per = (chunks + kFinGroups - 1) / kFinGroups, c0 = grp * per, c1 = std::min(chunks, c0 + per);
    float acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = 0.f;
    if (k < K) {
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            float v[8][P];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int p = 0; p < P; ++p) v[u][p] = part[((int64_t)(c + u) * P + p) * K + k];
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int p = 0; p < P; ++p) acc[p] += v[u][p];
        }
        for (; c < c1; ++c)
#pragma unroll
            for (int p = 0; p < P; ++p) acc[p] += part[((int64_t)c * P + p) * K + k];
    }
#pragma unroll
    for (int p = 0; p < P; ++p) red[grp][p][cl] = acc[p];
    __syncthreads();
#pragma unroll
    for (int p = 0; p < P; ++p) {
        float t = 0.f;
        for (int g = 0; g < kFinGroups; ++g) t += red[g][p][cl];
        out[p] = t;
    }
}

__global__ __launch_bounds__(kFinCols * kFinGroups) void col_stats_finish_kernel(const float* __restrict__ part, int64_t M, int K,
                                                                                 int chunks, int rows_per, float* __restrict__ mean,
                                                                                 float* __restrict__ var) {
    __shared__ float red[kFinGroups][3][kFinCols];
    const int cl = threadIdx.x % kFinCols, grp = threadIdx.x / kFinCols;
    const int k = blockIdx.x * kFinCols + cl;
    const int per = (chunks + kFinGroups - 1) / kFinGroups, c0 = grp * per, c1 = std::min(chunks, c0 + per);
    float n = 0.f, mu = 0.f, m2 = 0.f;
    auto combine = [&](float nb, float mb, float m2b) {
        if (nb <= 0.f) return;
        const float nn = n + nb, d = mb - mu;
        mu += d * (nb / nn);
        m2 += m2b + d * d * (n * nb / nn);
        n = nn;
    };
    auto rows = [&](int c) {
        const int64_t r0 = (int64_t)c * rows_per;
        return (float)std::max<int64_t>(0, std::min<int64_t>(M, r0 + rows_per) - r0);
    };
    if (k < K) {
        int c = c0;
        for (; c + 8 <= c1; c += 8) {
            float mb[8], m2b[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                mb[u] = part[(int64_t)(c + u) * 2 * K + k];
                m2b[u] = part[(int64_t)(c + u) * 2 * K + K + k];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) combine(rows(c + u), mb[u], m2b[u]);
        }
        for (; c < c1; ++c) combine(rows(c), part[(int64_t)c * 2 * K + k], part[(int64_t)c * 2 * K + K + k]);
    }
    red[grp][0][cl] = n;
    red[grp][1][cl] = mu;
    red[grp][2][cl] = m2;
    __syncthreads();
    if (grp != 0 || k >= K) return;
    n = mu = m2 = 0.f;
    for (int g = 0; g < kFinGroups; ++g) combine(red[g][0][cl], red[g][1][cl], red[g][2][cl]);
    mean[k] = mu;
    var[k] = m2 / (float)M;
}

// ---- BatchNormalization folded into the Dense that follows it ----------------------------------------------
// the fold's per-column affine a_k = gamma_k rstd_k, c_k = beta_k - mean_k a_k for columns k .. k + V
template <int V>
__device__ __forceinline__ void bn_affine(const float* gamma, const float* beta, const float* mean, const float* var, float eps,
                                          int k, typename vec_t<V>::T& a, typename vec_t<V>::T& c) {
    typename vec_t<V>::T g = ld<V>(gamma + k), be = ld<V>(beta + k), mu = ld<V>(mean + k), vr = ld<V>(var + k);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        lane<V>(a, i) = lane<V>(g, i) * (1.0f / sqrtf(lane<V>(vr, i) + eps));
        lane<V>(c, i) = lane<V>(be, i) - lane<V>(mu, i) * lane<V>(a, i);
    }
}

// one workgroup per output row n: W'[n][k] = W[n][k] a_k; b'[n] = b[n] + sum_k W[n][k] c_k (fixed order: each
// thread its strided subset, then a fixed tree)
template <int V>
__global__ __launch_bounds__(256) void bn_fold_kernel(const float* __restrict__ W, int K, const float* __restrict__ b,
                                                      const float* __restrict__ gamma, const float* __restrict__ beta,
                                                      const float* __restrict__ mean, const float* __restrict__ var,
                                                      float eps, float* __restrict__ Wo, float* __restrict__ bo) {
    __shared__ float red[256];
    const int64_t n = blockIdx.x;
    const float* w = W + n * K;
    float* wo = Wo + n * K;
    float acc = 0.f;
    for (int k = threadIdx.x * V; k < K; k += 256 * V) {
        typename vec_t<V>::T v = ld<V>(w + k), a, c, o;
        bn_affine<V>(gamma, beta, mean, var, eps, k, a, c);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            lane<V>(o, i) = lane<V>(v, i) * lane<V>(a, i);
            acc = fmaf(lane<V>(v, i), lane<V>(c, i), acc);
        }
        st<V>(wo + k, o);
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
template <int V>
__global__ __launch_bounds__(256) void bn_fold_grad_kernel(const float* __restrict__ G, int N, int K, const float* __restrict__ db,
                                                           const float* __restrict__ gamma, const float* __restrict__ beta,
                                                           const float* __restrict__ mean, const float* __restrict__ var,
                                                           float eps, float* __restrict__ dW) {
    const int k = (blockIdx.x * 256 + threadIdx.x) * V;
    if (k >= K) return;
    const int64_t e = (int64_t)blockIdx.y * K + k;
    typename vec_t<V>::T g = ld<V>(G + e), a, c, o;
    bn_affine<V>(gamma, beta, mean, var, eps, k, a, c);
    const float d = db[blockIdx.y];
#pragma unroll
    for (int i = 0; i < V; ++i) lane<V>(o, i) = fmaf(lane<V>(g, i), lane<V>(a, i), d * lane<V>(c, i));
    st<V>(dW + e, o);
}

// ---- dropout ------------------------------------------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(256) void dropout_fwd_kernel(const float* __restrict__ x, int64_t M, int N, int64_t ldx,
                                                          float rate, uint64_t seed, float* y, int64_t ldy) {
    const int c = (blockIdx.x * 256 + threadIdx.x) * V;
    if (c >= N) return;
    const int64_t r = blockIdx.y;
    typename vec_t<V>::T v = ld<V>(x + r * ldx + c);
    const float s = 1.0f / (1.0f - rate);
#pragma unroll
    for (int i = 0; i < V; ++i) lane<V>(v, i) = keep_elem(seed, r, N, c + i, rate) ? lane<V>(v, i) * s : 0.f;
    st<V>(y + r * ldy + c, v);
}

// ---- SELU + dropout backward, bias-gradient column partials ----------------------------------------------
// h = dropout(selu(pre)): for a kept element y = selu(pre) = h (1 - rate), and the gradient factor is TF's SeluGrad
// on the activations: y + scale alpha where y < 0, scale elsewhere; dropped elements get dpre = 0
template <int V>
__global__ __launch_bounds__(kColThreads) void selu_dropout_bwd_kernel(const float* __restrict__ dh, int64_t lddh,
                                                                       const float* __restrict__ h, int64_t ldh, int64_t M,
                                                                       int N, float rate, uint64_t seed, int rows_per,
                                                                       float* __restrict__ dpre, int64_t ldd,
                                                                       float* __restrict__ part) {
    constexpr float kScale = 1.0507009873554804934193349852946f, kAlpha = 1.6732632423543772848170429916717f;
    const int c = (blockIdx.x * kColThreads + threadIdx.x) * V;
    if (c >= N) return;
    const float s = 1.0f / (1.0f - rate), keepv = 1.0f - rate;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float acc[V];
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    constexpr int U = kUnroll / 2;
    int64_t r = r0;
    auto row = [&](int64_t rr, typename vec_t<V>::T g, typename vec_t<V>::T hv) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
            float o = 0.f;
            if (keep_elem(seed, rr, N, c + i, rate)) {
                const float y = lane<V>(hv, i) * keepv;
                o = lane<V>(g, i) * s * (y < 0.f ? y + kScale * kAlpha : kScale);
            }
            lane<V>(g, i) = o;
            acc[i] += o;
        }
        st<V>(dpre + rr * ldd + c, g);
    };
    for (; r + U <= r1; r += U) {
        typename vec_t<V>::T g[U], hv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            g[u] = ld<V>(dh + (r + u) * lddh + c);
            hv[u] = ld<V>(h + (r + u) * ldh + c);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) row(r + u, g[u], hv[u]);
    }
    for (; r < r1; ++r) row(r, ld<V>(dh + r * lddh + c), ld<V>(h + r * ldh + c));
    float* o = part + (int64_t)blockIdx.y * N + c;
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = acc[i];
}

__global__ __launch_bounds__(kFinCols * kFinGroups) void col_sum_finish_kernel(const float* __restrict__ part, int N, int chunks,
                                                                               float* __restrict__ out) {
    float t[1];
    finish_sums<1>(part, N, chunks, t);
    const int k = blockIdx.x * kFinCols + threadIdx.x;
    if (threadIdx.x < kFinCols && k < N) out[k] = t[0];
}

// ---- BatchNormalization backward -------------------------------------------------------------------------
// column partials of sum(dz) and sum(dz * xhat), xhat = (x - mean) rstd
template <int V>
__global__ __launch_bounds__(kColThreads) void bn_bwd_partial_kernel(const float* __restrict__ dz, int64_t lddz,
                                                                     const float* __restrict__ x, int64_t ldx, int64_t M, int K,
                                                                     const float* __restrict__ mean, const float* __restrict__ var,
                                                                     float eps, int rows_per, float* __restrict__ part) {
    const int k0 = (blockIdx.x * kColThreads + threadIdx.x) * V;
    if (k0 >= K) return;
    float mu[V], rstd[V], s1[V], s2[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        mu[i] = mean[k0 + i];
        rstd[i] = 1.0f / sqrtf(var[k0 + i] + eps);
        s1[i] = s2[i] = 0.f;
    }
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    constexpr int U = kUnroll / 2;
    int64_t r = r0;
    auto row = [&](typename vec_t<V>::T g, typename vec_t<V>::T xv) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
            s1[i] += lane<V>(g, i);
            s2[i] = fmaf(lane<V>(g, i), (lane<V>(xv, i) - mu[i]) * rstd[i], s2[i]);
        }
    };
    for (; r + U <= r1; r += U) {
        typename vec_t<V>::T g[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            g[u] = ld<V>(dz + (r + u) * lddz + k0);
            xv[u] = ld<V>(x + (r + u) * ldx + k0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) row(g[u], xv[u]);
    }
    for (; r < r1; ++r) row(ld<V>(dz + r * lddz + k0), ld<V>(x + r * ldx + k0));
    float* o = part + (int64_t)blockIdx.y * 2 * K + k0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        o[i] = s1[i];
        o[K + i] = s2[i];
    }
}

// dbeta, dgamma in chunk order; then the apply kernel's per-column constants: p_k = gamma_k rstd_k,
// q_k = dbeta_k / M, t_k = dgamma_k / M (written after dbeta, dgamma into ac[0..3K))
__global__ __launch_bounds__(kFinCols * kFinGroups) void bn_bwd_finish_kernel(const float* __restrict__ part, int64_t M, int K,
                                                                              int chunks, const float* __restrict__ gamma,
                                                                              const float* __restrict__ var, float eps,
                                                                              float* __restrict__ dbeta, float* __restrict__ dgamma,
                                                                              float* __restrict__ ac) {
    float t[2];
    finish_sums<2>(part, K, chunks, t);
    const int k = blockIdx.x * kFinCols + threadIdx.x;
    if (threadIdx.x >= kFinCols || k >= K) return;
    dbeta[k] = t[0];
    dgamma[k] = t[1];
    const float invM = 1.0f / (float)M;
    ac[k] = gamma[k] * (1.0f / sqrtf(var[k] + eps));
    ac[K + k] = t[0] * invM;
    ac[2 * K + k] = t[1] * invM;
}

// dx = gamma rstd (dz - dbeta / M - xhat dgamma / M)  (grid: x = column blocks, y = rows)
template <int V>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ dz, int64_t lddz, const float* __restrict__ x,
                                                           int64_t ldx, int K, const float* __restrict__ mean,
                                                           const float* __restrict__ var, float eps,
                                                           const float* __restrict__ ac, float* dx, int64_t lddx) {
    const int k = (blockIdx.x * 256 + threadIdx.x) * V;
    if (k >= K) return;
    const int64_t r = blockIdx.y;
    typename vec_t<V>::T g = ld<V>(dz + r * lddz + k), xv = ld<V>(x + r * ldx + k), mu = ld<V>(mean + k), vr = ld<V>(var + k),
                         p = ld<V>(ac + k), q = ld<V>(ac + K + k), t = ld<V>(ac + 2 * K + k), o;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const float xh = (lane<V>(xv, i) - lane<V>(mu, i)) * (1.0f / sqrtf(lane<V>(vr, i) + eps));
        lane<V>(o, i) = lane<V>(p, i) * (lane<V>(g, i) - lane<V>(q, i) - xh * lane<V>(t, i));
    }
    st<V>(dx + r * lddx + k, o);
}

// ---- LayerNorm MLP training stages (the ESIM input / output MLPs: create_mlp(.., gelu, LayerNormalization(1e-6)),
// esim.py:45-52, under model.fit) -----------------------------------------------------------------------------
// activation value and derivative at the pre-activation x (exact erf GELU: tf.keras.activations.gelu)
__device__ __forceinline__ void act_vd(int act, float x, float& y, float& dy) {
    switch (act) {
        case RF_ACT_GELU: {
            const float c = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
            y = x * c;
            dy = c + x * 0.39894228040143267794f * expf(-0.5f * x * x);
            break;
        }
        case RF_ACT_RELU: y = x > 0.f ? x : 0.f; dy = x > 0.f ? 1.f : 0.f; break;
        case RF_ACT_SELU: {
            const float alpha = 1.6732632423543772848170429916717f, scale = 1.0507009873554804934193349852946f;
            const float ex = expf(fminf(x, 0.f));
            y = x > 0.f ? scale * x : scale * alpha * (ex - 1.0f);
            dy = x > 0.f ? scale : scale * alpha * ex;
            break;
        }
        default: y = x; dy = 1.f; break;
    }
}

// h = Dropout(rate)(act(pre)): kept elements act(pre) / (1 - rate) (the rf_dropout_fwd mask), dropped 0
template <int V>
__global__ __launch_bounds__(256) void act_dropout_fwd_kernel(const float* __restrict__ pre, int64_t ldp, int N, int act,
                                                              float rate, uint64_t seed, float* __restrict__ h, int64_t ldh) {
    const int c = (blockIdx.x * 256 + threadIdx.x) * V;
    if (c >= N) return;
    const int64_t r = blockIdx.y;
    typename vec_t<V>::T v = ld<V>(pre + r * ldp + c);
    const float s = 1.0f / (1.0f - rate);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        float y, dy;
        act_vd(act, lane<V>(v, i), y, dy);
        lane<V>(v, i) = rate == 0.f || keep_elem(seed, r, N, c + i, rate) ? y * s : 0.f;
    }
    st<V>(h + r * ldh + c, v);
}

// dpre = dh keep / (1 - rate) act'(pre); bias-gradient column partials of dpre
template <int V>
__global__ __launch_bounds__(kColThreads) void act_dropout_bwd_kernel(const float* __restrict__ dh, int64_t lddh,
                                                                      const float* __restrict__ pre, int64_t ldp, int64_t M,
                                                                      int N, int act, float rate, uint64_t seed, int rows_per,
                                                                      float* __restrict__ dpre, int64_t ldd,
                                                                      float* __restrict__ part) {
    const int c = (blockIdx.x * kColThreads + threadIdx.x) * V;
    if (c >= N) return;
    const float s = 1.0f / (1.0f - rate);
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    float acc[V];
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        typename vec_t<V>::T g = ld<V>(dh + r * lddh + c), x = ld<V>(pre + r * ldp + c);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            float y, dy;
            act_vd(act, lane<V>(x, i), y, dy);
            const float o = rate == 0.f || keep_elem(seed, r, N, c + i, rate) ? lane<V>(g, i) * s * dy : 0.f;
            lane<V>(g, i) = o;
            acc[i] += o;
        }
        st<V>(dpre + r * ldd + c, g);
    }
    float* o = part + (int64_t)blockIdx.y * N + c;
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = acc[i];
}

// LayerNorm backward, rows: one wave per row. mean and (biased) variance as tf.nn.moments, xhat = (x - mean)
// rsqrt(var + eps); with u = dy gamma: dx = rstd (u - mean(u) - xhat mean(u xhat)). Row (mean, rstd) to rs.
__global__ __launch_bounds__(256) void ln_bwd_rows_kernel(const float* __restrict__ dy, int64_t lddy,
                                                          const float* __restrict__ x, int64_t ldx, int64_t M, int K,
                                                          const float* __restrict__ gamma, float eps, float* __restrict__ dx,
                                                          int64_t lddx, float* __restrict__ rs) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= M) return;
    const float* xr = x + r * ldx;
    const float* gr = dy + r * lddy;
    float s = 0.f;
    for (int k = lane; k < K; k += 64) s += xr[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s / (float)K;
    float q = 0.f;
    for (int k = lane; k < K; k += 64) {
        const float d = xr[k] - mean;
        q = fmaf(d, d, q);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = 1.0f / sqrtf(q / (float)K + eps);
    float a = 0.f, b = 0.f;
    for (int k = lane; k < K; k += 64) {
        const float u = gr[k] * gamma[k];
        a += u;
        b = fmaf(u, (xr[k] - mean) * rstd, b);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    a /= (float)K;
    b /= (float)K;
    float* dr = dx + r * lddx;
    for (int k = lane; k < K; k += 64) {
        const float xh = (xr[k] - mean) * rstd;
        dr[k] = rstd * (gr[k] * gamma[k] - a - xh * b);
    }
    if (lane == 0) {
        rs[2 * r] = mean;
        rs[2 * r + 1] = rstd;
    }
}

// LayerNorm backward, columns: chunk partials of dbeta = sum(dy), dgamma = sum(dy xhat) -> part[chunk][2][K]
template <int V>
__global__ __launch_bounds__(kColThreads) void ln_bwd_cols_kernel(const float* __restrict__ dy, int64_t lddy,
                                                                  const float* __restrict__ x, int64_t ldx, int64_t M, int K,
                                                                  const float* __restrict__ rs, int rows_per,
                                                                  float* __restrict__ part) {
    const int k0 = (blockIdx.x * kColThreads + threadIdx.x) * V;
    if (k0 >= K) return;
    float s1[V], s2[V];
#pragma unroll
    for (int i = 0; i < V; ++i) s1[i] = s2[i] = 0.f;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per;
    const int64_t r1 = std::min<int64_t>(M, r0 + rows_per);
    for (int64_t r = r0; r < r1; ++r) {
        typename vec_t<V>::T g = ld<V>(dy + r * lddy + k0), xv = ld<V>(x + r * ldx + k0);
        const float mean = rs[2 * r], rstd = rs[2 * r + 1];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            s1[i] += lane<V>(g, i);
            s2[i] = fmaf(lane<V>(g, i), (lane<V>(xv, i) - mean) * rstd, s2[i]);
        }
    }
    float* o = part + (int64_t)blockIdx.y * 2 * K + k0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        o[i] = s1[i];
        o[K + i] = s2[i];
    }
}

__global__ __launch_bounds__(kFinCols * kFinGroups) void col_sum2_finish_kernel(const float* __restrict__ part, int K,
                                                                                int chunks, float* __restrict__ out0,
                                                                                float* __restrict__ out1) {
    float t[2];
    finish_sums<2>(part, K, chunks, t);
    const int k = blockIdx.x * kFinCols + threadIdx.x;
    if (threadIdx.x < kFinCols && k < K) {
        out0[k] = t[0];
        out1[k] = t[1];
    }
}

}  // namespace

// chunk partials ([chunk][2][K] floats) + rf_bn_bwd's per-column constants (3 K floats)
extern "C" size_t rf_tower_ws_bytes(int64_t M, int32_t K) {
    const size_t k = (size_t)std::max(K, 1);
    return ((size_t)tower_chunks(std::max<int64_t>(M, 1), (int)k) * 2 + 3) * k * sizeof(float);
}

#define RF_TOWER_LAUNCH(kern, V, grid, ...)                                                    \
    do {                                                                                       \
        if (V == 4)                                                                            \
            hipLaunchKernelGGL(kern<4>, grid(4), dim3(256), 0, st, __VA_ARGS__);               \
        else                                                                                   \
            hipLaunchKernelGGL(kern<1>, grid(1), dim3(256), 0, st, __VA_ARGS__);               \
    } while (0)

extern "C" int rf_col_stats(const float* x, int64_t M, int32_t K, int64_t ldx, float* mean, float* var, void* ws,
                            size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && K > 0 && ldx >= K && x && mean && var, "rf_col_stats: bad arguments");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, K), "rf_col_stats: workspace too small");
    const int chunks = tower_chunks(M, K), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(K, {{x, ldx}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((K / v + kColThreads - 1) / kColThreads, chunks); };
    RF_TOWER_LAUNCH(col_stats_partial_kernel, V, grid, x, M, K, ldx, rows_per, (float*)ws);
    hipLaunchKernelGGL(col_stats_finish_kernel, dim3((K + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0, st,
                       (const float*)ws, M, K, chunks, rows_per, mean, var);
    return rf_check_launch("rf_col_stats");
}

extern "C" int rf_bn_fold(const float* W, int32_t N, int32_t K, const float* b, const float* gamma, const float* beta,
                          const float* mean, const float* var, float eps, float* W_out, float* b_out, void* stream) {
    RF_REQUIRE(N > 0 && K > 0 && W && gamma && beta && mean && var && W_out && b_out, "rf_bn_fold: bad arguments");
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(K, {{W, K}, {W_out, K}, {gamma, 0}, {beta, 0}, {mean, 0}, {var, 0}}) ? 4 : 1;
    auto grid = [&](int) { return dim3(N); };
    RF_TOWER_LAUNCH(bn_fold_kernel, V, grid, W, K, b, gamma, beta, mean, var, eps, W_out, b_out);
    return rf_check_launch("rf_bn_fold");
}

extern "C" int rf_bn_fold_grad(const float* G, int32_t N, int32_t K, const float* db, const float* gamma, const float* beta,
                               const float* mean, const float* var, float eps, float* dW, void* stream) {
    RF_REQUIRE(N > 0 && N <= 65535 && K > 0 && G && db && gamma && beta && mean && var && dW, "rf_bn_fold_grad: bad arguments");
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(K, {{G, K}, {dW, K}, {gamma, 0}, {beta, 0}, {mean, 0}, {var, 0}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((K / v + 255) / 256, N); };
    RF_TOWER_LAUNCH(bn_fold_grad_kernel, V, grid, G, N, K, db, gamma, beta, mean, var, eps, dW);
    return rf_check_launch("rf_bn_fold_grad");
}

extern "C" int rf_dropout_fwd(const float* x, int64_t M, int32_t N, int64_t ldx, float rate, uint64_t seed, float* y,
                              int64_t ldy, void* stream) {
    RF_REQUIRE(M >= 0 && M <= 65535 && N > 0 && ldx >= N && ldy >= N && rate >= 0.f && rate < 1.f,
               "rf_dropout_fwd: bad arguments");
    if (M == 0) return RF_OK;
    RF_REQUIRE(x && y, "rf_dropout_fwd: null pointer");
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(N, {{x, ldx}, {y, ldy}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((N / v + 255) / 256, (unsigned)M); };
    RF_TOWER_LAUNCH(dropout_fwd_kernel, V, grid, x, M, N, ldx, rate, seed, y, ldy);
    return rf_check_launch("rf_dropout_fwd");
}

extern "C" int rf_selu_dropout_bwd(const float* dh, int64_t lddh, const float* h, int64_t ldh, int64_t M, int32_t N,
                                   float rate, uint64_t seed, float* dpre, int64_t ldd, float* db, void* ws,
                                   size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && N > 0 && lddh >= N && ldh >= N && ldd >= N && rate >= 0.f && rate < 1.f,
               "rf_selu_dropout_bwd: bad arguments");
    RF_REQUIRE(dh && h && dpre && db, "rf_selu_dropout_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, N), "rf_selu_dropout_bwd: workspace too small");
    const int chunks = tower_chunks(M, N), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(N, {{dh, lddh}, {h, ldh}, {dpre, ldd}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((N / v + kColThreads - 1) / kColThreads, chunks); };
    RF_TOWER_LAUNCH(selu_dropout_bwd_kernel, V, grid, dh, lddh, h, ldh, M, N, rate, seed, rows_per, dpre, ldd, (float*)ws);
    hipLaunchKernelGGL(col_sum_finish_kernel, dim3((N + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0, st,
                       (const float*)ws, N, chunks, db);
    return rf_check_launch("rf_selu_dropout_bwd");
}

extern "C" int rf_bn_bwd(const float* dz, int64_t lddz, const float* x, int64_t ldx, int64_t M, int32_t K, const float* mean,
                         const float* var, const float* gamma, float eps, float* dx, int64_t lddx, float* dgamma,
                         float* dbeta, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && M <= 65535 && K > 0 && lddz >= K && ldx >= K && lddx >= K, "rf_bn_bwd: bad arguments");
    RF_REQUIRE(dz && x && mean && var && gamma && dx && dgamma && dbeta, "rf_bn_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, K), "rf_bn_bwd: workspace too small");
    const int chunks = tower_chunks(M, K), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    float* part = (float*)ws;
    float* ac = part + (size_t)chunks * 2 * K;
    const int V = vec4_ok(K, {{dz, lddz}, {x, ldx}, {dx, lddx}, {mean, 0}, {var, 0}, {ac, 0}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((K / v + kColThreads - 1) / kColThreads, chunks); };
    RF_TOWER_LAUNCH(bn_bwd_partial_kernel, V, grid, dz, lddz, x, ldx, M, K, mean, var, eps, rows_per, part);
    hipLaunchKernelGGL(bn_bwd_finish_kernel, dim3((K + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0, st,
                       (const float*)part, M, K, chunks, gamma, var, eps, dbeta, dgamma, ac);
    auto grid2 = [&](int v) { return dim3((K / v + 255) / 256, (unsigned)M); };
    RF_TOWER_LAUNCH(bn_bwd_apply_kernel, V, grid2, dz, lddz, x, ldx, K, mean, var, eps, (const float*)ac, dx, lddx);
    return rf_check_launch("rf_bn_bwd");
}

extern "C" int rf_act_dropout_fwd(const float* pre, int64_t ldp, int64_t M, int32_t N, int32_t act, float rate, uint64_t seed,
                                  float* h, int64_t ldh, void* stream) {
    RF_REQUIRE(M >= 0 && M <= 65535 && N > 0 && ldp >= N && ldh >= N && rate >= 0.f && rate < 1.f &&
                   act >= RF_ACT_NONE && act < RF_ACT_SOFTMAX,
               "rf_act_dropout_fwd: bad arguments");
    if (M == 0) return RF_OK;
    RF_REQUIRE(pre && h, "rf_act_dropout_fwd: null pointer");
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(N, {{pre, ldp}, {h, ldh}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((N / v + 255) / 256, (unsigned)M); };
    RF_TOWER_LAUNCH(act_dropout_fwd_kernel, V, grid, pre, ldp, N, act, rate, seed, h, ldh);
    return rf_check_launch("rf_act_dropout_fwd");
}

extern "C" int rf_act_dropout_bwd(const float* dh, int64_t lddh, const float* pre, int64_t ldp, int64_t M, int32_t N,
                                  int32_t act, float rate, uint64_t seed, float* dpre, int64_t ldd, float* db, void* ws,
                                  size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && N > 0 && lddh >= N && ldp >= N && ldd >= N && rate >= 0.f && rate < 1.f && act >= RF_ACT_NONE &&
                   act < RF_ACT_SOFTMAX,
               "rf_act_dropout_bwd: bad arguments");
    RF_REQUIRE(dh && pre && dpre && db, "rf_act_dropout_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_tower_ws_bytes(M, N), "rf_act_dropout_bwd: workspace too small");
    const int chunks = tower_chunks(M, N), rows_per = (int)((M + chunks - 1) / chunks);
    hipStream_t st = rf_stream(stream);
    const int V = vec4_ok(N, {{dh, lddh}, {pre, ldp}, {dpre, ldd}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((N / v + kColThreads - 1) / kColThreads, chunks); };
    RF_TOWER_LAUNCH(act_dropout_bwd_kernel, V, grid, dh, lddh, pre, ldp, M, N, act, rate, seed, rows_per, dpre, ldd,
                    (float*)ws);
    hipLaunchKernelGGL(col_sum_finish_kernel, dim3((N + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0, st,
                       (const float*)ws, N, chunks, db);
    return rf_check_launch("rf_act_dropout_bwd");
}

extern "C" size_t rf_layernorm_bwd_ws_bytes(int64_t M, int32_t K) {
    const size_t rows = ((size_t)std::max<int64_t>(M, 1) * 2 * sizeof(float) + 255) & ~(size_t)255;
    return rows + (size_t)tower_chunks(std::max<int64_t>(M, 1), std::max(K, 1)) * 2 * std::max(K, 1) * sizeof(float);
}

extern "C" int rf_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t M, int32_t K,
                                const float* gamma, float eps, float* dx, int64_t lddx, float* dgamma, float* dbeta, void* ws,
                                size_t ws_bytes, void* stream) {
    RF_REQUIRE(M > 0 && M <= (1 << 26) && K > 0 && lddy >= K && ldx >= K && lddx >= K, "rf_layernorm_bwd: bad arguments");
    RF_REQUIRE(dy && x && gamma && dx && dgamma && dbeta, "rf_layernorm_bwd: null pointer");
    RF_REQUIRE(ws && ws_bytes >= rf_layernorm_bwd_ws_bytes(M, K), "rf_layernorm_bwd: workspace too small");
    hipStream_t st = rf_stream(stream);
    float* rs = static_cast<float*>(ws);
    float* part = reinterpret_cast<float*>(static_cast<char*>(ws) + (((size_t)M * 2 * sizeof(float) + 255) & ~(size_t)255));
    hipLaunchKernelGGL(ln_bwd_rows_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, st, dy, lddy, x, ldx, M, K, gamma, eps,
                       dx, lddx, rs);
    const int chunks = tower_chunks(M, K), rows_per = (int)((M + chunks - 1) / chunks);
    const int V = vec4_ok(K, {{dy, lddy}, {x, ldx}}) ? 4 : 1;
    auto grid = [&](int v) { return dim3((K / v + kColThreads - 1) / kColThreads, chunks); };
    RF_TOWER_LAUNCH(ln_bwd_cols_kernel, V, grid, dy, lddy, x, ldx, M, K, (const float*)rs, rows_per, part);
    hipLaunchKernelGGL(col_sum2_finish_kernel, dim3((K + kFinCols - 1) / kFinCols), dim3(kFinCols * kFinGroups), 0, st,
                       (const float*)part, K, chunks, dbeta, dgamma);
    return rf_check_launch("rf_layernorm_bwd");
}
