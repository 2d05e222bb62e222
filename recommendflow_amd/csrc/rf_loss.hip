// rf_loss.hip — the two-tower training losses of SURVEY §8f.1, forward and gradient in one call.
//
// cosent_loss (backend/losses/match_losses.py:42-56):
//   x_ij = scale * (s_i - s_j) for pairs with y_i < y_j (other pairs get -1e12, i.e. exp -> 0)
//   loss = logsumexp([0, x_ij ...]) = m + log(exp(-m) + sum_valid exp(x_ij - m)),  m = max(0, max_valid x_ij)
//   dloss/ds_i = scale * (R_i - C_i) / Z,  R_i = sum_{j: y_i<y_j} e^{x_ij - m},  C_i = sum_{j: y_j<y_i} e^{x_ji - m}
// batch_neg_sample_scaled_multi_class_ce_loss (match_losses.py:150-165, Que2Search):
//   loss = mean_i( -log(exp(s P_ii) / sum_j exp(s P_ij)) * y_i ),  P = query . doc^T (a library GEMM)
//   dloss/dP_ij = s * y_i / B * (softmax_j(s P_i.) - [i == j])
// Deterministic: fixed-order block reductions, no atomics. cosent: (i block, j chunk) tiles of 256 x 64 pairs,
// the j scores and labels staged through LDS; the tile partials are summed in tile order, then row blocks in order.
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

// The B x B pairs run as (i block, j chunk) tiles: grid (ceil(B / 256), ceil(B / 64)), a thread per i walking its
// tile's 64 j through LDS, so a 4096 batch fills 1,024 workgroups (a thread per i over every j kept 16 busy).
constexpr int kCols = 64;  // j per tile

// pass A: per-tile max of the valid x_ij
__global__ __launch_bounds__(kRows) void cosent_max_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                                           int B, float scale, float* __restrict__ part) {
    __shared__ float sj[kCols], yj[kCols];
    __shared__ float red[kRows / 64];
    const int i = blockIdx.x * kRows + threadIdx.x;
    const float si = i < B ? s[i] : 0.f, yi = i < B ? y[i] : 0.f;
    const int j0 = blockIdx.y * kCols;
    if (threadIdx.x < kCols) {
        const int j = j0 + threadIdx.x;
        sj[threadIdx.x] = j < B ? s[j] : 0.f;
        yj[threadIdx.x] = j < B ? y[j] : -INFINITY;
    }
    __syncthreads();
    float m = -INFINITY;
    if (i < B) {
        const int n = min(kCols, B - j0);
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

// m = max(0, every tile maximum): a wave-parallel max over the tile maxima (max is order-free)
__device__ __forceinline__ float cosent_m(const float* __restrict__ part, int nparts) {
    float m = 0.f;
    for (int p = threadIdx.x & 63; p < nparts; p += 64) m = fmaxf(m, part[p]);
    return wave_max(m);
}

// pass B: per-tile partials of R_i and C_i with the global m
__global__ __launch_bounds__(kRows) void cosent_sums_kernel(const float* __restrict__ s, const float* __restrict__ y,
                                                            int B, float scale, const float* __restrict__ part, int nparts,
                                                            float* __restrict__ Rp, float* __restrict__ Cp) {
    __shared__ float sj[kCols], yj[kCols];
    const float m = cosent_m(part, nparts);
    const int i = blockIdx.x * kRows + threadIdx.x;
    const float si = i < B ? s[i] : 0.f, yi = i < B ? y[i] : 0.f;
    const int j0 = blockIdx.y * kCols;
    if (threadIdx.x < kCols) {
        const int j = j0 + threadIdx.x;
        sj[threadIdx.x] = j < B ? s[j] : 0.f;
        yj[threadIdx.x] = j < B ? y[j] : 0.f;
    }
    __syncthreads();
    if (i >= B) return;
    float r = 0.f, c = 0.f;
    const int n = min(kCols, B - j0);
    for (int k = 0; k < n; ++k) {
        if (yi < yj[k]) r += expf(scale * si - scale * sj[k] - m);
        if (yj[k] < yi) c += expf(scale * sj[k] - scale * si - m);
    }
    Rp[(int64_t)blockIdx.y * B + i] = r;
    Cp[(int64_t)blockIdx.y * B + i] = c;
}

// pass C: R_i, C_i = the tile partials summed in tile order; D_i = R_i - C_i and the block's sum of R_i
__global__ __launch_bounds__(kRows) void cosent_rows_kernel(const float* __restrict__ Rp, const float* __restrict__ Cp, int B,
                                                            int nj, float* __restrict__ D, float* __restrict__ rpart) {
    __shared__ float red[kRows / 64];
    const int i = blockIdx.x * kRows + threadIdx.x;
    float r = 0.f, c = 0.f;
    if (i < B)
        for (int t = 0; t < nj; ++t) {
            r += Rp[(int64_t)t * B + i];
            c += Cp[(int64_t)t * B + i];
        }
    if (i < B) D[i] = r - c;
    r = wave_sum(r);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
    __syncthreads();
    if (threadIdx.x == 0) rpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// pass D (one block): Z = e^-m + the row blocks' sums in block order, the loss, ds_i = scale D_i / Z
__global__ __launch_bounds__(1024) void cosent_final_kernel(const float* __restrict__ D, const float* __restrict__ rpart,
                                                            int B, int ni, float scale, const float* __restrict__ part,
                                                            int nparts, float* __restrict__ loss, float* __restrict__ ds) {
    __shared__ float s_z;
    const float m = cosent_m(part, nparts);
    if (threadIdx.x == 0) {
        float z = expf(-m);
        for (int b = 0; b < ni; ++b) z += rpart[b];
        s_z = z;
        *loss = m + logf(z);
    }
    __syncthreads();
    const float z = s_z;
    if (ds)
        for (int i = threadIdx.x; i < B; i += 1024) ds[i] = scale * D[i] / z;
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

// Dense(n, softmax) + sparse categorical cross-entropy (the ESIM click head, esim.py:53,88): Keras computes the CE
// of a softmax output from its logits, so per row loss_b = logsumexp(z_b) - z_b[y_b] and dz_b = (softmax(z_b) -
// onehot(y_b)) / B; the mean over the batch is mean_kernel's fixed-order sum. A label outside [0, n) gives that row
// a NaN loss and NaN gradients (never an out-of-range read).
__global__ __launch_bounds__(256) void softmax_ce_kernel(const float* __restrict__ z, int64_t ld, const int32_t* __restrict__ y,
                                                         int B, int N, float* __restrict__ rows, float* __restrict__ prob,
                                                         int64_t ldp, float* __restrict__ dz, int64_t ldd) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= B) return;
    const float* zr = z + (int64_t)b * ld;
    const int yb = y[b];
    const bool ok = yb >= 0 && yb < N;
    float m = -INFINITY;
    for (int j = 0; j < N; ++j) m = fmaxf(m, zr[j]);
    float s = 0.f;
    for (int j = 0; j < N; ++j) s += expf(zr[j] - m);
    rows[b] = ok ? m + logf(s) - zr[yb] : __builtin_nanf("");
    const float invB = 1.0f / (float)B;
    for (int j = 0; j < N; ++j) {
        const float p = expf(zr[j] - m) / s;
        if (prob) prob[(int64_t)b * ldp + j] = p;
        if (dz) dz[(int64_t)b * ldd + j] = ok ? (p - (j == yb ? 1.f : 0.f)) * invB : __builtin_nanf("");
    }
}

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// ---- l2-normalised row cosine (the DSSM score ahead of cosent_loss) ------------------------------------------
// s_i = <a_i / max(|a_i|, eps), b_i / max(|b_i|, eps)>: K.l2_normalize of both towers (dssm.py:35-36) then the
// row dot product of match_losses.py:46. One wave per row; each lane walks columns lane, lane + 64, ... and the
// three sums meet in a fixed butterfly (deterministic). nrm[2i], nrm[2i+1] = the unclamped |a_i|, |b_i|.
__global__ __launch_bounds__(256) void cosine_rows_fwd_kernel(const float* __restrict__ a, int64_t lda,
                                                              const float* __restrict__ b, int64_t ldb, int B, int N,
                                                              float eps, float* __restrict__ s, float* __restrict__ nrm) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= B) return;
    const float* ai = a + (int64_t)i * lda;
    const float* bi = b + (int64_t)i * ldb;
    float aa = 0.f, bb = 0.f, ab = 0.f;
    for (int j = lane; j < N; j += 64) {
        const float x = ai[j], y = bi[j];
        aa += x * x;
        bb += y * y;
        ab += x * y;
    }
    aa = wave_sum(aa);
    bb = wave_sum(bb);
    ab = wave_sum(ab);
    if (lane == 0) {
        const float ra = sqrtf(aa), rb = sqrtf(bb);
        s[i] = ab / (fmaxf(ra, eps) * fmaxf(rb, eps));
        nrm[2 * i] = ra;
        nrm[2 * i + 1] = rb;
    }
}

// d s_i / d a_i = (v_i - s_i u_i) / |a_i| while |a_i| > eps (the normalisation's Jacobian (I - u u^T) / |a|), and
// v_i / eps where the norm is clamped (u = a / eps is linear in a); likewise for b. da_i = g * ds_i * that, with ds
// the loss's per-score gradient and g the upstream scalar (*gscale, device) — the cosent backward fused in.
__global__ __launch_bounds__(256) void cosine_rows_bwd_kernel(const float* __restrict__ a, int64_t lda,
                                                              const float* __restrict__ b, int64_t ldb, int B, int N,
                                                              float eps, const float* __restrict__ s,
                                                              const float* __restrict__ nrm, const float* __restrict__ ds,
                                                              const float* __restrict__ gscale, float* __restrict__ da,
                                                              int64_t ldda, float* __restrict__ db, int64_t lddb) {
    const int lane = threadIdx.x & 63;
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= B) return;
    const float ra = nrm[2 * i], rb = nrm[2 * i + 1];
    const float na = fmaxf(ra, eps), nb = fmaxf(rb, eps);
    const float si = s[i];
    const float g = ds[i] * (gscale ? *gscale : 1.f);
    const bool ca = ra > eps, cb = rb > eps;  // unclamped
    const float* ai = a + (int64_t)i * lda;
    const float* bi = b + (int64_t)i * ldb;
    for (int j = lane; j < N; j += 64) {
        const float u = ai[j] / na, v = bi[j] / nb;
        da[(int64_t)i * ldda + j] = g * (ca ? (v - si * u) / na : v / eps);
        db[(int64_t)i * lddb + j] = g * (cb ? (u - si * v) / nb : u / eps);
    }
}

}  // namespace

extern "C" int rf_cosine_rows_fwd(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t batch, int32_t n,
                                  float eps, float* score, float* norms, void* stream) {
    RF_REQUIRE(batch >= 0 && n >= 1 && lda >= n && ldb >= n, "rf_cosine_rows_fwd: bad shape");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(a && b && score && norms, "rf_cosine_rows_fwd: null pointer");
    hipLaunchKernelGGL(cosine_rows_fwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, rf_stream(stream), a, lda, b, ldb,
                       batch, n, eps, score, norms);
    return rf_check_launch("rf_cosine_rows_fwd");
}

extern "C" int rf_cosine_rows_bwd(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t batch, int32_t n,
                                  float eps, const float* score, const float* norms, const float* dscore,
                                  const float* gscale, float* da, int64_t ldda, float* db, int64_t lddb, void* stream) {
    RF_REQUIRE(batch >= 0 && n >= 1 && lda >= n && ldb >= n && ldda >= n && lddb >= n, "rf_cosine_rows_bwd: bad shape");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(a && b && score && norms && dscore && da && db, "rf_cosine_rows_bwd: null pointer");
    hipLaunchKernelGGL(cosine_rows_bwd_kernel, dim3((batch + 3) / 4), dim3(256), 0, rf_stream(stream), a, lda, b, ldb,
                       batch, n, eps, score, norms, dscore, gscale, da, ldda, db, lddb);
    return rf_check_launch("rf_cosine_rows_bwd");
}

// tile maxima (ni x nj) | Rp, Cp (nj x B each) | D (B) | row-block sums (ni); also the in-batch CE's row losses
extern "C" size_t rf_loss_ws_bytes(int32_t batch) {
    if (batch < 0) return 0;
    const size_t B = (size_t)std::max(batch, 1), ni = (B + kRows - 1) / kRows, nj = (B + kCols - 1) / kCols;
    return a256(ni * nj * 4) + 2 * a256(nj * B * 4) + a256(B * 4) + a256(ni * 4);
}

extern "C" int rf_cosent_loss(const float* score, const float* label, int32_t batch, float scale, float* loss, float* dscore,
                              void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(batch >= 1, "rf_cosent_loss: batch must be >= 1");
    RF_REQUIRE(score && label && loss && ws, "rf_cosent_loss: null pointer");
    RF_REQUIRE(ws_bytes >= rf_loss_ws_bytes(batch), "rf_cosent_loss: workspace too small");
    hipStream_t st = rf_stream(stream);
    const size_t B = (size_t)batch;
    const int ni = (batch + kRows - 1) / kRows, nj = (batch + kCols - 1) / kCols;
    char* w = static_cast<char*>(ws);
    float* part = reinterpret_cast<float*>(w);
    w += a256((size_t)ni * nj * 4);
    float* Rp = reinterpret_cast<float*>(w);
    w += a256((size_t)nj * B * 4);
    float* Cp = reinterpret_cast<float*>(w);
    w += a256((size_t)nj * B * 4);
    float* D = reinterpret_cast<float*>(w);
    w += a256(B * 4);
    float* rpart = reinterpret_cast<float*>(w);
    const dim3 g(ni, nj);
    hipLaunchKernelGGL(cosent_max_kernel, g, dim3(kRows), 0, st, score, label, batch, scale, part);
    hipLaunchKernelGGL(cosent_sums_kernel, g, dim3(kRows), 0, st, score, label, batch, scale, part, ni * nj, Rp, Cp);
    hipLaunchKernelGGL(cosent_rows_kernel, dim3(ni), dim3(kRows), 0, st, Rp, Cp, batch, nj, D, rpart);
    hipLaunchKernelGGL(cosent_final_kernel, dim3(1), dim3(1024), 0, st, D, rpart, batch, ni, scale, part, ni * nj, loss, dscore);
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

extern "C" int rf_softmax_ce_loss(const float* logits, int64_t ld, const int32_t* label, int32_t batch, int32_t n_classes,
                                  float* loss, float* prob, int64_t ldp, float* dlogits, int64_t ldd, void* ws, size_t ws_bytes,
                                  void* stream) {
    RF_REQUIRE(batch >= 1 && n_classes >= 1 && ld >= n_classes && (!prob || ldp >= n_classes) &&
                   (!dlogits || ldd >= n_classes),
               "rf_softmax_ce_loss: bad shape");
    RF_REQUIRE(logits && label && loss && ws, "rf_softmax_ce_loss: null pointer");
    RF_REQUIRE(ws_bytes >= rf_loss_ws_bytes(batch), "rf_softmax_ce_loss: workspace too small");
    hipStream_t st = rf_stream(stream);
    float* rows = static_cast<float*>(ws);
    hipLaunchKernelGGL(softmax_ce_kernel, dim3((batch + 255) / 256), dim3(256), 0, st, logits, ld, label, batch, n_classes, rows,
                       prob, ldp, dlogits, ldd);
    hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(1024), 0, st, rows, batch, loss);
    return rf_check_launch("rf_softmax_ce_loss");
}
