// rf_esim_train.hip — the ESIM ranking model's attention block under model.fit, exact fp32 (models/ranking/esim.py:78-84
// trained by example/ranking_search/train.py:96-104 with Keras' float32 graph).
//
// Forward (SoftAttention, attention_layers.py:33-74, and the ESIM combine + pooling, esim.py:79-84), per example:
//   E[i][j] = a_i . q_j, S = softmax_j(E), att_q = S q, att_a = S a,
//   m_q = [q, att_q, q - att_q, q * att_q] (4L rows), avg_q / max_q over them (likewise m_a),
//   pooled = [avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a].
// TF's reduce_max gradient splits the gradient evenly over the elements equal to the maximum (_MinOrMaxGrad), so the
// forward also writes, per (example, side, column), how many of the 4L candidates equal the maximum (aux).
//
// Layout of the work: one eight-wave workgroup per example; q and a staged in LDS (fp32, rows padded to 16, row
// stride D + 4 floats); a wave owns a 16-column strip of i (rows of a) at a time and every product is a
// v_mfma_f32_16x16x4_f32 (exact fp32 products and accumulation, no xf32 on gfx950):
//   X = E^T strip [j][i] = q a^T       (A = q rows, B = a rows of the strip: both k-contiguous, float4 LDS reads)
//   softmax over j = down X's columns  (registers, then the two lane-group shuffles)
//   att_q^T [c][i] = q^T S^T           (S^T stays in the accumulator registers: its C layout IS the B operand of
//                                       the next product with the k order permuted to j = 16 jt + 4 g + r)
// Backward, stage 1 (same strip walk): the pooled gradient -> G_q = d/d att_q, G_a = d/d att_a and the direct terms
// of dq, da (avg: q * att and 2 q + q * att; max: the tied candidates' shares); dS^T = q G_q^T + a G_a^T, the softmax
// backward dE^T = S^T (dS^T - sum_j S^T dS^T); the strip-local da_i += sum_j dE_ij q_j. S^T, dE^T, G_q^T, G_a^T go
// to a workspace. Stage 2 (one workgroup per example): the products that sum over every strip,
//   dq_j += sum_i S_ij G_q,i + sum_i dE_ij a_i,   da_j += sum_i S_ij G_a,i,
// added onto stage 1's outputs (stream order makes the read-modify-write safe). Deterministic: fixed strip order,
// fixed k order, no atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "rf_common.h"

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mf(float a, float b, f4v c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ f4v zero4() { return f4v{0.f, 0.f, 0.f, 0.f}; }

template <int D>
struct Ex {
    static constexpr int RS = D + 4;  // LDS row stride (floats)
};

// stage rows [0, Lp) of one example's q and a into LDS (rows >= L zero)
// kStageBatch chunks per thread are loaded before any is written to LDS: a load -> write loop waits out one HBM round
// trip per chunk (14 of them per example at 112 x 128 with 512 threads)
constexpr int kStageBatch = 8;
template <int D, int NT>
__device__ __forceinline__ void stage_qa(const float* __restrict__ q, const float* __restrict__ a, int64_t ld, int L, int Lp,
                                         float* qs, float* as) {
    constexpr int RS = Ex<D>::RS, C4 = D / 4;
    const int n = 2 * Lp * C4;
    for (int t0 = threadIdx.x; t0 < n; t0 += kStageBatch * NT) {
        float4 v[kStageBatch];
#pragma unroll
        for (int b = 0; b < kStageBatch; ++b) {
            const int t = t0 + b * NT;
            const int side = t / (Lp * C4), rem = t - side * Lp * C4, r = rem / C4, c4 = rem - r * C4;
            v[b] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t < n && r < L) v[b] = *reinterpret_cast<const float4*>((side ? a : q) + (int64_t)r * ld + 4 * c4);
        }
#pragma unroll
        for (int b = 0; b < kStageBatch; ++b) {
            const int t = t0 + b * NT;
            const int side = t / (Lp * C4), rem = t - side * Lp * C4, r = rem / C4, c4 = rem - r * C4;
            if (t < n) *reinterpret_cast<float4*>((side ? as : qs) + r * RS + 4 * c4) = v[b];
        }
    }
}

__device__ __forceinline__ f4v lds4(const float* p) { return *reinterpret_cast<const f4v*>(p); }

// One strip's scores: S^T [NJ] (C layout: j = 16 jt + 4 g + r, i = ibase + li); the attention output is taken per
// 16-column tile from them (att_tile, or the forward's transposed tile).
// NJ (= Lp / 16 <= kMaxJ) is a runtime value: the j-tile loops are unrolled to kMaxJ with uniform guards, so each
// kernel holds one copy of its code (a copy per tile count put 140K lines of ISA in the forward and thrashed the
// instruction cache)
constexpr int kMaxJ = 8;
template <int D>
__device__ __forceinline__ void strip_scores(const float* qs, const float* as, int L, int NJ, int ibase, int li, int g,
                                             f4v (&S)[kMaxJ]) {
    constexpr int RS = Ex<D>::RS;
    // X = E^T strip
    f4v ar[D / 16];
#pragma unroll
    for (int k = 0; k < D / 16; ++k) ar[k] = lds4(as + (ibase + li) * RS + 16 * k + 4 * g);
    // two j tiles per pass: two independent accumulator chains (16x16x4 f32: 40-cycle dependent latency, 32-cycle issue)
#pragma unroll
    for (int jt = 0; jt < kMaxJ; jt += 2) {
        f4v acc0 = zero4(), acc1 = zero4();
        if (jt < NJ) {
            const bool two = jt + 1 < NJ;
#pragma unroll
            for (int k = 0; k < D / 16; ++k) {
                const f4v q0 = lds4(qs + (16 * jt + li) * RS + 16 * k + 4 * g);
                const f4v q1 = two ? lds4(qs + (16 * (jt + 1) + li) * RS + 16 * k + 4 * g) : zero4();
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    acc0 = mf(q0[s], ar[k][s], acc0);
                    acc1 = mf(q1[s], ar[k][s], acc1);
                }
            }
        }
        S[jt] = acc0;
        S[jt + 1] = acc1;
    }
    // softmax over j (rows of X) for every column i: max, exp, sum, divide (attention_layers.py:70-72)
    float m = -INFINITY;
#pragma unroll
    for (int jt = 0; jt < kMaxJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (16 * jt + 4 * g + r < L) m = fmaxf(m, S[jt][r]);
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float sum = 0.f;
#pragma unroll
    for (int jt = 0; jt < kMaxJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const float e = 16 * jt + 4 * g + r < L ? expf(S[jt][r] - m) : 0.f;
            S[jt][r] = e;
            sum += e;
        }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
#pragma unroll
    for (int jt = 0; jt < kMaxJ; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) S[jt][r] = S[jt][r] / sum;
}

// column tile ct of att^T = x^T S^T for x = q and a (A[c][j] = x[j][c], k order j = 16 jt + 4 g + r): two chains
template <int D>
__device__ __forceinline__ void att_tile(const float* qs, const float* as, int NJ, int ct, int li, int g,
                                         const f4v (&S)[kMaxJ], f4v& aq, f4v& aa) {
    constexpr int RS = Ex<D>::RS;
    aq = zero4();
    aa = zero4();
#pragma unroll
    for (int jt = 0; jt < kMaxJ; ++jt)
        if (jt < NJ) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 * jt + 4 * g + r;
                aq = mf(qs[j * RS + 16 * ct + li], S[jt][r], aq);
                aa = mf(as[j * RS + 16 * ct + li], S[jt][r], aa);
            }
        }
}

// (max, count) fold of the candidates equal to the maximum (exact comparisons: any combine order gives the same pair);
// selects, no branches
__device__ __forceinline__ void mc_merge(float& m, float& c, float m2, float c2) {
    const bool gt = m2 > m, eq = m2 == m;
    c = gt ? c2 : (eq ? c + c2 : c);
    m = gt ? m2 : m;
}

// per-wave partials of the pooled statistics in LDS: [wave][side][sum | max | count][D]. Eight waves (two per SIMD:
// one wave's LDS waits under the other's MFMAs; the forward needs < 256 registers), a strip per wave for L <= 128.
constexpr int kFwdWaves = 8;
template <int D>
__global__ __launch_bounds__(kFwdWaves * 64) void esim_train_fwd_kernel(const float* __restrict__ q, const float* __restrict__ a,
                                                                  int L, int64_t ex_stride, int64_t ld, float* __restrict__ out,
                                                                  int64_t out_stride, int64_t out_off, float* __restrict__ aux) {
    constexpr int RS = Ex<D>::RS;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int Lp = (L + 15) & ~15, NS = Lp / 16;
    float* qs = sm;
    float* as = qs + Lp * RS;
    float* part = as + Lp * RS;  // [kFwdWaves][2][3][D]
    const int64_t e = blockIdx.x;
    stage_qa<D, kFwdWaves * 64>(q + e * ex_stride, a + e * ex_stride, ld, L, Lp, qs, as);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    // [wave][side][stat][D]: (sum, max, count) = (0, -inf, 0)
    for (int t = threadIdx.x; t < kFwdWaves * 6 * D; t += kFwdWaves * 64) part[t] = (t / D) % 3 == 1 ? -INFINITY : 0.f;
    __syncthreads();
    for (int s = wave; s < NS; s += kFwdWaves) {
        const int ibase = 16 * s;
        f4v S[kMaxJ];
        strip_scores<D>(qs, as, L, NS, ibase, li, g, S);
#pragma unroll
        for (int ct2 = 0; ct2 < D / 16; ct2 += 2) {
            // att[i][c] (not att^T): S^T's C layout is the A operand of att = S x (k order j = 16 jt + 4 g + r), x the
            // B operand, so this lane holds rows i = ibase + 4 g + r of column c = 16 ct + li: the pooling over i is
            // four rows in the lane and two lane swaps, instead of a 16-lane reduction per (row, column) value.
            // Two column tiles at a time: four independent accumulator chains
            f4v at4[2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) at4[h][0] = at4[h][1] = zero4();
#pragma unroll
            for (int jt = 0; jt < kMaxJ; ++jt)
                if (jt < NS) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int j = 16 * jt + 4 * g + r;
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            at4[h][0] = mf(S[jt][r], qs[j * RS + 16 * (ct2 + h) + li], at4[h][0]);
                            at4[h][1] = mf(S[jt][r], as[j * RS + 16 * (ct2 + h) + li], at4[h][1]);
                        }
                    }
                }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
            const int ct = ct2 + h;
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const float* xs = side ? as : qs;
                const f4v at = at4[h][side];
                float sum = 0.f, cand[16];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = ibase + 4 * g + r;
                    const bool ok = i < L;
                    const float x = xs[i * RS + 16 * ct + li];
                    if (ok) sum += 2.f * x + x * at[r];
                    cand[4 * r] = ok ? x : -INFINITY;
                    cand[4 * r + 1] = ok ? at[r] : -INFINITY;
                    cand[4 * r + 2] = ok ? x - at[r] : -INFINITY;
                    cand[4 * r + 3] = ok ? x * at[r] : -INFINITY;
                }
                float mx = cand[0];
#pragma unroll
                for (int k = 1; k < 16; ++k) mx = fmaxf(mx, cand[k]);
                mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
                mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
                // the candidates equal to the strip's maximum (masked rows are -inf: never equal to a finite maximum)
                float cnt = 0.f;
#pragma unroll
                for (int k = 0; k < 16; ++k) cnt += (cand[k] == mx && cand[k] != -INFINITY) ? 1.f : 0.f;
                cnt += __shfl_xor(cnt, 16, 64);
                cnt += __shfl_xor(cnt, 32, 64);
                sum += __shfl_xor(sum, 16, 64);
                sum += __shfl_xor(sum, 32, 64);
                if (g == 0) {
                    float* p = part + ((wave * 2 + side) * 3) * D + 16 * ct + li;
                    p[0] += sum;
                    mc_merge(p[D], p[2 * D], mx, cnt);
                }
            }
            }
        }
    }
    __syncthreads();
    // combine the waves in order; pooled = [avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a]
    const float inv = 1.0f / (float)(4 * L);
    for (int c = threadIdx.x; c < D; c += kFwdWaves * 64) {
        float avg[2], mx[2], cn[2];
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            float s = 0.f, m = -INFINITY, k = 0.f;
            for (int w = 0; w < kFwdWaves; ++w) {
                const float* p = part + ((w * 2 + side) * 3) * D + c;
                s += p[0];
                mc_merge(m, k, p[D], p[2 * D]);
            }
            avg[side] = s * inv;
            mx[side] = m;
            cn[side] = k;
        }
        float* o = out + e * out_stride + out_off;
        o[c] = avg[0];
        o[D + c] = mx[0];
        o[2 * D + c] = avg[1];
        o[3 * D + c] = mx[1];
        o[4 * D + c] = avg[0] - avg[1];
        o[5 * D + c] = mx[0] - mx[1];
        aux[e * 2 * D + c] = cn[0];
        aux[e * 2 * D + D + c] = cn[1];
    }
}

// ---- backward, stage 1 -----------------------------------------------------------------------------------------
// workspace per example: S^T [Lp][Lp] ([j][i]), dE^T [Lp][Lp], G_q^T [D][Lp] ([c][i]), G_a^T [D][Lp]
// Eight waves (two per SIMD; the q / a images cap the kernel at one workgroup per CU), a strip each for L <= 128: the
// attention output is produced one 16-column tile at a time inside the gradient loop, so a wave holds S^T, dS^T and
// one tile of att instead of all of att (the four-wave form held att whole and ran one wave per SIMD)
#ifndef RF_BWD1_WAVES
#define RF_BWD1_WAVES 8
#endif
constexpr int kBwd1Waves = RF_BWD1_WAVES;
template <int D>
__global__ __launch_bounds__(kBwd1Waves * 64) void esim_train_bwd1_kernel(const float* __restrict__ q, const float* __restrict__ a,
                                                                   int L, int64_t ex_stride, int64_t ld,
                                                                   const float* __restrict__ pooled, int64_t p_stride,
                                                                   int64_t p_off, const float* __restrict__ dpooled,
                                                                   int64_t dp_stride, int64_t dp_off,
                                                                   const float* __restrict__ aux, float* __restrict__ dq,
                                                                   float* __restrict__ da, int64_t g_ex, int64_t ldg,
                                                                   float* __restrict__ ws) {
    constexpr int RS = Ex<D>::RS;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int Lp = (L + 15) & ~15, NS = Lp / 16;
    float* qs = sm;
    float* as = qs + Lp * RS;
    float* gc = as + Lp * RS;  // per column: gavg_q, gmax_q, M_q, gavg_a, gmax_a, M_a  [6][D]
    const int64_t e = blockIdx.x;
    stage_qa<D, kBwd1Waves * 64>(q + e * ex_stride, a + e * ex_stride, ld, L, Lp, qs, as);
    {
        const float inv = 1.0f / (float)(4 * L);
        const float* dp = dpooled + e * dp_stride + dp_off;
        const float* pp = pooled + e * p_stride + p_off;
        const float* cn = aux + e * 2 * D;
        for (int c = threadIdx.x; c < D; c += kBwd1Waves * 64) {
            const float d0 = dp[c], d1 = dp[D + c], d2 = dp[2 * D + c], d3 = dp[3 * D + c], d4 = dp[4 * D + c], d5 = dp[5 * D + c];
            gc[c] = (d0 + d4) * inv;
            gc[D + c] = (d1 + d5) / cn[c];
            gc[2 * D + c] = pp[D + c];
            gc[3 * D + c] = (d2 - d4) * inv;
            gc[4 * D + c] = (d3 - d5) / cn[D + c];
            gc[5 * D + c] = pp[3 * D + c];
        }
    }
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    float* wsS = ws + e * (int64_t)(2 * Lp * Lp + 2 * D * Lp);
    float* wsE = wsS + Lp * Lp;
    float* wsGq = wsE + Lp * Lp;
    float* wsGa = wsGq + D * Lp;
    for (int s = wave; s < NS; s += kBwd1Waves) {
        const int ibase = 16 * s, i = ibase + li;
        f4v S[kMaxJ];
        strip_scores<D>(qs, as, L, NS, ibase, li, g, S);
        // per 16-column tile of c: the tile of att, the pooled gradient's terms (G = d/d att, the direct d/d x), the direct terms
        // stored at once, G^T to the workspace, and dS^T[j][i] += sum_c x[j][c] G^T[c][i] for x = q, a
        // (A = x rows, k order c = 16 ct + 4 g + r); one tile's G / direct values live at a time
        f4v dS[kMaxJ];
#pragma unroll
        for (int jt = 0; jt < kMaxJ; ++jt) dS[jt] = zero4();
#pragma unroll
        for (int ct = 0; ct < D / 16; ++ct) {
            f4v attq, atta;
            att_tile<D>(qs, as, NS, ct, li, g, S, attq, atta);
            const f4v qv = lds4(qs + i * RS + 16 * ct + 4 * g), av = lds4(as + i * RS + 16 * ct + 4 * g);
            f4v G[2], Dx[2];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * ct + 4 * g + r;
#pragma unroll
                for (int side = 0; side < 2; ++side) {
                    const float x = side ? av[r] : qv[r], at = side ? atta[r] : attq[r];
                    const float gavg = gc[3 * side * D + c], gmax = gc[(3 * side + 1) * D + c], M = gc[(3 * side + 2) * D + c];
                    float gatt = 0.f, gx = 0.f;
                    if (i < L) {
                        const float dif = x - at, prd = x * at;
                        // avg: sum(x) + sum(at) + sum(x - at) + sum(x at) over 4L rows
                        gatt = x * gavg;
                        gx = (2.f + at) * gavg;
                        // max: an even share for every candidate equal to the maximum
                        if (x == M) gx += gmax;
                        if (at == M) gatt += gmax;
                        if (dif == M) {
                            gx += gmax;
                            gatt -= gmax;
                        }
                        if (prd == M) {
                            gx += gmax * at;
                            gatt += gmax * x;
                        }
                    }
                    G[side][r] = gatt;
                    Dx[side][r] = gx;
                }
            }
            // direct terms of rows i < L (float4 over r: c = 16 ct + 4 g .. + 3); da gets the strip-local
            // product added below by this same lane
            if (i < L) {
                *reinterpret_cast<f4v*>(dq + e * g_ex + (int64_t)i * ldg + 16 * ct + 4 * g) = Dx[0];
                *reinterpret_cast<f4v*>(da + e * g_ex + (int64_t)i * ldg + 16 * ct + 4 * g) = Dx[1];
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * ct + 4 * g + r;
                wsGq[c * Lp + i] = G[0][r];
                wsGa[c * Lp + i] = G[1][r];
            }
#pragma unroll
            for (int jt = 0; jt < kMaxJ; ++jt) {
                if (jt < NS) {
                    const f4v xq = lds4(qs + (16 * jt + li) * RS + 16 * ct + 4 * g);
                    const f4v xa = lds4(as + (16 * jt + li) * RS + 16 * ct + 4 * g);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        dS[jt] = mf(xq[r], G[0][r], dS[jt]);
                        dS[jt] = mf(xa[r], G[1][r], dS[jt]);
                    }
                }
            }
        }
        // softmax backward down each column i: dE = S (dS - sum_j S dS)
        float t = 0.f;
#pragma unroll
        for (int jt = 0; jt < kMaxJ; ++jt)
#pragma unroll
            for (int r = 0; r < 4; ++r) t += S[jt][r] * dS[jt][r];
        t += __shfl_xor(t, 16, 64);
        t += __shfl_xor(t, 32, 64);
#pragma unroll
        for (int jt = 0; jt < kMaxJ; ++jt)
#pragma unroll
            for (int r = 0; r < 4; ++r) dS[jt][r] = S[jt][r] * (dS[jt][r] - t);
        // workspace: S^T[j][i], dE^T[j][i] (j = 16 jt + 4 g + r)
#pragma unroll
        for (int jt = 0; jt < kMaxJ; ++jt)
            if (jt < NS) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 * jt + 4 * g + r;
                    wsS[j * Lp + i] = S[jt][r];
                    wsE[j * Lp + i] = dS[jt][r];
                }
            }
        // strip-local: da_i += sum_j dE^T[j][i] q_j  (da^T[c][i], A[c][j] = q[j][c])
        f4v* drow = reinterpret_cast<f4v*>(da + e * g_ex + (int64_t)(i < L ? i : 0) * ldg + 4 * g);
#pragma unroll
        for (int ct = 0; ct < D / 16; ct += 2) {
            // two tiles at a time (two independent accumulator chains); their direct terms loaded before the MFMAs
            const f4v p0 = i < L ? drow[4 * ct] : zero4();
            const f4v p1 = i < L ? drow[4 * ct + 4] : zero4();
            f4v acc0 = zero4(), acc1 = zero4();
#pragma unroll
            for (int jt = 0; jt < kMaxJ; ++jt)
                if (jt < NS) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float* qr = qs + (16 * jt + 4 * g + r) * RS + li;
                        acc0 = mf(qr[16 * ct], dS[jt][r], acc0);
                        acc1 = mf(qr[16 * ct + 16], dS[jt][r], acc1);
                    }
                }
            if (i < L) {
                drow[4 * ct] = p0 + acc0;
                drow[4 * ct + 4] = p1 + acc1;
            }
        }
    }
}

// ---- backward, stage 2: dq_j += sum_i S_ij G_q,i + dE_ij a_i, da_j += sum_i S_ij G_a,i ---------------------------
// D[j][c] tiles: A[j][i] = S^T / dE^T rows (float4 over i = 16 it + 4 g + s, from the workspace, one tile ahead),
// B[i][c] = G^T[c][i] and a[i][c] from LDS. The columns run in two halves: a half's G_q^T, G_a^T and a are staged in
// LDS once and read by every j tile (the round-one kernel read G^T from L2 once per j tile: 72 % of its wave cycles
// waited on those loads). Eight waves, a j tile each (7 at L = 100).
constexpr int kBwd2Waves = 8;
template <int D>
__global__ __launch_bounds__(kBwd2Waves * 64) void esim_train_bwd2_kernel(const float* __restrict__ a, int L, int64_t ex_stride,
                                                                          int64_t ld, const float* __restrict__ ws,
                                                                          float* __restrict__ dq, float* __restrict__ da,
                                                                          int64_t g_ex, int64_t ldg) {
    constexpr int H = D / 2, NT = kBwd2Waves * 64, HS = H + 4;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    const int Lp = (L + 15) & ~15, NS = Lp / 16, GS = Lp + 4;  // G^T row stride in LDS
    float* gq = sm;             // [H][GS]
    float* ga = gq + H * GS;    // [H][GS]
    float* as = ga + H * GS;    // [Lp][HS]
    const int64_t e = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    const float* wsS = ws + e * (int64_t)(2 * Lp * Lp + 2 * D * Lp);
    const float* wsE = wsS + Lp * Lp;
    const float* wsGq = wsE + Lp * Lp;
    const float* wsGa = wsGq + D * Lp;
    const float* ae = a + e * ex_stride;
    for (int half = 0; half < 2; ++half) {
        const int c0 = half * H;
        if (half) __syncthreads();  // the first half's reads are done
        // G_q^T, G_a^T and a of this half: every chunk of a batch loaded before any LDS write (see stage_qa)
        const int ng = 2 * H * (Lp / 4), na = Lp * (H / 4);
        for (int t0 = threadIdx.x; t0 < ng + na; t0 += kStageBatch * NT) {
            f4v v[kStageBatch];
#pragma unroll
            for (int b = 0; b < kStageBatch; ++b) {
                const int t = t0 + b * NT;
                v[b] = zero4();
                if (t < ng) {
                    const int side = t / (H * (Lp / 4)), rem = t - side * H * (Lp / 4), c = rem / (Lp / 4), i4 = rem - c * (Lp / 4);
                    v[b] = lds4((side ? wsGa : wsGq) + (int64_t)(c0 + c) * Lp + 4 * i4);
                } else if (t < ng + na) {
                    const int r = (t - ng) / (H / 4), c4 = (t - ng) - r * (H / 4);
                    if (r < L) v[b] = lds4(ae + (int64_t)r * ld + c0 + 4 * c4);
                }
            }
#pragma unroll
            for (int b = 0; b < kStageBatch; ++b) {
                const int t = t0 + b * NT;
                if (t < ng) {
                    const int side = t / (H * (Lp / 4)), rem = t - side * H * (Lp / 4), c = rem / (Lp / 4), i4 = rem - c * (Lp / 4);
                    *reinterpret_cast<f4v*>((side ? ga : gq) + c * GS + 4 * i4) = v[b];
                } else if (t < ng + na) {
                    const int r = (t - ng) / (H / 4), c4 = (t - ng) - r * (H / 4);
                    *reinterpret_cast<f4v*>(as + r * HS + 4 * c4) = v[b];
                }
            }
        }
        __syncthreads();
        for (int jt = wave; jt < NS; jt += kBwd2Waves) {
            f4v accq[H / 16], acca[H / 16];
#pragma unroll
            for (int ct = 0; ct < H / 16; ++ct) accq[ct] = acca[ct] = zero4();
            f4v nS = lds4(wsS + (16 * jt + li) * Lp + 4 * g), nE = lds4(wsE + (16 * jt + li) * Lp + 4 * g);
            for (int it = 0; it < NS; ++it) {
                const f4v sS = nS, sE = nE;
                if (it + 1 < NS) {
                    nS = lds4(wsS + (16 * jt + li) * Lp + 16 * (it + 1) + 4 * g);
                    nE = lds4(wsE + (16 * jt + li) * Lp + 16 * (it + 1) + 4 * g);
                }
#pragma unroll
                for (int ct = 0; ct < H / 16; ++ct) {
                    const f4v bq = lds4(gq + (16 * ct + li) * GS + 16 * it + 4 * g);
                    const f4v ba = lds4(ga + (16 * ct + li) * GS + 16 * it + 4 * g);
#pragma unroll
                    for (int s = 0; s < 4; ++s) {
                        accq[ct] = mf(sS[s], bq[s], accq[ct]);
                        accq[ct] = mf(sE[s], as[(16 * it + 4 * g + s) * HS + 16 * ct + li], accq[ct]);
                        acca[ct] = mf(sS[s], ba[s], acca[ct]);
                    }
                }
            }
            // stage 1's values of this lane's 2 x H / 16 x 4 outputs loaded together, then the adds and stores
            float oq[H / 16][4], oa[H / 16][4];
#pragma unroll
            for (int ct = 0; ct < H / 16; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 * jt + 4 * g + r;
                    const int64_t o = e * g_ex + (int64_t)min(j, L - 1) * ldg + c0 + 16 * ct + li;
                    oq[ct][r] = dq[o];
                    oa[ct][r] = da[o];
                }
#pragma unroll
            for (int ct = 0; ct < H / 16; ++ct)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int j = 16 * jt + 4 * g + r;
                    if (j < L) {
                        const int64_t o = e * g_ex + (int64_t)j * ldg + c0 + 16 * ct + li;
                        dq[o] = oq[ct][r] + accq[ct][r];
                        da[o] = oa[ct][r] + acca[ct][r];
                    }
                }
        }
    }
}

template <class K>
int set_lds(K kern, size_t bytes) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)bytes);
    return e == hipSuccess ? RF_OK : rf_set_error(RF_EHIP, "esim_train: LDS attribute: %s", hipGetErrorString(e));
}

size_t qa_lds_bytes(int L, int d) { return (size_t)2 * ((L + 15) & ~15) * (d + 4) * sizeof(float); }

}  // namespace

extern "C" size_t rf_esim_train_ws_bytes(int32_t batch, int32_t L, int32_t d) {
    const int64_t Lp = (std::max(L, 1) + 15) & ~15;
    return (size_t)std::max(batch, 0) * (size_t)(2 * Lp * Lp + 2 * (int64_t)d * Lp) * sizeof(float);
}

#define RF_ESIM_TRAIN_CHECK(name)                                                                                      \
    RF_REQUIRE(L >= 1 && L <= 128 && (d == 64 || d == 128) && batch >= 0, name ": need 1 <= L <= 128, d 64 or 128");  \
    RF_REQUIRE(ld >= d && ld % 4 == 0 && ex_stride % 4 == 0 && ex_stride >= (int64_t)(L - 1) * ld + d,                 \
               name ": ld / ex_stride must be multiples of 4 floats covering the L x d rows");                         \
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)a & 15) == 0, name ": q / a must be 16-byte aligned")

extern "C" int rf_esim_train_fwd_f32(const float* q, const float* a, int32_t batch, int32_t L, int32_t d, int64_t ex_stride,
                                     int64_t ld, float* out, int64_t out_stride, int64_t out_off, float* aux, void* stream) {
    RF_ESIM_TRAIN_CHECK("rf_esim_train_fwd_f32");
    RF_REQUIRE(out_stride >= out_off + 6 * d, "rf_esim_train_fwd_f32: out row too short");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q && a && out && aux, "rf_esim_train_fwd_f32: null pointer");
    const size_t lds = qa_lds_bytes(L, d) + (size_t)kFwdWaves * 6 * d * sizeof(float);
    hipStream_t st = rf_stream(stream);
    int rc;
    if (d == 64) {
        if ((rc = set_lds(esim_train_fwd_kernel<64>, lds))) return rc;
        hipLaunchKernelGGL(esim_train_fwd_kernel<64>, dim3(batch), dim3(kFwdWaves * 64), lds, st, q, a, L, ex_stride, ld, out,
                           out_stride, out_off, aux);
    } else {
        if ((rc = set_lds(esim_train_fwd_kernel<128>, lds))) return rc;
        hipLaunchKernelGGL(esim_train_fwd_kernel<128>, dim3(batch), dim3(kFwdWaves * 64), lds, st, q, a, L, ex_stride, ld, out,
                           out_stride, out_off, aux);
    }
    return rf_check_launch("esim_train_fwd_kernel");
}

extern "C" int rf_esim_train_bwd_f32(const float* q, const float* a, int32_t batch, int32_t L, int32_t d, int64_t ex_stride,
                                     int64_t ld, const float* pooled, int64_t p_stride, int64_t p_off, const float* dpooled,
                                     int64_t dp_stride, int64_t dp_off, const float* aux, float* dq, float* da,
                                     int64_t g_ex_stride, int64_t ldg, void* ws, size_t ws_bytes, void* stream) {
    RF_ESIM_TRAIN_CHECK("rf_esim_train_bwd_f32");
    RF_REQUIRE(ldg >= d && g_ex_stride >= (int64_t)(L - 1) * ldg + d && ldg % 4 == 0 && g_ex_stride % 4 == 0,
               "rf_esim_train_bwd_f32: gradient strides must be multiples of 4 floats covering the L x d rows");
    RF_REQUIRE(p_stride >= p_off + 6 * d && dp_stride >= dp_off + 6 * d, "rf_esim_train_bwd_f32: pooled rows too short");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q && a && pooled && dpooled && aux && dq && da && ws, "rf_esim_train_bwd_f32: null pointer");
    RF_REQUIRE(((uintptr_t)dq & 15) == 0 && ((uintptr_t)da & 15) == 0 && ((uintptr_t)ws & 15) == 0,
               "rf_esim_train_bwd_f32: dq / da / ws must be 16-byte aligned");
    RF_REQUIRE(ws_bytes >= rf_esim_train_ws_bytes(batch, L, d), "rf_esim_train_bwd_f32: workspace too small");
    const size_t Lp = (size_t)((L + 15) & ~15);
    const size_t lds1 = qa_lds_bytes(L, d) + (size_t)6 * d * sizeof(float),
                 lds2 = ((size_t)d * (Lp + 4) + Lp * (d / 2 + 4)) * sizeof(float);
    hipStream_t st = rf_stream(stream);
    float* w = static_cast<float*>(ws);
    int rc;
    if (d == 64) {
        if ((rc = set_lds(esim_train_bwd1_kernel<64>, lds1))) return rc;
        hipLaunchKernelGGL(esim_train_bwd1_kernel<64>, dim3(batch), dim3(kBwd1Waves * 64), lds1, st, q, a, L, ex_stride, ld, pooled,
                           p_stride, p_off, dpooled, dp_stride, dp_off, aux, dq, da, g_ex_stride, ldg, w);
        if ((rc = set_lds(esim_train_bwd2_kernel<64>, lds2))) return rc;
        hipLaunchKernelGGL(esim_train_bwd2_kernel<64>, dim3(batch), dim3(kBwd2Waves * 64), lds2, st, a, L, ex_stride, ld,
                           (const float*)w, dq, da, g_ex_stride, ldg);
    } else {
        if ((rc = set_lds(esim_train_bwd1_kernel<128>, lds1))) return rc;
        hipLaunchKernelGGL(esim_train_bwd1_kernel<128>, dim3(batch), dim3(kBwd1Waves * 64), lds1, st, q, a, L, ex_stride, ld, pooled,
                           p_stride, p_off, dpooled, dp_stride, dp_off, aux, dq, da, g_ex_stride, ldg, w);
        if ((rc = set_lds(esim_train_bwd2_kernel<128>, lds2))) return rc;
        hipLaunchKernelGGL(esim_train_bwd2_kernel<128>, dim3(batch), dim3(kBwd2Waves * 64), lds2, st, a, L, ex_stride, ld,
                           (const float*)w, dq, da, g_ex_stride, ldg);
    }
    return rf_check_launch("esim_train_bwd_kernels");
}
