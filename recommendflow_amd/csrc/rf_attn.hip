// rf_attn.hip — attention stages on gfx950 MFMA (v_mfma_f32_16x16x32_{bf16,f16}, fp32 accumulate).
//   rf_esim_soft_attention_fwd  SoftAttention + ESIM combine/pool  (attention_layers.py:15-74, esim.py:78-84)
//   rf_sdpa_fwd                 masked multi-head SDPA             (layer_utils.py:4-38, attention_layers.py:153-168)
//
// ESIM (pooled output) runs esim2_kernel: persistent 4-wave workgroups, two per CU, the next example
// prefetched into registers, x of each stripe taken from a selector MFMA, pooled features stored one example
// late; with the attention output requested, the 8-wave esim_kernel. SDPA: one (example, head)
// per 4-wave workgroup. Shared structure:
//   * the [L, d] operand images sit in LDS with a 16-byte row pad (conflict-free ds_read_b128 for the
//     16x16x32 A/B fragments, 8-byte aligned rows for ds_read_b64_tr_b16);
//   * each wave owns 16-row stripes of the score matrix; scores stay in registers (never HBM), the
//     row softmax runs in fp32 with 16-lane xor shuffles, P is rounded once to the MFMA dtype into a
//     per-wave LDS stripe;
//   * P @ V takes V's B fragments with the hardware transpose read (ds_read_b64_tr_b16, guide T10),
//     so V is staged once, row-major, straight from HBM.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "rf_common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef short s8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool F16>
struct Mfma;

template <>
struct Mfma<false> {  // bf16
    using frag = bf16x8;
    static __device__ __forceinline__ f4 mma(frag a, frag b, f4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ float to_f(uint16_t h) { return bf16_bits_to_f32(h); }
    static __device__ __forceinline__ uint16_t from_f(float f) { return (uint16_t)f32_to_bf16_bits(f); }
};

template <>
struct Mfma<true> {  // f16
    using frag = f16x8;
    static __device__ __forceinline__ f4 mma(frag a, frag b, f4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ float to_f(uint16_t h) { return __half2float(__ushort_as_half(h)); }
    static __device__ __forceinline__ uint16_t from_f(float f) { return __half_as_ushort(__float2half_rn(f)); }
};

template <typename frag>
__device__ __forceinline__ frag lds_frag(const uint16_t* p) {  // 16-byte aligned LDS address -> ds_read_b128
    return *reinterpret_cast<const frag*>(p);
}

__device__ __forceinline__ s4v tr_read(const uint16_t* p) {  // ds_read_b64_tr_b16
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)(p));
}

// B fragment of the 16x16x32 MFMA for B[k][n] = V[k0 + k][n0 + n] (V row-major in LDS, row stride rs):
// lane l needs V[k0 + 8*(l>>4) + j][n0 + (l&15)], j = 0..7 — two transposed 4-row reads.
template <typename frag>
__device__ __forceinline__ frag v_frag_tr(const uint16_t* V, int rs, int k0, int n0, int lane) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const uint16_t* base = V + (k0 + 8 * g + qq) * rs + n0 + 4 * p;
    const s4v lo = tr_read(base);
    const s4v hi = tr_read(base + 4 * rs);
    const s8v x = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(frag, x);
}

__device__ __forceinline__ float group16_max(float v) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float group16_sum(float v) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Reductions across the four 16-lane rows of a wave (lanes l, l^16, l^32, l^48) in VALU, no LDS:
// v_permlane16_swap(x, x) -> {row0,row0,row2,row2} / {row1,row1,row3,row3};
// v_permlane32_swap(x, x) -> {lo,lo} / {hi,hi} (semantics probed on MI355X, tools/probes/permlane.hip).
__device__ __forceinline__ float rows4_sum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
// IEEE-754 maximum (NaN-propagating): v_maximum3_f32 on gfx950, no operand canonicalisation
// (fmaxf costs an extra v_max_f32 per non-canonical operand: loads, MFMA results, bit casts)
__device__ __forceinline__ float fmx(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float fmx3(float a, float b, float c) { return fmx(fmx(a, b), c); }

__device__ __forceinline__ float rows4_maximum(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = __builtin_elementwise_maximum(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return __builtin_elementwise_maximum(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows4_max(float v) {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    const float s = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
    const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
    return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// B fragment with the k order of an accumulator-sourced A operand: element j of lane (lr, g) holds
// k = k0 + (j < 4 ? 4g + j : 16 + 4g + j - 4) — rows 4g..4g+3 and 16+4g..16+4g+3 of the 32-row step.
template <typename frag>
__device__ __forceinline__ frag v_frag_tr_acc(const uint16_t* V, int rs, int k0, int n0, int lane) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const uint16_t* base = V + (k0 + 4 * g + qq) * rs + n0 + 4 * p;
    const s4v lo = tr_read(base);
    const s4v hi = tr_read(base + 16 * rs);
    const s8v x = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(frag, x);
}

// ---------------------------------------------------------------------------------------------
// ESIM: persistent workgroups of 8 waves (2 per SIMD), one per CU; each loops over examples
//   stage   q, a of example e (prefetched into registers during example e - G) -> LDS images
//   prefetch the next example's q, a into registers (in flight during this example's compute)
//   wave w  owns score stripe w (16 rows of a): E = a_stripe q^T (MFMA), row softmax in fp32, P -> LDS,
//           att = P [q | a] (MFMA, transposed V reads), ESIM combine statistics -> per-wave LDS slots
//   reduce  threads n < D combine the 8 waves' statistics with the column sums of q / a
// ---------------------------------------------------------------------------------------------
constexpr int kEsimWaves = 8;

template <bool F16, int D>
__global__ __launch_bounds__(kEsimWaves * 64) void esim_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ a,
                                                           int batch, int L, int64_t ex_stride, int64_t ld,
                                                           float* __restrict__ out, int64_t out_stride, int64_t out_off,
                                                           float* __restrict__ att_out) {
    using M = Mfma<F16>;
    using frag = typename M::frag;
    constexpr int NTH = kEsimWaves * 64;
    constexpr int RS = D + 8;       // LDS row stride (elements) of the q / a images
    constexpr int DK = D / 32;      // k-steps of the score product
    constexpr int NT = D / 16;      // n-tiles of the P @ V product (per side)
    constexpr int CPR = D / 8;      // 16-byte chunks per row
    constexpr int NCH = 2 * 128 * CPR / NTH;  // chunks per thread at L <= 128
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int Lk = (L + 31) & ~31;  // k extent of P @ V (zero rows past L)
    const int nt = (L + 15) >> 4;   // 16-wide tiles over positions (<= 8 = waves)
    uint16_t* qs = reinterpret_cast<uint16_t*>(smem);
    uint16_t* as = qs + Lk * RS;
    float* st = reinterpret_cast<float*>(as + Lk * RS);  // [wave][stat 3][side*D + n]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;

    // chunk i of this thread: matrix m = i / (NCH/2) (q first), row r, 16-byte column ch; every index is a
    // compile-time power-of-two split (no runtime divisions on the staging path)
    constexpr int HALF = NCH / 2;
    constexpr int LOG_CPR = D == 128 ? 4 : 3;
    uint4 pre[NCH];
    auto prefetch = [&](int64_t e) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int cm = tid + (i % HALF) * NTH;
            const int r = cm >> LOG_CPR, ch = cm & (CPR - 1);
            pre[i] = make_uint4(0, 0, 0, 0);
            if (r < L) pre[i] = *reinterpret_cast<const uint4*>((i < HALF ? q : a) + e * ex_stride + (int64_t)r * ld + ch * 8);
        }
    };
    int64_t e = blockIdx.x;
    if (e < batch) prefetch(e);
    for (; e < batch; e += gridDim.x) {
        __syncthreads();  // the previous example's LDS images are no longer read
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int cm = tid + (i % HALF) * NTH;
            const int r = cm >> LOG_CPR, ch = cm & (CPR - 1);
            if (r < Lk) *reinterpret_cast<uint4*>((i < HALF ? qs : as) + r * RS + ch * 8) = pre[i];
        }
        __syncthreads();
        if (e + gridDim.x < batch) prefetch(e + gridDim.x);  // in flight while this example computes

        const int sp = wave;
        if (sp < nt) {
            float* wst = st + wave * 3 * 2 * D;
            // E^T[j, i] = sum_k q[j, k] a[i, k] for the stripe's 16 columns i (attention_layers.py:44-47):
            // A = q rows j, B = a rows i; the C layout puts j on (lane >> 4, register) and i on lane & 15
            frag bf[DK];
#pragma unroll
            for (int kk = 0; kk < DK; ++kk) bf[kk] = lds_frag<frag>(as + (sp * 16 + lr) * RS + kk * 32 + lg * 8);
            f4 ev[8];
#pragma unroll
            for (int jt = 0; jt < 8; ++jt) {
                ev[jt] = f4{0.f, 0.f, 0.f, 0.f};
                if (jt < nt) {
#pragma unroll
                    for (int kk = 0; kk < DK; ++kk)
                        ev[jt] = M::mma(lds_frag<frag>(qs + (jt * 16 + lr) * RS + kk * 32 + lg * 8), bf[kk], ev[jt]);
                }
            }
            // softmax over j < L for column i (attention_layers.py:69-72), fp32: in-lane over (tile, register),
            // then across the four 16-lane rows
            float mx = -INFINITY;
#pragma unroll
            for (int jt = 0; jt < 8; ++jt)
                if (jt < nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        if (jt * 16 + lg * 4 + r >= L) ev[jt][r] = -INFINITY;
                        mx = fmaxf(mx, ev[jt][r]);
                    }
            mx = rows4_max(mx);
            float sm = 0.f;
#pragma unroll
            for (int jt = 0; jt < 8; ++jt)
                if (jt < nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        ev[jt][r] = expf(ev[jt][r] - mx);
                        sm += ev[jt][r];
                    }
            const float inv = 1.0f / rows4_sum(sm);
            // P as the A operand of P @ V, straight from the accumulators: step kt takes tiles 2kt, 2kt+1
            frag pa[4];
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                uint16_t h[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h[r] = 2 * kt < nt ? M::from_f(ev[2 * kt][r] * inv) : (uint16_t)0;
                    h[4 + r] = 2 * kt + 1 < nt ? M::from_f(ev[2 * kt + 1][r] * inv) : (uint16_t)0;
                }
                const s8v x = {(short)h[0], (short)h[1], (short)h[2], (short)h[3], (short)h[4], (short)h[5], (short)h[6], (short)h[7]};
                pa[kt] = __builtin_bit_cast(frag, x);
            }

            // att_side = P @ side (attention_layers.py:74), then the ESIM combine statistics (esim.py:79-82)
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const uint16_t* V = side ? as : qs;
                f4 acc[NT];
#pragma unroll
                for (int nn = 0; nn < NT; ++nn) acc[nn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    if (kt * 32 < Lk) {
#pragma unroll
                        for (int nn = 0; nn < NT; ++nn)
                            acc[nn] = M::mma(pa[kt], v_frag_tr_acc<frag>(V, RS, kt * 32, nn * 16, lane), acc[nn]);
                    }
                }
#pragma unroll
                for (int nn = 0; nn < NT; ++nn) {
                    // mean over the 4L rows of [x; att; x - att; x * att] = (2 sum x + sum x*att) / 4L exactly
                    // (sum att + sum (x - att) = sum x); the four maxima fold into one (max is exact).
                    // x[i][n] for this lane's 4 rows i: one transposed read of the row-major image
                    const s4v xv = tr_read(V + (sp * 16 + lg * 4 + (lr >> 2)) * RS + nn * 16 + 4 * (lr & 3));
                    const int n = nn * 16 + lr;
                    float s_x = 0.f, s_mul = 0.f, m_all = -INFINITY;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = sp * 16 + lg * 4 + r;
                        if (row < L) {
                            const float x = M::to_f((uint16_t)xv[r]);
                            const float at = acc[nn][r];
                            const float ml = x * at;
                            s_x += x;
                            s_mul += ml;
                            m_all = fmaxf(m_all, fmaxf(fmaxf(x, at), fmaxf(x - at, ml)));
                            if (att_out) att_out[((e * 2 + side) * L + row) * D + n] = at;
                        }
                    }
                    s_x = rows4_sum(s_x);
                    s_mul = rows4_sum(s_mul);
                    m_all = rows4_max(m_all);
                    if (lg == 0) {
                        float* w = wst + side * D + n;
                        w[0] = s_x;
                        w[2 * D] = s_mul;
                        w[4 * D] = m_all;
                    }
                }
            }
        }
        __syncthreads();

        // pooled = [avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a]  (esim.py:82,84)
        for (int n = tid; n < D; n += NTH) {
            float avg[2], mxv[2];
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                float sx = 0.f, smul = 0.f, m3 = -INFINITY;  // waves in order: deterministic
                for (int w = 0; w < nt; ++w) {
                    const float* ws = st + w * 3 * 2 * D + side * D + n;
                    sx += ws[0];
                    smul += ws[2 * D];
                    m3 = fmaxf(m3, ws[4 * D]);
                }
                avg[side] = (2.0f * sx + smul) / (float)(4 * L);
                mxv[side] = m3;
            }
            float* o = out + e * out_stride + out_off + n;
            o[0] = avg[0];
            o[D] = mxv[0];
            o[2 * D] = avg[1];
            o[3 * D] = mxv[1];
            o[4 * D] = avg[0] - avg[1];
            o[5 * D] = mxv[0] - mxv[1];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// ESIM v2: 4-wave workgroups, two per CU (LDS <= 80 KB each), so two examples are in flight per CU and
// one workgroup's barriers / softmax / statistics overlap the other's MFMA and LDS phases. Wave w owns
// the score stripes w and w + 4 and runs them jointly: every q fragment (scores) and every transposed V
// fragment (P @ V) read from LDS feeds both stripes' MFMAs, halving the LDS read traffic per example.
// The LDS images stop at the 16-row tile edge (not the 32-row k-step): the upper half of a P @ V k-step
// past the last tile reads zeros instead of LDS.
// ---------------------------------------------------------------------------------------------
constexpr int kEsim2Waves = 4;

template <typename frag>
__device__ __forceinline__ frag v_frag_tr_acc_h(const uint16_t* V, int rs, int k0, int n0, int lane, bool hi_ok) {
    const int g = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
    const uint16_t* base = V + (k0 + 4 * g + qq) * rs + n0 + 4 * p;
    const s4v lo = tr_read(base);
    s4v hi = s4v{0, 0, 0, 0};
    if (hi_ok) hi = tr_read(base + 16 * rs);
    const s8v x = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(frag, x);
}

typedef float f2v __attribute__((ext_vector_type(2)));

// LDS row stride (elements) of the ESIM v2 images: D + 16 puts the 8 rows of a ds_read_b64_tr_b16 lane
// group (and the 16 rows of a ds_read_b128 fragment) on disjoint banks; D + 8 (2-way conflicts) only
// where the wider images would push the workgroup past 80 KB (two per CU)
// images + statistics + (d = 64) a 2 KB dummy area for the staging chunks of rows past the image (d = 64 rows
// are 8 chunks, so a 256-chunk group can end mid-tile); it sits apart from the statistics, which the v6 loop
// reduces while the next images are written
__host__ __device__ constexpr size_t esim2_lds_bytes(int D, int ntt, int rs) {
    return (size_t)2 * ntt * 16 * rs * 2 + (size_t)kEsim2Waves * 3 * 2 * D * 4 + (D == 64 ? 128 * 16 : 0);
}
// offset of the GATHER id buffers past the statistics (and the d = 64 dummy area), from the statistics base
__host__ __device__ constexpr size_t esim2_stats_dummy_bytes(int D) {
    return (size_t)kEsim2Waves * 3 * 2 * D * 4 + (D == 64 ? 128 * 16 : 0);
}
// the GATHER kernel's LDS: the same images (row stride of the plain kernel) + two id buffers of 4 x 16 ntt dwords
__host__ __device__ constexpr size_t esim2_gather_lds_bytes(int D, int ntt, int rs) {
    return esim2_lds_bytes(D, ntt, rs) + (size_t)2 * 4 * 16 * ntt * 4;
}
__host__ __device__ constexpr int esim2_rs(int D, int ntt) {
    return esim2_lds_bytes(D, ntt, D + 16) <= 80 * 1024 ? D + 16 : D + 8;
}

// ---------------------------------------------------------------------------------------------
// ESIM wave body (v3 statistics; v2 masked every padding row and reduced each statistic separately):
//  * padding rows i >= L of a stripe get P = 0 (inv = 0), so att = 0 there, and x = 0 (zero image rows):
//    they add 0 to both sums and a 0 to the max, which never changes it, because every row's max of
//    [x, att, x - att, x * att] is >= 0 (x > 0: x; x < 0 and att >= 0: att; x < 0 and att < 0: x * att > 0;
//    x = 0: x * att = 0). No per-row validity masks in the statistics.
//  * the statistics of a side (NT columns tiles x {sum x, sum x*att, max}) leave the wave by reduce-scatter:
//    two lane swaps + two ops reduce FOUR values over the four 16-lane rows (1.5 instructions per value
//    instead of 4), and every lane then stores one reduced value.
//  * the x reads of a side are issued before its P @ V MFMAs.
// ---------------------------------------------------------------------------------------------

// four values a, b, c, d (one per call site, same op) summed / maxed over the four 16-lane rows of the wave;
// row 0 of the result holds a, row 1 c, row 2 b, row 3 d (v_permlane32_swap: a' = [a.lo, b.lo],
// b' = [a.hi, b.hi]; v_permlane16_swap: a' = [a.r0, b.r0, a.r2, b.r2], b' = [a.r1, b.r1, a.r3, b.r3])
template <bool MAX>
__device__ __forceinline__ float rs4(float a, float b, float c, float d) {
    auto op = [](float x, float y) { return MAX ? __builtin_elementwise_maximum(x, y) : x + y; };
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const float s1 = op(__uint_as_float(p[0]), __uint_as_float(p[1]));
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(d), false, false);
    const float s2 = op(__uint_as_float(q[0]), __uint_as_float(q[1]));
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s1), __float_as_uint(s2), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Sum over each 32-lane half of the wave, in every lane of the half, without LDS: the 16-lane rows by DPP (quad_perm
// [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror, row_mirror), then rows 0 + 1 and 2 + 3 by one v_permlane16_swap
// (a' = [r0, r0, r2, r2], b' = [r1, r1, r3, r3] for a = b = v)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float half32_sum(float v) {
    v += dpp_f<0xB1>(v);
    v += dpp_f<0x4E>(v);
    v += dpp_f<0x141>(v);
    v += dpp_f<0x140>(v);
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(p[0]) + __uint_as_float(p[1]);
}

// v[0..N) reduced as a balanced tree (maximum3 / add pairs): dependent depth ~log instead of N
template <int N, bool MAX>
__device__ __forceinline__ float tree_reduce(float (&v)[8]) {
    if constexpr (N == 1) return v[0];
    if constexpr (MAX) {
        if constexpr (N == 2) return fmx(v[0], v[1]);
        if constexpr (N == 3) return fmx3(v[0], v[1], v[2]);
        if constexpr (N == 4) return fmx3(v[0], v[1], fmx(v[2], v[3]));
        if constexpr (N == 5) return fmx3(fmx3(v[0], v[1], v[2]), v[3], v[4]);
        if constexpr (N == 6) return fmx(fmx3(v[0], v[1], v[2]), fmx3(v[3], v[4], v[5]));
        if constexpr (N == 7) return fmx3(fmx3(v[0], v[1], v[2]), fmx3(v[3], v[4], v[5]), v[6]);
        if constexpr (N == 8) return fmx3(fmx3(v[0], v[1], v[2]), fmx3(v[3], v[4], v[5]), fmx(v[6], v[7]));
    } else {
        if constexpr (N == 2) return v[0] + v[1];
        if constexpr (N == 3) return (v[0] + v[1]) + v[2];
        if constexpr (N == 4) return (v[0] + v[1]) + (v[2] + v[3]);
        if constexpr (N == 5) return ((v[0] + v[1]) + (v[2] + v[3])) + v[4];
        if constexpr (N == 6) return ((v[0] + v[1]) + (v[2] + v[3])) + (v[4] + v[5]);
        if constexpr (N == 7) return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + v[6]);
        if constexpr (N == 8) return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
    }
    return 0.f;
}

// column softmax of one E^T stripe (as stripe_softmax) with the stripe's padding rows zeroed: i = lane & 15
template <typename M, int nt, typename frag>
__device__ __forceinline__ void stripe_softmax3(f4 (&ev)[8], int L, int lg, bool row_ok, frag (&pa)[4]) {
    using elem = decltype(frag{}[0]);
    constexpr float kL2E = 1.4426950408889634f;
    if (L < nt * 16) {  // only the last tile can hold rows j >= L
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if ((nt - 1) * 16 + lg * 4 + r >= L) ev[nt - 1][r] = -INFINITY;
    }
    // the maximum and the sum as trees over the tiles (the tile-serial chains were 2 nt dependent VALU deep; the
    // maximum is exact in any order, the sum's fp32 order is this tree's)
    float tm[8];
#pragma unroll
    for (int jt = 0; jt < nt; ++jt) tm[jt] = fmx3(ev[jt][0], ev[jt][1], fmx(ev[jt][2], ev[jt][3]));
    const float mx = rows4_maximum(tree_reduce<nt, true>(tm));
    const float mo = -mx * kL2E;
#pragma unroll
    for (int jt = 0; jt < nt; ++jt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) ev[jt][r] = __builtin_amdgcn_exp2f(fmaf(ev[jt][r], kL2E, mo));
        tm[jt] = (ev[jt][0] + ev[jt][1]) + (ev[jt][2] + ev[jt][3]);
    }
    float inv = 1.0f / rows4_sum(tree_reduce<nt, false>(tm));
    inv = row_ok ? inv : 0.f;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
        frag f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            f[r] = (elem)(2 * kt < nt ? ev[2 * kt][r] * inv : 0.f);
            f[4 + r] = (elem)(2 * kt + 1 < nt ? ev[2 * kt + 1][r] * inv : 0.f);
        }
        pa[kt] = f;
    }
}

// statistics of 4 rows of one column: x (4 MFMA-dtype values), att (accumulator rows)
template <typename M>
__device__ __forceinline__ void esim_acc4(s4v xv, f4 at, f2v& sx, f2v& sm, float& mx) {
    const f2v x01 = {M::to_f((uint16_t)xv[0]), M::to_f((uint16_t)xv[1])};
    const f2v x23 = {M::to_f((uint16_t)xv[2]), M::to_f((uint16_t)xv[3])};
    const f2v t01 = {at[0], at[1]}, t23 = {at[2], at[3]};
    const f2v m01 = x01 * t01, m23 = x23 * t23;
    const f2v d01 = x01 - t01, d23 = x23 - t23;
    sx += x01 + x23;
    sm += m01 + m23;
    mx = fmx3(mx, x01[0], t01[0]);
    mx = fmx3(mx, d01[0], m01[0]);
    mx = fmx3(mx, x01[1], t01[1]);
    mx = fmx3(mx, d01[1], m01[1]);
    mx = fmx3(mx, x23[0], t23[0]);
    mx = fmx3(mx, d23[0], m23[0]);
    mx = fmx3(mx, x23[1], t23[1]);
    mx = fmx3(mx, d23[1], m23[1]);
}

// statistics of 4 rows of one column with x in fp32 (from the selector MFMA, v5): scalar ops only — packed
// f32 VALU beside MFMAs costs more than the two scalar ops it replaces (MI355X_MICROARCH constants table;
// rf_attn.hip is built with -fno-slp-vectorize so the compiler does not re-pack them)
__device__ __forceinline__ void esim_acc4x(f4 x, f4 at, float& sx, float& sm, float& mx) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float m = x[r] * at[r];
        const float d = x[r] - at[r];
        sx += x[r];
        sm += m;
        mx = fmx3(mx, x[r], at[r]);
        mx = fmx3(mx, d, m);
    }
}

// maximum of v[0..N) as a tree of maximum3 (N - 1 values folded 2 per instruction, depth ~log3 N); exact in any order
template <int N>
__device__ __forceinline__ float max3_tree(float (&v)[N]) {
    if constexpr (N == 1) {
        return v[0];
    } else if constexpr (N == 2) {
        return fmx(v[0], v[1]);
    } else {
        constexpr int M = N / 3 + (N % 3 ? 1 : 0);
        float w[M];
#pragma unroll
        for (int i = 0; i < N / 3; ++i) w[i] = fmx3(v[3 * i], v[3 * i + 1], v[3 * i + 2]);
        if constexpr (N % 3 == 1) w[M - 1] = v[N - 1];
        if constexpr (N % 3 == 2) w[M - 1] = fmx(v[N - 2], v[N - 1]);
        return max3_tree<M>(w);
    }
}

// the statistics of one column over the wave's 4 (one stripe) or 8 (TWO) rows as trees: sum x, sum x * att, and the
// maximum of [x, att, x - att, x * att] (v7; the v5 chains were 8 / 8 / 16 dependent VALU deep per column)
template <bool TWO>
__device__ __forceinline__ void esim_stats(f4 x0, f4 a0, f4 x1, f4 a1, float& sx, float& sm, float& mx) {
    float m[8], d[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        m[r] = x0[r] * a0[r];
        d[r] = x0[r] - a0[r];
        if (TWO) {
            m[4 + r] = x1[r] * a1[r];
            d[4 + r] = x1[r] - a1[r];
        }
    }
    constexpr int NV = TWO ? 32 : 16;
    float v[NV];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        v[4 * r] = x0[r];
        v[4 * r + 1] = a0[r];
        v[4 * r + 2] = d[r];
        v[4 * r + 3] = m[r];
        if (TWO) {
            v[16 + 4 * r] = x1[r];
            v[16 + 4 * r + 1] = a1[r];
            v[16 + 4 * r + 2] = d[4 + r];
            v[16 + 4 * r + 3] = m[4 + r];
        }
    }
    mx = max3_tree<NV>(v);
    if (TWO) {
        sx = ((x0[0] + x0[1]) + (x0[2] + x0[3])) + ((x1[0] + x1[1]) + (x1[2] + x1[3]));
        sm = ((m[0] + m[1]) + (m[2] + m[3])) + ((m[4] + m[5]) + (m[6] + m[7]));
    } else {
        sx = (x0[0] + x0[1]) + (x0[2] + x0[3]);
        sm = (m[0] + m[1]) + (m[2] + m[3]);
    }
}

// A operand selecting the 16 rows of stripe sp out of its 32-row P @ V k-step, in the k order of
// stripe_softmax3's accumulator-sourced fragments (element j of lane (lr, g): k = 4g + j for j < 4,
// 16 + 4g + j - 4 for j >= 4): row lr picks k = 16 (sp & 1) + lr, so sel @ V_kstep = x of the stripe,
// exactly, in the accumulator layout of att (one 1.0 per row, fp32 accumulation of one product)
template <typename M>
__device__ __forceinline__ typename M::frag stripe_selector(int sp, int lr, int lg) {
    using frag = typename M::frag;
    using elem = decltype(frag{}[0]);
    frag f;
    const int jh = 4 * (sp & 1) + (lr & 3);
    const bool mine = lg == (lr >> 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (elem)((mine && j == jh) ? 1.0f : 0.0f);
    return f;
}

// Diagnostic phase stamps (rf_diag_esim_gather_stamped only; STAMP = false compiles them out): the low 32 bits of
// the shader clock, one vector store from lane 0 of the wave into the caller's buffer
__device__ __forceinline__ void esim_stamp(uint32_t* p, int k, int lane) {
    const uint32_t t = (uint32_t)__builtin_amdgcn_s_memtime();
    if (lane == 0) __builtin_nontemporal_store(t, p + k);
}
constexpr int kStampPts = 10;  // stamps per (wave, example)
constexpr int kPfParts = 4;    // GATHER: the next example's row loads in this many parts (esim3_wave's pf hook)

// the 4 values of the lower (HI = 0) or upper (HI = 1) half of a B fragment widened to fp32
template <typename M, int HI, typename frag>
__device__ __forceinline__ f4 frag_rows_f32(frag vf) {
    const s8v b = __builtin_bit_cast(s8v, vf);
    f4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = M::to_f((uint16_t)b[4 * HI + j]);
    return r;
}

// KT0 = sp0 >> 1: the P @ V k-step holding stripe sp0's rows (sp1 = sp0 + 4: k-step KT0 + 2), a template
// parameter so the selector MFMAs are placed at compile time and each half's P @ V is one basic block (a runtime
// wave-uniform test split it into per-k-step blocks, each waiting out its own LDS reads before its MFMAs)
template <typename M, int D, int NTT, bool TWO, int XM = 0, int KT0 = 0, int XHI = 0, bool STAMP = false,
          typename PF = void (*)(int)>
__device__ __forceinline__ void esim3_wave(const uint16_t* qs, const uint16_t* as, float* wst, int sp0, int sp1, int L,
                                           int lane, uint32_t* stp, PF&& pf) {
    constexpr int nt = NTT;
    using frag = typename M::frag;
    constexpr int RS = esim2_rs(D, NTT);
    constexpr int DK = D / 32;
    constexpr int NT = D / 16;
    const int lr = lane & 15, lg = lane >> 4;
    frag pa0[4], pa1[4];
    {
        frag b0[DK], b1[DK];
#pragma unroll
        for (int kk = 0; kk < DK; ++kk) {
            b0[kk] = lds_frag<frag>(as + (sp0 * 16 + lr) * RS + kk * 32 + lg * 8);
            b1[kk] = b0[kk];
            if (TWO) b1[kk] = lds_frag<frag>(as + (sp1 * 16 + lr) * RS + kk * 32 + lg * 8);
        }
        f4 e0[8], e1[8];
#pragma unroll
        for (int jt = 0; jt < 8; ++jt) {
            e0[jt] = f4{0.f, 0.f, 0.f, 0.f};
            e1[jt] = f4{0.f, 0.f, 0.f, 0.f};
        }
        if constexpr (NTT < 8) {
#pragma unroll
            for (int kk = 0; kk < DK; ++kk) {
#pragma unroll
                for (int jt = 0; jt < nt; ++jt) {
                    const frag qf = lds_frag<frag>(qs + (jt * 16 + lr) * RS + kk * 32 + lg * 8);
                    e0[jt] = M::mma(qf, b0[kk], e0[jt]);
                    if (TWO) e1[jt] = M::mma(qf, b1[kk], e1[jt]);
                }
            }
        } else {
#pragma unroll
            for (int jt = 0; jt < nt; ++jt) {
#pragma unroll
                for (int kk = 0; kk < DK; ++kk) {
                    const frag qf = lds_frag<frag>(qs + (jt * 16 + lr) * RS + kk * 32 + lg * 8);
                    e0[jt] = M::mma(qf, b0[kk], e0[jt]);
                    if (TWO) e1[jt] = M::mma(qf, b1[kk], e1[jt]);
                }
            }
        }
        pf(1);
        if constexpr (STAMP) esim_stamp(stp, 7, lane);  // scores done
        stripe_softmax3<M, NTT>(e0, L, lg, sp0 * 16 + lr < L, pa0);
        if (TWO) stripe_softmax3<M, NTT>(e1, L, lg, sp1 * 16 + lr < L, pa1);
    }
    pf(2);
    if constexpr (STAMP) esim_stamp(stp, 8, lane);  // softmax done
#pragma unroll
    for (int side = 0; side < 2; ++side) {
        if (side == 1) pf(3);
        if constexpr (STAMP) {
            if (side == 1) esim_stamp(stp, 9, lane);  // side 0 done
        }
        const uint16_t* V = side ? as : qs;
        f4 c0[NT], c1[NT];
#pragma unroll
        for (int nn = 0; nn < NT; ++nn) {
            c0[nn] = f4{0.f, 0.f, 0.f, 0.f};
            c1[nn] = f4{0.f, 0.f, 0.f, 0.f};
        }
        float sx[NT], sm[NT], mx[NT];
        if constexpr (XM == 0) {
#pragma unroll
            for (int kt = 0; kt < 4; ++kt) {
                if (2 * kt < nt) {
                    const bool hi_ok = 2 * kt + 1 < nt;
#pragma unroll
                    for (int nn = 0; nn < NT; ++nn) {
                        const frag vf = v_frag_tr_acc_h<frag>(V, RS, kt * 32, nn * 16, lane, hi_ok);
                        c0[nn] = M::mma(pa0[kt], vf, c0[nn]);
                        if (TWO) c1[nn] = M::mma(pa1[kt], vf, c1[nn]);
                    }
                }
            }
#pragma unroll
            for (int nn = 0; nn < NT; ++nn) {
                // this lane's x values: rows sp*16 + 4*lg .. +3 of column nn*16 + lr
                f2v sx2 = {0.f, 0.f}, sm2 = {0.f, 0.f};
                float m = -INFINITY;
                esim_acc4<M>(tr_read(V + (sp0 * 16 + lg * 4 + (lr >> 2)) * RS + nn * 16 + 4 * (lr & 3)), c0[nn], sx2, sm2, m);
                if (TWO)
                    esim_acc4<M>(tr_read(V + (sp1 * 16 + lg * 4 + (lr >> 2)) * RS + nn * 16 + 4 * (lr & 3)), c1[nn], sx2, sm2, m);
                sx[nn] = sx2[0] + sx2[1];
                sm[nn] = sm2[0] + sm2[1];
                mx[nn] = m;
            }
        } else {
            // v5: x of the wave's stripes comes out of the MFMA pipe in fp32 (selector @ the k-step's V
            // fragments, already loaded for P @ V): no x reads, no bf16 -> f32 conversions. The columns run
            // in halves at d = 128 (att and x of both stripes for 4 column tiles at a time: 64 accumulator
            // registers instead of 128, no spills next to the 64 prefetch registers)
            constexpr int NH = NT >= 8 ? 2 : 1, NC = NT / NH;
            const frag sel = stripe_selector<M>(sp0, lr, lg);  // sp1 = sp0 + 4: the same row half
            constexpr int kt0 = KT0, kt1 = KT0 + 2;  // sp0 >> 1, sp1 >> 1
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                f4 a0[NC], a1[NC], x0[NC], x1[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    a0[c] = f4{0.f, 0.f, 0.f, 0.f};
                    a1[c] = f4{0.f, 0.f, 0.f, 0.f};
                }
#pragma unroll
                for (int kt = 0; kt < 4; ++kt) {
                    if (2 * kt < nt) {
                        const bool hi_ok = 2 * kt + 1 < nt;
                        // wave-uniform: this k-step holds the rows of stripe sp0 (kt < 2) or sp1 (kt >= 2)
                        if (kt < 2 ? kt == kt0 : (TWO && kt == kt1)) {
#pragma unroll
                            for (int c = 0; c < NC; ++c) {
                                const frag vf = v_frag_tr_acc_h<frag>(V, RS, kt * 32, (h * NC + c) * 16, lane, hi_ok);
                                a0[c] = M::mma(pa0[kt], vf, a0[c]);
                                if (TWO) a1[c] = M::mma(pa1[kt], vf, a1[c]);
                                if constexpr (XM == 2) {
                                    // v7: x of the stripe's rows is already in this B fragment, in the accumulator
                                    // layout of att (element j of lane (lr, g): row 4 g + j of the k-step's lower (j < 4)
                                    // or upper 16 rows = stripe row 4 g + j, column lr): 4 widenings, no MFMA
                                    if (kt < 2) x0[c] = frag_rows_f32<M, XHI>(vf);
                                    else x1[c] = frag_rows_f32<M, XHI>(vf);
                                } else {
                                    if (kt < 2) x0[c] = M::mma(sel, vf, f4{0.f, 0.f, 0.f, 0.f});
                                    else x1[c] = M::mma(sel, vf, f4{0.f, 0.f, 0.f, 0.f});
                                }
                            }
                        } else {
#pragma unroll
                            for (int c = 0; c < NC; ++c) {
                                const frag vf = v_frag_tr_acc_h<frag>(V, RS, kt * 32, (h * NC + c) * 16, lane, hi_ok);
                                a0[c] = M::mma(pa0[kt], vf, a0[c]);
                                if (TWO) a1[c] = M::mma(pa1[kt], vf, a1[c]);
                            }
                        }
                    }
                }
                float hx[NC], hm[NC], hmx[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) esim_stats<TWO>(x0[c], a0[c], x1[c], a1[c], hx[c], hm[c], hmx[c]);
                // this half's reduce-scatter and stores now (nothing carried into the next half)
                const int pk = (lg == 1) ? 2 : (lg == 2) ? 1 : lg;
                float* w = wst + side * D + lr;
#pragma unroll
                for (int g = 0; g < NC / 4; ++g) {
                    const int n = (h * NC + 4 * g + pk) * 16;
                    w[n] = rs4<false>(hx[4 * g], hx[4 * g + 1], hx[4 * g + 2], hx[4 * g + 3]);
                    w[2 * D + n] = rs4<false>(hm[4 * g], hm[4 * g + 1], hm[4 * g + 2], hm[4 * g + 3]);
                    w[4 * D + n] = rs4<true>(hmx[4 * g], hmx[4 * g + 1], hmx[4 * g + 2], hmx[4 * g + 3]);
                }
            }
            continue;  // statistics stored
        }
        // reduce-scatter over the four 16-lane rows: row k of group g holds tile nn = 4g + perm[k]
        const int pk = (lg == 1) ? 2 : (lg == 2) ? 1 : lg;
        float* w = wst + side * D + lr;
#pragma unroll
        for (int g = 0; g < NT / 4; ++g) {
            const int n = (4 * g + pk) * 16;
            w[n] = rs4<false>(sx[4 * g], sx[4 * g + 1], sx[4 * g + 2], sx[4 * g + 3]);
            w[2 * D + n] = rs4<false>(sm[4 * g], sm[4 * g + 1], sm[4 * g + 2], sm[4 * g + 3]);
            w[4 * D + n] = rs4<true>(mx[4 * g], mx[4 * g + 1], mx[4 * g + 2], mx[4 * g + 3]);
        }
    }
}

// GATHER (rf_esim_gather_fwd): the q / a images are gathered from the two fused tables by row id (a token's
// row = [table row of hash 0 | table row of hash 1], D / 2 elements each) instead of read from the encoders'
// [B, L, D] outputs, which are then never written: the single-token ids (rf_single_token_ids_fwd) of example
// e + 2G are LDS-DMA'd while e computes, and the staging of e + G reads its ids from LDS (double-buffered), so
// no dependent global round trip sits in front of a compute phase.
struct EsimGatherArgs {
    const uint32_t* qid;   // [batch][L][2]
    const uint32_t* aid;
    const uint16_t* qtab;  // [rows + 2][D / 2]: rows, then the NaN row and the zero row (RF_FLAG_SPEC_ROWS ids)
    const uint16_t* atab;
    uint32_t qzero, azero;  // the zero row's id in each table (rows + 1): image rows L .. L16 - 1
    uint32_t* stamps;      // STAMP only: [grid][waves][stamp_ex][kStampPts]
    int stamp_ex;
    uint16_t* outb;        // OB only: the pooled features as bf16 (row stride out_stride, column out_off) ...
    float* ostats;         // ... and per 32-column slice (sum, squared deviations from the slice mean) of the fp32
    int oP, op0;           // values: ostats[row][op0 + slice], oP pairs per row (rf_linear_lnfold_* consume them)
    // plain (non-GATHER) path, rf_esim_soft_attention_idx_fwd: example e reads q example e / q_rep (q_rep >= 1; 0 = 1)
    // and a example a_rows[e] (a_stride elements apart; a_rows == nullptr: e, ex_stride apart); a row outside
    // [0, a_count) reads nothing (an empty descriptor) and its example's pooled features are NaN
    int q_rep;
    const int64_t* a_rows;
    int64_t a_stride;
    int64_t a_count;
};

template <bool F16, int D, int NTT, int XM, bool GATHER = false, bool STAMP = false, bool OB = false>
__global__ __launch_bounds__(kEsim2Waves * 64, 2) void esim2_kernel(const uint16_t* __restrict__ q,
                                                                     const uint16_t* __restrict__ a, int batch, int L,
                                                                     int64_t ex_stride, int64_t ld, float* __restrict__ out,
                                                                     int64_t out_stride, int64_t out_off,
                                                                     EsimGatherArgs ga = {}) {
    using M = Mfma<F16>;
    constexpr int NTH = kEsim2Waves * 64;
    constexpr int RS = esim2_rs(D, NTT);
    constexpr int CPR = D / 8;
    constexpr int NCH = 2 * 128 * CPR / NTH;
    constexpr int HALF = NCH / 2;
    constexpr int LOG_CPR = D == 128 ? 4 : 3;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int L16 = NTT * 16;  // LDS rows per image
    constexpr int nt = NTT;        // 16-row tiles (<= 8)
    uint16_t* qs = reinterpret_cast<uint16_t*>(smem);
    uint16_t* as = qs + L16 * RS;
    float* st = reinterpret_cast<float*>(as + L16 * RS);  // [wave][stat 3][side*D + n]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;

    // staging loads through buffer descriptors over the example's L rows: the chunks of rows >= L fall past
    // the descriptor's range and read as zeros (the zero padding rows of the images), with no per-chunk
    // branch, select or zero-fill (a conditional load makes hipcc branch around every load; an
    // unconditional one with a clamped row demotes pre[] to scratch)
    uint4 pre[NCH];
    const int img_bytes = L * (int)ld * 2;
    auto prefetch = [&](int64_t e) __attribute__((always_inline)) {
        const int64_t eq = ga.q_rep > 1 ? e / ga.q_rep : e;
        const uint16_t* ap = a + e * ex_stride;
        int a_bytes = img_bytes;
        if (ga.a_rows) {
            const int64_t r = ga.a_rows[e];
            const bool ok = r >= 0 && r < ga.a_count;
            ap = a + (ok ? r : 0) * ga.a_stride;
            a_bytes = ok ? img_bytes : 0;
        }
        const auto rq = __builtin_amdgcn_make_buffer_rsrc((void*)(q + eq * ex_stride), 0, img_bytes, 0x00020000);
        const auto ra = __builtin_amdgcn_make_buffer_rsrc((void*)ap, 0, a_bytes, 0x00020000);
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int cm = tid + (i % HALF) * NTH;
            const int r = cm >> LOG_CPR, ch = cm & (CPR - 1);
            pre[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(i < HALF ? rq : ra, (r * (int)ld + ch * 8) * 2, 0, 0));
        }
    };
    // a chunk of a row past the image (only where 16-row tiles end inside a 256-chunk group: d = 64, odd
    // tile counts) goes to this thread's slot of the dummy area past the statistics
    uint16_t* dummy = reinterpret_cast<uint16_t*>(st + kEsim2Waves * 3 * 2 * D) + (tid & 127) * 8;
    // GATHER: two id buffers past the dummy area, each [side][row < L16][hash]; the DMAs write rows < L, rows L ..
    // L16 - 1 hold the zero row's id from the kernel start on (no per-chunk row test)
    constexpr int IDS = 2 * L16, IDW = 2 * IDS;
    uint32_t* idb = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(st) + esim2_stats_dummy_bytes(D));
    if constexpr (GATHER) {
        for (int w = tid; w < 2 * 2 * 2 * (L16 - L); w += NTH) {  // [buffer][side][row L ..][hash]
            const int hh = w & 1, q = w >> 1, r = L + q % (L16 - L), bs = q / (L16 - L);
            idb[(bs >> 1) * IDW + (bs & 1) * IDS + 2 * r + hh] = (bs & 1) ? ga.azero : ga.qzero;
        }
    }
    // ids of example ee -> buffer buf, one side at a time (64 dwords per wave instruction)
    auto ids_dma = [&](int64_t ee, int buf) __attribute__((always_inline)) {
        const int nc = (2 * L + 63) >> 6;
        for (int k = wave; k < 2 * nc; k += kEsim2Waves) {
            const int sd = k >= nc ? 1 : 0, j = k - sd * nc, w = j * 64 + lane;
            if (w < 2 * L)
                __builtin_amdgcn_global_load_lds((sd ? ga.aid : ga.qid) + ee * 2 * L + w,
                                                 (__attribute__((address_space(3))) void*)(idb + buf * IDW + sd * IDS + j * 64),
                                                 4, 0, 0);
        }
    };
    // the row loads of the next example in kPfParts parts: part 0 at the loop top, parts 1.. between the compute
    // phases (esim3_wave's pf hook), so a wave never stalls issuing NCH loads in one burst behind the CU's other
    // waves' bursts (r04 phase stamps: 2.9 K of 17.3 K cycles per example at the loop top with one burst)
    auto prefetch_g = [&](int buf, int part) __attribute__((always_inline)) {
        constexpr int HC = CPR / 2;  // 16-byte chunks per table row
        constexpr int PC = NCH / kPfParts;
        // every id of the part read from LDS first, then the row loads: left to itself hipcc interleaves them as
        // read -> lgkmcnt(0) -> address -> load per chunk (dependent LDS round trips)
        // chunk groups wholly past the image (cfg3: 2 of 16) are neither loaded nor staged; a group that straddles
        // the image end (d = 64) reads a valid id slot and stages into the dummy area
        auto live = [](int i) { return i % HALF * NTH < L16 * CPR; };
        auto straddles = [](int i) { return (i % HALF + 1) * NTH > L16 * CPR; };
        uint32_t idv[NCH];
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if (i / PC != part || !live(i)) continue;
            const int cm = tid + (i % HALF) * NTH;
            const int r = straddles(i) ? min(cm >> LOG_CPR, L16 - 1) : cm >> LOG_CPR, ch = cm & (CPR - 1);
            const int side = i < HALF ? 0 : 1;
            idv[i] = idb[buf * IDW + side * IDS + 2 * r + (ch >= HC ? 1 : 0)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            if (i / PC != part || !live(i)) continue;
            const int ch = (tid + (i % HALF) * NTH) & (CPR - 1);
            // every id indexes its table directly (the NaN and zero rows sit past the table's rows): one 64-bit
            // multiply-add per chunk, the side and the chunk offset folded into the base at compile time
            const char* tab = reinterpret_cast<const char*>(i < HALF ? ga.qtab : ga.atab) + (ch & (HC - 1)) * 16;
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            pre[i] = __builtin_bit_cast(uint4, *reinterpret_cast<const u32x4*>(tab + (uint64_t)idv[i] * (D / 2 * 2)));
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    int64_t e = blockIdx.x;
    uint32_t it = 0;
    // the pooled features of the previous example, stored one example late (right before the next prefetch):
    // vmcnt counts stores as well as loads, in issue order, so stores issued after a prefetch make the next
    // staging wait for them (hipcc emits vmcnt(0) for the last chunk); issued before it, they have the whole
    // compute phase to land. Four buffer stores per thread, unused ones at an offset past the descriptor.
    constexpr int kOff = 1 << 30;
    float pv[4] = {0.f, 0.f, 0.f, 0.f};
    int po[4] = {kOff, kOff, kOff, kOff};
    int64_t pe = -1;
    auto flush = [&]() __attribute__((always_inline)) {
        if constexpr (OB) {
            const auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)(ga.outb + pe * out_stride + out_off), 0, 6 * D * 2, 0x00020000);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)f32_to_bf16_bits(pv[k]), ro, po[k] >> 1, 0, 0);
            // slice statistics of the previous example's features, here (after the barrier, beside this example's
            // prefetch and compute) rather than inside the barrier-bounded reduction: the 32 lanes of a half-wave
            // hold columns wave * 32 .. + 31 of each feature (D <= NTH / 2); one pass around a pivot (the half's
            // first value): S = sum d + 32 p, M2 = sum d^2 - (sum d)^2 / 32, d = v - p, 8 independent DPP chains
            static_assert(NTH / 2 >= D && D % 32 == 0, "one 32-column slice per half-wave and feature");
            const int side = lane >> 5;
            const bool ok = po[0] != kOff;  // column wave * 32 + (lane & 31) < D
            float sd[4], sq[4], pvt[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float p0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pv[k]), 0));
                const float p1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, pv[k]), 32));
                pvt[k] = side ? p1 : p0;
                const float d = ok ? pv[k] - pvt[k] : 0.f;
                sd[k] = d;
                sq[k] = d * d;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                sd[k] = half32_sum(sd[k]);
                sq[k] = half32_sum(sq[k]);
            }
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(ga.ostats + (pe * ga.oP + ga.op0) * 2), 0, 6 * D / 32 * 8,
                                                              0x00020000);
            const bool lead = (lane & 31) == 0 && ok;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int sl = ((k < 2 ? (2 * side + k) * D : (4 + k - 2) * D) + wave * 32) / 32;
                const int off = lead && (k < 2 || side == 0) ? sl * 8 : kOff;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sd[k] + 32.0f * pvt[k]), rs, off, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaxf(sq[k] - sd[k] * sd[k] * (1.0f / 32.0f), 0.f)),
                                                      rs, off + 4, 0, 0);
            }
        } else {
            const auto ro = __builtin_amdgcn_make_buffer_rsrc((void*)(out + pe * out_stride + out_off), 0, 6 * D * 4, 0x00020000);
#pragma unroll
            for (int k = 0; k < 4; ++k) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(pv[k]), ro, po[k], 0, 0);
        }
    };
    // v6 loop: two barriers per example. The images of example e + G are written right after the barrier that
    // ends e's compute phase (nothing reads them after it; the prefetched registers landed under that compute),
    // beside e's statistics reduction, which reads only the statistics area; the second barrier publishes the
    // new images and retires the statistics reads before the next compute phase rewrites them (v5 had a third
    // barrier before the staging writes).
    auto stage_images = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
            const int cm = tid + (i % HALF) * NTH;
            const int r = cm >> LOG_CPR, ch = cm & (CPR - 1);
            if (i % HALF * NTH < L16 * CPR) {  // compile-time: chunk groups wholly past the image never exist
                uint16_t* dst = (i % HALF + 1) * NTH <= L16 * CPR || r < L16 ? (i < HALF ? qs : as) + r * RS + ch * 8 : dummy;
                *reinterpret_cast<uint4*>(dst) = pre[i];
            }
        }
    };
    int pbuf = 0;  // GATHER: the id buffer holding example e's ids (the other: e + G's)
    if (e < batch) {
        if constexpr (GATHER) {
            ids_dma(e, 0);
            __syncthreads();  // (its release fence waits for the DMA) ids of e visible
#pragma unroll
            for (int part = 0; part < kPfParts; ++part) prefetch_g(0, part);
            if (e + gridDim.x < batch) ids_dma(e + gridDim.x, 1);
        } else {
            prefetch(e);
        }
        stage_images();
        __syncthreads();
    }
    for (; e < batch; e += gridDim.x) {
        if constexpr (STAMP) {
            const int ex = (int)it;
            esim_stamp(ga.stamps + (((int64_t)blockIdx.x * kEsim2Waves + wave) * ga.stamp_ex + min(ex, ga.stamp_ex - 1)) * kStampPts, 0, lane);
        }
        if (pe >= 0) flush();
        const bool more = e + gridDim.x < batch;
        const int rbuf = pbuf ^ 1;  // GATHER: the id buffer holding e + G's ids
        if constexpr (GATHER) {
            if (more) {
                prefetch_g(rbuf, 0);
                if (e + 2 * (int64_t)gridDim.x < batch) ids_dma(e + 2 * (int64_t)gridDim.x, pbuf);
            }
            pbuf ^= 1;
        } else if (more) {
            prefetch(e + gridDim.x);
        }
        // the later load parts, called by esim3_wave between its phases
        auto pf = [&](int part) __attribute__((always_inline)) {
            if constexpr (GATHER) {
                if (more) prefetch_g(rbuf, part);
            }
        };

        // v3: the stripe pairs rotate over the waves from one example to the next, so the wave left with one
        // stripe (7 tiles over 4 waves) is a different SIMD each time; statistics slots follow the stripe
        const int rot = (int)(it++ & 3);
        const int sp0 = (wave + rot) & 3, sp1 = sp0 + kEsim2Waves;
        uint32_t* stp = nullptr;
        if constexpr (STAMP) {
            const int ex = (int)(it - 1);
            stp = ga.stamps + (((int64_t)blockIdx.x * kEsim2Waves + wave) * ga.stamp_ex + min(ex, ga.stamp_ex - 1)) * kStampPts;
            esim_stamp(stp, 1, lane);  // prefetch issued
        }
        if (sp0 < nt) {
            float* wst = st + sp0 * 3 * 2 * D;
            // both-stripe / one-stripe waves are separate instantiations: no predicated MFMAs
            // (KT0, XHI) = (sp0 >> 1, sp0 & 1) at compile time (XHI only matters for XM = 2)
            auto run = [&](auto two, auto kt0, auto xhi) __attribute__((always_inline)) {
                esim3_wave<M, D, NTT, decltype(two)::value, XM, decltype(kt0)::value, decltype(xhi)::value, STAMP>(
                    qs, as, wst, sp0, sp1, L, lane, stp, pf);
            };
            using T_ = std::true_type;
            using F_ = std::false_type;
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            const int xh = XM == 2 ? (sp0 & 1) : 0;
            if (sp1 < nt) {
                if (sp0 >> 1) { if (xh) run(T_{}, I1{}, I1{}); else run(T_{}, I1{}, I0{}); }
                else { if (xh) run(T_{}, I0{}, I1{}); else run(T_{}, I0{}, I0{}); }
            } else {
                if (sp0 >> 1) { if (xh) run(F_{}, I1{}, I1{}); else run(F_{}, I1{}, I0{}); }
                else { if (xh) run(F_{}, I0{}, I1{}); else run(F_{}, I0{}, I0{}); }
            }
        }
        else {
#pragma unroll
            for (int part = 1; part < kPfParts; ++part) pf(part);
        }
        if constexpr (STAMP) esim_stamp(stp, 2, lane);  // compute done
        __syncthreads();  // compute done: images free, statistics complete
        if constexpr (STAMP) esim_stamp(stp, 3, lane);
        if (more) stage_images();
        if constexpr (STAMP) esim_stamp(stp, 4, lane);  // next images written (prefetched rows landed)

        // pooled = [avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a]  (esim.py:82,84)
        // every thread of the workgroup: lane l of wave w reduces side l >> 5 of the columns
        // n = (w * 32 + (l & 31)) + j * 128; the two sides of a column meet with one lane swap (l ^ 32)
        constexpr int nw = nt < kEsim2Waves ? nt : kEsim2Waves;
        const int side = lane >> 5;
#pragma unroll
        for (int n0 = 0; n0 < D; n0 += NTH / 2) {
            const int n = n0 + wave * 32 + (lane & 31);
            float sx = 0.f, smul = 0.f, m3 = -INFINITY;
            if (n < D) {
#pragma unroll
                for (int w = 0; w < nw; ++w) {
                    const float* ws = st + w * 3 * 2 * D + side * D + n;
                    sx += ws[0];
                    smul += ws[2 * D];
                    m3 = fmx(m3, ws[4 * D]);
                }
            }
            float avg = (2.0f * sx + smul) / (float)(4 * L);
            if constexpr (!GATHER) {
                if (ga.a_rows) {  // an a row outside the catalog: NaN features (nothing was read for it)
                    const int64_t r = ga.a_rows[e];
                    if (r < 0 || r >= ga.a_count) avg = m3 = __builtin_nanf("");
                }
            }
            const float avg_o = __shfl_xor(avg, 32, 64), mx_o = __shfl_xor(m3, 32, 64);
            {
                static_assert(NTH / 2 >= D, "one column per thread and side: four pending values");
                const bool ok = n < D, ok0 = ok && side == 0;
                pv[0] = avg;
                pv[1] = m3;
                pv[2] = avg - avg_o;
                pv[3] = m3 - mx_o;
                po[0] = ok ? (2 * side * D + n) * 4 : kOff;
                po[1] = ok ? ((2 * side + 1) * D + n) * 4 : kOff;
                po[2] = ok0 ? (4 * D + n) * 4 : kOff;
                po[3] = ok0 ? (5 * D + n) * 4 : kOff;
                pe = e;
            }
        }
        if constexpr (STAMP) esim_stamp(stp, 5, lane);
        __syncthreads();  // next images visible; statistics reads retired
        if constexpr (STAMP) esim_stamp(stp, 6, lane);
    }
    if (pe >= 0) flush();  // the last example's features
}

// ---------------------------------------------------------------------------------------------
// masked multi-head SDPA: one workgroup per (example, head)
// ---------------------------------------------------------------------------------------------
template <bool F16, int DEP>
__global__ __launch_bounds__(256) void sdpa_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ k,
                                                   const uint16_t* __restrict__ v, int heads, int Lq, int Lk,
                                                   const float* __restrict__ mask, float* __restrict__ out) {
    using M = Mfma<F16>;
    using frag = typename M::frag;
    constexpr int RS = DEP + 8, DK = DEP / 32, NT = DEP / 16, MAXT = 16;  // up to 256 keys
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int64_t b = blockIdx.x / heads;
    const int h = blockIdx.x - (int)(b * heads);
    const int64_t rowstride = (int64_t)heads * DEP;
    const int Lkp = (Lk + 31) & ~31, nt = (Lk + 15) >> 4, SS = Lkp + 8;
    uint16_t* ks = reinterpret_cast<uint16_t*>(smem);
    uint16_t* vs = ks + Lkp * RS;
    uint16_t* pbuf = vs + Lkp * RS;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    constexpr int CPR = DEP / 8;
    for (int c = tid; c < 2 * Lkp * CPR; c += 256) {
        const int m = c / (Lkp * CPR), rem = c - m * Lkp * CPR, r = rem / CPR, ch = rem - r * CPR;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (r < Lk) x = *reinterpret_cast<const uint4*>((m ? v : k) + (b * Lk + r) * rowstride + h * DEP + ch * 8);
        *reinterpret_cast<uint4*>((m ? vs : ks) + r * RS + ch * 8) = x;
    }
    __syncthreads();
    const float scale = 1.0f / sqrtf((float)DEP);
    uint16_t* pw = pbuf + wave * 16 * SS;
    const int ntq = (Lq + 15) >> 4;
    for (int sp = wave; sp < ntq; sp += 4) {
        const int qrow = sp * 16 + lr;
        frag af[DK];
#pragma unroll
        for (int kk = 0; kk < DK; ++kk) {
            if (qrow < Lq)
                af[kk] = *reinterpret_cast<const frag*>(q + (b * Lq + qrow) * rowstride + h * DEP + kk * 32 + lg * 8);
            else
                af[kk] = __builtin_bit_cast(frag, s8v{0, 0, 0, 0, 0, 0, 0, 0});
        }
        f4 e[MAXT];
#pragma unroll
        for (int jt = 0; jt < MAXT; ++jt) {
            e[jt] = f4{0.f, 0.f, 0.f, 0.f};
            if (jt < nt) {
#pragma unroll
                for (int kk = 0; kk < DK; ++kk)
                    e[jt] = M::mma(af[kk], lds_frag<frag>(ks + (jt * 16 + lr) * RS + kk * 32 + lg * 8), e[jt]);
            }
        }
        // rows of this lane: sp*16 + lg*4 + r ; query-row mask replaces the whole row (layer_utils.py:13-14)
        bool masked[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = sp * 16 + lg * 4 + r;
            masked[r] = mask != nullptr && row < Lq && mask[b * Lq + row] == 0.0f;
        }
        float mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
        for (int jt = 0; jt < MAXT; ++jt)
            if (jt < nt) {
                const bool valid = jt * 16 + lr < Lk;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float x = e[jt][r] * scale;
                    if (masked[r]) x = -4294967295.0f;
                    if (!valid) x = -INFINITY;
                    e[jt][r] = x;
                    mx[r] = fmaxf(mx[r], x);
                }
            }
        float sm[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            mx[r] = group16_max(mx[r]);
            sm[r] = 0.f;
        }
#pragma unroll
        for (int jt = 0; jt < MAXT; ++jt)
            if (jt < nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    e[jt][r] = expf(e[jt][r] - mx[r]);
                    sm[r] += e[jt][r];
                }
#pragma unroll
        for (int r = 0; r < 4; ++r) sm[r] = 1.0f / group16_sum(sm[r]);
#pragma unroll
        for (int jt = 0; jt < MAXT; ++jt)
            if (jt * 16 < Lkp)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    pw[(lg * 4 + r) * SS + jt * 16 + lr] = jt < nt ? M::from_f(e[jt][r] * sm[r]) : (uint16_t)0;
        wave_lds_sync();
        f4 acc[NT];
#pragma unroll
        for (int nn = 0; nn < NT; ++nn) acc[nn] = f4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < Lkp; kt += 32) {
            const frag pa = lds_frag<frag>(pw + lr * SS + kt + lg * 8);
#pragma unroll
            for (int nn = 0; nn < NT; ++nn) acc[nn] = M::mma(pa, v_frag_tr<frag>(vs, RS, kt, nn * 16, lane), acc[nn]);
        }
#pragma unroll
        for (int nn = 0; nn < NT; ++nn)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = sp * 16 + lg * 4 + r;
                if (row < Lq) out[(b * Lq + row) * rowstride + h * DEP + nn * 16 + lr] = acc[nn][r];
            }
        wave_lds_sync();
    }
}

template <typename K>
int launch_big_lds(K kernel, int grid, size_t lds, hipStream_t st, const char* name) {
    (void)kernel;
    (void)grid;
    (void)st;
    if (lds > 160 * 1024) return rf_set_error(RF_EINVAL, "%s: needs %zu bytes of LDS (> 160 KiB)", name, lds);
    if (lds > 64 * 1024) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "%s: hipFuncSetAttribute: %s", name, hipGetErrorString(e));
    }
    return RF_OK;
}

template <bool F16, int D, int NTT>
int launch_esim2_nt(int grid, size_t lds, hipStream_t st, const void* q, const void* a, int batch, int L, int64_t ex_stride,
                    int64_t ld, float* out, int64_t out_stride, int64_t out_off, const EsimGatherArgs& ga) {
    // RF_ESIM_XM=0 keeps the v3 statistics (x read from LDS and converted on the VALU); A/B runs only
    static const int xm = [] {
        const char* e = getenv("RF_ESIM_XM");
        return e && e[0] == '0' ? 0 : 1;
    }();
    auto kern = xm == 0 ? esim2_kernel<F16, D, NTT, 0> : esim2_kernel<F16, D, NTT, 1>;
    const int rc = launch_big_lds(kern, grid, lds, st, "esim2_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kEsim2Waves * 64), lds, st, (const uint16_t*)q, (const uint16_t*)a, batch, L,
                       ex_stride, ld, out, out_stride, out_off, ga);
    return RF_OK;
}

template <bool F16, int D>
int launch_esim2(int nt, int grid, size_t lds, hipStream_t st, const void* q, const void* a, int batch, int L,
                 int64_t ex_stride, int64_t ld, float* out, int64_t out_stride, int64_t out_off, const EsimGatherArgs& ga) {
    switch (nt) {
#define RF_NT(N) \
    case N: return launch_esim2_nt<F16, D, N>(grid, lds, st, q, a, batch, L, ex_stride, ld, out, out_stride, out_off, ga);
        RF_NT(1) RF_NT(2) RF_NT(3) RF_NT(4) RF_NT(5) RF_NT(6) RF_NT(7) RF_NT(8)
#undef RF_NT
        default: return rf_set_error(RF_EINVAL, "esim2: bad tile count %d", nt);
    }
}

// the 4-wave persistent kernel (two workgroups per CU when the images fit 80 KB)
int esim2_dispatch(const void* q, const void* a, int32_t dtype, int32_t batch, int32_t L, int32_t d, int64_t ex_stride,
                   int64_t ld, float* out, int64_t out_stride, int64_t out_off, hipStream_t st,
                   const EsimGatherArgs& ga = EsimGatherArgs{}) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int nt = (L + 15) >> 4;
    const size_t lds2 = esim2_lds_bytes(d, nt, esim2_rs(d, nt));
    const int per_cu = lds2 <= 80 * 1024 ? 2 : 1;
    const int grid2 = (int)std::min<int64_t>(batch, (int64_t)per_cu * cus);
    if (dtype == RF_DTYPE_BF16)
        return d == 64 ? launch_esim2<false, 64>(nt, grid2, lds2, st, q, a, batch, L, ex_stride, ld, out, out_stride, out_off, ga)
                       : launch_esim2<false, 128>(nt, grid2, lds2, st, q, a, batch, L, ex_stride, ld, out, out_stride, out_off, ga);
    return d == 64 ? launch_esim2<true, 64>(nt, grid2, lds2, st, q, a, batch, L, ex_stride, ld, out, out_stride, out_off, ga)
                   : launch_esim2<true, 128>(nt, grid2, lds2, st, q, a, batch, L, ex_stride, ld, out, out_stride, out_off, ga);
}

// GATHER: bf16 tables, the v5 statistics, two workgroups per CU when images + id buffers fit 80 KB
template <int D, int NTT>
int launch_esim2g_nt(int grid, size_t lds, hipStream_t st, int batch, int L, float* out, int64_t out_stride,
                     int64_t out_off, const EsimGatherArgs& ga) {
    // (XM = 2, x widened from the P @ V B fragments instead of the selector MFMA, measured equal: r04g3 0.0875 /
    // 0.0869 vs 0.0872 / 0.0865 ms; the template keeps it, no launcher instantiates it)
    auto kern = ga.outb ? esim2_kernel<false, D, NTT, 1, true, false, true> : esim2_kernel<false, D, NTT, 1, true>;
    if constexpr (D == 128 && NTT == 7) {  // the diagnostic stamped build: cfg3's shape only
        if (ga.stamps) kern = esim2_kernel<false, D, NTT, 1, true, true>;
    } else {
        if (ga.stamps) return rf_set_error(RF_EINVAL, "stamped ESIM: only d = 128, 97 <= L <= 112");
    }
    if (ga.stamps && ga.outb) return rf_set_error(RF_EINVAL, "stamped ESIM: fp32 output only");
    const int rc = launch_big_lds(kern, grid, lds, st, "esim2_kernel (gather)");
    if (rc) return rc;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kEsim2Waves * 64), lds, st, nullptr, nullptr, batch, L, (int64_t)0,
                       (int64_t)D, out, out_stride, out_off, ga);
    return RF_OK;
}

template <int D>
int launch_esim2g(int nt, int grid, size_t lds, hipStream_t st, int batch, int L, float* out, int64_t out_stride,
                  int64_t out_off, const EsimGatherArgs& ga) {
    switch (nt) {
#define RF_NT(N) case N: return launch_esim2g_nt<D, N>(grid, lds, st, batch, L, out, out_stride, out_off, ga);
        RF_NT(1) RF_NT(2) RF_NT(3) RF_NT(4) RF_NT(5) RF_NT(6) RF_NT(7) RF_NT(8)
#undef RF_NT
        default: return rf_set_error(RF_EINVAL, "esim2 gather: bad tile count %d", nt);
    }
}

}  // namespace


extern "C" int rf_esim_soft_attention_fwd(const void* q, const void* a, int32_t dtype, int32_t batch, int32_t L, int32_t d,
                                          int64_t ex_stride, int64_t ld, float* out, int64_t out_stride, int64_t out_off,
                                          float* att_out, void* stream) {
    RF_REQUIRE(dtype == RF_DTYPE_BF16 || dtype == RF_DTYPE_F16, "rf_esim_soft_attention_fwd: dtype must be BF16 or F16");
    RF_REQUIRE(L >= 1 && L <= 128, "rf_esim_soft_attention_fwd: need 1 <= L <= 128 (got %d)", L);
    RF_REQUIRE(d == 64 || d == 128, "rf_esim_soft_attention_fwd: d must be 64 or 128 (got %d)", d);
    RF_REQUIRE(batch >= 0, "rf_esim_soft_attention_fwd: batch < 0");
    RF_REQUIRE(ld % 8 == 0 && ex_stride % 8 == 0 && ld >= d, "rf_esim_soft_attention_fwd: ld/ex_stride must be multiples of 8 elements (16-byte rows)");
    RF_REQUIRE((int64_t)L * ld * 2 < ((int64_t)1 << 31), "rf_esim_soft_attention_fwd: one example's rows must span < 2 GiB");
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)a & 15) == 0, "rf_esim_soft_attention_fwd: q/a must be 16-byte aligned");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q && a && out, "rf_esim_soft_attention_fwd: null pointer");
    hipStream_t st = rf_stream(stream);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    // v2 (default): 4-wave workgroups, two per CU. RF_ESIM_V1=1 selects the 8-wave one-per-CU kernel (A/B only).
    static const bool v1 = [] {
        const char* e = getenv("RF_ESIM_V1");
        return e && e[0] == '1';
    }();
    if (!v1 && !att_out) {
        const int rc = esim2_dispatch(q, a, dtype, batch, L, d, ex_stride, ld, out, out_stride, out_off, st);
        if (rc) return rc;
        return rf_check_launch("rf_esim_soft_attention_fwd");
    }
    // the attention-output variant (tests, diagnostics) and RF_ESIM_V1=1 run the 8-wave kernel
    const int Lk = (L + 31) & ~31;
    const size_t lds = (size_t)2 * Lk * (d + 8) * 2 + (size_t)kEsimWaves * 3 * 2 * d * 4;
    const int grid = (int)std::min<int64_t>(batch, cus);  // persistent: one 8-wave workgroup per CU
#define RF_ESIM_LAUNCH(F16, D)                                                                                     \
    {                                                                                                              \
        auto kern = esim_kernel<F16, D>;                                                                           \
        int rc = launch_big_lds(kern, grid, lds, st, "esim_kernel");                                               \
        if (rc) return rc;                                                                                         \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kEsimWaves * 64), lds, st, (const uint16_t*)q, (const uint16_t*)a, \
                           batch, L, ex_stride, ld, out, out_stride, out_off, att_out);                            \
    }
    if (dtype == RF_DTYPE_BF16) {
        if (d == 64) RF_ESIM_LAUNCH(false, 64) else RF_ESIM_LAUNCH(false, 128)
    } else {
        if (d == 64) RF_ESIM_LAUNCH(true, 64) else RF_ESIM_LAUNCH(true, 128)
    }
#undef RF_ESIM_LAUNCH
    return rf_check_launch("esim_kernel");
}

extern "C" int rf_esim_soft_attention_idx_fwd(const void* q, int32_t q_rep, const void* a, const int64_t* a_rows,
                                              int64_t a_count, int64_t a_stride, int32_t dtype, int32_t batch, int32_t L, int32_t d,
                                              int64_t q_stride, int64_t ld, float* out, int64_t out_stride, int64_t out_off,
                                              void* stream) {
    RF_REQUIRE(dtype == RF_DTYPE_BF16 || dtype == RF_DTYPE_F16, "rf_esim_soft_attention_idx_fwd: dtype must be BF16 or F16");
    RF_REQUIRE(L >= 1 && L <= 128 && (d == 64 || d == 128) && batch >= 0 && q_rep >= 1,
               "rf_esim_soft_attention_idx_fwd: need 1 <= L <= 128, d 64 or 128, batch >= 0, q_rep >= 1");
    RF_REQUIRE(ld % 8 == 0 && q_stride % 8 == 0 && a_stride % 8 == 0 && ld >= d,
               "rf_esim_soft_attention_idx_fwd: ld / q_stride / a_stride must be multiples of 8 elements");
    RF_REQUIRE((int64_t)L * ld * 2 < ((int64_t)1 << 31), "rf_esim_soft_attention_idx_fwd: one example's rows must span < 2 GiB");
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)a & 15) == 0, "rf_esim_soft_attention_idx_fwd: q/a must be 16-byte aligned");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q && a && a_rows && out, "rf_esim_soft_attention_idx_fwd: null pointer");
    RF_REQUIRE(a_count >= 1, "rf_esim_soft_attention_idx_fwd: a_count must be >= 1");
    EsimGatherArgs ga{};
    ga.q_rep = q_rep;
    ga.a_rows = a_rows;
    ga.a_stride = a_stride;
    ga.a_count = a_count;
    const int rc = esim2_dispatch(q, a, dtype, batch, L, d, q_stride, ld, out, out_stride, out_off, rf_stream(stream), ga);
    if (rc) return rc;
    return rf_check_launch("rf_esim_soft_attention_idx_fwd");
}

extern "C" int rf_sdpa_fwd(const void* q, const void* k, const void* v, int32_t dtype, int32_t batch, int32_t heads,
                           int32_t Lq, int32_t Lk, int32_t depth, const float* mask, float* out, void* stream) {
    RF_REQUIRE(dtype == RF_DTYPE_BF16 || dtype == RF_DTYPE_F16, "rf_sdpa_fwd: dtype must be BF16 or F16");
    RF_REQUIRE(depth == 32 || depth == 64 || depth == 128, "rf_sdpa_fwd: depth must be 32, 64 or 128 (got %d)", depth);
    RF_REQUIRE(Lq >= 1 && Lq <= 4096 && Lk >= 1 && Lk <= 256, "rf_sdpa_fwd: need 1 <= Lk <= 256 and Lq >= 1");
    RF_REQUIRE(batch >= 0 && heads >= 1, "rf_sdpa_fwd: batch >= 0, heads >= 1");
    RF_REQUIRE(((uintptr_t)q & 15) == 0 && ((uintptr_t)k & 15) == 0 && ((uintptr_t)v & 15) == 0, "rf_sdpa_fwd: q/k/v must be 16-byte aligned");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q && k && v && out, "rf_sdpa_fwd: null pointer");
    const int Lkp = (Lk + 31) & ~31;
    const size_t lds = (size_t)2 * Lkp * (depth + 8) * 2 + (size_t)4 * 16 * (Lkp + 8) * 2;
    hipStream_t st = rf_stream(stream);
    const int grid = batch * heads;
#define RF_SDPA_LAUNCH(F16, DEP)                                                                                    \
    {                                                                                                               \
        auto kern = sdpa_kernel<F16, DEP>;                                                                          \
        int rc = launch_big_lds(kern, grid, lds, st, "sdpa_kernel");                                                \
        if (rc) return rc;                                                                                          \
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, (const uint16_t*)q, (const uint16_t*)k,            \
                           (const uint16_t*)v, heads, Lq, Lk, mask, out);                                          \
    }
    if (dtype == RF_DTYPE_BF16) {
        if (depth == 32) RF_SDPA_LAUNCH(false, 32) else if (depth == 64) RF_SDPA_LAUNCH(false, 64) else RF_SDPA_LAUNCH(false, 128)
    } else {
        if (depth == 32) RF_SDPA_LAUNCH(true, 32) else if (depth == 64) RF_SDPA_LAUNCH(true, 64) else RF_SDPA_LAUNCH(true, 128)
    }
#undef RF_SDPA_LAUNCH
    return rf_check_launch("sdpa_kernel");
}

namespace {
int esim_gather_impl(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows, const void* a_table,
                     int64_t a_rows, int32_t dtype, int32_t batch, int32_t L, int32_t d, float* out, int64_t out_stride,
                     int64_t out_off, uint32_t* stamps, int32_t stamp_ex, void* stream, uint16_t* outb = nullptr,
                     float* ostats = nullptr, int32_t oP = 0, int32_t op0 = 0) {
    RF_REQUIRE(dtype == RF_DTYPE_BF16, "rf_esim_gather_fwd: tables must be BF16");
    RF_REQUIRE(L >= 1 && L <= 128, "rf_esim_gather_fwd: need 1 <= L <= 128 (got %d)", L);
    RF_REQUIRE(d == 64 || d == 128, "rf_esim_gather_fwd: d must be 64 or 128 (got %d)", d);
    RF_REQUIRE(batch >= 0, "rf_esim_gather_fwd: batch < 0");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(q_ids && a_ids && q_table && a_table && (out || (outb && ostats)), "rf_esim_gather_fwd: null pointer");
    RF_REQUIRE(q_rows >= 1 && a_rows >= 1 && q_rows + 1 < (int64_t)kRowNaN && a_rows + 1 < (int64_t)kRowNaN,
               "rf_esim_gather_fwd: table rows must be in [1, 2^32 - 3)");
    RF_REQUIRE(((uintptr_t)q_table & 15) == 0 && ((uintptr_t)a_table & 15) == 0 && ((uintptr_t)q_ids & 3) == 0 &&
                   ((uintptr_t)a_ids & 3) == 0,
               "rf_esim_gather_fwd: tables must be 16-byte and ids 4-byte aligned");
    hipStream_t st = rf_stream(stream);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int nt = (L + 15) >> 4;
    const size_t lds = esim2_gather_lds_bytes(d, nt, esim2_rs(d, nt));
    const int per_cu = lds <= 80 * 1024 ? 2 : 1;
    const int grid = (int)std::min<int64_t>(batch, (int64_t)per_cu * cus);
    const EsimGatherArgs ga{q_ids, a_ids, (const uint16_t*)q_table, (const uint16_t*)a_table, (uint32_t)(q_rows + 1),
                            (uint32_t)(a_rows + 1), stamps, stamp_ex, outb, ostats, oP, op0};
    const int rc = d == 64 ? launch_esim2g<64>(nt, grid, lds, st, batch, L, out, out_stride, out_off, ga)
                           : launch_esim2g<128>(nt, grid, lds, st, batch, L, out, out_stride, out_off, ga);
    if (rc) return rc;
    return rf_check_launch("rf_esim_gather_fwd");
}
}  // namespace

extern "C" int rf_esim_gather_fwd(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows,
                                  const void* a_table, int64_t a_rows, int32_t dtype, int32_t batch, int32_t L, int32_t d,
                                  float* out, int64_t out_stride, int64_t out_off, void* stream) {
    return esim_gather_impl(q_ids, a_ids, q_table, q_rows, a_table, a_rows, dtype, batch, L, d, out, out_stride, out_off,
                            nullptr, 0, stream);
}

// the same attention with the pooled features written as bf16 plus per-32-column-slice (sum, squared deviations
// from the slice mean) pairs of their fp32 values: stats[row][stats_p0 + s], s = 0 .. 6 d / 32 - 1 the slices of the
// 6 d features (column out_off + 32 s ..), stats_P pairs per row — the producer side of rf_linear_lnfold_stats_fwd
// (cfg3: out_off = 32 stats_p0, the slices line up with the consumer's)
extern "C" int rf_esim_gather_stats_fwd(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows,
                                        const void* a_table, int64_t a_rows, int32_t dtype, int32_t batch, int32_t L,
                                        int32_t d, void* out_bf16, int64_t out_stride, int64_t out_off, float* stats,
                                        int32_t stats_P, int32_t stats_p0, void* stream) {
    RF_REQUIRE(out_bf16 && stats, "rf_esim_gather_stats_fwd: null pointer");
    RF_REQUIRE(stats_p0 >= 0 && stats_P >= stats_p0 + 6 * d / 32, "rf_esim_gather_stats_fwd: stats slots out of range");
    RF_REQUIRE(out_off >= 0 && out_stride >= out_off + 6 * d, "rf_esim_gather_stats_fwd: bad output stride / offset");
    return esim_gather_impl(q_ids, a_ids, q_table, q_rows, a_table, a_rows, dtype, batch, L, d, nullptr, out_stride, out_off,
                            nullptr, 0, stream, static_cast<uint16_t*>(out_bf16), stats, stats_P, stats_p0);
}

extern "C" int rf_diag_esim_gather_stamped(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table,
                                           int64_t q_rows, const void* a_table, int64_t a_rows, int32_t dtype,
                                           int32_t batch, int32_t L, int32_t d, float* out, int64_t out_stride,
                                           int64_t out_off, uint32_t* stamps, int32_t stamp_ex, void* stream) {
    RF_REQUIRE(stamps && stamp_ex >= 1, "rf_diag_esim_gather_stamped: need a stamp buffer");
    return esim_gather_impl(q_ids, a_ids, q_table, q_rows, a_table, a_rows, dtype, batch, L, d, out, out_stride, out_off,
                            stamps, stamp_ex, stream);
}
