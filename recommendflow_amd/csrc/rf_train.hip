// rf_train.hip — training backward of the sparse hot path.
//
// Reference: model.fit with tf.keras.optimizers.Adam (example/ranking_search/train.py:96-104). The
// gradient of every Keras Embedding gather is an IndexedSlices over ALL gathered positions of the
// padded [B, Lmax] id tensor (padding positions gather bin 0, dataloader.py:32-33 + Hashing
// mask_value=""), shaped by the pooling combiner's gradient (EmbeddingBag.get_combiner,
// backend/layers/preprocess_layers.py:44-64: reduce_sum / reduce_mean / reduce_max / reduce_min /
// t[0] / t[-1]). OptimizerV2 first deduplicates it (_deduplicate_indexed_slices: unique +
// unsorted_segment_sum, summing in (b, l) order on CPU), then Adam._resource_apply_sparse decays m and v
// over the WHOLE variable, scatter-adds the scaled gradient, and updates every row.
//
// Here (one fused table, all slots of a tower):
//   1. enum      thread per position p -> key = fused-table row (SipHash of its token, or the slot's pad
//                row), value = p; positions are enumerated example-major, so within one row they are
//                already in the reference's (b, l) order
//   2. sort      hipcub radix sort of (row, p) pairs over the row's significant bits (stable)
//   3. heads     segment heads + inclusive scan -> distinct rows (ascending) and segment starts
//   4. reduce    a team of D/4 lanes per distinct row walks its segment IN ORDER, recomputes each
//                position's gradient vector from dout (and, for max/min, from the forward output and
//                the tie counts), and accumulates acc = 0; acc += v like unsorted_segment_sum
//   5. adam      rf_adam_apply: Keras-exact dense Adam (map row -> distinct id, one fused pass over the
//                table: var, m, v read + written once) or lazy (touched rows only; TF-Addons LazyAdam)
// No atomics anywhere: the result is deterministic and bit-identical to oracle/rf_oracle.c.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include "rf_common.h"

namespace {

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

int key_bits(uint64_t max_key) {
    int b = 1;
    while (b < 32 && (max_key >> b) != 0) ++b;
    return b;
}

struct BwdLayout {
    int64_t n;
    int end_bit;
    size_t sort_bytes, scan_bytes;
    size_t off_kin, off_kout, off_vin, off_vout, off_scan, off_seg, off_posoff, off_flag, off_tmp, total;
};

BwdLayout bwd_layout(int64_t n_positions, int32_t n_slots, int64_t table_rows) {
    BwdLayout L{};
    L.n = std::max<int64_t>(n_positions, 1);
    L.end_bit = key_bits((uint64_t)table_rows);  // sentinel key = table_rows (masked padding / bad rows)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, L.sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)L.n, 0, L.end_bit);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, L.scan_bytes, (const int32_t*)nullptr, (int32_t*)nullptr, (int)L.n);
    size_t o = 0;
    const size_t v = a256((size_t)L.n * 4);
    L.off_kin = o; o += v;
    L.off_kout = o; o += v;
    L.off_vin = o; o += v;
    L.off_vout = o; o += v;
    L.off_scan = o; o += v;
    L.off_seg = o; o += a256((size_t)(L.n + 1) * 4);
    L.off_posoff = o; o += a256((size_t)(n_slots + 2) * 8);
    L.off_flag = o; o += 256;
    L.off_tmp = o; o += a256(std::max(L.sort_bytes, L.scan_bytes));
    L.total = o;
    return L;
}

// pos_off[s] = sum_{s' < s} 2 * lmax[s'] (int64), pos_off[S] = positions per example; one block
__global__ __launch_bounds__(1024) void posoff_kernel(const int32_t* __restrict__ lmax, int S, int64_t* __restrict__ pos_off) {
    __shared__ int64_t s_carry;
    __shared__ int64_t s_wave[16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int c0 = 0; c0 < S; c0 += 1024) {
        const int s = c0 + threadIdx.x;
        const int64_t x = s < S ? 2 * (int64_t)max(lmax[s], 0) : 0;
        int64_t incl = x;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        int64_t base = s_carry;
        for (int w = 0; w < wave; ++w) base += s_wave[w];
        if (s < S) pos_off[s] = base + incl - x;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = base + incl;
        __syncthreads();
    }
    if (threadIdx.x == 0) pos_off[S] = s_carry;
}

// last s with pos_off[s] <= r (pos_off strictly increasing except for lmax == 0 slots, which own no positions)
__device__ __forceinline__ int find_slot(const int64_t* __restrict__ pos_off, int S, int64_t r) {
    int lo = 0, hi = S - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pos_off[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

struct Pos {
    int b, s, k, l, L, len;
};

__device__ __forceinline__ Pos decode_pos(uint32_t p, const int64_t* __restrict__ pos_off, int S,
                                          const int32_t* __restrict__ lmax, const int32_t* __restrict__ bag_off) {
    Pos q;
    const int64_t per = pos_off[S];
    q.b = (int)((int64_t)p / per);
    const int64_t r = (int64_t)p - (int64_t)q.b * per;
    q.s = find_slot(pos_off, S, r);
    const int lm = lmax[q.s];
    const int64_t w = r - pos_off[q.s];
    q.k = (int)(w / lm);
    q.l = (int)(w - (int64_t)q.k * lm);
    const int64_t u = (int64_t)q.b * S + q.s;
    const int t0 = bag_off[u];
    q.len = bag_off[u + 1] - t0;
    q.L = lm;
    return q;
}

// Row of table k for bag position l of (b, s): the hashed token (or the slot's pad row) — or, for pooled
// pre-gathered rows (rf_pool_rows_bwd), the distinct-row index row_map gives the logical row 2t + k
// (pad rows: 2 n_tok + 2 s + k), exactly the rows rf_pool_rows_fwd read.
__device__ __forceinline__ int64_t position_row(const rf_slot_desc* sd, int s, int k, int t, bool real,
                                                const uint8_t* __restrict__ tok_bytes, const int32_t* __restrict__ tok_off,
                                                const int32_t* __restrict__ row_map, int64_t n_tok) {
    if (row_map) return real ? (int64_t)row_map[2 * (int64_t)t + k] : (int64_t)row_map[2 * n_tok + 2 * s + k];
    if (real) {
        const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
        return sd->row_base[k] + hash_bucket_dev(sd->salt[k], sd->salt[k], tok_bytes + b0, n, sd->num_bins, sd->mask_empty);
    }
    return sd->row_base[k] + (sd->mask_empty ? 0 : hash_bucket_dev(sd->salt[k], sd->salt[k], tok_bytes, 0, sd->num_bins, 0));
}

__global__ __launch_bounds__(256) void enum_kernel(const rf_slot_desc* __restrict__ slots, int S,
                                                   const uint8_t* __restrict__ tok_bytes,
                                                   const int32_t* __restrict__ tok_off,
                                                   const int32_t* __restrict__ bag_off,
                                                   const int32_t* __restrict__ lmax, int batch, int64_t n_pos,
                                                   const int64_t* __restrict__ pos_off, int64_t table_rows, int masked,
                                                   const int32_t* __restrict__ row_map, int64_t n_tok,
                                                   uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                   int32_t* __restrict__ flag) {
    const uint32_t sentinel = (uint32_t)table_rows;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_pos; p += (int64_t)gridDim.x * blockDim.x) {
        vals[p] = (uint32_t)p;
        const int64_t per = pos_off[S];
        if (p == 0 && n_pos != (int64_t)batch * per) atomicOr(flag, 2);  // caller's n_positions is wrong
        if (per == 0 || p / per >= batch) {
            keys[p] = sentinel;
            continue;
        }
        const Pos q = decode_pos((uint32_t)p, pos_off, S, lmax, bag_off);
        const rf_slot_desc* sd = slots + q.s;
        if (q.len > q.L) atomicOr(flag, 4);  // a bag longer than its lmax: invalid batch
        if (q.l >= q.len && masked) {
            keys[p] = sentinel;
            continue;
        }
        const int t = bag_off[(int64_t)q.b * S + q.s] + q.l;
        const int64_t row = position_row(sd, q.s, q.k, t, q.l < q.len, tok_bytes, tok_off, row_map, n_tok);
        if (row < 0 || row >= table_rows) {
            atomicOr(flag, 1);
            keys[p] = sentinel;
        } else {
            keys[p] = (uint32_t)row;
        }
    }
}

__global__ __launch_bounds__(256) void heads_kernel(const uint32_t* __restrict__ keys, int64_t n, int32_t* __restrict__ head) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

__global__ __launch_bounds__(256) void emit_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ scan,
                                                   int64_t n, uint32_t sentinel, int64_t cap,
                                                   int64_t* __restrict__ uniq_rows, int32_t* __restrict__ seg) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (i != 0 && keys[i] == keys[i - 1]) continue;
        const int64_t u = scan[i] - 1;
        seg[u] = (int32_t)i;  // the sentinel segment (if any) starts where the real ones end
        if (keys[i] != sentinel && u < cap) uniq_rows[u] = keys[i];
    }
}

// n_uniq = distinct rows, or -(error bits) for an invalid batch: 1 row out of range, 2 n_positions !=
// batch * sum_s 2 * lmax[s], 4 a bag longer than its lmax (then the reduce and Adam kernels do nothing)
__global__ void count_kernel(const uint32_t* __restrict__ keys, const int32_t* __restrict__ scan, int64_t n,
                             uint32_t sentinel, const int32_t* __restrict__ flag, int32_t* __restrict__ seg,
                             int32_t* __restrict__ n_uniq) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int32_t total = scan[n - 1];
    const bool has_sentinel = keys[n - 1] == sentinel;
    const int32_t nu = has_sentinel ? total - 1 : total;
    if (!has_sentinel) seg[nu] = (int32_t)n;
    *n_uniq = *flag ? -*flag : nu;
}

// flags raised after count_kernel (prep's alignment check) reach the caller through n_uniq too
__global__ void flag_kernel(const int32_t* __restrict__ flag, int32_t* __restrict__ n_uniq) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && *flag) *n_uniq = -*flag;
}

// max/min tie counts: cnt[b][col + d] = #{l < L : T[row_l][d] == out[b][col + d]} (tf _MinOrMaxGrad num_selected)
__global__ __launch_bounds__(256) void minmax_count_kernel(const rf_slot_desc* __restrict__ slots, int S,
                                                           const uint8_t* __restrict__ tok_bytes,
                                                           const int32_t* __restrict__ tok_off,
                                                           const int32_t* __restrict__ bag_off,
                                                           const int32_t* __restrict__ lmax, int batch, int masked,
                                                           const int32_t* __restrict__ row_map, int64_t n_tok,
                                                           const float* __restrict__ table, int64_t table_rows, int D,
                                                           const float* __restrict__ out, int64_t stride,
                                                           int32_t* __restrict__ cnt) {
    const int64_t n = (int64_t)batch * S * 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(i & 1);
        const int64_t u = i >> 1;
        const int s = (int)(u % S), b = (int)(u / S);
        const rf_slot_desc* sd = slots + s;
        if (sd->combiner != RF_COMB_MAX && sd->combiner != RF_COMB_MIN) continue;
        const int t0 = bag_off[u], len = bag_off[u + 1] - t0;
        const int L = masked ? len : max(lmax[s], len);
        const int64_t pad = position_row(sd, s, k, 0, false, tok_bytes, tok_off, row_map, n_tok);
        const float* o = out + (int64_t)b * stride + sd->out_off + (int64_t)k * D;
        int32_t* c = cnt + (int64_t)b * stride + sd->out_off + (int64_t)k * D;
        for (int d = 0; d < D; ++d) c[d] = 0;
        for (int l = 0; l < L; ++l) {
            const int64_t row = l < len ? position_row(sd, s, k, t0 + l, true, tok_bytes, tok_off, row_map, n_tok) : pad;
            if (row < 0 || row >= table_rows) continue;
            const float* tr = table + row * D;
            for (int d = 0; d < D; ++d) c[d] += tr[d] == o[d] ? 1 : 0;
        }
    }
}

// ---- ordered segment reduce -------------------------------------------------------------------
// After the sort, a parallel prep pass turns every position into (src, aux): src = the float4 index of
// its [slot, k] block in dout (kZero for the exact-zero gradients of first/last at other positions),
// aux = combiner << 24 | L. The reduce then only streams dout rows and adds them in order; no decode
// sits on the serial chain. An accumulator that starts at +0.0 can never become -0.0 under round-to-
// nearest, so adding +0.0 changes nothing: kZero positions add nothing (their row still counts as touched).
constexpr uint32_t kZero = 0xffffffffu;
constexpr int kLong = 256;  // segments longer than this go to the block-per-segment kernel

__global__ __launch_bounds__(256) void prep_kernel(const rf_slot_desc* __restrict__ slots, int S,
                                                   const int32_t* __restrict__ bag_off,
                                                   const int32_t* __restrict__ lmax,
                                                   const int64_t* __restrict__ pos_off, int masked,
                                                   const uint32_t* __restrict__ vals,
                                                   const int32_t* __restrict__ seg,
                                                   const int32_t* __restrict__ n_uniq_p, int D, int64_t stride,
                                                   uint32_t* __restrict__ src, uint32_t* __restrict__ aux,
                                                   int32_t* __restrict__ flag) {
    const int32_t nu = *n_uniq_p;
    if (nu <= 0) return;
    const int64_t n = seg[nu];  // positions of real rows (the sentinel segment, if any, follows)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const Pos q = decode_pos(vals[i], pos_off, S, lmax, bag_off);
        const rf_slot_desc* sd = slots + q.s;
        const int L = masked ? q.len : max(q.L, q.len);
        const int64_t col = (int64_t)q.b * stride + sd->out_off + (int64_t)q.k * D;
        if (col & 3) atomicOr(flag, 8);
        const int comb = sd->combiner;
        const bool zero = (comb == RF_COMB_FIRST && q.l != 0) || (comb == RF_COMB_LAST && q.l != L - 1);
        src[i] = zero ? kZero : (uint32_t)(col >> 2);
        aux[i] = ((uint32_t)comb << 24) | ((uint32_t)L & 0xffffffu);
    }
}

__global__ __launch_bounds__(256) void classify_kernel(const int32_t* __restrict__ seg, const int32_t* __restrict__ n_uniq_p,
                                                       int64_t cap, int32_t* __restrict__ long_list,
                                                       int32_t* __restrict__ long_cnt) {
    const int64_t nu = min<int64_t>(*n_uniq_p, cap);
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (int64_t)gridDim.x * blockDim.x)
        if (seg[u + 1] - seg[u] > kLong) long_list[atomicAdd(long_cnt, 1)] = (int32_t)u;
}

// gradient contribution of one position to the lane's 4 columns
__device__ __forceinline__ float4 pos_value(uint32_t s4, uint32_t a, int lane, const float4& trow,
                                            const float4* __restrict__ dout4, const float4* __restrict__ out4,
                                            const int4* __restrict__ cnt4) {
    if (s4 == kZero) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 g = dout4[(int64_t)s4 + lane];
    const int comb = (int)(a >> 24);
    if (comb == RF_COMB_AVG) {  // tf.reduce_mean gradient: g / L
        const float L = (float)(a & 0xffffffu);
        return make_float4(g.x / L, g.y / L, g.z / L, g.w / L);
    }
    if (comb == RF_COMB_MAX || comb == RF_COMB_MIN) {  // tf _MinOrMaxGrad: (x == y) / num_selected * grad
        const float4 o = out4[(int64_t)s4 + lane];
        const int4 c = cnt4[(int64_t)s4 + lane];
        return make_float4(((trow.x == o.x ? 1.f : 0.f) / (float)c.x) * g.x, ((trow.y == o.y ? 1.f : 0.f) / (float)c.y) * g.y,
                           ((trow.z == o.z ? 1.f : 0.f) / (float)c.z) * g.z, ((trow.w == o.w ? 1.f : 0.f) / (float)c.w) * g.w);
    }
    return g;  // sum, and first/last at their position
}

__device__ __forceinline__ void add4(float4& a, const float4& v) {
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
}

// Short segments: a team of TPR lanes (>= D/4) per row, 4 positions' loads in flight per step.
template <int TPR>
__global__ __launch_bounds__(256) void reduce_short_kernel(const uint32_t* __restrict__ src, const uint32_t* __restrict__ aux,
                                                           const int32_t* __restrict__ seg,
                                                           const int32_t* __restrict__ n_uniq_p, int64_t cap,
                                                           const int64_t* __restrict__ uniq_rows,
                                                           const float* __restrict__ table, int D,
                                                           const float* __restrict__ out, const float* __restrict__ dout,
                                                           const int32_t* __restrict__ cnt, float* __restrict__ uniq_grad) {
    constexpr int TEAMS = 256 / TPR;
    const int team = threadIdx.x / TPR, lane = threadIdx.x % TPR;
    const int64_t nu = min<int64_t>(*n_uniq_p, cap);
    const bool active = lane * 4 < D;
    const auto* dout4 = reinterpret_cast<const float4*>(dout);
    const auto* out4 = reinterpret_cast<const float4*>(out);
    const auto* cnt4 = reinterpret_cast<const int4*>(cnt);
    for (int64_t u = (int64_t)blockIdx.x * TEAMS + team; u < nu; u += (int64_t)gridDim.x * TEAMS) {
        const int i0 = seg[u], i1 = seg[u + 1];
        if (i1 - i0 > kLong || !active) continue;
        const int64_t row = uniq_rows[u];
        const float4 trow = table ? reinterpret_cast<const float4*>(table + row * D)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        int i = i0;
        for (; i + 4 <= i1; i += 4) {
            uint32_t s4[4], a[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                s4[k] = src[i + k];
                a[k] = aux[i + k];
            }
            float4 v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = pos_value(s4[k], a[k], lane, trow, dout4, out4, cnt4);
#pragma unroll
            for (int k = 0; k < 4; ++k) add4(acc, v[k]);
        }
        for (; i < i1; ++i) add4(acc, pos_value(src[i], aux[i], lane, trow, dout4, out4, cnt4));
        reinterpret_cast<float4*>(uniq_grad + u * D)[lane] = acc;
    }
}

// Long segments (Zipf-hot tokens, the padding rows of multi-valued slots): one 1024-thread block per
// row. Every thread computes one (position, float4) value of a chunk of P = 1024 / TPR positions. Two
// register rings keep kDepth chunks in flight: the (src, aux) pairs of chunk c + 2 kDepth and the dout
// values of chunk c + kDepth, so a dout load never waits on its index load. A chunk goes through a
// double-buffered LDS image (one barrier per chunk) and the first team adds it in order: only the adds
// are serial.
template <int TPR>
__global__ __launch_bounds__(1024) void reduce_long_kernel(const uint32_t* __restrict__ src, const uint32_t* __restrict__ aux,
                                                           const int32_t* __restrict__ seg,
                                                           const int32_t* __restrict__ long_list,
                                                           const int32_t* __restrict__ long_cnt,
                                                           const int64_t* __restrict__ uniq_rows,
                                                           const float* __restrict__ table, int D,
                                                           const float* __restrict__ out, const float* __restrict__ dout,
                                                           const int32_t* __restrict__ cnt, float* __restrict__ uniq_grad) {
    constexpr int PPT = TPR >= 32 ? 2 : 1;  // positions per thread per chunk (register budget: 1024 threads)
    constexpr int PT = 1024 / TPR;     // positions per pass of the block
    constexpr int P = PPT * PT;        // positions per chunk (one barrier)
    constexpr int kDepth = 8 / PPT;
    constexpr int G4 = 4;  // 16-byte LDS reads in flight per add group (16 positions)
    constexpr int KD = TPR >= 16 ? TPR / 16 : 1;  // float columns per lane of the adding wave (TPR * 4 floats a row)
    // chunk image transposed, column-major: column j's P values at buf[j * PS + q] (PS = P + 4 keeps the
    // columns 16-byte aligned for the adding wave's ds_read_b128 of 4 positions and spreads their banks)
    constexpr int PS = P + 4;
    __shared__ __attribute__((aligned(16))) float buf[2][TPR * 4 * PS];
    const int t = threadIdx.x, pi = t / TPR, lane = t % TPR;
    const bool active = lane * 4 < D;
    const auto* dout4 = reinterpret_cast<const float4*>(dout);
    const auto* out4 = reinterpret_cast<const float4*>(out);
    const auto* cnt4 = reinterpret_cast<const int4*>(cnt);
    const int nl = *long_cnt;
    for (int j = blockIdx.x; j < nl; j += gridDim.x) {
        const int32_t u = long_list[j];
        const int i0 = seg[u], i1 = seg[u + 1];
        const int64_t row = uniq_rows[u];
        const float4 trow = (active && table) ? reinterpret_cast<const float4*>(table + row * D)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
        const int nch = (i1 - i0 + P - 1) / P;
        // index of this thread's h-th position in chunk c (chunk-local q = h * PT + pi), or -1
        auto pos_of = [&](int c, int h) -> int {
            const int i = i0 + c * P + h * PT + pi;
            return (c < nch && i < i1 && active) ? i : -1;
        };
        uint32_t rs[kDepth][PPT], ra[kDepth][PPT];
        float4 rv[kDepth][PPT];
#pragma unroll
        for (int k = 0; k < kDepth; ++k)
#pragma unroll
            for (int h = 0; h < PPT; ++h) {
                const int i = pos_of(k, h);
                rs[k][h] = i >= 0 ? src[i] : kZero;
                ra[k][h] = i >= 0 ? aux[i] : 0u;
            }
#pragma unroll
        for (int k = 0; k < kDepth; ++k)
#pragma unroll
            for (int h = 0; h < PPT; ++h) {
                rv[k][h] = pos_value(rs[k][h], ra[k][h], lane, trow, dout4, out4, cnt4);
                const int i = pos_of(k + kDepth, h);
                rs[k][h] = i >= 0 ? src[i] : kZero;
                ra[k][h] = i >= 0 ? aux[i] : 0u;
            }
        float acc[KD];
#pragma unroll
        for (int k = 0; k < KD; ++k) acc[k] = 0.f;
        for (int c0 = 0; c0 < nch; c0 += kDepth) {
#pragma unroll
            for (int k = 0; k < kDepth; ++k) {
                const int c = c0 + k;
                if (c < nch) {  // block-uniform
                    float* b = buf[c & 1];
#pragma unroll
                    for (int h = 0; h < PPT; ++h) {  // position q = h * PT + pi, columns lane * 4 .. + 3
                        float* o = b + (lane * 4) * PS + h * PT + pi;
                        o[0] = rv[k][h].x;
                        o[PS] = rv[k][h].y;
                        o[2 * PS] = rv[k][h].z;
                        o[3 * PS] = rv[k][h].w;
                    }
                    __syncthreads();
#pragma unroll
                    for (int h = 0; h < PPT; ++h) {
                        rv[k][h] = pos_value(rs[k][h], ra[k][h], lane, trow, dout4, out4, cnt4);  // chunk c + kDepth
                        const int i = pos_of(c + 2 * kDepth, h);
                        rs[k][h] = i >= 0 ? src[i] : kZero;
                        ra[k][h] = i >= 0 ? aux[i] : 0u;
                    }
                    if (t < 64) {  // wave 0, a lane per float column: one add per position and column, reading
                                   // 4 positions of its column per ds_read_b128
                        const int np = min(P, i1 - (i0 + c * P));
                        const float* col[KD];  // this lane's columns (a dead lane re-reads column 0; never stored)
#pragma unroll
                        for (int k = 0; k < KD; ++k) col[k] = b + (k * 64 + t < D ? k * 64 + t : 0) * PS;
                        int q = 0;
                        for (; q + 4 * G4 <= np; q += 4 * G4) {
                            float4 v[G4][KD];
#pragma unroll
                            for (int r = 0; r < G4; ++r)
#pragma unroll
                                for (int k = 0; k < KD; ++k) v[r][k] = *reinterpret_cast<const float4*>(col[k] + q + 4 * r);
#pragma unroll
                            for (int r = 0; r < G4; ++r)
#pragma unroll
                                for (int k = 0; k < KD; ++k) {
                                    acc[k] += v[r][k].x;
                                    acc[k] += v[r][k].y;
                                    acc[k] += v[r][k].z;
                                    acc[k] += v[r][k].w;
                                }
                        }
                        for (; q < np; ++q)
#pragma unroll
                            for (int k = 0; k < KD; ++k) acc[k] += col[k][q];
                    }
                }
            }
        }
        if (t < 64)
#pragma unroll
            for (int k = 0; k < KD; ++k)
                if (k * 64 + t < D) uniq_grad[(int64_t)u * D + k * 64 + t] = acc[k];
        __syncthreads();
    }
}

// Long segments, RF_FLAG_TREE_REDUCE (opt-in, SURVEY §8d's |d| <= L 2^-23 sum|x| bar instead of the reference's
// CPU order): position group pi (of PT = 1024 / TPR) sums positions i0 + pi, i0 + pi + PT, ... in that order in
// registers (8 positions' loads in flight, no LDS, no barrier per chunk), then the PT partials meet in a fixed
// pairwise tree through LDS. The same assignment and tree for every launch: replay-deterministic.
template <int TPR>
__global__ __launch_bounds__(1024) void reduce_long_tree_kernel(const uint32_t* __restrict__ src,
                                                                const uint32_t* __restrict__ aux,
                                                                const int32_t* __restrict__ seg,
                                                                const int32_t* __restrict__ long_list,
                                                                const int32_t* __restrict__ long_cnt,
                                                                const int64_t* __restrict__ uniq_rows,
                                                                const float* __restrict__ table, int D,
                                                                const float* __restrict__ out,
                                                                const float* __restrict__ dout,
                                                                const int32_t* __restrict__ cnt,
                                                                float* __restrict__ uniq_grad) {
    constexpr int PT = 1024 / TPR;
    constexpr int DEPTH = 8;
    __shared__ float4 part[PT][TPR];
    const int t = threadIdx.x, pi = t / TPR, lane = t % TPR;
    const bool active = lane * 4 < D;
    const auto* dout4 = reinterpret_cast<const float4*>(dout);
    const auto* out4 = reinterpret_cast<const float4*>(out);
    const auto* cnt4 = reinterpret_cast<const int4*>(cnt);
    const int nl = *long_cnt;
    for (int j = blockIdx.x; j < nl; j += gridDim.x) {
        const int32_t u = long_list[j];
        const int i0 = seg[u], i1 = seg[u + 1];
        const int64_t row = uniq_rows[u];
        const float4 trow = (active && table) ? reinterpret_cast<const float4*>(table + row * D)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        // this group's positions i0 + pi + PT * k, DEPTH at a time: every load of a step issued before its adds
        for (int base = i0 + pi; base < i1; base += PT * DEPTH) {
            uint32_t rs[DEPTH], ra[DEPTH];
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) {
                const int i = base + PT * k;
                rs[k] = (i < i1 && active) ? src[i] : kZero;
                ra[k] = (i < i1 && active) ? aux[i] : 0u;
            }
            float4 v[DEPTH];
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) v[k] = pos_value(rs[k], ra[k], lane, trow, dout4, out4, cnt4);
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) add4(acc, v[k]);
        }
        part[pi][lane] = acc;
        __syncthreads();
#pragma unroll
        for (int s = PT / 2; s >= 1; s >>= 1) {
            if (pi < s) {
                float4 a = part[pi][lane];
                add4(a, part[pi + s][lane]);
                part[pi][lane] = a;
            }
            __syncthreads();
        }
        if (pi == 0 && active) reinterpret_cast<float4*>(uniq_grad + (int64_t)u * D)[lane] = part[0][lane];
        __syncthreads();
    }
}

// Long segments, exact CPU order, streamed (D <= 128): the serial adds are the whole critical path of a Zipf-hot
// or padding row (a cfg2 padding row has ~57 K positions), so nothing else waits on them. Wave 0 only adds; the
// other NW - 1 waves produce. Producer wave w takes chunks w - 1, w - 1 + NP, ... of Q positions: one
// index load per lane, then all Q row loads of the chunk in flight at once (lane l = columns l, l + 64, ...; one load
// per position), the mean / max / min transform, a wait for its ring slot to be free, the chunk written column-
// major into the slot, and the slot's ready mark (release). Wave 0 waits for a slot's mark (acquire), reads 4
// positions of each of its columns per ds_read_b128, adds them in order and marks the slot consumed. The marks are
// LDS words at workgroup scope; no block barrier per chunk. Same value per position (pos_value's arithmetic) and
// the same order as reduce_long_kernel: bit-identical results.
// NW waves, Q positions per chunk: <KD 1: 16 waves, Q 64> (15 producers x 64 values), <KD 2: 8 waves, Q 64> (7 producers
// x 128 values, two waves per SIMD for the registers; RF_BWD_LONG_KD2_NARROW=1: 16 waves, Q 32 for A/B)
template <int KD, int NW, int Q>
__global__ __launch_bounds__(64 * NW) void reduce_long_stream_kernel(
    const uint32_t* __restrict__ src, const uint32_t* __restrict__ aux, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ long_list, const int32_t* __restrict__ long_cnt, const int64_t* __restrict__ uniq_rows,
    const float* __restrict__ table, int D, const float* __restrict__ out, const float* __restrict__ dout,
    const int32_t* __restrict__ cnt, float* __restrict__ uniq_grad) {
    static_assert(Q % 4 == 0 && Q <= 64, "Q: 4 .. 64 positions per chunk");
    constexpr int PS = Q + 4;        // column stride: 16-byte aligned, and lane l's column at 4 l (mod 64) banks for
                                     // 16 lanes (PS = 68 or 36), so each 16-lane pass of a ds_read_b128 is conflict-free
    constexpr int SLOT = 64 * KD * PS;
    constexpr int R = KD * Q <= 64 ? 8 : 4;  // ring slots: 139 KB (KD 1, Q 64), 147 KB (KD 2, Q 32), 139 KB (KD 2, Q 64)
    constexpr int NP = NW - 1;
    __shared__ __attribute__((aligned(16))) float ring[R * SLOT];
    __shared__ int ready[R];
    __shared__ int consumed;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int nl = *long_cnt;
    for (int j = blockIdx.x; j < nl; j += gridDim.x) {
        if (threadIdx.x < R) ready[threadIdx.x] = 0;
        if (threadIdx.x == 0) consumed = 0;
        __syncthreads();
        const int32_t u = long_list[j];
        const int i0 = seg[u], i1 = seg[u + 1];
        const int nch = (i1 - i0 + Q - 1) / Q;
        if (wave == 0) {
            float acc[KD];
#pragma unroll
            for (int k = 0; k < KD; ++k) acc[k] = 0.f;
            for (int c = 0; c < nch; ++c) {
                const int sl = c % R;
                while (__hip_atomic_load(&ready[sl], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != c + 1) {
                }
                const float* b = ring + sl * SLOT + lane * PS;  // this lane's columns c * 64 + lane
                const int np = min(Q, i1 - i0 - c * Q);
                if (np == Q) {
                    float4 v[Q / 4][KD];
#pragma unroll
                    for (int r = 0; r < Q / 4; ++r)
#pragma unroll
                        for (int k = 0; k < KD; ++k) v[r][k] = *reinterpret_cast<const float4*>(b + k * 64 * PS + 4 * r);
#pragma unroll
                    for (int r = 0; r < Q / 4; ++r)
#pragma unroll
                        for (int k = 0; k < KD; ++k) {
                            acc[k] += v[r][k].x;
                            acc[k] += v[r][k].y;
                            acc[k] += v[r][k].z;
                            acc[k] += v[r][k].w;
                        }
                } else {
                    for (int q = 0; q < np; ++q)
#pragma unroll
                        for (int k = 0; k < KD; ++k) acc[k] += b[k * 64 * PS + q];
                }
                if (lane == 0) __hip_atomic_store(&consumed, c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#pragma unroll
            for (int k = 0; k < KD; ++k)
                if (k * 64 + lane < D) uniq_grad[(int64_t)u * D + k * 64 + lane] = acc[k];
        } else {
            const int64_t row = uniq_rows[u];
            float tr[KD];
#pragma unroll
            for (int k = 0; k < KD; ++k) tr[k] = (table && k * 64 + lane < D) ? table[row * D + k * 64 + lane] : 0.f;
            // this producer's next chunk's (src, aux) are loaded while the current chunk's rows are in flight, so a
            // chunk costs one memory round trip (its rows), not two (indices, then rows)
            auto idx_load = [&](int c, uint32_t& ms, uint32_t& ma) {
                const int ib = i0 + c * Q;
                const int np = c < nch ? min(Q, i1 - ib) : 0;
                ms = lane < np ? src[ib + lane] : kZero;
                ma = lane < np ? aux[ib + lane] : 0u;
            };
            uint32_t ms_next, ma_next;
            idx_load(wave - 1, ms_next, ma_next);
            for (int c = wave - 1; c < nch; c += NP) {
                const int ib = i0 + c * Q;
                const int np = min(Q, i1 - ib);
                const uint32_t ms = ms_next;
                const uint32_t ma = ma_next;
                float v[Q][KD];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const uint32_t s4 = (uint32_t)__builtin_amdgcn_readlane((int)ms, q);
                    const float* g = dout + (int64_t)s4 * 4 + lane;
                    if (s4 == kZero) {
#pragma unroll
                        for (int k = 0; k < KD; ++k) v[q][k] = 0.f;
                    } else {
#pragma unroll
                        for (int k = 0; k < KD; ++k) v[q][k] = k * 64 + lane < D ? g[k * 64] : 0.f;
                    }
                }
                idx_load(c + NP, ms_next, ma_next);
                // mean / max / min (block-uniform test: any such position in the chunk)
                const int comb_any = __builtin_amdgcn_readfirstlane(
                    (int)(__ballot((lane < np) && ((ma >> 24) == RF_COMB_AVG || (ma >> 24) == RF_COMB_MAX ||
                                                   (ma >> 24) == RF_COMB_MIN)) != 0));
                if (comb_any) {
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        const uint32_t s4 = (uint32_t)__builtin_amdgcn_readlane((int)ms, q);
                        const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)ma, q);
                        if (s4 == kZero) continue;
                        const int comb = (int)(a >> 24);
                        if (comb == RF_COMB_AVG) {
                            const float L = (float)(a & 0xffffffu);
#pragma unroll
                            for (int k = 0; k < KD; ++k) v[q][k] = v[q][k] / L;
                        } else if (comb == RF_COMB_MAX || comb == RF_COMB_MIN) {
#pragma unroll
                            for (int k = 0; k < KD; ++k) {
                                const int64_t e = (int64_t)s4 * 4 + k * 64 + lane;
                                if (k * 64 + lane < D)
                                    v[q][k] = ((tr[k] == out[e] ? 1.f : 0.f) / (float)cnt[e]) * v[q][k];
                            }
                        }
                    }
                }
                while (__hip_atomic_load(&consumed, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < c + 1 - R)
                    __builtin_amdgcn_s_sleep(1);
                float* b = ring + (c % R) * SLOT + lane * PS;
#pragma unroll
                for (int k = 0; k < KD; ++k)
#pragma unroll
                    for (int r = 0; r < Q / 4; ++r)
                        *reinterpret_cast<float4*>(b + k * 64 * PS + 4 * r) =
                            make_float4(v[4 * r][k], v[4 * r + 1][k], v[4 * r + 2][k], v[4 * r + 3][k]);
                if (lane == 0) __hip_atomic_store(&ready[c % R], c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
    }
}

// exact-order long segments: the streamed kernel for D <= 128 (RF_BWD_LONG_LEGACY=1 keeps the barrier-per-chunk one
// for A/B), reduce_long_kernel beyond
bool long_legacy() {
    static const bool v = [] {
        const char* e = std::getenv("RF_BWD_LONG_LEGACY");
        return e && e[0] == '1';
    }();
    return v;
}

bool kd1_eight() {  // RF_BWD_LONG_KD1_8W=1: D <= 64 with 8 waves (A/B)
    static const bool v = [] {
        const char* e = std::getenv("RF_BWD_LONG_KD1_8W");
        return e && e[0] == '1';
    }();
    return v;
}

bool kd2_narrow() {
    static const bool v = [] {
        const char* e = std::getenv("RF_BWD_LONG_KD2_NARROW");
        return e && e[0] == '1';
    }();
    return v;
}

template <int TPR>
void launch_long_exact(int lgrid, hipStream_t st, const uint32_t* src, const uint32_t* aux, const int32_t* seg,
                       const int32_t* long_list, const int32_t* long_cnt, const int64_t* rows, const float* table, int dim,
                       const float* out, const float* dout, const int32_t* cnt, float* grad) {
    if (dim <= 64 && !long_legacy())
        if (kd1_eight())
            hipLaunchKernelGGL((reduce_long_stream_kernel<1, 8, 64>), dim3(lgrid), dim3(64 * 8), 0, st, src, aux, seg,
                               long_list, long_cnt, rows, table, dim, out, dout, cnt, grad);
        else
            hipLaunchKernelGGL((reduce_long_stream_kernel<1, 16, 64>), dim3(lgrid), dim3(64 * 16), 0, st, src, aux, seg,
                               long_list, long_cnt, rows, table, dim, out, dout, cnt, grad);
    else if (dim <= 128 && !long_legacy())
        if (kd2_narrow())
            hipLaunchKernelGGL((reduce_long_stream_kernel<2, 16, 32>), dim3(lgrid), dim3(64 * 16), 0, st, src, aux, seg,
                               long_list, long_cnt, rows, table, dim, out, dout, cnt, grad);
        else
            hipLaunchKernelGGL((reduce_long_stream_kernel<2, 8, 64>), dim3(lgrid), dim3(64 * 8), 0, st, src, aux, seg,
                               long_list, long_cnt, rows, table, dim, out, dout, cnt, grad);
    else
        hipLaunchKernelGGL(reduce_long_kernel<TPR>, dim3(lgrid), dim3(1024), 0, st, src, aux, seg, long_list, long_cnt,
                           rows, table, dim, out, dout, cnt, grad);
}

// ---- owner-side gradient sum (sharded training) ------------------------------------------------
__global__ __launch_bounds__(256) void ids_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t range,
                                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t id = ids[i];
        keys[i] = (id >= 0 && id < range) ? (uint32_t)id : (uint32_t)range;
        vals[i] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void prep_sum_kernel(const uint32_t* __restrict__ vals, const int32_t* __restrict__ seg,
                                                       const int32_t* __restrict__ n_uniq_p, int D4,
                                                       uint32_t* __restrict__ src, uint32_t* __restrict__ aux) {
    const int32_t nu = *n_uniq_p;
    if (nu <= 0) return;
    const int64_t n = seg[nu];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        src[i] = vals[i] * (uint32_t)D4;
        aux[i] = ((uint32_t)RF_COMB_SUM << 24) | 1u;
    }
}

// ---- Adam --------------------------------------------------------------------------------------
struct AdamCoef {
    float lr, b1, b2, omb1, omb2, eps;
};

__device__ __forceinline__ void adam_elem(float& w, float& m, float& v, bool touched, float g, const AdamCoef& c) {
    // Adam._resource_apply_sparse: m_t = m * beta_1; m_t = scatter_add(m_t, g * (1 - beta_1)); likewise v
    // with g * g; var -= lr * m_t / (sqrt(v_t) + epsilon)   (lr already carries sqrt(1-b2^t)/(1-b1^t))
    float mt = m * c.b1;
    float vt = v * c.b2;
    if (touched) {
        mt = mt + g * c.omb1;
        vt = vt + (g * g) * c.omb2;
    }
    m = mt;
    v = vt;
    w = w - (c.lr * mt) / (sqrtf(vt) + c.eps);
}

__global__ __launch_bounds__(256) void map_fill_kernel(const int64_t* __restrict__ uniq_rows, const int32_t* __restrict__ n_uniq_p,
                                                       int64_t cap, int32_t* __restrict__ map) {
    const int64_t nu = min<int64_t>(*n_uniq_p, cap);
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < nu; u += (int64_t)gridDim.x * blockDim.x)
        map[uniq_rows[u]] = (int32_t)u;
}

// dense: every element of the table (float4 granules); row -> distinct id through `map`
__global__ __launch_bounds__(256) void adam_dense_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                                         int64_t n4, int D4, const int32_t* __restrict__ map,
                                                         const float* __restrict__ grad, AdamCoef c) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t row = i / D4;
        const int j = (int)(i - row * D4);
        const int32_t u = map[row];
        float4 wv = reinterpret_cast<float4*>(w)[i];
        float4 mv = reinterpret_cast<float4*>(m)[i];
        float4 vv = reinterpret_cast<float4*>(v)[i];
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool t = u >= 0;
        if (t) g = reinterpret_cast<const float4*>(grad)[(int64_t)u * D4 + j];
        adam_elem(wv.x, mv.x, vv.x, t, g.x, c);
        adam_elem(wv.y, mv.y, vv.y, t, g.y, c);
        adam_elem(wv.z, mv.z, vv.z, t, g.z, c);
        adam_elem(wv.w, mv.w, vv.w, t, g.w, c);
        reinterpret_cast<float4*>(w)[i] = wv;
        reinterpret_cast<float4*>(m)[i] = mv;
        reinterpret_cast<float4*>(v)[i] = vv;
    }
}

// the rows NOT in the gradient (map < 0) only: their Keras update needs no gradient, so it can run before the
// gradient exists; the listed rows then take the lazy kernel with their gradient (together: exactly the dense step)
// U float4 slots per thread per pass, every load issued before the first update: this kernel runs on a capped
// grid beside the towers' GEMMs, so its bandwidth comes from loads in flight per wave, not from more waves
template <int U>
__global__ __launch_bounds__(256) void adam_untouched_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                                             int64_t n4, int D4, const int32_t* __restrict__ map,
                                                             const int32_t* __restrict__ n_uniq, AdamCoef c) {
    // an invalid batch (the plan's error flag, n_uniq < 0) lists no row: its step still counts and every row takes
    // the untouched update, as adam_dense_kernel and the deferred replay of that step do (one rule for all modes)
    (void)n_uniq;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n4; base += stride) {
        bool act[U];
        float4 wv[U], mv[U], vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + (int64_t)u * blockDim.x;
            act[u] = i < n4 && map[i / D4] < 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (act[u]) {
                const int64_t i = base + (int64_t)u * blockDim.x;
                wv[u] = reinterpret_cast<float4*>(w)[i];
                mv[u] = reinterpret_cast<float4*>(m)[i];
                vv[u] = reinterpret_cast<float4*>(v)[i];
            }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (act[u]) {
                const int64_t i = base + (int64_t)u * blockDim.x;
                adam_elem(wv[u].x, mv[u].x, vv[u].x, false, 0.f, c);
                adam_elem(wv[u].y, mv[u].y, vv[u].y, false, 0.f, c);
                adam_elem(wv[u].z, mv[u].z, vv[u].z, false, 0.f, c);
                adam_elem(wv[u].w, mv[u].w, vv[u].w, false, 0.f, c);
                reinterpret_cast<float4*>(w)[i] = wv[u];
                reinterpret_cast<float4*>(m)[i] = mv[u];
                reinterpret_cast<float4*>(v)[i] = vv[u];
            }
    }
}

// Deferred dense step (exact): a row's untouched Keras steps l + 1 .. t_now are applied when the row is next
// listed (before a forward reads it, or before its touched update), one step at a time with that step's lr
// (lr_log[s]) through adam_elem's untouched branch — the fp32 expressions adam_untouched_kernel would have run
// step by step, in the same order, so the row's bits are the same. A team of TPR lanes per row (one wave holds a
// whole team); lane 0 claims the row by swapping last[r] from the value it read to t_set (compare-and-swap), so a
// row listed twice (the ids several ranks requested from one shard) is replayed once. uniq_rows == nullptr: every
// row (materialize); n_uniq_p == nullptr: all cap listed rows; rows outside [0, table_rows) are skipped.
template <int TPR>
__global__ __launch_bounds__(256) void adam_replay_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                                          int64_t table_rows, int D4, const int64_t* __restrict__ uniq_rows,
                                                          const int32_t* __restrict__ n_uniq_p, int64_t cap,
                                                          int32_t* __restrict__ last, int t_now, int t_set,
                                                          const float* __restrict__ lr_log, AdamCoef c) {
    constexpr int TEAMS = 256 / TPR;
    const int team = threadIdx.x / TPR, lane = threadIdx.x % TPR;
    int64_t nu = table_rows;
    if (uniq_rows) {
        const int32_t n = n_uniq_p ? *n_uniq_p : 0;
        if (n < 0) return;  // invalid batch (the plan's error flag): no row moves
        nu = n_uniq_p ? min<int64_t>(n, cap) : cap;
    }
    const int base = (threadIdx.x & 63) - lane;  // the team's first lane in the wave
    for (int64_t u = (int64_t)blockIdx.x * TEAMS + team; u < nu; u += (int64_t)gridDim.x * TEAMS) {
        const int64_t r = uniq_rows ? uniq_rows[u] : u;
        if (r < 0 || r >= table_rows) continue;  // team-uniform
        int l = 0;
        if (lane == 0) {
            l = __hip_atomic_load(&last[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (l < t_set) {
                int e = l;
                if (!__hip_atomic_compare_exchange_strong(&last[r], &e, t_set, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT))
                    l = t_set;  // another team holds this row
            }
        }
        l = __shfl(l, base, 64);
        if (l < t_now) {
            for (int j = lane; j < D4; j += TPR) {
                const int64_t i = r * D4 + j;
                float4 wv = reinterpret_cast<float4*>(w)[i];
                float4 mv = reinterpret_cast<float4*>(m)[i];
                float4 vv = reinterpret_cast<float4*>(v)[i];
                AdamCoef cs = c;
                for (int s = l + 1; s <= t_now; ++s) {
                    cs.lr = lr_log[s];
                    adam_elem(wv.x, mv.x, vv.x, false, 0.f, cs);
                    adam_elem(wv.y, mv.y, vv.y, false, 0.f, cs);
                    adam_elem(wv.z, mv.z, vv.z, false, 0.f, cs);
                    adam_elem(wv.w, mv.w, vv.w, false, 0.f, cs);
                }
                reinterpret_cast<float4*>(w)[i] = wv;
                reinterpret_cast<float4*>(m)[i] = mv;
                reinterpret_cast<float4*>(v)[i] = vv;
            }
        }
    }
}

// lazy: touched rows only
// last != nullptr (the deferred step, rows already current): also marks each row current through t_set
__global__ __launch_bounds__(256) void adam_lazy_kernel(float* __restrict__ w, float* __restrict__ m, float* __restrict__ v,
                                                        int D4, const int64_t* __restrict__ uniq_rows,
                                                        const int32_t* __restrict__ n_uniq_p, int64_t cap,
                                                        const float* __restrict__ grad, AdamCoef c,
                                                        int32_t* __restrict__ last = nullptr, int t_set = 0) {
    const int64_t nu = min<int64_t>(*n_uniq_p, cap);
    const int64_t n4 = nu * D4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = i / D4;
        const int j = (int)(i - u * D4);
        if (last && j == 0) last[uniq_rows[u]] = t_set;
        const int64_t e = uniq_rows[u] * D4 + j;
        float4 wv = reinterpret_cast<float4*>(w)[e];
        float4 mv = reinterpret_cast<float4*>(m)[e];
        float4 vv = reinterpret_cast<float4*>(v)[e];
        const float4 g = reinterpret_cast<const float4*>(grad)[i];
        adam_elem(wv.x, mv.x, vv.x, true, g.x, c);
        adam_elem(wv.y, mv.y, vv.y, true, g.y, c);
        adam_elem(wv.z, mv.z, vv.z, true, g.z, c);
        adam_elem(wv.w, mv.w, vv.w, true, g.w, c);
        reinterpret_cast<float4*>(w)[e] = wv;
        reinterpret_cast<float4*>(m)[e] = mv;
        reinterpret_cast<float4*>(v)[e] = vv;
    }
}

// Dense variables (the towers): ResourceApplyAdam, the form Keras' Adam._resource_apply_dense runs —
// m += (g - m)(1 - beta_1); v += (g^2 - v)(1 - beta_2); var -= m lr / (sqrt(v) + epsilon)
__device__ __forceinline__ void adam_dense_elem(float& w, float& m, float& v, float g, const AdamCoef& c) {
    m = m + (g - m) * c.omb1;
    v = v + (g * g - v) * c.omb2;
    w = w - (m * c.lr) / (sqrtf(v) + c.eps);
}

template <int V>
__global__ __launch_bounds__(256) void adam_dense_flat_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                              float* __restrict__ m, float* __restrict__ v, int64_t n, AdamCoef c) {
    const int64_t nv = n / V;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
        if constexpr (V == 4) {
            float4 wv = reinterpret_cast<float4*>(w)[i], mv = reinterpret_cast<float4*>(m)[i], vv = reinterpret_cast<float4*>(v)[i];
            const float4 gv = reinterpret_cast<const float4*>(g)[i];
            adam_dense_elem(wv.x, mv.x, vv.x, gv.x, c);
            adam_dense_elem(wv.y, mv.y, vv.y, gv.y, c);
            adam_dense_elem(wv.z, mv.z, vv.z, gv.z, c);
            adam_dense_elem(wv.w, mv.w, vv.w, gv.w, c);
            reinterpret_cast<float4*>(w)[i] = wv;
            reinterpret_cast<float4*>(m)[i] = mv;
            reinterpret_cast<float4*>(v)[i] = vv;
        } else {
            adam_dense_elem(w[i], m[i], v[i], g[i], c);
        }
    }
}

// every tensor of a list in one launch: blockIdx.y = tensor, blockIdx.x strides its elements (float4 when the
// tensor's four pointers are 16-byte aligned and n % 4 == 0)
__global__ __launch_bounds__(256) void adam_dense_multi_kernel(const rf_adam_tensor* __restrict__ ts, AdamCoef c) {
    const rf_adam_tensor t = ts[blockIdx.y];
    const bool v4 = t.n % 4 == 0 && ((((uintptr_t)t.w | (uintptr_t)t.g | (uintptr_t)t.m | (uintptr_t)t.v) & 15) == 0);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    if (v4) {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n / 4; i += stride) {
            float4 wv = reinterpret_cast<float4*>(t.w)[i], mv = reinterpret_cast<float4*>(t.m)[i],
                   vv = reinterpret_cast<float4*>(t.v)[i];
            const float4 gv = reinterpret_cast<const float4*>(t.g)[i];
            adam_dense_elem(wv.x, mv.x, vv.x, gv.x, c);
            adam_dense_elem(wv.y, mv.y, vv.y, gv.y, c);
            adam_dense_elem(wv.z, mv.z, vv.z, gv.z, c);
            adam_dense_elem(wv.w, mv.w, vv.w, gv.w, c);
            reinterpret_cast<float4*>(t.w)[i] = wv;
            reinterpret_cast<float4*>(t.m)[i] = mv;
            reinterpret_cast<float4*>(t.v)[i] = vv;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < t.n; i += stride)
            adam_dense_elem(t.w[i], t.m[i], t.v[i], t.g[i], c);
    }
}

int grid_of(int64_t n, int cap = 256 * 64) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, cap)); }

}  // namespace

extern "C" size_t rf_embed_bwd_ws_bytes(int64_t n_positions, int32_t n_slots, int64_t table_rows) {
    if (n_positions < 0 || n_slots < 1 || table_rows < 1) return 0;
    return bwd_layout(n_positions, n_slots, table_rows).total;
}

namespace {
// shared by rf_fused_hash_embed_bwd (rows = hashed tokens) and rf_pool_rows_bwd (rows = row_map of the
// pre-gathered logical rows; `table` = the gathered rows, table_rows = their count)
int embed_bwd_impl(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                   const int32_t* row_map, int64_t n_tok, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                   int64_t n_positions, const float* table, int64_t table_rows, int32_t dim, const float* out,
                   const float* dout, int64_t out_stride, int32_t flags, int32_t* minmax_count, int64_t* uniq_rows,
                   float* uniq_grad, int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream,
                   int mode = 0) {
    // mode 0: everything; 1: the plan (enumerate, sort, segment, classify: the batch alone decides it, so it can
    // run before dout exists); 2: the reduce of a plan already in ws (minmax counts, segment sums, flag)
    RF_REQUIRE(n_slots >= 1 && batch >= 0 && n_positions >= 0, "rf_fused_hash_embed_bwd: need n_slots >= 1, batch >= 0, n_positions >= 0");
    RF_REQUIRE(n_positions < ((int64_t)1 << 32) - 1, "rf_fused_hash_embed_bwd: n_positions must be < 2^32 - 1");
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 32) - 1, "rf_fused_hash_embed_bwd: table_rows must be in [1, 2^32 - 1)");
    RF_REQUIRE(dim >= 4 && dim <= 256 && dim % 4 == 0, "rf_fused_hash_embed_bwd: dim must be a multiple of 4 in [4, 256]");
    RF_REQUIRE(out_stride % 4 == 0 && out_stride >= 2 * (int64_t)dim, "rf_fused_hash_embed_bwd: out_stride must be a multiple of 4");
    RF_REQUIRE((flags & ~(RF_FLAG_MASK_PADDING | RF_FLAG_TREE_REDUCE)) == 0,
               "rf_fused_hash_embed_bwd: only RF_FLAG_MASK_PADDING and RF_FLAG_TREE_REDUCE are accepted");
    RF_REQUIRE(uniq_cap >= 0 && n_uniq && ws, "rf_fused_hash_embed_bwd: null pointer");
    const BwdLayout lay = bwd_layout(n_positions, n_slots, table_rows);
    RF_REQUIRE(ws_bytes >= lay.total, "rf_fused_hash_embed_bwd: workspace too small (%zu < %zu)", ws_bytes, lay.total);
    hipStream_t st = rf_stream(stream);
    if (n_positions == 0 || batch == 0) {
        if (hipMemsetAsync(n_uniq, 0, sizeof(int32_t), st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_fused_hash_embed_bwd: memset failed");
        return RF_OK;
    }
    RF_REQUIRE(d_slots && (row_map || (tok_bytes && tok_off)) && bag_off && lmax && uniq_rows, "rf_fused_hash_embed_bwd: null pointer");
    if (mode != 1) {
        RF_REQUIRE(table && dout && uniq_grad, "rf_fused_hash_embed_bwd: null pointer");
        RF_REQUIRE(((uintptr_t)table & 15) == 0 && ((uintptr_t)dout & 15) == 0 && ((uintptr_t)uniq_grad & 15) == 0 &&
                   (!out || ((uintptr_t)out & 15) == 0) && (!minmax_count || ((uintptr_t)minmax_count & 15) == 0),
                   "rf_fused_hash_embed_bwd: buffers must be 16-byte aligned");
    }
    const int masked = (flags & RF_FLAG_MASK_PADDING) ? 1 : 0;
    char* w = static_cast<char*>(ws);
    auto* kin = reinterpret_cast<uint32_t*>(w + lay.off_kin);
    auto* kout = reinterpret_cast<uint32_t*>(w + lay.off_kout);
    auto* vin = reinterpret_cast<uint32_t*>(w + lay.off_vin);
    auto* vout = reinterpret_cast<uint32_t*>(w + lay.off_vout);
    auto* scan = reinterpret_cast<int32_t*>(w + lay.off_scan);
    auto* seg = reinterpret_cast<int32_t*>(w + lay.off_seg);
    auto* pos_off = reinterpret_cast<int64_t*>(w + lay.off_posoff);
    auto* flag = reinterpret_cast<int32_t*>(w + lay.off_flag);
    void* tmp = w + lay.off_tmp;
    const int64_t n = n_positions;
    const uint32_t sentinel = (uint32_t)table_rows;
    uint32_t* src = kin;
    uint32_t* aux = vin;
    int32_t* long_list = scan;
    int32_t* long_cnt = flag + 1;
    const int64_t max_u = std::min<int64_t>(std::min<int64_t>(n, table_rows), uniq_cap);
    if (mode != 2) {
    if (hipMemsetAsync(flag, 0, 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_fused_hash_embed_bwd: memset failed");
    hipLaunchKernelGGL(posoff_kernel, dim3(1), dim3(1024), 0, st, lmax, n_slots, pos_off);
    hipLaunchKernelGGL(enum_kernel, dim3(grid_of(n)), dim3(256), 0, st, d_slots, n_slots, tok_bytes, tok_off, bag_off,
                       lmax, batch, n, pos_off, table_rows, masked, row_map, n_tok, kin, vin, flag);
    size_t sb = lay.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, sb, kin, kout, vin, vout, (int)n, 0, lay.end_bit, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_fused_hash_embed_bwd: radix sort failed");
    hipLaunchKernelGGL(heads_kernel, dim3(grid_of(n)), dim3(256), 0, st, kout, n, scan);
    size_t cb = lay.scan_bytes;
    if (hipcub::DeviceScan::InclusiveSum(tmp, cb, scan, scan, (int)n, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_fused_hash_embed_bwd: scan failed");
    hipLaunchKernelGGL(emit_kernel, dim3(grid_of(n)), dim3(256), 0, st, kout, scan, n, sentinel, uniq_cap, uniq_rows, seg);
    hipLaunchKernelGGL(count_kernel, dim3(1), dim3(64), 0, st, kout, scan, n, sentinel, flag, seg, n_uniq);
    // prep (src/aux into the now-free pre-sort buffers) and the long-segment list (into the free scan buffer)
    if (hipMemsetAsync(long_cnt, 0, 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_fused_hash_embed_bwd: memset failed");
    hipLaunchKernelGGL(prep_kernel, dim3(grid_of(n)), dim3(256), 0, st, d_slots, n_slots, bag_off, lmax, pos_off, masked,
                       vout, seg, n_uniq, dim, out_stride, src, aux, flag);
    hipLaunchKernelGGL(classify_kernel, dim3(grid_of(max_u)), dim3(256), 0, st, seg, n_uniq, uniq_cap, long_list, long_cnt);
    }
    if (mode == 1) {
        // the plan half reports prep's alignment flag through n_uniq too, so a consumer of the plan alone (the
        // untouched-row Adam on the side stream) sees an invalid batch before it moves any row
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, n_uniq);
        return rf_check_launch("rf_fused_hash_embed_bwd_plan");
    }
    if (minmax_count) {
        RF_REQUIRE(out, "rf_fused_hash_embed_bwd: max/min pooling needs the forward output");
        hipLaunchKernelGGL(minmax_count_kernel, dim3(grid_of((int64_t)batch * n_slots * 2)), dim3(256), 0, st, d_slots,
                           n_slots, tok_bytes, tok_off, bag_off, lmax, batch, masked, row_map, n_tok, table, table_rows, dim, out,
                           out_stride, minmax_count);
    }
    auto launch = [&](auto tpr) {
        constexpr int TPR = decltype(tpr)::value;
        const int teams = 256 / TPR;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((max_u + teams - 1) / teams, 256 * 64));
        const int lgrid = (int)std::max<int64_t>(1, std::min<int64_t>(n / kLong + 1, 1024));
        if (flags & RF_FLAG_TREE_REDUCE)
            hipLaunchKernelGGL(reduce_long_tree_kernel<TPR>, dim3(lgrid), dim3(1024), 0, st, src, aux, seg, long_list,
                               long_cnt, uniq_rows, table, dim, out, dout, minmax_count, uniq_grad);
        else
            launch_long_exact<TPR>(lgrid, st, src, aux, seg, long_list, long_cnt, uniq_rows, table, dim, out, dout,
                                   minmax_count, uniq_grad);
        hipLaunchKernelGGL(reduce_short_kernel<TPR>, dim3(grid), dim3(256), 0, st, src, aux, seg, n_uniq, uniq_cap,
                           uniq_rows, table, dim, out, dout, minmax_count, uniq_grad);
    };
    const int d4 = dim / 4;
    if (d4 <= 1) launch(std::integral_constant<int, 1>{});
    else if (d4 <= 2) launch(std::integral_constant<int, 2>{});
    else if (d4 <= 4) launch(std::integral_constant<int, 4>{});
    else if (d4 <= 8) launch(std::integral_constant<int, 8>{});
    else if (d4 <= 16) launch(std::integral_constant<int, 16>{});
    else if (d4 <= 32) launch(std::integral_constant<int, 32>{});
    else launch(std::integral_constant<int, 64>{});
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, n_uniq);  // prep's alignment flag
    return rf_check_launch("rf_fused_hash_embed_bwd");
}
}  // namespace

extern "C" int rf_fused_hash_embed_bwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                       const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                       int32_t batch, int64_t n_positions, const float* table, int64_t table_rows,
                                       int32_t dim, const float* out, const float* dout, int64_t out_stride,
                                       int32_t flags, int32_t* minmax_count, int64_t* uniq_rows, float* uniq_grad,
                                       int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream) {
    return embed_bwd_impl(d_slots, n_slots, tok_bytes, tok_off, nullptr, 0, bag_off, lmax, batch, n_positions, table,
                          table_rows, dim, out, dout, out_stride, flags, minmax_count, uniq_rows, uniq_grad, uniq_cap,
                          n_uniq, ws, ws_bytes, stream);
}

extern "C" int rf_fused_hash_embed_bwd_plan(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                            const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                            int32_t batch, int64_t n_positions, int64_t table_rows, int32_t dim,
                                            int64_t out_stride, int32_t flags, int64_t* uniq_rows, int64_t uniq_cap,
                                            int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream) {
    return embed_bwd_impl(d_slots, n_slots, tok_bytes, tok_off, nullptr, 0, bag_off, lmax, batch, n_positions, nullptr,
                          table_rows, dim, nullptr, nullptr, out_stride, flags, nullptr, uniq_rows, nullptr, uniq_cap, n_uniq,
                          ws, ws_bytes, stream, 1);
}

extern "C" int rf_fused_hash_embed_bwd_reduce(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                              const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                              int32_t batch, int64_t n_positions, const float* table, int64_t table_rows,
                                              int32_t dim, const float* out, const float* dout, int64_t out_stride,
                                              int32_t flags, int32_t* minmax_count, int64_t* uniq_rows, float* uniq_grad,
                                              int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream) {
    return embed_bwd_impl(d_slots, n_slots, tok_bytes, tok_off, nullptr, 0, bag_off, lmax, batch, n_positions, table,
                          table_rows, dim, out, dout, out_stride, flags, minmax_count, uniq_rows, uniq_grad, uniq_cap,
                          n_uniq, ws, ws_bytes, stream, 2);
}

extern "C" int rf_pool_rows_bwd(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                                int32_t batch, int64_t n_tok, int64_t n_positions, const int32_t* row_map,
                                const float* gathered, int64_t n_rows, int32_t dim, const float* out, const float* dout,
                                int64_t out_stride, int32_t flags, int32_t* minmax_count, int64_t* uniq_rows,
                                float* uniq_grad, int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes,
                                void* stream) {
    RF_REQUIRE(row_map, "rf_pool_rows_bwd: row_map is required");
    return embed_bwd_impl(d_slots, n_slots, nullptr, nullptr, row_map, n_tok, bag_off, lmax, batch, n_positions, gathered,
                          n_rows, dim, out, dout, out_stride, flags, minmax_count, uniq_rows, uniq_grad, uniq_cap, n_uniq,
                          ws, ws_bytes, stream);
}

extern "C" size_t rf_segment_sum_ws_bytes(int64_t n, int64_t id_range) {
    if (n < 0 || id_range < 1) return 0;
    return bwd_layout(n, 1, id_range).total;
}

extern "C" int rf_segment_sum_rows(const int64_t* ids, const float* vals, int64_t n, int32_t dim, int64_t id_range,
                                   int64_t* uniq_ids, float* uniq_vals, int64_t uniq_cap, int32_t* n_uniq, void* ws,
                                   size_t ws_bytes, void* stream) {
    RF_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "rf_segment_sum_rows: n must be in [0, 2^31)");
    RF_REQUIRE(id_range >= 1 && id_range < ((int64_t)1 << 32) - 1, "rf_segment_sum_rows: id_range must be in [1, 2^32 - 1)");
    RF_REQUIRE(dim >= 4 && dim <= 256 && dim % 4 == 0, "rf_segment_sum_rows: dim must be a multiple of 4 in [4, 256]");
    RF_REQUIRE(n_uniq && ws && uniq_cap >= 0, "rf_segment_sum_rows: null pointer");
    const BwdLayout lay = bwd_layout(n, 1, id_range);
    RF_REQUIRE(ws_bytes >= lay.total, "rf_segment_sum_rows: workspace too small (%zu < %zu)", ws_bytes, lay.total);
    hipStream_t st = rf_stream(stream);
    if (n == 0) {
        if (hipMemsetAsync(n_uniq, 0, 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_segment_sum_rows: memset failed");
        return RF_OK;
    }
    RF_REQUIRE(ids && vals && uniq_ids && uniq_vals, "rf_segment_sum_rows: null pointer");
    RF_REQUIRE((((uintptr_t)vals | (uintptr_t)uniq_vals) & 15) == 0, "rf_segment_sum_rows: buffers must be 16-byte aligned");
    char* w = static_cast<char*>(ws);
    auto* kin = reinterpret_cast<uint32_t*>(w + lay.off_kin);
    auto* kout = reinterpret_cast<uint32_t*>(w + lay.off_kout);
    auto* vin = reinterpret_cast<uint32_t*>(w + lay.off_vin);
    auto* vout = reinterpret_cast<uint32_t*>(w + lay.off_vout);
    auto* scan = reinterpret_cast<int32_t*>(w + lay.off_scan);
    auto* seg = reinterpret_cast<int32_t*>(w + lay.off_seg);
    auto* flag = reinterpret_cast<int32_t*>(w + lay.off_flag);
    void* tmp = w + lay.off_tmp;
    const uint32_t sentinel = (uint32_t)id_range;
    if (hipMemsetAsync(flag, 0, 8, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_segment_sum_rows: memset failed");
    hipLaunchKernelGGL(ids_kernel, dim3(grid_of(n)), dim3(256), 0, st, ids, n, id_range, kin, vin);
    size_t sb = lay.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, sb, kin, kout, vin, vout, (int)n, 0, lay.end_bit, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_segment_sum_rows: radix sort failed");
    hipLaunchKernelGGL(heads_kernel, dim3(grid_of(n)), dim3(256), 0, st, kout, n, scan);
    size_t cb = lay.scan_bytes;
    if (hipcub::DeviceScan::InclusiveSum(tmp, cb, scan, scan, (int)n, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_segment_sum_rows: scan failed");
    hipLaunchKernelGGL(emit_kernel, dim3(grid_of(n)), dim3(256), 0, st, kout, scan, n, sentinel, uniq_cap, uniq_ids, seg);
    hipLaunchKernelGGL(count_kernel, dim3(1), dim3(64), 0, st, kout, scan, n, sentinel, flag, seg, n_uniq);
    uint32_t* src = kin;
    uint32_t* aux = vin;
    int32_t* long_list = scan;
    int32_t* long_cnt = flag + 1;
    hipLaunchKernelGGL(prep_sum_kernel, dim3(grid_of(n)), dim3(256), 0, st, vout, seg, n_uniq, dim / 4, src, aux);
    const int64_t max_u = std::min<int64_t>(std::min<int64_t>(n, id_range), uniq_cap);
    hipLaunchKernelGGL(classify_kernel, dim3(grid_of(max_u)), dim3(256), 0, st, seg, n_uniq, uniq_cap, long_list, long_cnt);
    auto launch = [&](auto tpr) {
        constexpr int TPR = decltype(tpr)::value;
        const int teams = 256 / TPR;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((max_u + teams - 1) / teams, 256 * 64));
        hipLaunchKernelGGL(reduce_short_kernel<TPR>, dim3(grid), dim3(256), 0, st, src, aux, seg, n_uniq, uniq_cap,
                           uniq_ids, nullptr, dim, nullptr, vals, nullptr, uniq_vals);
        const int lgrid = (int)std::max<int64_t>(1, std::min<int64_t>(n / kLong + 1, 1024));
        launch_long_exact<TPR>(lgrid, st, src, aux, seg, long_list, long_cnt, uniq_ids, nullptr, dim, nullptr, vals,
                               nullptr, uniq_vals);
    };
    const int d4 = dim / 4;
    if (d4 <= 1) launch(std::integral_constant<int, 1>{});
    else if (d4 <= 2) launch(std::integral_constant<int, 2>{});
    else if (d4 <= 4) launch(std::integral_constant<int, 4>{});
    else if (d4 <= 8) launch(std::integral_constant<int, 8>{});
    else if (d4 <= 16) launch(std::integral_constant<int, 16>{});
    else if (d4 <= 32) launch(std::integral_constant<int, 32>{});
    else launch(std::integral_constant<int, 64>{});
    return rf_check_launch("rf_segment_sum_rows");
}

extern "C" size_t rf_adam_ws_bytes(int64_t table_rows, int32_t lazy) {
    if (table_rows < 1) return 0;
    return lazy ? 256 : a256((size_t)table_rows * 4);
}

extern "C" int rf_adam_apply(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                             const float* uniq_grad, const int32_t* n_uniq, int64_t uniq_cap, float lr, float beta1,
                             float beta2, float epsilon, int32_t lazy, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 31), "rf_adam_apply: table_rows must be in [1, 2^31)");
    RF_REQUIRE(dim >= 4 && dim % 4 == 0, "rf_adam_apply: dim must be a multiple of 4");
    RF_REQUIRE(table && m && v && n_uniq && (uniq_cap == 0 || (uniq_rows && uniq_grad)), "rf_adam_apply: null pointer");
    RF_REQUIRE((((uintptr_t)table | (uintptr_t)m | (uintptr_t)v | (uintptr_t)uniq_grad) & 15) == 0,
               "rf_adam_apply: buffers must be 16-byte aligned");
    RF_REQUIRE(ws_bytes >= rf_adam_ws_bytes(table_rows, lazy) && (lazy || ws), "rf_adam_apply: workspace too small");
    hipStream_t st = rf_stream(stream);
    AdamCoef c;
    c.lr = lr;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;  // one_minus_beta_1_t (fp32, as Keras computes it)
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    const int D4 = dim / 4;
    if (lazy) {
        if (uniq_cap > 0)
            hipLaunchKernelGGL(adam_lazy_kernel, dim3(grid_of(uniq_cap * D4)), dim3(256), 0, st, table, m, v, D4, uniq_rows,
                               n_uniq, uniq_cap, uniq_grad, c, (int32_t*)nullptr, 0);
        return rf_check_launch("adam_lazy_kernel");
    }
    auto* map = static_cast<int32_t*>(ws);
    if (hipMemsetAsync(map, 0xff, (size_t)table_rows * 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_adam_apply: memset failed");
    if (uniq_cap > 0)
        hipLaunchKernelGGL(map_fill_kernel, dim3(grid_of(uniq_cap)), dim3(256), 0, st, uniq_rows, n_uniq, uniq_cap, map);
    hipLaunchKernelGGL(adam_dense_kernel, dim3(grid_of(table_rows * D4, 256 * 256)), dim3(256), 0, st, table, m, v,
                       table_rows * D4, D4, map, uniq_grad, c);
    return rf_check_launch("adam_dense_kernel");
}

extern "C" int rf_adam_untouched(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                                 const int32_t* n_uniq, int64_t uniq_cap, float lr, float beta1, float beta2, float epsilon,
                                 void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 31), "rf_adam_untouched: table_rows must be in [1, 2^31)");
    RF_REQUIRE(dim >= 4 && dim % 4 == 0, "rf_adam_untouched: dim must be a multiple of 4");
    RF_REQUIRE(table && m && v && n_uniq && (uniq_cap == 0 || uniq_rows), "rf_adam_untouched: null pointer");
    RF_REQUIRE((((uintptr_t)table | (uintptr_t)m | (uintptr_t)v) & 15) == 0, "rf_adam_untouched: buffers must be 16-byte aligned");
    RF_REQUIRE(ws && ws_bytes >= rf_adam_ws_bytes(table_rows, 0), "rf_adam_untouched: workspace too small");
    hipStream_t st = rf_stream(stream);
    AdamCoef c;
    c.lr = lr;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    auto* map = static_cast<int32_t*>(ws);
    if (hipMemsetAsync(map, 0xff, (size_t)table_rows * 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_adam_untouched: memset failed");
    if (uniq_cap > 0)
        hipLaunchKernelGGL(map_fill_kernel, dim3(grid_of(uniq_cap)), dim3(256), 0, st, uniq_rows, n_uniq, uniq_cap, map);
    // a persistent-size grid (one workgroup per CU; 128 / 256 / 512 / 65536 measured 16.2 / 13.2 / 13.4 / 13.9 ms
    // per cfg2 train step, profiles/r03/r03y_train_ab.txt): this runs beside the towers' GEMMs on another stream, so it
    // takes a bounded share of every CU instead of queueing 65,536 workgroups ahead of them
    static const int gmax = [] {
        const char* e = getenv("RF_ADAM_SIDE_GRID");
        return e ? std::max(1, atoi(e)) : 256;
    }();
    hipLaunchKernelGGL(adam_untouched_kernel<4>, dim3(grid_of(table_rows * (dim / 4), gmax)), dim3(256), 0, st, table, m, v,
                       table_rows * (dim / 4), dim / 4, map, n_uniq, c);
    return rf_check_launch("rf_adam_untouched");
}

extern "C" int rf_adam_apply_current(float* table, float* m, float* v, int64_t table_rows, int32_t dim,
                                     const int64_t* uniq_rows, const float* uniq_grad, const int32_t* n_uniq,
                                     int64_t uniq_cap, float lr, float beta1, float beta2, float epsilon, int32_t* last,
                                     int32_t t_set, void* stream) {
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 31), "rf_adam_apply_current: table_rows must be in [1, 2^31)");
    RF_REQUIRE(dim >= 4 && dim % 4 == 0, "rf_adam_apply_current: dim must be a multiple of 4");
    RF_REQUIRE(table && m && v && n_uniq && last && uniq_cap >= 0 && (uniq_cap == 0 || (uniq_rows && uniq_grad)),
               "rf_adam_apply_current: null pointer");
    RF_REQUIRE((((uintptr_t)table | (uintptr_t)m | (uintptr_t)v | (uintptr_t)uniq_grad) & 15) == 0,
               "rf_adam_apply_current: buffers must be 16-byte aligned");
    if (uniq_cap == 0) return RF_OK;
    AdamCoef c;
    c.lr = lr;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    const int D4 = dim / 4;
    hipLaunchKernelGGL(adam_lazy_kernel, dim3(grid_of(uniq_cap * D4)), dim3(256), 0, rf_stream(stream), table, m, v, D4,
                       uniq_rows, n_uniq, uniq_cap, uniq_grad, c, last, t_set);
    return rf_check_launch("rf_adam_apply_current");
}

extern "C" int rf_adam_replay(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                              const int32_t* n_uniq, int64_t uniq_cap, int32_t* last, int32_t t_now, int32_t t_set,
                              const float* lr_log, float beta1, float beta2, float epsilon, void* stream) {
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 31), "rf_adam_replay: table_rows must be in [1, 2^31)");
    RF_REQUIRE(dim >= 4 && dim % 4 == 0, "rf_adam_replay: dim must be a multiple of 4");
    RF_REQUIRE(t_now >= 0 && (t_set == t_now || t_set == t_now + 1), "rf_adam_replay: t_set must be t_now or t_now + 1");
    RF_REQUIRE(table && m && v && last && (t_now == 0 || lr_log), "rf_adam_replay: null pointer");
    RF_REQUIRE(uniq_cap >= 0, "rf_adam_replay: uniq_cap must be >= 0");
    RF_REQUIRE((((uintptr_t)table | (uintptr_t)m | (uintptr_t)v) & 15) == 0, "rf_adam_replay: buffers must be 16-byte aligned");
    hipStream_t st = rf_stream(stream);
    const int64_t nu = uniq_rows ? uniq_cap : table_rows;
    if (nu == 0) return RF_OK;
    AdamCoef c;
    c.lr = 0.f;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    const int D4 = dim / 4;
    auto launch = [&](auto tpr) {
        constexpr int TPR = decltype(tpr)::value;
        const int64_t teams = 256 / TPR;
        hipLaunchKernelGGL(adam_replay_kernel<TPR>, dim3(grid_of((nu + teams - 1) / teams * 256, 256 * 64)), dim3(256), 0, st,
                           table, m, v, table_rows, D4, uniq_rows, n_uniq, uniq_cap, last, t_now, t_set, lr_log, c);
    };
    if (D4 <= 4) launch(std::integral_constant<int, 4>{});
    else if (D4 <= 8) launch(std::integral_constant<int, 8>{});
    else if (D4 <= 16) launch(std::integral_constant<int, 16>{});
    else if (D4 <= 32) launch(std::integral_constant<int, 32>{});
    else launch(std::integral_constant<int, 64>{});
    return rf_check_launch("rf_adam_replay");
}

extern "C" int rf_adam_dense(float* w, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                             float epsilon, void* stream) {
    RF_REQUIRE(n >= 0, "rf_adam_dense: n must be >= 0");
    if (n == 0) return RF_OK;
    RF_REQUIRE(w && g && m && v, "rf_adam_dense: null pointer");
    AdamCoef c;
    c.lr = lr;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    hipStream_t st = rf_stream(stream);
    const bool v4 = n % 4 == 0 && ((((uintptr_t)w | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0);
    if (v4)
        hipLaunchKernelGGL(adam_dense_flat_kernel<4>, dim3(grid_of(n / 4, 4096)), dim3(256), 0, st, w, g, m, v, n, c);
    else
        hipLaunchKernelGGL(adam_dense_flat_kernel<1>, dim3(grid_of(n, 4096)), dim3(256), 0, st, w, g, m, v, n, c);
    return rf_check_launch("rf_adam_dense");
}

extern "C" int rf_adam_dense_multi(const rf_adam_tensor* tensors, int32_t n_tensors, int64_t max_n, float lr, float beta1,
                                   float beta2, float epsilon, void* stream) {
    RF_REQUIRE(n_tensors >= 0 && n_tensors <= 65535 && max_n >= 0, "rf_adam_dense_multi: bad arguments");
    if (n_tensors == 0 || max_n == 0) return RF_OK;
    RF_REQUIRE(tensors, "rf_adam_dense_multi: null pointer");
    AdamCoef c;
    c.lr = lr;
    c.b1 = beta1;
    c.b2 = beta2;
    c.omb1 = 1.0f - beta1;
    c.omb2 = 1.0f - beta2;
    c.eps = epsilon;
    const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((max_n / 4 + 255) / 256, 1024));
    hipLaunchKernelGGL(adam_dense_multi_kernel, dim3(gx, n_tensors), dim3(256), 0, rf_stream(stream), tensors, c);
    return rf_check_launch("rf_adam_dense_multi");
}
