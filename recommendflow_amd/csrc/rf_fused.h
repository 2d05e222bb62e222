// rf_fused.h — the fused multi-slot hash -> gather -> pool kernel (rf_fused_hash_embed_fwd), shared by the
// per-table-dtype instantiation units rf_fused_f32.hip / rf_fused_bf16.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <type_traits>

#include "rf_common.h"

namespace rf {


// waves per workgroup (each wave walks its own items): 4 measured 0.7-1.1 % faster than 1 on the cfg2 headline (the
// same 12 waves per CU, a quarter of the workgroups to dispatch); 8 and 16 slower (LDS per workgroup)
// (profiles/r06/headline_waves_per_wg_ab.txt)
#ifndef RF_FUSED_WAVES
#define RF_FUSED_WAVES 4
#endif
// waves per workgroup: items are wave-independent, and one-wave workgroups release their slots as soon
// as their own item is done (a 4-wave workgroup holds its slots until the slowest of 4 items ends)
constexpr int kWaves = RF_FUSED_WAVES;
constexpr int kCap = 768;    // tokens per wave item kept in the LDS row bucket (more: hashed inline)
constexpr int kUnits = 64;   // examples per wave item (one slot per item)
constexpr int kDefaultMaxLpr = 16;  // lanes per row cap (tuned on MI355X)

template <typename T>
struct Elem {
    static constexpr int EPV = 16 / (int)sizeof(T);  // elements per 16-byte chunk
};

template <typename TT>
__device__ __forceinline__ void unpack16(const uint4& v, float* f) {
    if constexpr (sizeof(TT) == 4) {
        f[0] = __uint_as_float(v.x);
        f[1] = __uint_as_float(v.y);
        f[2] = __uint_as_float(v.z);
        f[3] = __uint_as_float(v.w);
    } else {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = bf16_bits_to_f32(w[i] & 0xffffu);
            f[2 * i + 1] = bf16_bits_to_f32(w[i] >> 16);
        }
    }
}

template <typename OT, int EPV>
__device__ __forceinline__ void store_chunk(OT* dst, const float* f) {
    if constexpr (sizeof(OT) == 4) {
        // fp32 pooled rows stream out with nontemporal stores: the 480 MB of cfg2 output per launch then does not
        // evict the tables' Zipf-hot rows from L2 / MALL (same-box A/B, profiles/r06/headline_nt_store_ab.txt:
        // 0.2559 -> 0.2534 ms). RF_TEMPORAL_OUT=1 at build time restores plain stores.
#pragma unroll
        for (int i = 0; i < EPV; i += 4) {
#ifdef RF_TEMPORAL_OUT
            *reinterpret_cast<float4*>(dst + i) = make_float4(f[i], f[i + 1], f[i + 2], f[i + 3]);
#else
            typedef float f4nt __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(f4nt{f[i], f[i + 1], f[i + 2], f[i + 3]}, reinterpret_cast<f4nt*>(dst + i));
#endif
        }
    } else {
        uint32_t w[EPV / 2];
#pragma unroll
        for (int i = 0; i < EPV / 2; ++i) w[i] = f32_to_bf16_bits(f[2 * i]) | (f32_to_bf16_bits(f[2 * i + 1]) << 16);
        if constexpr (EPV == 4)
            *reinterpret_cast<uint2*>(dst) = make_uint2(w[0], w[1]);
        else
            *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__device__ __forceinline__ uint4 nan_chunk() {
    const uint32_t q = 0x7fc07fc0u;  // NaN as f32 and as a bf16 pair
    return make_uint4(q, q, q, q);
}

template <typename TT>
__device__ __forceinline__ uint4 load_chunk(const TT* __restrict__ table, int64_t row, int64_t table_rows, int dim,
                                            int c) {
    constexpr int EPV = Elem<TT>::EPV;
    if (row < 0 || row >= table_rows) return nan_chunk();
    return *reinterpret_cast<const uint4*>(table + row * (int64_t)dim + (int64_t)c * EPV);
}

// the mean of zero positions (a slot with Lmax = 0 unmasked): 0/0 with the x86 default-NaN bits (sign set),
// what the reference's CPU reduce_mean and the oracle produce; GPU division would give the positive NaN
#define kMeanOfNothing __uint_as_float(0xffc00000u)

__device__ __forceinline__ float comb_init(int comb) {
    return comb == RF_COMB_MAX ? -INFINITY : comb == RF_COMB_MIN ? INFINITY : 0.0f;
}

__device__ __forceinline__ float comb_step(int comb, float a, float v) {
    // sum/avg: one fp32 add per position in order (no fma, no reassociation)
    return comb == RF_COMB_MAX ? (v > a ? v : a) : comb == RF_COMB_MIN ? (v < a ? v : a) : __fadd_rn(a, v);
}

// a[e] += f[e] for e < N (N even), two lanes of fp32 per v_pk_add_f32: the same RN add per element,
// half the VALU issue of scalar adds (sum/avg pooling and the padded-position adds are VALU-heavy)
template <int N>
__device__ __forceinline__ void add_pk(float* a, const float* f) {
    typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int e = 0; e < N; e += 2) {
        f2 x = {a[e], a[e + 1]};
        const f2 y = {f[e], f[e + 1]};
        x = x + y;
        a[e] = x.x;
        a[e + 1] = x.y;
    }
}

// ---------------------------------------------------------------------------------------------
// fused multi-slot hash -> gather -> pool
// ---------------------------------------------------------------------------------------------
// row r (already clamped into the table), 16-byte chunk c: no bounds branch on the hot path
template <typename TT>
__device__ __forceinline__ uint4 row_chunk(const TT* __restrict__ table, uint32_t r, int dim, int c) {
    return *reinterpret_cast<const uint4*>(table + (int64_t)r * dim + (int64_t)c * Elem<TT>::EPV);
}

// PRE (rf_pool_rows_fwd): a row id with bit 31 set is row (r & 0x7fffffff) of the caller's LOCAL table
// (the rank's own shard: rows it owns are read in place instead of travelling through the receive buffer),
// any other id a row of the gathered buffer. One select per row load; with local == nullptr no id has bit 31.
template <bool PRE, typename TT>
__device__ __forceinline__ uint4 row_chunk_src(const TT* __restrict__ table, const TT* __restrict__ local, uint32_t r,
                                               int dim, int c) {
    if constexpr (PRE) {
        const bool loc = (r & 0x80000000u) != 0u;
        return row_chunk(loc ? local : table, r & 0x7fffffffu, dim, c);
    } else {
        return row_chunk(table, r, dim, c);
    }
}

// Slot-major items: item = (slot s, examples b0 .. b0+kUnits-1). Every unit of an item shares the slot's
// combiner, Lmax, salts, table segments and pad rows — all wave-uniform (scalar loads, one pad-row
// prefetch per item) — and unit lengths follow one distribution, so the teams stay balanced.
//  1a. lane j < nu reads unit j's token range; a wave prefix-scan lays the item's tokens out
//      contiguously (item-local index i) in LDS;
//  1b. lane-per-token: both SipHash-2-4 states over one read of the token, fused-table rows of both
//      tables into the LDS bucket (indices never touch HBM);
//  2.  the wave splits into TEAMS of LPR lanes (one 16-byte chunk per lane per row, CPL chunks);
//      team t takes the units whose first token falls in the t-th share of the item's tokens and
//      streams them through a two-stage software pipeline, accumulating in position order
//      l = 0 .. L-1 with one fp32 add per position (bit-exact with the oracle); padded positions
//      reuse the item's prefetched pad rows. Loads carry no branches: rows are clamped into the
//      table in phase 1, and a slot whose descriptor does not fit the table is written as NaN.
#ifndef RF_FUSED_MIN_WAVES
#define RF_FUSED_MIN_WAVES 1
#endif
template <int LPR, int CPL, bool FULL, typename TT, typename OT, bool PRE>
__global__ __launch_bounds__(kWaves * 64, RF_FUSED_MIN_WAVES) void fused_hash_embed_kernel(
    const rf_slot_desc* __restrict__ slots, int n_slots, const uint8_t* __restrict__ tok_bytes,
    const int32_t* __restrict__ tok_off, const int32_t* __restrict__ bag_off, const int32_t* __restrict__ lmax,
    int64_t n_units, const TT* __restrict__ table, int64_t table_rows, int dim, OT* __restrict__ out,
    int64_t out_stride, int flags, int64_t* __restrict__ idx_out) {
    constexpr int EPV = Elem<TT>::EPV;
    constexpr int TEAMS = 64 / LPR;
#ifdef RF_TOKENS_IN_FLIGHT
    constexpr int C = RF_TOKENS_IN_FLIGHT;
#else
    constexpr int C = CPL >= 2 ? 1 : 2;  // tokens per pipeline stage per team (2 stages in flight)
#endif
    __shared__ uint32_t s_row[kWaves][2][kCap];
    __shared__ int32_t s_loc[kWaves][kUnits + 1];
    __shared__ int32_t s_gbeg[kWaves][kUnits];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int team = lane / LPR, tl = lane % LPR;
    const int nchunks = dim / EPV;
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const bool emit = (flags & RF_FLAG_EMIT_IDX) != 0 && idx_out != nullptr;
    const bool abl_nohash = (flags & (1 << 12)) != 0, abl_nopool = (flags & (1 << 13)) != 0,
               abl_nopad = (flags & (1 << 14)) != 0;  // result-changing ablations: rf_diag_fused_hash_embed_fwd only (include/rf_diag.h)
    const bool no_lean = (flags & (1 << 15)) != 0;  // A/B: force the general phase 2 on single-token items
    // rf_pool_rows_fwd: `table` holds pre-gathered rows (token t, table k -> row 2t + k; pad rows after)
    constexpr bool pregathered = PRE;
    // PRE: tok_bytes is unused and tok_off carries the optional row map (logical row j of the pre-gathered
    // buffer lives at row_map[j]; nullptr = identity) — rf_pool_rows_fwd's un-permute, fused into the loads
    const int32_t* row_map = PRE ? tok_off : nullptr;
    // PRE: tok_bytes carries the rank-local table (row ids with bit 31 set), or nullptr
    const TT* local_tab = PRE ? reinterpret_cast<const TT*>(tok_bytes) : nullptr;
    const int batch = (int)(n_units / n_slots);
    const int nbb = (batch + kUnits - 1) / kUnits;
    const int64_t n_items = (int64_t)n_slots * nbb;
    int cidx[CPL];
    bool cown[CPL];
#pragma unroll
    for (int cc = 0; cc < CPL; ++cc) {
        const int c = tl + cc * LPR;
        cown[cc] = FULL || c < nchunks;
        cidx[cc] = FULL ? c : min(c, nchunks - 1);  // a lane past the row re-reads the last chunk, stores nothing
    }

    // slot-interleaved XCD order (diagnostic, opt-in via flag bit 11; a bijection on the items): work
    // index v is dealt to XCD v % 8 (round-robin dispatch), and XCD x walks ALL b-blocks of slots x,
    // x + 8, x + 16, ... so a slot's Zipf-hot rows stay in one XCD's L2. Measured SLOWER than the plain
    // order on MI355X (cfg3 encoder 0.0676 vs 0.0615 ms, cfg2 0.2626 vs 0.2603 ms), so it is off by default.
    const int64_t s8_items = (int64_t)(n_slots & ~7) * nbb;
    const bool xcd_order = (flags & (1 << 11)) != 0;
    for (int64_t v = (int64_t)blockIdx.x * kWaves + wave; v < n_items; v += (int64_t)gridDim.x * kWaves) {
        int64_t item = v;
        if (xcd_order && v < s8_items) {
            const int64_t x = v & 7, p = v >> 3, jj = p / nbb, bb = p - jj * nbb;
            item = (x + 8 * jj) * nbb + bb;
        }
        // ---- slot descriptor: wave-uniform ----
        const int s = (int)(item / nbb);
        const int b0 = (int)(item - (int64_t)s * nbb) * kUnits;
        const int nu = min(kUnits, batch - b0);
        const rf_slot_desc* sd = slots + s;
        const int comb = sd->combiner;
        const int64_t rb0 = sd->row_base[0], rb1 = sd->row_base[1], nbins = sd->num_bins;
        const uint64_t salt0 = sd->salt[0], salt1 = sd->salt[1];
        const int mask_empty = sd->mask_empty;
        const BucketMod bmod = bucket_mod_init(nbins, mask_empty);  // once per item (the slot is wave-uniform)
        const int64_t out_off = sd->out_off;
        const int lm = lmax[s];
        const bool ok = pregathered || (rb0 >= 0 && rb1 >= 0 && rb0 + nbins <= table_rows && rb1 + nbins <= table_rows);
        // padded position = b"": bin 0 with mask_value "", else the bin of b""
        int64_t pb0 = 0, pb1 = 0;
        if (!mask_empty && !pregathered) {
            pb0 = (int64_t)(siphash24_dev(salt0, salt0, tok_bytes, 0) % (uint64_t)nbins);
            pb1 = (int64_t)(siphash24_dev(salt1, salt1, tok_bytes, 0) % (uint64_t)nbins);
        }
        uint32_t pad0 = ok ? (uint32_t)(rb0 + pb0) : 0u, pad1 = ok ? (uint32_t)(rb1 + pb1) : 0u;
        if (pregathered) {  // pad rows follow the 2 * n_tok token rows (through the row map when given)
            pad0 = (uint32_t)(table_rows - 2 * (int64_t)n_slots + 2 * s);
            pad1 = pad0 + 1;
            if (row_map) {
                pad0 = (uint32_t)row_map[pad0];
                pad1 = (uint32_t)row_map[pad1];
            }
        }

        // ---- phase 1a: unit token ranges, wave prefix scan -> item-local token layout ----
        int g0 = 0, len = 0;
        if (lane < nu) {
            const int64_t u = (int64_t)(b0 + lane) * n_slots + s;
            g0 = bag_off[u];
            len = bag_off[u + 1] - g0;
        }
        int incl = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane < nu) {
            s_loc[wave][lane + 1] = incl;
            s_gbeg[wave][lane] = g0;
        }
        if (lane == 0) s_loc[wave][0] = 0;
        const int ntok = __shfl(incl, 63, 64);
        // single-token items (Lmax = 1, every bag 0 or 1 token): phase 2 is one row pair per bag, so the
        // lean path below issues every team's loads up front instead of running the pooling pipeline
        // (PRE too: the bucket then holds the row-mapped rows of the pre-gathered buffer or, bit 31, the local shard)
        const bool lean = !no_lean && lm == 1 && comb != RF_COMB_NULL && !emit && !abl_nohash && !abl_nopad &&
                          __all(len <= 1);
        wave_lds_sync();

        // ---- phase 1b: lane-per-token double hashing into the LDS bucket ----
        // (with RF_FLAG_EMIT_IDX every token of the item is hashed here, so ids past the bucket are
        //  emitted even when the pooling never visits them — first/last/null)
        const int nh = min(ntok, kCap);
        if (pregathered) {
            for (int i = lane; i < nh; i += 64) {
                int lo = 0, hi = nu - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_loc[wave][mid] <= i) lo = mid; else hi = mid - 1;
                }
                const uint32_t t = (uint32_t)(s_gbeg[wave][lo] + (i - s_loc[wave][lo]));
                s_row[wave][0][i] = row_map ? (uint32_t)row_map[2 * t] : 2 * t;
                s_row[wave][1][i] = row_map ? (uint32_t)row_map[2 * t + 1] : 2 * t + 1;
            }
        }
        if (abl_nohash) {
            for (int i = lane; i < nh; i += 64) {
                s_row[wave][0][i] = (uint32_t)(((uint64_t)i * 2654435761u + item) % (uint64_t)table_rows);
                s_row[wave][1][i] = (uint32_t)(((uint64_t)i * 40503u + 7u + item) % (uint64_t)table_rows);
            }
        }
        const int nhash = (abl_nohash || pregathered) ? 0 : (emit ? ntok : nh);
        for (int i = lane; i < nhash; i += 64) {
            int lo = 0, hi = nu - 1;  // unit of item-local token i: last j with s_loc[j] <= i
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_loc[wave][mid] <= i) lo = mid; else hi = mid - 1;
            }
            const int t = s_gbeg[wave][lo] + (i - s_loc[wave][lo]);
            const int tb = tok_off[t], n = tok_off[t + 1] - tb;
            uint64_t h0, h1;
            siphash24x2_dev(salt0, salt1, tok_bytes + tb, n, h0, h1);
            const int64_t i0 = bucket_from_hash(h0, n, bmod);
            const int64_t i1 = bucket_from_hash(h1, n, bmod);
            if (i < kCap) {
                s_row[wave][0][i] = ok ? (uint32_t)(rb0 + i0) : 0u;
                s_row[wave][1][i] = ok ? (uint32_t)(rb1 + i1) : 0u;
            }
            if (emit) {
                idx_out[2 * (int64_t)t] = i0;
                idx_out[2 * (int64_t)t + 1] = i1;
            }
        }
        wave_lds_sync();
        if (abl_nopool) continue;

        // ---- lean phase 2 (single-token items): a team per bag, GU bags' row pairs in flight per team.
        // Same values as the general path with Lu = 1: sum/avg = 0 + x (avg / 1 is exact), max/min =
        // comb_step(init, x), first/last = x; an empty bag reads the pad rows, or is zeros when masked.
        if (lean) {
            constexpr int UPT = kUnits / TEAMS;     // bags per team
#ifdef RF_LEAN_GU
            constexpr int GU = RF_LEAN_GU;
#else
            constexpr int GU = CPL >= 2 ? 2 : 4;    // bags per load group
#endif
#ifdef RF_LEAN_PIPE
            constexpr bool LPIPE = RF_LEAN_PIPE != 0;  // A/B build option: group q0 + GU's loads issued before q0 is consumed
#else
            constexpr bool LPIPE = false;
#endif
            // the element rule is wave-uniform per item: resolved once here, not as a chain of uniform branches
            // per element (as the single-token kernel)
            auto lean_body = [&](auto rule) __attribute__((always_inline)) {
                auto lean_issue = [&](uint4 (&v)[GU][2][CPL], bool (&has)[GU], int q0) __attribute__((always_inline)) {
#pragma unroll
                    for (int g = 0; g < GU; ++g) {
                        const int jj = min(team + TEAMS * (q0 + g), nu - 1);
                        const int i = s_loc[wave][jj];
                        has[g] = s_loc[wave][jj + 1] - i == 1;
                        const uint32_t r0 = has[g] ? s_row[wave][0][i] : pad0;
                        const uint32_t r1 = has[g] ? s_row[wave][1][i] : pad1;
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            v[g][0][cc] = row_chunk_src<PRE>(table, local_tab, r0, dim, cidx[cc]);
                            v[g][1][cc] = row_chunk_src<PRE>(table, local_tab, r1, dim, cidx[cc]);
                        }
                    }
                };
                auto lean_consume = [&](const uint4 (&v)[GU][2][CPL], const bool (&has)[GU], int q0) __attribute__((always_inline)) {
#pragma unroll
                    for (int g = 0; g < GU; ++g) {
                        const int j = team + TEAMS * (q0 + g);
                        if (j >= nu) continue;
                        const int64_t ob = (int64_t)(b0 + j) * out_stride + out_off;
                        const bool zero = !has[g] && mask_pad;
#pragma unroll
                        for (int k = 0; k < 2; ++k)
#pragma unroll
                            for (int cc = 0; cc < CPL; ++cc) {
                                float f[EPV], a[EPV];
                                unpack16<TT>(v[g][k][cc], f);
#pragma unroll
                                for (int e = 0; e < EPV; ++e) a[e] = zero ? 0.0f : rule(f[e]);
                                if (!ok) {
#pragma unroll
                                    for (int e = 0; e < EPV; ++e) a[e] = __builtin_nanf("");
                                }
                                if (cown[cc]) store_chunk<OT, EPV>(out + ob + (int64_t)k * dim + cidx[cc] * EPV, a);
                            }
                    }
                };
                if constexpr (LPIPE) {
                    uint4 va[GU][2][CPL], vb[GU][2][CPL];
                    bool ha[GU], hb[GU];
                    lean_issue(va, ha, 0);
#pragma unroll 1
                    for (int q0 = 0; q0 < UPT; q0 += 2 * GU) {
                        if (q0 + GU < UPT) lean_issue(vb, hb, q0 + GU);
                        lean_consume(va, ha, q0);
                        if (q0 + GU >= UPT) break;
                        if (q0 + 2 * GU < UPT) lean_issue(va, ha, q0 + 2 * GU);
                        lean_consume(vb, hb, q0 + GU);
                    }
                } else {
#pragma unroll 1
                    for (int q0 = 0; q0 < UPT; q0 += GU) {
                        uint4 v[GU][2][CPL];
                        bool has[GU];
                        lean_issue(v, has, q0);
                        lean_consume(v, has, q0);
                    }
                }
            };
            if (comb == RF_COMB_SUM || comb == RF_COMB_AVG) lean_body([](float x) { return __fadd_rn(0.0f, x); });
            else if (comb == RF_COMB_MAX) lean_body([](float x) { return comb_step(RF_COMB_MAX, -INFINITY, x); });
            else if (comb == RF_COMB_MIN) lean_body([](float x) { return comb_step(RF_COMB_MIN, INFINITY, x); });
            else lean_body([](float x) { return x; });
            continue;
        }

        // ---- phase 2: token-balanced teams, pipelined gather + pool ----
        auto bound = [&](int tm) -> int {  // first unit j whose first token lies in team tm's share
            if (tm <= 0) return 0;
            if (tm >= TEAMS) return nu;
            int lo = 0, hi = nu;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if ((int64_t)s_loc[wave][mid] * TEAMS >= (int64_t)tm * ntok) hi = mid; else lo = mid + 1;
            }
            return lo;
        };
        const int ja = bound(team), jb = bound(team + 1);

        // the slot's pad rows, once per item
        uint4 padv[2][CPL];
#pragma unroll
        for (int cc = 0; cc < CPL; ++cc) {
            padv[0][cc] = row_chunk_src<PRE>(table, local_tab, pad0, dim, cidx[cc]);
            padv[1][cc] = row_chunk_src<PRE>(table, local_tab, pad1, dim, cidx[cc]);
        }
        const float init = comb_init(comb);
        int j = ja, ubeg = 0, uend = 0, Lu = 0;
        int64_t obase = 0;
        float acc[2][CPL][EPV];
        auto start_unit = [&]() {
            ubeg = s_loc[wave][j];
            uend = s_loc[wave][j + 1];
            const int ul = uend - ubeg;
            Lu = comb == RF_COMB_NULL ? lm : ((mask_pad || abl_nopad) ? ul : max(lm, ul));
            obase = (int64_t)(b0 + j) * out_stride + out_off;
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                    for (int e = 0; e < EPV; ++e) acc[k][cc][e] = init;
        };
        auto put = [&](int64_t off, const float* f) {  // one chunk; NaN if the slot does not fit the table
            float g[EPV];
#pragma unroll
            for (int e = 0; e < EPV; ++e) g[e] = ok ? f[e] : __builtin_nanf("");
            store_chunk<OT, EPV>(out + off, g);
        };
        auto finish_unit = [&]() {
            const int ul = uend - ubeg;
            const int npad = Lu - ul;
            if (comb == RF_COMB_NULL) {
                for (int p = ul; p < Lu; ++p)
#pragma unroll
                    for (int k = 0; k < 2; ++k)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            if (!cown[cc]) continue;
                            float f[EPV];
                            unpack16<TT>(padv[k][cc], f);
                            if (mask_pad) {
#pragma unroll
                                for (int e = 0; e < EPV; ++e) f[e] = 0.0f;
                            }
                            put(obase + ((int64_t)k * Lu + p) * dim + cidx[cc] * EPV, f);
                        }
                return;
            }
            if (npad > 0 && (comb == RF_COMB_SUM || comb == RF_COMB_AVG)) {
                // one add per padded position, in order; both tables' chains in one loop, unrolled by 2
                float pf[2][CPL][EPV];
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int cc = 0; cc < CPL; ++cc) unpack16<TT>(padv[k][cc], pf[k][cc]);
                int p = 0;
                for (; p + 2 <= npad; p += 2) {
#pragma unroll
                    for (int r = 0; r < 2; ++r)
#pragma unroll
                        for (int k = 0; k < 2; ++k)
#pragma unroll
                            for (int cc = 0; cc < CPL; ++cc) add_pk<EPV>(acc[k][cc], pf[k][cc]);
                }
                if (p < npad) {
#pragma unroll
                    for (int k = 0; k < 2; ++k)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) add_pk<EPV>(acc[k][cc], pf[k][cc]);
                }
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc) {
                    float* a = acc[k][cc];
                    if (npad > 0) {
                        float f[EPV];
                        unpack16<TT>(padv[k][cc], f);
                        if (comb == RF_COMB_MAX || comb == RF_COMB_MIN) {
#pragma unroll
                            for (int e = 0; e < EPV; ++e) a[e] = comb_step(comb, a[e], f[e]);
                        } else if (comb == RF_COMB_LAST || (comb == RF_COMB_FIRST && ul == 0)) {
#pragma unroll
                            for (int e = 0; e < EPV; ++e) a[e] = f[e];
                        }
                    }
                    if (comb == RF_COMB_AVG) {
                        const float fl = (float)Lu;
#pragma unroll
                        for (int e = 0; e < EPV; ++e) a[e] = Lu == 0 ? kMeanOfNothing : __fdiv_rn(a[e], fl);
                    }
                    if (Lu == 0 && (mask_pad || comb == RF_COMB_FIRST || comb == RF_COMB_LAST)) {
#pragma unroll
                        for (int e = 0; e < EPV; ++e) a[e] = 0.0f;  // empty (masked) bag / no position -> zeros
                    }
                    if (cown[cc]) put(obase + (int64_t)k * dim + cidx[cc] * EPV, a);
                }
        };
        auto consume = [&](const uint4 (&v)[2][CPL], int pos) {
            if (comb == RF_COMB_NULL) {
                if (pos < Lu)
#pragma unroll
                    for (int k = 0; k < 2; ++k)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            if (!cown[cc]) continue;
                            float f[EPV];
                            unpack16<TT>(v[k][cc], f);
                            put(obase + ((int64_t)k * Lu + pos) * dim + cidx[cc] * EPV, f);
                        }
                return;
            }
            if (comb == RF_COMB_FIRST && pos != 0) return;
            if (comb == RF_COMB_LAST && pos != Lu - 1) return;
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc) {
                    float f[EPV];
                    unpack16<TT>(v[k][cc], f);
                    if (comb == RF_COMB_FIRST || comb == RF_COMB_LAST) {
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[k][cc][e] = f[e];
                    } else if (comb == RF_COMB_SUM || comb == RF_COMB_AVG) {
                        add_pk<EPV>(acc[k][cc], f);
                    } else {
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[k][cc][e] = comb_step(comb, acc[k][cc][e], f[e]);
                    }
                }
        };

        if (ja < jb) {
            start_unit();
            const int tb0 = s_loc[wave][ja], tb1 = s_loc[wave][jb];
            const int th = min(tb1, kCap);  // hot range: rows staged in LDS
            auto issue = [&](uint4 (&v)[C][2][CPL], int c0) {
#pragma unroll
                for (int q = 0; q < C; ++q) {
                    const int i = min(c0 + q, th - 1);  // past the range: re-read a valid row, ignored
                    const uint32_t r0 = s_row[wave][0][i], r1 = s_row[wave][1][i];
#pragma unroll
                    for (int cc = 0; cc < CPL; ++cc) {
                        v[q][0][cc] = row_chunk_src<PRE>(table, local_tab, r0, dim, cidx[cc]);
                        v[q][1][cc] = row_chunk_src<PRE>(table, local_tab, r1, dim, cidx[cc]);
                    }
                }
            };
            auto drain = [&](const uint4 (&v)[C][2][CPL], int c0) {
#pragma unroll
                for (int q = 0; q < C; ++q) {
                    const int i = c0 + q;
                    if (i < th) {
                        while (i >= uend) {  // close the current unit (and any empty ones after it)
                            finish_unit();
                            ++j;
                            start_unit();
                        }
                        consume(v[q], i - ubeg);
                    }
                }
            };
            uint4 va[C][2][CPL], vb[C][2][CPL];
            int c0 = tb0;
            if (c0 < th) issue(va, c0);
            while (c0 < th) {
                if (c0 + C < th) issue(vb, c0 + C);
                drain(va, c0);
                c0 += C;
                if (c0 >= th) break;
                if (c0 + C < th) issue(va, c0 + C);
                drain(vb, c0);
                c0 += C;
            }
            // cold range (item holds more than kCap tokens): hash inline, one token at a time
            for (int i = max(tb0, kCap); i < tb1; ++i) {
                while (i >= uend) {
                    finish_unit();
                    ++j;
                    start_unit();
                }
                const int t = s_gbeg[wave][j] + (i - ubeg);
                uint32_t r0, r1;
                if (pregathered) {
                    r0 = 2u * (uint32_t)t;
                    r1 = r0 + 1;
                    if (row_map) {
                        r0 = (uint32_t)row_map[r0];
                        r1 = (uint32_t)row_map[r1];
                    }
                } else {
                    const int tb = tok_off[t], n = tok_off[t + 1] - tb;
                    uint64_t h0, h1;
                    siphash24x2_dev(salt0, salt1, tok_bytes + tb, n, h0, h1);
                    r0 = ok ? (uint32_t)(rb0 + bucket_from_hash(h0, n, bmod)) : 0u;
                    r1 = ok ? (uint32_t)(rb1 + bucket_from_hash(h1, n, bmod)) : 0u;
                }
                uint4 v[2][CPL];
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc) {
                    v[0][cc] = row_chunk_src<PRE>(table, local_tab, r0, dim, cidx[cc]);
                    v[1][cc] = row_chunk_src<PRE>(table, local_tab, r1, dim, cidx[cc]);
                }
                consume(v, i - ubeg);
            }
            while (true) {
                finish_unit();
                if (++j >= jb) break;
                start_unit();
            }
        }
        wave_lds_sync();  // the LDS bucket is rewritten by the next item
    }
}

// ---------------------------------------------------------------------------------------------
// single-token slots (RF_FLAG_SINGLE_TOKEN: the caller knows every slot's batch Lmax is <= 1, e.g. cfg3's
// 200 single-valued slots). The general kernel's pooling pipeline sets its register allocation (~195
// VGPRs: two waves per SIMD), so its lean path cannot overlap one item's hashing with another's
// gather. This kernel keeps only what an Lmax = 1 item needs (~100 VGPRs): lane j hashes bag j's token
// (both keys, one read), the rows move to the gathering teams by lane shuffles (no LDS, no barrier),
// and every team issues all of its bags' row loads at once (the whole row: one 16-byte chunk per lane).
// Values are the general kernel's for Lmax = 1 (its lean phase 2): sum/avg 0 + x, max/min
// comb_step(init, x), first/last/null x, an empty bag reads the pad rows (zeros when masked), NaN for a
// slot that does not fit the table; a slot with Lmax = 0 gets the empty-reduction values (sum/first/
// last 0, avg 0/0, max -inf, min +inf; zeros when masked; null: nothing) and one with Lmax > 1 (a
// broken promise) NaN.
template <int LPR, typename TT, typename OT>
__global__ __launch_bounds__(64) void single_token_embed_kernel(
    const rf_slot_desc* __restrict__ slots, int n_slots, const uint8_t* __restrict__ tok_bytes,
    const int32_t* __restrict__ tok_off, const int32_t* __restrict__ bag_off, const int32_t* __restrict__ lmax,
    int64_t n_units, const TT* __restrict__ table, int64_t table_rows, int dim, OT* __restrict__ out,
    int64_t out_stride, int flags) {
    constexpr int EPV = Elem<TT>::EPV;
    constexpr int TEAMS = 64 / LPR;   // one team per bag at a time, one 16-byte chunk per lane
    constexpr int G = kUnits / TEAMS;  // bags per team per item
    constexpr int GH = G > 8 ? 8 : G;  // bags per load batch (16 row chunks per lane in flight)
    const int lane = threadIdx.x, team = lane / LPR, tl = lane % LPR;
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const int batch = (int)(n_units / n_slots);
    const int nbb = (batch + kUnits - 1) / kUnits;
    const int64_t n_items = (int64_t)n_slots * nbb;
    for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
        const int s = (int)(item / nbb);
        const int b0 = (int)(item - (int64_t)s * nbb) * kUnits;
        const int nu = min(kUnits, batch - b0);
        const rf_slot_desc* sd = slots + s;
        const int comb = sd->combiner;
        const int64_t rb0 = sd->row_base[0], rb1 = sd->row_base[1], nbins = sd->num_bins;
        const uint64_t salt0 = sd->salt[0], salt1 = sd->salt[1];
        const int mask_empty = sd->mask_empty;
        const BucketMod bmod = bucket_mod_init(nbins, mask_empty);  // once per item (the slot is wave-uniform)
        const int64_t out_off = sd->out_off;
        const int lm = lmax[s];
        const bool ok = rb0 >= 0 && rb1 >= 0 && rb0 + nbins <= table_rows && rb1 + nbins <= table_rows;
        int64_t pb0 = 0, pb1 = 0;
        if (!mask_empty) {
            pb0 = (int64_t)(siphash24_dev(salt0, salt0, tok_bytes, 0) % (uint64_t)nbins);
            pb1 = (int64_t)(siphash24_dev(salt1, salt1, tok_bytes, 0) % (uint64_t)nbins);
        }
        // lane j: bag b0 + j -> its two rows (the pad rows when empty)
        uint32_t r0 = ok ? (uint32_t)(rb0 + pb0) : 0u, r1 = ok ? (uint32_t)(rb1 + pb1) : 0u;
        int has = 0;
        if (lane < nu) {
            const int64_t u = (int64_t)(b0 + lane) * n_slots + s;
            const int t = bag_off[u];
            if (bag_off[u + 1] > t) {
                const int tb = tok_off[t], n = tok_off[t + 1] - tb;
                uint64_t h0, h1;
                siphash24x2_dev(salt0, salt1, tok_bytes + tb, n, h0, h1);
                if (ok) {
                    r0 = (uint32_t)(rb0 + bucket_from_hash(h0, n, bmod));
                    r1 = (uint32_t)(rb1 + bucket_from_hash(h1, n, bmod));
                }
                has = 1;
            }
        }
        if (lm == 0 && comb == RF_COMB_NULL) continue;  // no positions: nothing to write
        const float initv = comb_init(comb);
        float special = 0.0f;  // the value of every element when the slot's Lmax is not 1
        if (lm == 0 && !mask_pad)
            special = comb == RF_COMB_AVG ? kMeanOfNothing : (comb == RF_COMB_MAX || comb == RF_COMB_MIN) ? initv : 0.0f;
        if (lm > 1 || !ok) special = __builtin_nanf("");
        const bool use_special = lm != 1 || !ok;
        const bool full = nu == kUnits;  // every team's bag exists: no per-bag guard on the stores
        // the element rule is wave-uniform per item: resolved once here, not per element (a chain of uniform
        // branches per element was most of this loop's issue)
        auto body = [&](auto rule, auto zero_ok) {  // zero_ok: mask_pad zeros apply (not to the special values)
#pragma unroll
            for (int g0 = 0; g0 < G; g0 += GH) {
                uint4 v[GH][2];
#pragma unroll
                for (int g = 0; g < GH; ++g) {
                    const int j = team + TEAMS * (g0 + g);
                    const uint32_t q0 = (uint32_t)__shfl((int)r0, j, 64), q1 = (uint32_t)__shfl((int)r1, j, 64);
                    v[g][0] = row_chunk(table, q0, dim, tl);
                    v[g][1] = row_chunk(table, q1, dim, tl);
                }
#pragma unroll
                for (int g = 0; g < GH; ++g) {
                    const int j = team + TEAMS * (g0 + g);
                    const int hj = __shfl(has, j, 64);
                    if (!full && j >= nu) continue;
                    const bool zero = mask_pad && !hj;
                    const int64_t ob = (int64_t)(b0 + j) * out_stride + out_off;
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        float f[EPV], a[EPV];
                        unpack16<TT>(v[g][k], f);
#pragma unroll
                        for (int e = 0; e < EPV; ++e) a[e] = (decltype(zero_ok)::value && zero) ? 0.0f : rule(f[e]);
                        store_chunk<OT, EPV>(out + ob + (int64_t)k * dim + tl * EPV, a);
                    }
                }
            }
        };
        if (use_special) {
            body([=](float) { return special; }, std::false_type{});
        } else if (comb == RF_COMB_SUM || comb == RF_COMB_AVG) {
            body([](float x) { return __fadd_rn(0.0f, x); }, std::true_type{});
        } else if (comb == RF_COMB_MAX) {
            body([](float x) { return comb_step(RF_COMB_MAX, -INFINITY, x); }, std::true_type{});
        } else if (comb == RF_COMB_MIN) {
            body([](float x) { return comb_step(RF_COMB_MIN, INFINITY, x); }, std::true_type{});
        } else {
            body([](float x) { return x; }, std::true_type{});
        }
    }
}

template <typename TT, typename OT>
int launch_single_token(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                        const int32_t* bag_off, const int32_t* lmax, int64_t n_units, const void* table,
                        int64_t table_rows, int32_t dim, void* out, int64_t out_stride, int32_t flags, int grid,
                        hipStream_t st) {
    const int nchunks = dim / Elem<TT>::EPV;
#define RF_ST(L)                                                                                                      \
    hipLaunchKernelGGL((single_token_embed_kernel<L, TT, OT>), dim3(grid), dim3(64), 0, st, d_slots, n_slots, tok_bytes, \
                       tok_off, bag_off, lmax, n_units, (const TT*)table, table_rows, dim, (OT*)out, out_stride, flags)
    if (nchunks == 4) RF_ST(4);
    else if (nchunks == 8) RF_ST(8);
    else if (nchunks == 16) RF_ST(16);
    else return rf_set_error(RF_EINVAL, "single-token kernel: rows of %d 16-byte chunks (4, 8 or 16 supported)", nchunks);
#undef RF_ST
    return rf_check_launch("single_token_embed_kernel");
}

// lanes per row / 16-byte chunks per lane for `nchunks` 16-byte chunks per row: teams of up to
// kDefaultMaxLpr = 16 lanes (tuned on MI355X: 16 > 8 >> 4, 2), at most 4 chunks per lane.
template <typename F>
int dispatch_fused(int nchunks, F&& f) {
    using std::integral_constant;
    int lpr = 1;
    while (lpr < nchunks && lpr < kDefaultMaxLpr) lpr <<= 1;
    while ((nchunks + lpr - 1) / lpr > 4 && lpr < 64) lpr <<= 1;
    const int cpl = (nchunks + lpr - 1) / lpr;
    const int c = cpl <= 1 ? 1 : cpl <= 2 ? 2 : cpl <= 4 ? 4 : 0;
    if (c == 0) return rf_set_error(RF_EINVAL, "embedding dim too large (> 256 16-byte chunks per row)");
#define RF_CASE(L, CP) \
    if (lpr == L && c == CP) return f(integral_constant<int, L>{}, integral_constant<int, CP>{});
    RF_CASE(1, 1) RF_CASE(2, 1) RF_CASE(4, 1) RF_CASE(8, 1) RF_CASE(16, 1) RF_CASE(16, 2) RF_CASE(16, 4)
    RF_CASE(32, 4) RF_CASE(64, 4)
#undef RF_CASE
    return rf_set_error(RF_EINVAL, "no kernel for %d lanes x %d chunks", lpr, c);
}

// One launcher per (table dtype, mode, output dtype), each in its own translation unit (parallel build).
// PRE = pooling of pre-gathered rows (rf_pool_rows_fwd): a separate instantiation so the hashing
// kernel's register allocation is not affected by the extra mode.
template <typename TT, bool PRE, typename OT>
int launch_fused_impl(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                      const int32_t* bag_off, const int32_t* lmax, int64_t n_units, const void* table,
                      int64_t table_rows, int32_t dim, void* out, int64_t out_stride, int32_t flags,
                      int64_t* idx_out, int grid, hipStream_t st) {
    constexpr int epv = Elem<TT>::EPV;
    return dispatch_fused(dim / epv, [&](auto lpr, auto cpl) -> int {
        constexpr int LPR = decltype(lpr)::value, CPL = decltype(cpl)::value;
        const bool full = dim / epv == LPR * CPL;
#define RF_FUSED_LAUNCH(FULL)                                                                                        \
    hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, FULL, TT, OT, PRE>), dim3(grid), dim3(kWaves * 64), 0, st, \
                       d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const TT*)table, table_rows,     \
                       dim, (OT*)out, out_stride, flags, idx_out)
        if (full) RF_FUSED_LAUNCH(true); else RF_FUSED_LAUNCH(false);
#undef RF_FUSED_LAUNCH
        return rf_check_launch(PRE ? "fused_pool_rows_kernel" : "fused_hash_embed_kernel");
    });
}

#define RF_FUSED_LAUNCH_DECL(NAME)                                                                                     \
    int NAME(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,          \
             const int32_t* bag_off, const int32_t* lmax, int64_t n_units, const void* table, int64_t table_rows,      \
             int32_t dim, void* out, int64_t out_stride, int32_t flags, int64_t* idx_out, int grid, hipStream_t st)
// rf_{fused,pool}_<table dtype>_o<out dtype>.hip
RF_FUSED_LAUNCH_DECL(launch_fused_f32_of32);
RF_FUSED_LAUNCH_DECL(launch_fused_f32_obf16);
RF_FUSED_LAUNCH_DECL(launch_fused_bf16_of32);
RF_FUSED_LAUNCH_DECL(launch_fused_bf16_obf16);
RF_FUSED_LAUNCH_DECL(launch_pool_f32_of32);
RF_FUSED_LAUNCH_DECL(launch_pool_f32_obf16);
RF_FUSED_LAUNCH_DECL(launch_pool_bf16_of32);
RF_FUSED_LAUNCH_DECL(launch_pool_bf16_obf16);

// rf_single.hip: the single-token kernel for (table dtype, output dtype)
int launch_single_token_any(int32_t table_dtype, int32_t out_dtype, const rf_slot_desc* d_slots, int32_t n_slots,
                            const uint8_t* tok_bytes, const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                            int64_t n_units, const void* table, int64_t table_rows, int32_t dim, void* out,
                            int64_t out_stride, int32_t flags, int grid, hipStream_t st);

// picks the launcher for (table dtype, output dtype)
inline int launch_fused_any(bool pre, int32_t table_dtype, int32_t out_dtype, const rf_slot_desc* d_slots,
                            int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off, const int32_t* bag_off,
                            const int32_t* lmax, int64_t n_units, const void* table, int64_t table_rows, int32_t dim,
                            void* out, int64_t out_stride, int32_t flags, int64_t* idx_out, int grid, hipStream_t st) {
    const bool tf = table_dtype == RF_DTYPE_F32, of = out_dtype == RF_DTYPE_F32;
    auto* fn = pre ? (tf ? (of ? launch_pool_f32_of32 : launch_pool_f32_obf16)
                         : (of ? launch_pool_bf16_of32 : launch_pool_bf16_obf16))
                   : (tf ? (of ? launch_fused_f32_of32 : launch_fused_f32_obf16)
                         : (of ? launch_fused_bf16_of32 : launch_fused_bf16_obf16));
    return fn(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table, table_rows, dim, out, out_stride,
              flags, idx_out, grid, st);
}

}  // namespace rf
