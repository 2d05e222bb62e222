// rf_embed.hip — sparse-feature hot path for gfx950:
//   rf_siphash_bucket        Keras Hashing                       (preprocess_layers.py:89-90)
//   rf_fused_hash_embed_fwd  DoubleHashingEmbedding x all slots  (preprocess_layers.py:79-106, preprocess_utils.py:10-20)
//   rf_embedding_bag_fwd     EmbeddingBag over integer ids       (preprocess_layers.py:16-76)
//   rf_table_init_uniform    counter-based 'uniform' init        (preprocess_layers.py:24,31-39)
//
// Fused kernel layout: one wave owns an "item" of kUnits consecutive
// (example, slot) units of the example-major CSR batch.
//   phase 1  lane-per-token: both SipHash-2-4 states over one read of the token bytes, bucket ids
//            into a per-wave LDS index bucket (indices never touch HBM);
//   phase 2  the wave splits into teams of LPR lanes (one 16-byte chunk of a row per lane); a team
//            pools its units' rows with fp32 accumulation in position order l = 0..Lmax-1 (bit-exact
//            with the oracle), then writes [pool(T1) | pool(T2)] straight to the slot's output offset.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "rf_fused.h"

namespace {
using namespace rf;
// ---------------------------------------------------------------------------------------------
// EmbeddingBag over dense ids [batch][len]
// ---------------------------------------------------------------------------------------------
template <int LPR, int CPL, typename TT, typename OT>
__global__ __launch_bounds__(256) void embedding_bag_kernel(const int64_t* __restrict__ ids, int batch, int len,
                                                            int64_t row_base, const TT* __restrict__ table,
                                                            int64_t table_rows, int dim, int comb,
                                                            OT* __restrict__ out, int64_t out_stride, int64_t out_off) {
    constexpr int EPV = Elem<TT>::EPV;
    constexpr int TEAMS = 64 / LPR;
    const int lane = threadIdx.x & 63, team = lane / LPR, tl = lane % LPR;
    const int nchunks = dim / EPV;
    const int64_t gteam = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * TEAMS + team;
    const int64_t nteams = (int64_t)gridDim.x * (blockDim.x >> 6) * TEAMS;
    for (int64_t b = gteam; b < batch; b += nteams) {
        const int64_t* bid = ids + b * len;
        OT* orow = out + b * out_stride + out_off;
        if (comb == RF_COMB_NULL) {
            for (int l = 0; l < len; ++l) {
                const int64_t r = row_base + bid[l];
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc) {
                    const int c = tl + cc * LPR;
                    if (c >= nchunks) continue;
                    float f[EPV];
                    unpack16<TT>(load_chunk(table, r, table_rows, dim, c), f);
                    store_chunk<OT, EPV>(orow + (int64_t)l * dim + c * EPV, f);
                }
            }
            continue;
        }
        float acc[CPL][EPV];
        if (comb == RF_COMB_FIRST || comb == RF_COMB_LAST) {
            const int p = comb == RF_COMB_FIRST ? 0 : len - 1;
            const int64_t r = len > 0 ? row_base + bid[p] : -1;
#pragma unroll
            for (int cc = 0; cc < CPL; ++cc) {
                const int c = tl + cc * LPR;
                if (len == 0 || c >= nchunks) {
#pragma unroll
                    for (int e = 0; e < EPV; ++e) acc[cc][e] = 0.0f;
                } else {
                    unpack16<TT>(load_chunk(table, r, table_rows, dim, c), acc[cc]);
                }
            }
        } else {
            const float init = comb_init(comb);
#pragma unroll
            for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                for (int e = 0; e < EPV; ++e) acc[cc][e] = init;
            for (int l = 0; l < len; l += 4) {
                uint4 v[4][CPL];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (l + q < len) {
                        const int64_t r = row_base + bid[l + q];
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            const int c = tl + cc * LPR;
                            v[q][cc] = c < nchunks ? load_chunk(table, r, table_rows, dim, c) : make_uint4(0, 0, 0, 0);
                        }
                    }
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (l + q < len)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            float f[EPV];
                            unpack16<TT>(v[q][cc], f);
#pragma unroll
                            for (int e = 0; e < EPV; ++e) acc[cc][e] = comb_step(comb, acc[cc][e], f[e]);
                        }
            }
            if (comb == RF_COMB_AVG) {
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                    for (int e = 0; e < EPV; ++e) acc[cc][e] = __fdiv_rn(acc[cc][e], (float)len);
            }
        }
#pragma unroll
        for (int cc = 0; cc < CPL; ++cc) {
            const int c = tl + cc * LPR;
            if (c < nchunks) store_chunk<OT, EPV>(orow + c * EPV, acc[cc]);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Keras Hashing, lane per token
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void siphash_bucket_kernel(const uint8_t* __restrict__ tok_bytes,
                                                             const int32_t* __restrict__ tok_off, int64_t n_tok,
                                                             uint64_t k0, uint64_t k1, int64_t num_bins,
                                                             int mask_empty, int64_t* __restrict__ out) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_tok; t += (int64_t)gridDim.x * blockDim.x) {
        const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
        out[t] = hash_bucket_dev(k0, k1, tok_bytes + b0, n, num_bins, mask_empty);
    }
}

// ---------------------------------------------------------------------------------------------
// counter-based uniform init (4 consecutive elements per thread)
// ---------------------------------------------------------------------------------------------
template <typename TT>
__global__ __launch_bounds__(256) void table_init_kernel(TT* __restrict__ table, int64_t rows, int dim, int64_t row0,
                                                         int64_t row_stride, uint64_t seed, float lo, float hi) {
    const int64_t total = rows * (int64_t)dim;
    const float span = hi - lo;
    for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < total;
         i += (int64_t)gridDim.x * blockDim.x * 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t x = i + e;
            if (x >= total) break;
            const int64_t r = x / dim;
            const int d = (int)(x - r * dim);
            const uint64_t g = (uint64_t)(row0 + r * row_stride);
            const uint64_t h = splitmix64_dev(seed ^ (g * (uint64_t)dim + (uint64_t)d));
            const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
            const float v = __fmaf_rn(span, u, lo);
            if constexpr (sizeof(TT) == 4)
                table[x] = v;
            else
                table[x] = (TT)f32_to_bf16_bits(v);
        }
    }
}

// rf_hash_rows: a block takes 256 consecutive (example, slot) units = one contiguous token range; a
// thread per TOKEN (its unit found by binary search over the block's 257 bag offsets in LDS), so the
// multi-valued slots do not serialise a thread; both salts over one read of each token, 16-byte stores.
constexpr int kHashUnits = 256;
__global__ __launch_bounds__(kHashUnits) void hash_rows_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                               const uint8_t* __restrict__ tok_bytes,
                                                               const int32_t* __restrict__ tok_off,
                                                               const int32_t* __restrict__ bag_off, int64_t n_units,
                                                               int64_t* __restrict__ rows_out) {
    __shared__ int32_t s_off[kHashUnits + 1];
    for (int64_t u0 = (int64_t)blockIdx.x * kHashUnits; u0 < n_units; u0 += (int64_t)gridDim.x * kHashUnits) {
        const int nu = (int)min<int64_t>(kHashUnits, n_units - u0);
        __syncthreads();
        for (int j = threadIdx.x; j <= nu; j += kHashUnits) s_off[j] = bag_off[u0 + j];
        __syncthreads();
        const int t0 = s_off[0], t1 = s_off[nu];
        const uint32_t s_first = (uint32_t)(u0 % n_slots);  // slot of unit u0 (one 64-bit remainder per block step)
        for (int t = t0 + (int)threadIdx.x; t < t1; t += kHashUnits) {
            int lo = 0, hi = nu - 1;  // last unit j with s_off[j] <= t
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] <= t) lo = mid; else hi = mid - 1;
            }
            const rf_slot_desc* sd = slots + (int)((s_first + (uint32_t)lo) % (uint32_t)n_slots);
            const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
            uint64_t h0, h1;
            siphash24x2_dev(sd->salt[0], sd->salt[1], tok_bytes + b0, n, h0, h1);
            // both keys share the slot's modulus: one reciprocal instead of two 64-bit remainders
            const BucketMod bm = bucket_mod_init(sd->num_bins, sd->mask_empty);
            longlong2 r;
            r.x = sd->row_base[0] + bucket_from_hash(h0, n, bm);
            r.y = sd->row_base[1] + bucket_from_hash(h1, n, bm);
            reinterpret_cast<longlong2*>(rows_out)[t] = r;
        }
    }
}

int grid_for(int64_t work_items, int per_block, int cap = 256 * 16) {
    int64_t g = (work_items + per_block - 1) / per_block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// choose (LPR, CPL) for `nchunks` 16-byte chunks per row
template <typename F>
int dispatch_lpr(int nchunks, F&& f) {
    if (nchunks <= 1) return f(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 2) return f(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 4) return f(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 8) return f(std::integral_constant<int, 8>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 16) return f(std::integral_constant<int, 16>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 32) return f(std::integral_constant<int, 32>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 64) return f(std::integral_constant<int, 64>{}, std::integral_constant<int, 1>{});
    if (nchunks <= 128) return f(std::integral_constant<int, 64>{}, std::integral_constant<int, 2>{});
    if (nchunks <= 256) return f(std::integral_constant<int, 64>{}, std::integral_constant<int, 4>{});
    return rf_set_error(RF_EINVAL, "embedding dim too large (> 256 16-byte chunks per row)");
}

}  // namespace

// ===============================================================================================
// C ABI
// ===============================================================================================
extern "C" int rf_siphash_bucket(const uint8_t* tok_bytes, const int32_t* tok_off, int64_t n_tok, uint64_t k0,
                                 uint64_t k1, int64_t num_bins, int32_t mask_empty, int64_t* out, void* stream) {
    RF_REQUIRE(n_tok >= 0, "rf_siphash_bucket: n_tok < 0");
    RF_REQUIRE(num_bins >= 1, "rf_siphash_bucket: num_bins must be >= 1 (Keras: non-positive num_bins is an error)");
    if (n_tok == 0) return RF_OK;
    RF_REQUIRE(tok_bytes && tok_off && out, "rf_siphash_bucket: null pointer");
    hipLaunchKernelGGL(siphash_bucket_kernel, dim3(grid_for(n_tok, 256)), dim3(256), 0, rf_stream(stream), tok_bytes,
                       tok_off, n_tok, k0, k1, num_bins, mask_empty, out);
    return rf_check_launch("siphash_bucket_kernel");
}

static int fused_hash_embed_fwd_impl(uint32_t allowed_diag, const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                       const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                       int32_t batch, const void* table, int32_t table_dtype, int64_t table_rows,
                                       int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags,
                                       int64_t* idx_out, void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0, "rf_fused_hash_embed_fwd: need n_slots >= 1, batch >= 0");
    RF_REQUIRE(table_dtype == RF_DTYPE_F32 || table_dtype == RF_DTYPE_BF16, "rf_fused_hash_embed_fwd: table dtype must be F32 or BF16");
    RF_REQUIRE(out_dtype == RF_DTYPE_F32 || out_dtype == RF_DTYPE_BF16, "rf_fused_hash_embed_fwd: out dtype must be F32 or BF16");
    const int epv = table_dtype == RF_DTYPE_F32 ? 4 : 8;
    RF_REQUIRE(dim > 0 && dim % epv == 0, "rf_fused_hash_embed_fwd: dim (%d) must be a positive multiple of %d (16-byte rows chunks)", dim, epv);
    RF_REQUIRE(out_stride % epv == 0, "rf_fused_hash_embed_fwd: out_stride must be a multiple of %d", epv);
    RF_REQUIRE(((uintptr_t)table & 15) == 0 && ((uintptr_t)out & 15) == 0, "rf_fused_hash_embed_fwd: table/out must be 16-byte aligned");
    RF_REQUIRE((flags & ~(RF_FLAG_MASK_PADDING | RF_FLAG_EMIT_IDX | RF_FLAG_SINGLE_TOKEN | (int32_t)allowed_diag)) == 0,
               "rf_fused_hash_embed_fwd: unknown flags (result-changing ablation bits 12-14 are only accepted by "
               "rf_diag_fused_hash_embed_fwd)");
    RF_REQUIRE(table_rows >= 1 && table_rows <= (int64_t)0xffffffff, "rf_fused_hash_embed_fwd: table_rows must be in [1, 2^32) (32-bit row ids in LDS)");
    const int64_t n_units = (int64_t)batch * n_slots;
    if (n_units == 0) return RF_OK;
    RF_REQUIRE(d_slots && tok_bytes && tok_off && bag_off && lmax && table && out, "rf_fused_hash_embed_fwd: null pointer");
    const int64_t items = (int64_t)n_slots * ((batch + kUnits - 1) / kUnits);  // slot-major items
    hipStream_t st = rf_stream(stream);
    if (flags & RF_FLAG_SINGLE_TOKEN) {
        RF_REQUIRE(!(flags & RF_FLAG_EMIT_IDX), "rf_fused_hash_embed_fwd: RF_FLAG_SINGLE_TOKEN does not emit ids");
        RF_REQUIRE(!(flags & 0xF800), "rf_fused_hash_embed_fwd: RF_FLAG_SINGLE_TOKEN takes no diagnostic bits");
        return launch_single_token_any(table_dtype, out_dtype, d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units,
                                       table, table_rows, dim, out, out_stride, flags, grid_for(items, 1, 256 * 32 * 2), st);
    }
    static const int grid_cap = [] {  // RF_FUSED_GRID_CAP: A/B of a persistent grid (waves walk several items)
        const char* e = getenv("RF_FUSED_GRID_CAP");
        return e ? std::max(1, atoi(e)) : 256 * 32 * 2;
    }();
    const int grid = grid_for(items, kWaves, grid_cap);
    return launch_fused_any(false, table_dtype, out_dtype, d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units,
                            table, table_rows, dim, out, out_stride, flags, idx_out, grid, st);
}

namespace {
// The index half of the single-token kernel (rf_single_token_ids_fwd; the ESIM gather path, rf_attn.hip):
// ids[u][k] = the fused-table row of hash k for unit u = b * n_slots + s (its one token; an empty bag: the
// slot's pad rows, or kRowZero when padding is masked); a slot whose batch Lmax is not 1, or that does not fit
// the table, gets kRowNaN (the embedding kernel writes NaN there). One wave per item (a slot x 64 bags),
// lane j hashes bag b0 + j exactly as single_token_embed_kernel does.
__global__ __launch_bounds__(64) void single_token_ids_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                             const uint8_t* __restrict__ tok_bytes,
                                                             const int32_t* __restrict__ tok_off,
                                                             const int32_t* __restrict__ bag_off,
                                                             const int32_t* __restrict__ lmax, int64_t n_units,
                                                             int64_t table_rows, uint32_t* __restrict__ ids, int flags) {
    const int lane = threadIdx.x;
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const int batch = (int)(n_units / n_slots);
    const int nbb = (batch + kUnits - 1) / kUnits;
    const int64_t n_items = (int64_t)n_slots * nbb;
    for (int64_t item = blockIdx.x; item < n_items; item += gridDim.x) {
        const int s = (int)(item / nbb);
        const int b0 = (int)(item - (int64_t)s * nbb) * kUnits;
        const int nu = min(kUnits, batch - b0);
        if (lane >= nu) continue;
        const rf_slot_desc* sd = slots + s;
        const int64_t rb0 = sd->row_base[0], rb1 = sd->row_base[1], nbins = sd->num_bins;
        const uint64_t salt0 = sd->salt[0], salt1 = sd->salt[1];
        const int mask_empty = sd->mask_empty;
        const BucketMod bmod = bucket_mod_init(nbins, mask_empty);
        const bool ok = rb0 >= 0 && rb1 >= 0 && rb0 + nbins <= table_rows && rb1 + nbins <= table_rows;
        const int64_t u = (int64_t)(b0 + lane) * n_slots + s;
        uint32_t r0 = kRowNaN, r1 = kRowNaN;
        if (ok && lmax[s] == 1) {
            const int t = bag_off[u];
            if (bag_off[u + 1] > t) {
                const int tb = tok_off[t], n = tok_off[t + 1] - tb;
                uint64_t h0, h1;
                siphash24x2_dev(salt0, salt1, tok_bytes + tb, n, h0, h1);
                r0 = (uint32_t)(rb0 + bucket_from_hash(h0, n, bmod));
                r1 = (uint32_t)(rb1 + bucket_from_hash(h1, n, bmod));
            } else if (mask_pad) {
                r0 = r1 = kRowZero;
            } else {
                int64_t pb0 = 0, pb1 = 0;
                if (!mask_empty) {
                    pb0 = (int64_t)(siphash24_dev(salt0, salt0, tok_bytes, 0) % (uint64_t)nbins);
                    pb1 = (int64_t)(siphash24_dev(salt1, salt1, tok_bytes, 0) % (uint64_t)nbins);
                }
                r0 = (uint32_t)(rb0 + pb0);
                r1 = (uint32_t)(rb1 + pb1);
            }
        }
        if (flags & RF_FLAG_SPEC_ROWS) {
            r0 = r0 == kRowNaN ? (uint32_t)table_rows : r0 == kRowZero ? (uint32_t)table_rows + 1u : r0;
            r1 = r1 == kRowNaN ? (uint32_t)table_rows : r1 == kRowZero ? (uint32_t)table_rows + 1u : r1;
        }
        *reinterpret_cast<uint2*>(ids + 2 * u) = make_uint2(r0, r1);
    }
}


// The same ids, example-major (round 3): thread per unit u = b * n_slots + s, so the bag_off / tok_off reads and
// the ids stores of a wave are consecutive (the slot-major kernel touches 64 units n_slots apart per load and
// store). Each workgroup first stages every slot's constants in LDS (salts, row bases, the bucket modulus: one
// 64-bit division per slot), so a unit's only global reads are its CSR offsets and token bytes; u < 2^31, 32-bit
// index arithmetic (round 4: the per-lane descriptor gathers and the 64-bit u % n_slots were a third of the
// cfg3 id pass, profiles/r04/cfg3_*).
constexpr int kIdsMaxSlots = 512;
#ifndef RF_IDS_UNITS
#define RF_IDS_UNITS 1
#endif
constexpr int kIdsUnits = RF_IDS_UNITS;  // units per thread (single_token_ids_em_body)
struct IdsSlot {
    uint64_t salt0, salt1;
    BucketMod bm;
    int64_t rb0, rb1, nbins;
    int32_t live;  // the slot fits the table and its batch Lmax is 1
    int32_t mask_empty;
};

__device__ __forceinline__ void single_token_ids_em_body(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                        const uint8_t* __restrict__ tok_bytes,
                                                        const int32_t* __restrict__ tok_off,
                                                        const int32_t* __restrict__ bag_off,
                                                        const int32_t* __restrict__ lmax, int64_t n_units,
                                                        int64_t table_rows, uint32_t* __restrict__ ids, int flags,
                                                        int64_t block, int64_t n_blocks, IdsSlot* ssl) {
    for (int s = threadIdx.x; s < n_slots; s += blockDim.x) {
        const rf_slot_desc& sd = slots[s];
        IdsSlot v;
        v.salt0 = sd.salt[0];
        v.salt1 = sd.salt[1];
        v.bm = bucket_mod_init(sd.num_bins, sd.mask_empty);
        v.rb0 = sd.row_base[0];
        v.rb1 = sd.row_base[1];
        v.nbins = sd.num_bins;
        v.live = v.rb0 >= 0 && v.rb1 >= 0 && v.rb0 + v.nbins <= table_rows && v.rb1 + v.nbins <= table_rows && lmax[s] == 1;
        v.mask_empty = sd.mask_empty;
        ssl[s] = v;
    }
    __syncthreads();
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const uint32_t ns = (uint32_t)n_slots, nu = (uint32_t)n_units;
    const uint32_t stride = (uint32_t)(n_blocks * blockDim.x);
    // kIdsUnits units per thread in lockstep: the CSR offsets, then the token offsets, then the token's dwords of
    // every unit are loaded before any is hashed (siphash24x2_dev's message reads sit inside its rounds). One unit
    // per thread measured best (tools/ids_probe.py: 16.0 us for 1, 16.7 for 2, 21.2 for 4 units per thread)
    for (uint32_t u0 = (uint32_t)(block * blockDim.x) + threadIdx.x; u0 < nu; u0 += kIdsUnits * stride) {
        uint32_t uu[kIdsUnits], ss[kIdsUnits];
        bool live[kIdsUnits];
        int t0[kIdsUnits], t1[kIdsUnits];
#pragma unroll
        for (int k = 0; k < kIdsUnits; ++k) {
            uu[k] = u0 + (uint32_t)k * stride;
            ss[k] = uu[k] < nu ? uu[k] % ns : 0u;
            live[k] = uu[k] < nu && ssl[ss[k]].live;
            t0[k] = live[k] ? bag_off[uu[k]] : 0;
            t1[k] = live[k] ? bag_off[uu[k] + 1] : 0;
        }
        int tb[kIdsUnits], n[kIdsUnits];
#pragma unroll
        for (int k = 0; k < kIdsUnits; ++k) {
            const bool has = live[k] && t1[k] > t0[k];
            tb[k] = has ? tok_off[t0[k]] : 0;
            n[k] = has ? tok_off[t0[k] + 1] - tb[k] : -1;  // -1: empty bag or dead slot
        }
        uint32_t wv[kIdsUnits][kSipRegWords + 1];
        uint32_t sh[kIdsUnits];
#pragma unroll
        for (int k = 0; k < kIdsUnits; ++k) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(tok_bytes + tb[k]);
            sh[k] = (uint32_t)(a & 3);
            const uint32_t* w = reinterpret_cast<const uint32_t*>(a - sh[k]);
            const int nw = n[k] > 0 && (int)sh[k] + n[k] <= 4 * kSipRegWords ? (int)((sh[k] + (uint32_t)n[k] + 3) >> 2) : 0;
#pragma unroll
            for (int j = 0; j < kSipRegWords; ++j) wv[k][j] = j < nw ? w[j] : 0u;
            wv[k][kSipRegWords] = 0u;
        }
#pragma unroll
        for (int k = 0; k < kIdsUnits; ++k) {
            if (uu[k] >= nu) continue;
            const IdsSlot& sl = ssl[ss[k]];
            uint32_t r0 = kRowNaN, r1 = kRowNaN;
            if (live[k]) {
                if (n[k] >= 0) {
                    uint64_t h0, h1;
                    if ((int)sh[k] + n[k] <= 4 * kSipRegWords)
                        siphash24x2_regs(sl.salt0, sl.salt1, wv[k], sh[k], n[k], h0, h1);
                    else  // long token: the streaming form
                        siphash24x2_dev(sl.salt0, sl.salt1, tok_bytes + tb[k], n[k], h0, h1);
                    r0 = (uint32_t)(sl.rb0 + bucket_from_hash(h0, n[k], sl.bm));
                    r1 = (uint32_t)(sl.rb1 + bucket_from_hash(h1, n[k], sl.bm));
                } else if (mask_pad) {
                    r0 = r1 = kRowZero;
                } else {
                    int64_t pb0 = 0, pb1 = 0;
                    if (!sl.mask_empty) {
                        pb0 = (int64_t)(siphash24_dev(sl.salt0, sl.salt0, tok_bytes, 0) % (uint64_t)sl.nbins);
                        pb1 = (int64_t)(siphash24_dev(sl.salt1, sl.salt1, tok_bytes, 0) % (uint64_t)sl.nbins);
                    }
                    r0 = (uint32_t)(sl.rb0 + pb0);
                    r1 = (uint32_t)(sl.rb1 + pb1);
                }
            }
            if (flags & RF_FLAG_SPEC_ROWS) {  // the NaN / zero rows at table_rows / table_rows + 1
                r0 = r0 == kRowNaN ? (uint32_t)table_rows : r0 == kRowZero ? (uint32_t)table_rows + 1u : r0;
                r1 = r1 == kRowNaN ? (uint32_t)table_rows : r1 == kRowZero ? (uint32_t)table_rows + 1u : r1;
            }
            *reinterpret_cast<uint2*>(ids + 2 * (size_t)uu[k]) = make_uint2(r0, r1);
        }
    }
}

__global__ __launch_bounds__(256) void single_token_ids_em_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                                 const uint8_t* __restrict__ tok_bytes,
                                                                 const int32_t* __restrict__ tok_off,
                                                                 const int32_t* __restrict__ bag_off,
                                                                 const int32_t* __restrict__ lmax, int64_t n_units,
                                                                 int64_t table_rows, uint32_t* __restrict__ ids, int flags) {
    extern __shared__ IdsSlot ssl[];
    single_token_ids_em_body(slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table_rows, ids, flags,
                             blockIdx.x, gridDim.x, ssl);
}

// several towers in one launch (rf_single_token_ids_multi_fwd): workgroups [first[k], first[k + 1]) run task k
struct IdsTasks {
    rf_ids_task t[4];
    int64_t first[5];
    int n;
};
__global__ __launch_bounds__(256) void single_token_ids_multi_kernel(const IdsTasks tasks) {
    extern __shared__ IdsSlot ssl[];
    int k = 0;
    while (k + 1 < tasks.n && (int64_t)blockIdx.x >= tasks.first[k + 1]) ++k;
    const rf_ids_task& t = tasks.t[k];
    single_token_ids_em_body(t.slots, t.n_slots, t.tok_bytes, t.tok_off, t.bag_off, t.lmax, (int64_t)t.batch * t.n_slots,
                             t.table_rows, t.ids, t.flags, (int64_t)blockIdx.x - tasks.first[k],
                             tasks.first[k + 1] - tasks.first[k], ssl);
}

}  // namespace

extern "C" int rf_single_token_ids_multi_fwd(const rf_ids_task* tasks, int32_t n_tasks, void* stream) {
    RF_REQUIRE(tasks && n_tasks >= 1 && n_tasks <= 4, "rf_single_token_ids_multi_fwd: need 1 <= n_tasks <= 4 (got %d)", n_tasks);
    IdsTasks a{};
    a.n = n_tasks;
    int64_t blocks = 0;
    for (int k = 0; k < n_tasks; ++k) {
        const rf_ids_task& t = tasks[k];
        RF_REQUIRE(t.n_slots >= 1 && t.n_slots <= kIdsMaxSlots && t.batch >= 0,
                   "rf_single_token_ids_multi_fwd: task %d needs 1 <= n_slots <= %d, batch >= 0", k, kIdsMaxSlots);
        RF_REQUIRE((t.flags & ~(RF_FLAG_MASK_PADDING | RF_FLAG_SPEC_ROWS)) == 0 && t.reserved == 0,
                   "rf_single_token_ids_multi_fwd: task %d: only RF_FLAG_MASK_PADDING and RF_FLAG_SPEC_ROWS are accepted", k);
        RF_REQUIRE(t.table_rows >= 1 && t.table_rows < (int64_t)kRowNaN,
                   "rf_single_token_ids_multi_fwd: task %d: table_rows must be in [1, 2^32 - 2)", k);
        const int64_t n_units = (int64_t)t.batch * t.n_slots;
        RF_REQUIRE(n_units < ((int64_t)1 << 31), "rf_single_token_ids_multi_fwd: task %d: batch * n_slots must be < 2^31", k);
        if (n_units)
            RF_REQUIRE(t.slots && t.tok_bytes && t.tok_off && t.bag_off && t.lmax && t.ids && ((uintptr_t)t.ids & 7) == 0,
                       "rf_single_token_ids_multi_fwd: task %d: null pointer or ids not 8-byte aligned", k);
        a.t[k] = t;
        a.first[k] = blocks;
        blocks += std::min<int64_t>((n_units + 256 * kIdsUnits - 1) / (256 * kIdsUnits), 256 * 32 / n_tasks);
    }
    a.first[n_tasks] = blocks;
    if (blocks == 0) return RF_OK;
    int max_slots = 1;
    for (int k = 0; k < n_tasks; ++k) max_slots = std::max(max_slots, tasks[k].n_slots);
    hipLaunchKernelGGL(single_token_ids_multi_kernel, dim3((unsigned)blocks), dim3(256), sizeof(IdsSlot) * max_slots,
                       rf_stream(stream), a);
    return rf_check_launch("single_token_ids_multi_kernel");
}

extern "C" int rf_single_token_ids_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                       const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                       int32_t batch, int64_t table_rows, uint32_t* ids, int32_t flags, void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0, "rf_single_token_ids_fwd: need n_slots >= 1, batch >= 0");
    RF_REQUIRE((flags & ~(RF_FLAG_MASK_PADDING | RF_FLAG_SPEC_ROWS)) == 0,
               "rf_single_token_ids_fwd: only RF_FLAG_MASK_PADDING and RF_FLAG_SPEC_ROWS are accepted");
    RF_REQUIRE(table_rows >= 1 && table_rows < (int64_t)kRowNaN, "rf_single_token_ids_fwd: table_rows must be in [1, 2^32 - 2)");
    const int64_t n_units = (int64_t)batch * n_slots;
    if (n_units == 0) return RF_OK;
    RF_REQUIRE(d_slots && tok_bytes && tok_off && bag_off && lmax && ids, "rf_single_token_ids_fwd: null pointer");
    RF_REQUIRE(((uintptr_t)ids & 7) == 0, "rf_single_token_ids_fwd: ids must be 8-byte aligned");
    static const int slot_major = [] {  // RF_IDS_SLOT_MAJOR=1: the slot-major kernel (A/B only)
        const char* e = getenv("RF_IDS_SLOT_MAJOR");
        return e && e[0] == '1';
    }();
    if (n_slots <= kIdsMaxSlots && !slot_major && n_units < ((int64_t)1 << 31)) {
        const int64_t blocks = std::min<int64_t>((n_units + 256 * kIdsUnits - 1) / (256 * kIdsUnits), 256 * 32);
        hipLaunchKernelGGL(single_token_ids_em_kernel, dim3((unsigned)blocks), dim3(256), sizeof(IdsSlot) * n_slots,
                           rf_stream(stream), d_slots,
                           n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table_rows, ids, flags);
        return rf_check_launch("single_token_ids_em_kernel");
    }
    const int64_t items = (int64_t)n_slots * ((batch + kUnits - 1) / kUnits);
    hipLaunchKernelGGL(single_token_ids_kernel, dim3(grid_for(items, 1, 256 * 32 * 2)), dim3(64), 0, rf_stream(stream),
                       d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table_rows, ids, flags);
    return rf_check_launch("single_token_ids_kernel");
}

extern "C" int rf_fused_hash_embed_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                       const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                       int32_t batch, const void* table, int32_t table_dtype, int64_t table_rows,
                                       int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags,
                                       int64_t* idx_out, void* stream) {
    // public ABI: only the result-preserving switches (bit 11 XCD item order, bit 15 general phase 2)
    return fused_hash_embed_fwd_impl(RF_FLAG_DIAG_XCD_ORDER | RF_FLAG_DIAG_GENERAL_PHASE2, d_slots, n_slots, tok_bytes,
                                     tok_off, bag_off, lmax, batch, table, table_dtype, table_rows, dim, out, out_dtype,
                                     out_stride, flags, idx_out, stream);
}

extern "C" int rf_diag_fused_hash_embed_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                            const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                                            int32_t batch, const void* table, int32_t table_dtype, int64_t table_rows,
                                            int32_t dim, void* out, int32_t out_dtype, int64_t out_stride,
                                            int32_t flags, int64_t* idx_out, void* stream) {
    // tools only (include/rf_diag.h): additionally accepts the ablation bits 12-14, which CHANGE results
    return fused_hash_embed_fwd_impl(0xF800u, d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, batch, table,
                                     table_dtype, table_rows, dim, out, out_dtype, out_stride, flags, idx_out, stream);
}

extern "C" int rf_hash_rows(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                            const int32_t* tok_off, const int32_t* bag_off, int32_t batch, int64_t* rows_out,
                            void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0, "rf_hash_rows: need n_slots >= 1, batch >= 0");
    const int64_t n_units = (int64_t)batch * n_slots;
    if (n_units == 0) return RF_OK;
    RF_REQUIRE(d_slots && tok_bytes && tok_off && bag_off && rows_out, "rf_hash_rows: null pointer");
    RF_REQUIRE(((uintptr_t)rows_out & 15) == 0, "rf_hash_rows: rows_out must be 16-byte aligned");
    hipLaunchKernelGGL(hash_rows_kernel, dim3(grid_for(n_units, kHashUnits, 256 * 64)), dim3(kHashUnits), 0, rf_stream(stream), d_slots,
                       n_slots, tok_bytes, tok_off, bag_off, n_units, rows_out);
    return rf_check_launch("hash_rows_kernel");
}

extern "C" int rf_pool_rows_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off,
                                const int32_t* lmax, int32_t batch, int64_t n_tok, const void* gathered,
                                const int32_t* row_map, const void* local_table, int32_t dtype, int32_t dim, void* out,
                                int32_t out_dtype, int64_t out_stride, int32_t flags, void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0 && n_tok >= 0, "rf_pool_rows_fwd: need n_slots >= 1, batch, n_tok >= 0");
    RF_REQUIRE(dtype == RF_DTYPE_F32 || dtype == RF_DTYPE_BF16, "rf_pool_rows_fwd: dtype must be F32 or BF16");
    RF_REQUIRE(out_dtype == RF_DTYPE_F32 || out_dtype == RF_DTYPE_BF16, "rf_pool_rows_fwd: out dtype must be F32 or BF16");
    const int epv = dtype == RF_DTYPE_F32 ? 4 : 8;
    RF_REQUIRE(dim > 0 && dim % epv == 0 && out_stride % epv == 0, "rf_pool_rows_fwd: dim/out_stride must be multiples of %d", epv);
    RF_REQUIRE((flags & ~RF_FLAG_MASK_PADDING) == 0, "rf_pool_rows_fwd: only RF_FLAG_MASK_PADDING is accepted");
    const int64_t rows = 2 * n_tok + 2 * (int64_t)n_slots;
    RF_REQUIRE(rows <= (int64_t)0xffffffff, "rf_pool_rows_fwd: too many rows");
    RF_REQUIRE(((uintptr_t)gathered & 15) == 0 && ((uintptr_t)out & 15) == 0 && ((uintptr_t)local_table & 15) == 0,
               "rf_pool_rows_fwd: buffers must be 16-byte aligned");
    RF_REQUIRE(!local_table || row_map, "rf_pool_rows_fwd: local_table needs a row_map");
    const int64_t n_units = (int64_t)batch * n_slots;
    if (n_units == 0) return RF_OK;
    RF_REQUIRE(d_slots && bag_off && lmax && gathered && out, "rf_pool_rows_fwd: null pointer");
    const int64_t items = (int64_t)n_slots * ((batch + kUnits - 1) / kUnits);
    const int grid = grid_for(items, kWaves, 256 * 32 * 2);
    hipStream_t st = rf_stream(stream);
    const int fl = flags;
    // the PRE kernel takes the local table through its (otherwise unused) token-bytes pointer
    return launch_fused_any(true, dtype, out_dtype, d_slots, n_slots, (const uint8_t*)local_table, row_map, bag_off, lmax, n_units,
                            gathered, rows, dim, out, out_stride, fl, nullptr, grid, st);
}

extern "C" int rf_embedding_bag_fwd(const int64_t* ids, int32_t batch, int32_t len, int64_t row_base, const void* table,
                                    int32_t table_dtype, int64_t table_rows, int32_t dim, int32_t combiner, void* out,
                                    int32_t out_dtype, int64_t out_stride, int64_t out_off, void* stream) {
    RF_REQUIRE(batch >= 0 && len >= 0, "rf_embedding_bag_fwd: batch/len must be >= 0");
    RF_REQUIRE(combiner >= RF_COMB_SUM && combiner <= RF_COMB_NULL, "rf_embedding_bag_fwd: Do not support combiner = %d", combiner);
    RF_REQUIRE(table_dtype == RF_DTYPE_F32 || table_dtype == RF_DTYPE_BF16, "rf_embedding_bag_fwd: table dtype must be F32 or BF16");
    RF_REQUIRE(out_dtype == RF_DTYPE_F32 || out_dtype == RF_DTYPE_BF16, "rf_embedding_bag_fwd: out dtype must be F32 or BF16");
    const int epv = table_dtype == RF_DTYPE_F32 ? 4 : 8;
    RF_REQUIRE(dim > 0 && dim % epv == 0, "rf_embedding_bag_fwd: dim (%d) must be a positive multiple of %d", dim, epv);
    RF_REQUIRE(out_stride % epv == 0 && out_off % epv == 0, "rf_embedding_bag_fwd: out_stride/out_off must be multiples of %d", epv);
    RF_REQUIRE(((uintptr_t)table & 15) == 0 && ((uintptr_t)out & 15) == 0, "rf_embedding_bag_fwd: table/out must be 16-byte aligned");
    if (batch == 0) return RF_OK;
    RF_REQUIRE(table && out && (ids || len == 0), "rf_embedding_bag_fwd: null pointer");
    hipStream_t st = rf_stream(stream);
    return dispatch_lpr(dim / epv, [&](auto lpr, auto cpl) -> int {
        constexpr int LPR = decltype(lpr)::value, CPL = decltype(cpl)::value;
        const int grid = grid_for((int64_t)batch, 4 * (64 / LPR));
#define RF_EB_LAUNCH(TT, OT)                                                                                        \
    hipLaunchKernelGGL((embedding_bag_kernel<LPR, CPL, TT, OT>), dim3(grid), dim3(256), 0, st, ids, batch, len,    \
                       row_base, (const TT*)table, table_rows, dim, combiner, (OT*)out, out_stride, out_off)
        if (table_dtype == RF_DTYPE_F32) {
            if (out_dtype == RF_DTYPE_F32) RF_EB_LAUNCH(float, float); else RF_EB_LAUNCH(float, uint16_t);
        } else {
            if (out_dtype == RF_DTYPE_F32) RF_EB_LAUNCH(uint16_t, float); else RF_EB_LAUNCH(uint16_t, uint16_t);
        }
#undef RF_EB_LAUNCH
        return rf_check_launch("embedding_bag_kernel");
    });
}

extern "C" int rf_table_init_uniform(void* table, int32_t dtype, int64_t rows, int32_t dim, int64_t row0,
                                     int64_t row_stride, uint64_t seed, float lo, float hi, void* stream) {
    RF_REQUIRE(rows >= 0 && dim > 0, "rf_table_init_uniform: rows >= 0, dim > 0 required");
    RF_REQUIRE(dtype == RF_DTYPE_F32 || dtype == RF_DTYPE_BF16, "rf_table_init_uniform: dtype must be F32 or BF16");
    if (rows == 0) return RF_OK;
    RF_REQUIRE(table != nullptr, "rf_table_init_uniform: null table");
    const int grid = grid_for(rows * (int64_t)dim / 4 + 1, 256, 256 * 32);
    if (dtype == RF_DTYPE_F32)
        hipLaunchKernelGGL(table_init_kernel<float>, dim3(grid), dim3(256), 0, rf_stream(stream), (float*)table, rows,
                           dim, row0, row_stride, seed, lo, hi);
    else
        hipLaunchKernelGGL(table_init_kernel<uint16_t>, dim3(grid), dim3(256), 0, rf_stream(stream), (uint16_t*)table,
                           rows, dim, row0, row_stride, seed, lo, hi);
    return rf_check_launch("table_init_kernel");
}
