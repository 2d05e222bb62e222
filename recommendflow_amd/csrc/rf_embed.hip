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

#include "rf_common.h"

namespace {

constexpr int kWaves = 4;    // waves per workgroup
constexpr int kCap = 256;    // tokens per wave item kept in the LDS index bucket
constexpr int kUnits = 64;   // (example, slot) units per wave item

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
#pragma unroll
        for (int i = 0; i < EPV; i += 4)
            *reinterpret_cast<float4*>(dst + i) = make_float4(f[i], f[i + 1], f[i + 2], f[i + 3]);
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

__device__ __forceinline__ float comb_init(int comb) {
    return comb == RF_COMB_MAX ? -INFINITY : comb == RF_COMB_MIN ? INFINITY : 0.0f;
}

__device__ __forceinline__ float comb_step(int comb, float a, float v) {
    // sum/avg: one fp32 add per position in order (no fma, no reassociation)
    return comb == RF_COMB_MAX ? (v > a ? v : a) : comb == RF_COMB_MIN ? (v < a ? v : a) : __fadd_rn(a, v);
}

// ---------------------------------------------------------------------------------------------
// fused multi-slot hash -> gather -> pool
// ---------------------------------------------------------------------------------------------
template <int LPR, int CPL, typename TT, typename OT>
__global__ __launch_bounds__(kWaves * 64) void fused_hash_embed_kernel(
    const rf_slot_desc* __restrict__ slots, int n_slots, const uint8_t* __restrict__ tok_bytes,
    const int32_t* __restrict__ tok_off, const int32_t* __restrict__ bag_off, const int32_t* __restrict__ lmax,
    int64_t n_units, const TT* __restrict__ table, int64_t table_rows, int dim, OT* __restrict__ out,
    int64_t out_stride, int flags, int64_t* __restrict__ idx_out) {
    constexpr int EPV = Elem<TT>::EPV;
    constexpr int TEAMS = 64 / LPR;
    constexpr int KPT = kUnits / TEAMS;  // units per team per item
    __shared__ int32_t s_bin[kWaves][2][kCap];
    __shared__ int32_t s_bag[kWaves][kUnits + 1];

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int team = lane / LPR, tl = lane % LPR;
    const int nchunks = dim / EPV;
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const bool emit = (flags & RF_FLAG_EMIT_IDX) != 0 && idx_out != nullptr;
    const int64_t n_items = (n_units + kUnits - 1) / kUnits;

    for (int64_t item = (int64_t)blockIdx.x * kWaves + wave; item < n_items; item += (int64_t)gridDim.x * kWaves) {
        const int64_t u0 = item * kUnits;
        const int nu = (int)min((int64_t)kUnits, n_units - u0);
        for (int i = lane; i <= nu; i += 64) s_bag[wave][i] = bag_off[u0 + i];
        wave_lds_sync();
        const int t0 = s_bag[wave][0];
        const int ntok = s_bag[wave][nu] - t0;
        const int nh = min(ntok, kCap);

        // ---- phase 1: lane-per-token double hashing into the LDS bucket ----
        for (int i = lane; i < nh; i += 64) {
            const int t = t0 + i;
            int lo = 0, hi = nu - 1;  // unit of token t: last j with s_bag[j] <= t
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_bag[wave][mid] <= t) lo = mid; else hi = mid - 1;
            }
            const int s = (int)((u0 + lo) % n_slots);
            const rf_slot_desc* sd = slots + s;
            const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
            uint64_t h0, h1;
            siphash24x2_dev(sd->salt[0], sd->salt[1], tok_bytes + b0, n, h0, h1);
            const int64_t i0 = bucket_from_hash(h0, n, sd->num_bins, sd->mask_empty);
            const int64_t i1 = bucket_from_hash(h1, n, sd->num_bins, sd->mask_empty);
            s_bin[wave][0][i] = (int32_t)i0;
            s_bin[wave][1][i] = (int32_t)i1;
            if (emit) {
                idx_out[2 * (int64_t)t] = i0;
                idx_out[2 * (int64_t)t + 1] = i1;
            }
        }
        wave_lds_sync();

        // ---- phase 2: team-per-unit gather + pool ----
        for (int kk = 0; kk < KPT; ++kk) {
            const int j = team * KPT + kk;
            if (j >= nu) break;
            const int64_t u = u0 + j;
            const int s = (int)(u % n_slots);
            const int64_t b = u / n_slots;
            const rf_slot_desc* sd = slots + s;
            const int comb = sd->combiner;
            const int64_t rb0 = sd->row_base[0], rb1 = sd->row_base[1];
            const int64_t nbins = sd->num_bins;
            const int mask_empty = sd->mask_empty;
            const int tb = s_bag[wave][j] - t0, len = s_bag[wave][j + 1] - s_bag[wave][j];
            const int lm = lmax[s];
            const int L = mask_pad ? len : max(lm, len);
            OT* orow = out + b * out_stride + sd->out_off;
            // poison rather than fault if the descriptor does not fit the table
            const bool bad = rb0 < 0 || rb1 < 0 || rb0 + nbins > table_rows || rb1 + nbins > table_rows;
            const int64_t trows = bad ? -1 : table_rows;

            // token position -> fused-table row of table k
            auto row_of = [&](int k, int l) -> int64_t {
                const int i = tb + l;
                int64_t bin;
                if (i < kCap) {
                    bin = s_bin[wave][k][i];
                } else {  // bucket overflow (very long bags): hash inline
                    const int t = t0 + i;
                    const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
                    uint64_t h0, h1;
                    siphash24x2_dev(sd->salt[0], sd->salt[1], tok_bytes + b0, n, h0, h1);
                    bin = bucket_from_hash(k ? h1 : h0, n, nbins, mask_empty);
                    if (emit && tl == 0) idx_out[2 * (int64_t)t + k] = bin;
                }
                return (k ? rb1 : rb0) + bin;
            };
            // padded position (b"" after parse_example): bin 0 with mask_value="", else hash of b""
            auto pad_row = [&](int k) -> int64_t {
                if (mask_empty) return k ? rb1 : rb0;
                const uint64_t h = siphash24_dev(sd->salt[k], sd->salt[k], tok_bytes, 0);
                return (k ? rb1 : rb0) + (int64_t)(h % (uint64_t)nbins);
            };

            if (comb == RF_COMB_NULL) {
                const int Lo = lm;  // output positions are fixed by the batch max
                for (int l = 0; l < Lo; ++l) {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const bool real = l < len;
                        const int64_t r = real ? row_of(k, l) : pad_row(k);
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            const int c = tl + cc * LPR;
                            if (c >= nchunks) continue;
                            float f[EPV];
                            if (!real && mask_pad) {
#pragma unroll
                                for (int e = 0; e < EPV; ++e) f[e] = 0.0f;
                            } else {
                                unpack16<TT>(load_chunk(table, r, trows, dim, c), f);
                            }
                            store_chunk<OT, EPV>(orow + ((int64_t)k * Lo + l) * dim + c * EPV, f);
                        }
                    }
                }
                continue;
            }

            float acc[2][CPL][EPV];
            if (comb == RF_COMB_FIRST || comb == RF_COMB_LAST) {
                const int p = comb == RF_COMB_FIRST ? 0 : L - 1;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int64_t r = L == 0 ? -1 : (p < len ? row_of(k, p) : pad_row(k));
#pragma unroll
                    for (int cc = 0; cc < CPL; ++cc) {
                        const int c = tl + cc * LPR;
                        if (L == 0 || c >= nchunks) {
#pragma unroll
                            for (int e = 0; e < EPV; ++e) acc[k][cc][e] = 0.0f;
                        } else {
                            unpack16<TT>(load_chunk(table, r, trows, dim, c), acc[k][cc]);
                        }
                    }
                }
            } else {
                const float init = comb_init(comb);
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                        for (int e = 0; e < EPV; ++e) acc[k][cc][e] = init;
                // real positions, 4 in flight per table
                for (int l = 0; l < len; l += 4) {
                    uint4 v[4][2][CPL];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (l + q < len) {
#pragma unroll
                            for (int k = 0; k < 2; ++k) {
                                const int64_t r = row_of(k, l + q);
#pragma unroll
                                for (int cc = 0; cc < CPL; ++cc) {
                                    const int c = tl + cc * LPR;
                                    v[q][k][cc] = c < nchunks ? load_chunk(table, r, trows, dim, c) : make_uint4(0, 0, 0, 0);
                                }
                            }
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (l + q < len) {
#pragma unroll
                            for (int k = 0; k < 2; ++k)
#pragma unroll
                                for (int cc = 0; cc < CPL; ++cc) {
                                    float f[EPV];
                                    unpack16<TT>(v[q][k][cc], f);
#pragma unroll
                                    for (int e = 0; e < EPV; ++e) acc[k][cc][e] = comb_step(comb, acc[k][cc][e], f[e]);
                                }
                        }
                    }
                }
                // padding positions len..L-1 (reference parity): row pad, added one position at a time
                const int npad = L - len;
                if (npad > 0) {
#pragma unroll
                    for (int k = 0; k < 2; ++k) {
                        const int64_t r = pad_row(k);
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc) {
                            const int c = tl + cc * LPR;
                            if (c >= nchunks) continue;
                            float f[EPV];
                            unpack16<TT>(load_chunk(table, r, trows, dim, c), f);
                            if (comb == RF_COMB_MAX || comb == RF_COMB_MIN) {
#pragma unroll
                                for (int e = 0; e < EPV; ++e) acc[k][cc][e] = comb_step(comb, acc[k][cc][e], f[e]);
                            } else {
                                for (int p = 0; p < npad; ++p)
#pragma unroll
                                    for (int e = 0; e < EPV; ++e) acc[k][cc][e] = __fadd_rn(acc[k][cc][e], f[e]);
                            }
                        }
                    }
                }
                if (comb == RF_COMB_AVG) {
                    const float fl = (float)L;
#pragma unroll
                    for (int k = 0; k < 2; ++k)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                            for (int e = 0; e < EPV; ++e) acc[k][cc][e] = __fdiv_rn(acc[k][cc][e], fl);
                }
                if (mask_pad && L == 0) {  // masked empty bag -> zeros
#pragma unroll
                    for (int k = 0; k < 2; ++k)
#pragma unroll
                        for (int cc = 0; cc < CPL; ++cc)
#pragma unroll
                            for (int e = 0; e < EPV; ++e) acc[k][cc][e] = 0.0f;
                }
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int cc = 0; cc < CPL; ++cc) {
                    const int c = tl + cc * LPR;
                    if (c < nchunks) store_chunk<OT, EPV>(orow + (int64_t)k * dim + c * EPV, acc[k][cc]);
                }
        }
        wave_lds_sync();  // s_bag / s_bin are rewritten by the next item
    }
}

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

extern "C" int rf_fused_hash_embed_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
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
    RF_REQUIRE((flags & ~(RF_FLAG_MASK_PADDING | RF_FLAG_EMIT_IDX)) == 0, "rf_fused_hash_embed_fwd: unknown flags");
    const int64_t n_units = (int64_t)batch * n_slots;
    if (n_units == 0) return RF_OK;
    RF_REQUIRE(d_slots && tok_bytes && tok_off && bag_off && lmax && table && out, "rf_fused_hash_embed_fwd: null pointer");
    const int64_t items = (n_units + kUnits - 1) / kUnits;
    const int grid = grid_for(items, kWaves, 256 * 8 * 2);
    hipStream_t st = rf_stream(stream);
    return dispatch_lpr(dim / epv, [&](auto lpr, auto cpl) -> int {
        constexpr int LPR = decltype(lpr)::value, CPL = decltype(cpl)::value;
        if (table_dtype == RF_DTYPE_F32) {
            if (out_dtype == RF_DTYPE_F32)
                hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, float, float>), dim3(grid), dim3(kWaves * 64), 0, st,
                                   d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const float*)table,
                                   table_rows, dim, (float*)out, out_stride, flags, idx_out);
            else
                hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, float, uint16_t>), dim3(grid), dim3(kWaves * 64), 0, st,
                                   d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const float*)table,
                                   table_rows, dim, (uint16_t*)out, out_stride, flags, idx_out);
        } else {
            if (out_dtype == RF_DTYPE_F32)
                hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, uint16_t, float>), dim3(grid), dim3(kWaves * 64), 0, st,
                                   d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const uint16_t*)table,
                                   table_rows, dim, (float*)out, out_stride, flags, idx_out);
            else
                hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, uint16_t, uint16_t>), dim3(grid), dim3(kWaves * 64), 0, st,
                                   d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const uint16_t*)table,
                                   table_rows, dim, (uint16_t*)out, out_stride, flags, idx_out);
        }
        return rf_check_launch("fused_hash_embed_kernel");
    });
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
