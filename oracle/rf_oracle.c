/*
 * rf_oracle.c — CPU restatement of the reference's hash -> gather -> pool path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker and the timed CPU baseline
 * ("port") for the HIP path in recommendflow_amd/csrc. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product never links or calls it.
 *
 * The reference hot path is Keras on TensorFlow (absent from this image); the arithmetic lives in
 * third-party code that is not vendored and whose version is unpinned (TF 2.6-2.11 inferred, SURVEY
 * §8c). Restated here:
 *   - keras.layers.Hashing(num_bins, mask_value, salt=int s)  (called at
 *     backend/layers/preprocess_layers.py:89-90) -> tf.strings.to_hash_bucket_strong with key [s, s]
 *     = SipHash-2-4 (highwayhash SipHash, standard 2-4 rounds, 64-bit LE words), bucket = h mod N;
 *     with mask_value set: masked token -> 0, else 1 + h mod (N - 1).
 *   - EmbeddingBag (preprocess_layers.py:16-76): Embedding gather (:67) + combiner over axis 1
 *     (:44-64) on the [B, Lmax] tensor padded with b"" by parse_example (dataloader.py:32-33,86).
 *   - DoubleHashingEmbedding.call (preprocess_layers.py:94-97): concat([pool(T1), pool(T2)], axis=1).
 * Pins (tests/test_oracle_kats.py): the SipHash-2-4 reference vectors (key 00..0f), CPython's own
 * siphash24 (PYTHONHASHSEED=0 => key (0,0)), and the TF/Keras API docstring examples.
 *
 * Build: oracle/Makefile -> oracle/build/librf_oracle.so (gcc -O3 -fopenmp).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rf_api.h"

#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                                                    \
    do {                                                                                            \
        v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);                                   \
        v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                                                      \
        v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                                                      \
        v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);                                   \
    } while (0)

/* SipHash-2-4 (Aumasson & Bernstein 2012), key (k0, k1) as two little-endian 64-bit words. */
uint64_t orf_siphash24(uint64_t k0, uint64_t k1, const uint8_t* m, int64_t n) {
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
    uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
    uint64_t v3 = 0x7465646279746573ULL ^ k1;
    int64_t nb = n / 8;
    for (int64_t i = 0; i < nb; ++i) {
        uint64_t w = 0;
        for (int j = 0; j < 8; ++j) w |= (uint64_t)m[8 * i + j] << (8 * j);
        v3 ^= w;
        SIPROUND;
        SIPROUND;
        v0 ^= w;
    }
    uint64_t b = ((uint64_t)n) << 56;
    for (int j = 0; j < (int)(n & 7); ++j) b |= (uint64_t)m[8 * nb + j] << (8 * j);
    v3 ^= b;
    SIPROUND;
    SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

/* Keras Hashing._hash_values_to_bins for string input with an int salt (key [salt, salt]). */
int64_t orf_hash_bucket(uint64_t k0, uint64_t k1, const uint8_t* m, int64_t n, int64_t num_bins,
                        int32_t mask_empty) {
    if (mask_empty) {
        if (n == 0) return 0;
        if (num_bins > 1) return 1 + (int64_t)(orf_siphash24(k0, k1, m, n) % (uint64_t)(num_bins - 1));
    }
    return (int64_t)(orf_siphash24(k0, k1, m, n) % (uint64_t)num_bins);
}

void orf_hash_tokens(const uint8_t* tok_bytes, const int32_t* tok_off, int64_t n_tok, uint64_t k0,
                     uint64_t k1, int64_t num_bins, int32_t mask_empty, int64_t* out) {
    for (int64_t t = 0; t < n_tok; ++t)
        out[t] = orf_hash_bucket(k0, k1, tok_bytes + tok_off[t], tok_off[t + 1] - tok_off[t], num_bins,
                                 mask_empty);
}

static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

static inline float bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

/* round-to-nearest-even, NaN kept NaN (quiet) */
static inline uint16_t f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

/* value of the counter-based init, see rf_table_init_uniform in include/rf_api.h */
float orf_table_value(uint64_t seed, int64_t g, int32_t dim, int32_t d, float lo, float hi) {
    uint64_t r = splitmix64(seed ^ ((uint64_t)g * (uint64_t)dim + (uint64_t)d));
    float u = (float)(r >> 40) * (1.0f / 16777216.0f); /* exact: 24-bit integer times 2^-24 */
    return fmaf(hi - lo, u, lo);                        /* one rounding; the HIP kernel uses the same fma */
}

void orf_table_init_uniform(void* table, int32_t dtype, int64_t rows, int32_t dim, int64_t row0,
                            int64_t row_stride, uint64_t seed, float lo, float hi) {
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < rows; ++r) {
        int64_t g = row0 + r * row_stride;
        for (int32_t d = 0; d < dim; ++d) {
            float v = orf_table_value(seed, g, dim, d, lo, hi);
            if (dtype == RF_DTYPE_F32)
                ((float*)table)[r * dim + d] = v;
            else
                ((uint16_t*)table)[r * dim + d] = f32_to_bf16(v);
        }
    }
}

static inline float load_elem(const void* table, int32_t dtype, int64_t idx) {
    return dtype == RF_DTYPE_F32 ? ((const float*)table)[idx] : bf16_to_f32(((const uint16_t*)table)[idx]);
}

static inline void store_elem(void* out, int32_t dtype, int64_t idx, float v) {
    if (dtype == RF_DTYPE_F32)
        ((float*)out)[idx] = v;
    else
        ((uint16_t*)out)[idx] = f32_to_bf16(v);
}

/*
 * Pool one bag of `len` real rows plus (L - len) padding rows (row `pad_row`) with `comb`,
 * positions in order l = 0 .. L-1 (preprocess_layers.py:44-64 over the padded [B, Lmax, D] tensor).
 * rows[l] for l < len are absolute table rows. acc receives D fp32 values (pooled combiners).
 * Returns 0, or RF_EOOB if a row is outside [0, table_rows).
 */
static int pool_bag(const void* table, int32_t dtype, int64_t table_rows, int32_t D, const int64_t* rows,
                    int32_t len, int32_t L, int64_t pad_row, int32_t comb, float* acc) {
    for (int32_t l = 0; l < len; ++l)
        if (rows[l] < 0 || rows[l] >= table_rows) return RF_EOOB;
    if (L > len && (pad_row < 0 || pad_row >= table_rows)) return RF_EOOB;
    for (int32_t d = 0; d < D; ++d) {
        float a;
        switch (comb) {
            case RF_COMB_SUM:
            case RF_COMB_AVG:
                a = 0.0f;
                for (int32_t l = 0; l < L; ++l) a += load_elem(table, dtype, (l < len ? rows[l] : pad_row) * D + d);
                if (comb == RF_COMB_AVG) a = a / (float)L; /* tf.reduce_mean: sum / count (0/0 -> NaN) */
                break;
            case RF_COMB_MAX:
                a = -INFINITY;
                for (int32_t l = 0; l < L; ++l) {
                    float v = load_elem(table, dtype, (l < len ? rows[l] : pad_row) * D + d);
                    a = v > a ? v : a;
                }
                break;
            case RF_COMB_MIN:
                a = INFINITY;
                for (int32_t l = 0; l < L; ++l) {
                    float v = load_elem(table, dtype, (l < len ? rows[l] : pad_row) * D + d);
                    a = v < a ? v : a;
                }
                break;
            case RF_COMB_FIRST:
                a = L == 0 ? 0.0f : load_elem(table, dtype, (len > 0 ? rows[0] : pad_row) * D + d);
                break;
            case RF_COMB_LAST:
                a = L == 0 ? 0.0f : load_elem(table, dtype, (len >= L ? rows[L - 1] : pad_row) * D + d);
                break;
            default:
                return RF_EINVAL;
        }
        acc[d] = a;
    }
    return 0;
}

/* Same contract as rf_fused_hash_embed_fwd (include/rf_api.h), host memory. n_threads<=0: OpenMP default. */
int orf_fused_hash_embed_fwd(const rf_slot_desc* slots, int32_t n_slots, const uint8_t* tok_bytes,
                             const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                             int32_t batch, const void* table, int32_t table_dtype, int64_t table_rows,
                             int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags,
                             int64_t* idx_out, int32_t n_threads) {
    int status = 0;
    int32_t maxL = 1;
    for (int32_t s = 0; s < n_slots; ++s) {
        if (slots[s].dim != dim) return RF_EINVAL;
        if (lmax[s] > maxL) maxL = lmax[s];
    }
    for (int64_t u = 0; u < (int64_t)batch * n_slots; ++u)
        if (bag_off[u + 1] - bag_off[u] > maxL) maxL = bag_off[u + 1] - bag_off[u];
#pragma omp parallel num_threads(n_threads > 0 ? n_threads : omp_get_max_threads())
    {
        int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)maxL);
        float* acc = (float*)malloc(sizeof(float) * (size_t)dim);
#pragma omp for schedule(static)
        for (int32_t b = 0; b < batch; ++b) {
            for (int32_t s = 0; s < n_slots; ++s) {
                const rf_slot_desc* sd = &slots[s];
                int64_t u = (int64_t)b * n_slots + s;
                int32_t t0 = bag_off[u], len = bag_off[u + 1] - t0;
                int32_t L = (flags & RF_FLAG_MASK_PADDING) ? len : (lmax[s] > len ? lmax[s] : len);
                for (int k = 0; k < 2; ++k) {
                    for (int32_t l = 0; l < len; ++l) {
                        int32_t t = t0 + l;
                        int64_t bin = orf_hash_bucket(sd->salt[k], sd->salt[k], tok_bytes + tok_off[t],
                                                      tok_off[t + 1] - tok_off[t], sd->num_bins, sd->mask_empty);
                        if (idx_out && (flags & RF_FLAG_EMIT_IDX)) idx_out[2 * (int64_t)t + k] = bin;
                        rows[l] = sd->row_base[k] + bin;
                    }
                    /* padded position: b"" -> Hashing(mask_value="") bin 0; without a mask, hash of b"" */
                    int64_t pad_bin = sd->mask_empty ? 0 : orf_hash_bucket(sd->salt[k], sd->salt[k], (const uint8_t*)"", 0,
                                                                           sd->num_bins, 0);
                    int64_t pad_row = sd->row_base[k] + pad_bin;
                    char* ob = (char*)out;
                    if (sd->combiner == RF_COMB_NULL) {
                        for (int32_t l = 0; l < L; ++l) {
                            int64_t r = l < len ? rows[l] : pad_row;
                            if (r < 0 || r >= table_rows) {
#pragma omp atomic write
                                status = RF_EOOB;
                                continue;
                            }
                            for (int32_t d = 0; d < dim; ++d)
                                store_elem(ob, out_dtype, (int64_t)b * out_stride + sd->out_off + ((int64_t)k * L + l) * dim + d,
                                           load_elem(table, table_dtype, r * dim + d));
                        }
                        continue;
                    }
                    int rc = 0;
                    if (L == 0 && (flags & RF_FLAG_MASK_PADDING))
                        memset(acc, 0, sizeof(float) * (size_t)dim); /* masked empty bag -> zeros */
                    else
                        rc = pool_bag(table, table_dtype, table_rows, dim, rows, len, L, pad_row, sd->combiner, acc);
                    if (rc) {
#pragma omp atomic write
                        status = rc;
                        continue;
                    }
                    for (int32_t d = 0; d < dim; ++d)
                        store_elem(ob, out_dtype, (int64_t)b * out_stride + sd->out_off + (int64_t)k * dim + d, acc[d]);
                }
            }
        }
        free(rows);
        free(acc);
    }
    return status;
}

/* Same contract as rf_embedding_bag_fwd, host memory. */
int orf_embedding_bag_fwd(const int64_t* ids, int32_t batch, int32_t len, int64_t row_base, const void* table,
                          int32_t table_dtype, int64_t table_rows, int32_t dim, int32_t combiner, void* out,
                          int32_t out_dtype, int64_t out_stride, int64_t out_off) {
    int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)(len > 0 ? len : 1));
    float* acc = (float*)malloc(sizeof(float) * (size_t)dim);
    int status = 0;
    for (int32_t b = 0; b < batch && !status; ++b) {
        for (int32_t l = 0; l < len; ++l) rows[l] = row_base + ids[(int64_t)b * len + l];
        if (combiner == RF_COMB_NULL) {
            for (int32_t l = 0; l < len; ++l) {
                if (rows[l] < 0 || rows[l] >= table_rows) { status = RF_EOOB; break; }
                for (int32_t d = 0; d < dim; ++d)
                    store_elem(out, out_dtype, (int64_t)b * out_stride + out_off + (int64_t)l * dim + d,
                               load_elem(table, table_dtype, rows[l] * dim + d));
            }
            continue;
        }
        status = pool_bag(table, table_dtype, table_rows, dim, rows, len, len, 0, combiner, acc);
        if (status) break;
        for (int32_t d = 0; d < dim; ++d)
            store_elem(out, out_dtype, (int64_t)b * out_stride + out_off + d, acc[d]);
    }
    free(rows);
    free(acc);
    return status;
}

/* Owner routing of the row-sharded table: owner = g mod P, local = g div P, stable. */
void orf_bucketize_owner(const int64_t* rows, int64_t n, int32_t nranks, int32_t* counts, int32_t* perm,
                         int32_t* inv_perm, int64_t* local_rows) {
    int64_t* start = (int64_t*)calloc((size_t)nranks + 1, sizeof(int64_t));
    for (int32_t p = 0; p < nranks; ++p) counts[p] = 0;
    for (int64_t i = 0; i < n; ++i) counts[rows[i] % nranks]++;
    for (int32_t p = 0; p < nranks; ++p) start[p + 1] = start[p] + counts[p];
    for (int64_t i = 0; i < n; ++i) {
        int32_t p = (int32_t)(rows[i] % nranks);
        int64_t pos = start[p]++;
        perm[pos] = (int32_t)i;
        if (inv_perm) inv_perm[i] = (int32_t)pos;
        local_rows[pos] = rows[i] / nranks;
    }
    free(start);
}

/* rf_hash_rows restated: rows_out[2t + k] = row_base[k] + bucket_k(token t). */
void orf_hash_rows(const rf_slot_desc* slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                   const int32_t* bag_off, int32_t batch, int64_t* rows_out) {
    for (int64_t u = 0; u < (int64_t)batch * n_slots; ++u) {
        const rf_slot_desc* sd = &slots[u % n_slots];
        for (int32_t t = bag_off[u]; t < bag_off[u + 1]; ++t)
            for (int k = 0; k < 2; ++k)
                rows_out[2 * (int64_t)t + k] = sd->row_base[k] + orf_hash_bucket(sd->salt[k], sd->salt[k], tok_bytes + tok_off[t],
                                                                                tok_off[t + 1] - tok_off[t], sd->num_bins,
                                                                                sd->mask_empty);
    }
}

/* rf_pool_rows_fwd restated: the pooling of orf_fused_hash_embed_fwd over pre-gathered rows (token t,
   table k -> row 2t + k; pad row of slot s, table k -> row 2*n_tok + 2s + k). */
int orf_pool_rows_fwd(const rf_slot_desc* slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                      int32_t batch, int64_t n_tok, const void* gathered, const int32_t* row_map, int32_t dtype,
                      int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags) {
    int32_t maxL = 1;
    for (int32_t s = 0; s < n_slots; ++s) if (lmax[s] > maxL) maxL = lmax[s];
    for (int64_t u = 0; u < (int64_t)batch * n_slots; ++u)
        if (bag_off[u + 1] - bag_off[u] > maxL) maxL = bag_off[u + 1] - bag_off[u];
    int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)maxL);
    float* acc = (float*)malloc(sizeof(float) * (size_t)dim);
    const int64_t nrows = 2 * n_tok + 2 * (int64_t)n_slots;
    int status = 0;
    for (int32_t b = 0; b < batch && !status; ++b)
        for (int32_t s = 0; s < n_slots && !status; ++s) {
            const rf_slot_desc* sd = &slots[s];
            const int64_t u = (int64_t)b * n_slots + s;
            const int32_t t0 = bag_off[u], len = bag_off[u + 1] - t0;
            const int32_t L = (flags & RF_FLAG_MASK_PADDING) ? len : (lmax[s] > len ? lmax[s] : len);
            for (int k = 0; k < 2; ++k) {
                for (int32_t l = 0; l < len; ++l) {
                    rows[l] = 2 * (int64_t)(t0 + l) + k;
                    if (row_map) rows[l] = row_map[rows[l]];
                }
                int64_t pad = 2 * n_tok + 2 * (int64_t)s + k;
                if (row_map) pad = row_map[pad];
                char* ob = (char*)out;
                if (sd->combiner == RF_COMB_NULL) {
                    for (int32_t l = 0; l < L; ++l)
                        for (int32_t d = 0; d < dim; ++d)
                            store_elem(ob, out_dtype, (int64_t)b * out_stride + sd->out_off + ((int64_t)k * L + l) * dim + d,
                                       (l >= len && (flags & RF_FLAG_MASK_PADDING)) ? 0.0f
                                                                                   : load_elem(gathered, dtype, (l < len ? rows[l] : pad) * dim + d));
                    continue;
                }
                if (L == 0 && (flags & RF_FLAG_MASK_PADDING))
                    memset(acc, 0, sizeof(float) * (size_t)dim);
                else
                    status = pool_bag(gathered, dtype, nrows, dim, rows, len, L, pad, sd->combiner, acc);
                for (int32_t d = 0; d < dim; ++d)
                    store_elem(ob, out_dtype, (int64_t)b * out_stride + sd->out_off + (int64_t)k * dim + d, acc[d]);
            }
        }
    free(rows);
    free(acc);
    return status;
}

/* ============================================================================================
 * Training backward, restated sequentially:
 *   the Embedding gradient of each (slot, table) is an IndexedSlices over every gathered position of
 *   the padded [B, Lmax] ids (preprocess_layers.py:67 + the combiner gradient of :44-64:
 *   reduce_sum -> g; reduce_mean -> g / L; reduce_max/min -> (x == y) / num_selected * g
 *   (tf _MinOrMaxGrad); t[0] / t[-1] -> g at that position, 0 elsewhere);
 *   Keras _deduplicate_indexed_slices = unique + unsorted_segment_sum, which on CPU adds the values
 *   of one row into a zero-initialised accumulator in (b, l) order.
 * Output: distinct rows ascending, their summed gradients. Returns n_uniq, or -1 on a bad row.
 * ============================================================================================ */
static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* Row read at (slot s, table k, bag position l) of an example whose bag starts at token t0 and holds len
 * tokens: the hashed row (row_map == NULL), or — the sharded requester — the slot in the receive buffer
 * of logical row 2t + k (real token) / 2 n_tok + 2 s + k (padding), as rf_pool_rows_fwd reads it. */
static int64_t bwd_row(const rf_slot_desc* sd, int32_t s, int k, int32_t l, int32_t t0, int32_t len,
                       const uint8_t* tok_bytes, const int32_t* tok_off, const int32_t* row_map, int64_t n_tok) {
    if (row_map) return l < len ? row_map[2 * (int64_t)(t0 + l) + k] : row_map[2 * n_tok + 2 * (int64_t)s + k];
    if (l < len) {
        const int32_t t = t0 + l;
        return sd->row_base[k] + orf_hash_bucket(sd->salt[k], sd->salt[k], tok_bytes + tok_off[t],
                                                 tok_off[t + 1] - tok_off[t], sd->num_bins, sd->mask_empty);
    }
    return sd->row_base[k] + (sd->mask_empty ? 0 : orf_hash_bucket(sd->salt[k], sd->salt[k], (const uint8_t*)"", 0,
                                                                     sd->num_bins, 0));
}

static int64_t embed_bwd(const rf_slot_desc* slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                         const int32_t* bag_off, const int32_t* lmax, int32_t batch, const int32_t* row_map,
                         int64_t n_tok, const float* table, int64_t table_rows, int32_t dim, const float* out,
                         const float* dout, int64_t out_stride, int32_t flags, int64_t* uniq_rows, float* uniq_grad) {
    const int masked = (flags & RF_FLAG_MASK_PADDING) != 0;
    int64_t per = 0;
    int64_t* pos_off = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_slots + 1));
    for (int32_t s = 0; s < n_slots; ++s) { pos_off[s] = per; per += 2 * (int64_t)lmax[s]; }
    pos_off[n_slots] = per;
    const int64_t n = per * batch;
    uint64_t* keys = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(n > 0 ? n : 1));
    int64_t m = 0;
    int status = 0;
    /* positions p in (b, s, k, l) order; key = row << 32 | p */
    for (int32_t b = 0; b < batch; ++b)
        for (int32_t s = 0; s < n_slots; ++s) {
            const rf_slot_desc* sd = &slots[s];
            const int64_t u = (int64_t)b * n_slots + s;
            const int32_t t0 = bag_off[u], len = bag_off[u + 1] - t0;
            for (int k = 0; k < 2; ++k)
                for (int32_t l = 0; l < lmax[s]; ++l) {
                    const int64_t p = (int64_t)b * per + pos_off[s] + (int64_t)k * lmax[s] + l;
                    if (l >= len && masked) continue;
                    const int64_t row = bwd_row(sd, s, k, l, t0, len, tok_bytes, tok_off, row_map, n_tok);
                    if (row < 0 || row >= table_rows) { status = -1; continue; }
                    keys[m++] = ((uint64_t)row << 32) | (uint64_t)p;
                }
        }
    qsort(keys, (size_t)m, sizeof(uint64_t), cmp_u64);
    int64_t nu = 0;
    for (int64_t i = 0; i < m;) {
        const uint64_t row = keys[i] >> 32;
        float* acc = uniq_grad + nu * dim;
        for (int32_t d = 0; d < dim; ++d) acc[d] = 0.0f;
        const float* tr = table + (int64_t)row * dim;
        for (; i < m && (keys[i] >> 32) == row; ++i) {
            const int64_t p = (int64_t)(keys[i] & 0xffffffffu);
            const int32_t b = (int32_t)(p / per);
            const int64_t r = p - (int64_t)b * per;
            int32_t s = 0;
            while (s + 1 < n_slots && pos_off[s + 1] <= r) ++s;
            const int32_t k = (int32_t)((r - pos_off[s]) / lmax[s]);
            const int32_t l = (int32_t)(r - pos_off[s] - (int64_t)k * lmax[s]);
            const rf_slot_desc* sd = &slots[s];
            const int64_t u = (int64_t)b * n_slots + s;
            const int32_t t0 = bag_off[u], len = bag_off[u + 1] - t0;
            const int32_t L = masked ? len : (lmax[s] > len ? lmax[s] : len);
            const int64_t col = (int64_t)b * out_stride + sd->out_off + (int64_t)k * dim;
            for (int32_t d = 0; d < dim; ++d) {
                const float g = dout[col + d];
                float v = 0.0f;
                switch (sd->combiner) {
                    case RF_COMB_SUM: v = g; break;
                    case RF_COMB_AVG: v = g / (float)L; break;
                    case RF_COMB_MAX:
                    case RF_COMB_MIN: {
                        /* num_selected over the bag's L positions (pads included unless masked) */
                        int32_t c = 0;
                        for (int32_t l2 = 0; l2 < L; ++l2) {
                            const int64_t r2 = bwd_row(sd, s, k, l2, t0, len, tok_bytes, tok_off, row_map, n_tok);
                            if (r2 >= 0 && r2 < table_rows && table[r2 * dim + d] == out[col + d]) ++c;
                        }
                        v = ((tr[d] == out[col + d] ? 1.0f : 0.0f) / (float)c) * g;
                        break;
                    }
                    case RF_COMB_FIRST: v = l == 0 ? g : 0.0f; break;
                    case RF_COMB_LAST: v = l == L - 1 ? g : 0.0f; break;
                    default: break;
                }
                acc[d] += v;
            }
        }
        uniq_rows[nu++] = (int64_t)row;
    }
    free(keys);
    free(pos_off);
    return status ? -1 : nu;
}

int64_t orf_fused_hash_embed_bwd(const rf_slot_desc* slots, int32_t n_slots, const uint8_t* tok_bytes,
                                 const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                                 const float* table, int64_t table_rows, int32_t dim, const float* out,
                                 const float* dout, int64_t out_stride, int32_t flags, int64_t* uniq_rows,
                                 float* uniq_grad) {
    return embed_bwd(slots, n_slots, tok_bytes, tok_off, bag_off, lmax, batch, NULL, 0, table, table_rows, dim, out,
                     dout, out_stride, flags, uniq_rows, uniq_grad);
}

/* rf_pool_rows_bwd: the same gradient with rows read through row_map from gathered [n_rows][dim]
 * (uniq_rows index the gathered rows). */
int64_t orf_pool_rows_bwd(const rf_slot_desc* slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                          int32_t batch, int64_t n_tok, const int32_t* row_map, const float* gathered, int64_t n_rows,
                          int32_t dim, const float* out, const float* dout, int64_t out_stride, int32_t flags,
                          int64_t* uniq_rows, float* uniq_grad) {
    return embed_bwd(slots, n_slots, NULL, NULL, bag_off, lmax, batch, row_map, n_tok, gathered, n_rows, dim, out,
                     dout, out_stride, flags, uniq_rows, uniq_grad);
}

/* Keras Adam (OptimizerV2 Adam._resource_apply_sparse after dedup), fp32, one step:
 *   m = m * b1 (every row); m[r] = m[r] + g_r * (1 - b1) (touched rows); likewise v with g_r * g_r;
 *   var = var - lr * m / (sqrt(v) + eps) (every row); lr = lr_t * sqrt(1 - b2^t) / (1 - b1^t) (host).
 * lazy != 0: touched rows only (TF-Addons LazyAdam). uniq_rows must be distinct. */
void orf_adam_apply(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                    const float* uniq_grad, int64_t n_uniq, float lr, float b1, float b2, float eps, int32_t lazy) {
    const float omb1 = 1.0f - b1, omb2 = 1.0f - b2;
    int32_t* map = NULL;
    if (!lazy) {
        map = (int32_t*)malloc(sizeof(int32_t) * (size_t)table_rows);
        for (int64_t r = 0; r < table_rows; ++r) map[r] = -1;
        for (int64_t u = 0; u < n_uniq; ++u) map[uniq_rows[u]] = (int32_t)u;
    }
    const int64_t nrows = lazy ? n_uniq : table_rows;
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t row = lazy ? uniq_rows[i] : i;
        const int64_t u = lazy ? i : map[i];
        for (int32_t d = 0; d < dim; ++d) {
            const int64_t e = row * dim + d;
            float mt = m[e] * b1, vt = v[e] * b2;
            if (u >= 0) {
                const float g = uniq_grad[u * dim + d];
                mt = mt + g * omb1;
                vt = vt + (g * g) * omb2;
            }
            m[e] = mt;
            v[e] = vt;
            table[e] = table[e] - (lr * mt) / (sqrtf(vt) + eps);
        }
    }
    free(map);
}
