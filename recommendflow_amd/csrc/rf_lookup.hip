// rf_lookup.hip — GPU index producers for the Lookup / Discrete embeddings.
//
// Reference (backend/layers/preprocess_layers.py):
//   LookupEmbedding   (:135-169)  StringLookup / IntegerLookup(vocabulary, output_mode="int") -> EmbeddingBag
//   DiscreteEmbedding (:172-200)  Discretization(bin_boundaries)                           -> EmbeddingBag
// Keras (TF 2.6+ defaults, num_oov_indices = 1, mask_token = None): vocab[i] -> i + 1, anything else -> 0;
// Discretization = tf.raw_ops.Bucketize: index = #{boundaries <= x} (upper_bound; NaN -> n_boundaries).
// Both produce the padded [B, Lmax] id tensor parse_example + the layer would (padding = the feature's
// default, "" / 0 / 0.0, mapped through the same rule), which rf_embedding_bag_fwd then pools.
//
// The vocabulary is an open-addressing table built on the host (rf_vocab_build, linear probing,
// capacity = pow2 >= 2 * |vocab|); string keys are a SipHash-2-4 of the bytes and every hit is verified
// byte for byte against the vocabulary, integer keys are the value itself.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../include/rf_api.h"
#include "rf_common.h"

namespace {

constexpr uint64_t kVocabK0 = 0x5246766f63616231ull, kVocabK1 = 0x6c6f6f6b75702121ull;  // fixed table key

uint64_t siphash24_host(uint64_t k0, uint64_t k1, const uint8_t* m, int64_t n) {
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0, v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0, v3 = 0x7465646279746573ULL ^ k1;
    auto rotl = [](uint64_t x, int b) { return (x << b) | (x >> (64 - b)); };
    auto round = [&]() {
        v0 += v1; v1 = rotl(v1, 13); v1 ^= v0; v0 = rotl(v0, 32);
        v2 += v3; v3 = rotl(v3, 16); v3 ^= v2;
        v0 += v3; v3 = rotl(v3, 21); v3 ^= v0;
        v2 += v1; v1 = rotl(v1, 17); v1 ^= v2; v2 = rotl(v2, 32);
    };
    const int64_t nb = n / 8;
    for (int64_t i = 0; i < nb; ++i) {
        uint64_t w;
        std::memcpy(&w, m + 8 * i, 8);
        v3 ^= w; round(); round(); v0 ^= w;
    }
    uint64_t b = (uint64_t)n << 56;
    for (int j = 0; j < (int)(n & 7); ++j) b |= (uint64_t)m[8 * nb + j] << (8 * j);
    v3 ^= b; round(); round(); v0 ^= b;
    v2 ^= 0xff;
    round(); round(); round(); round();
    return v0 ^ v1 ^ v2 ^ v3;
}

uint64_t mix64_host(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// string token -> id (vocab hit verified byte for byte)
__device__ int64_t lookup_bytes(const rf_vocab_entry* __restrict__ tab, int64_t cap, const uint8_t* __restrict__ vb,
                                const int32_t* __restrict__ voff, const uint8_t* p, int n) {
    const uint64_t key = siphash24_dev(kVocabK0, kVocabK1, p, n);
    for (int64_t h = (int64_t)(key & (uint64_t)(cap - 1)), probe = 0; probe < cap; ++probe, h = (h + 1) & (cap - 1)) {
        const rf_vocab_entry e = tab[h];
        if (e.id < 0) return 0;  // empty slot: OOV
        if (e.key != key) continue;
        const int32_t b0 = voff[e.ref], bn = voff[e.ref + 1] - b0;
        if (bn != n) continue;
        bool same = true;
        for (int i = 0; i < n && same; ++i) same = vb[b0 + i] == p[i];
        if (same) return e.id;
    }
    return 0;
}

__device__ int64_t lookup_int(const rf_vocab_entry* __restrict__ tab, int64_t cap, int64_t v) {
    const uint64_t key = (uint64_t)v;
    for (int64_t h = (int64_t)(splitmix64_dev(key) & (uint64_t)(cap - 1)), probe = 0; probe < cap;
         ++probe, h = (h + 1) & (cap - 1)) {
        const rf_vocab_entry e = tab[h];
        if (e.id < 0) return 0;
        if (e.key == key) return e.id;
    }
    return 0;
}

// one thread per (example, position < Lmax)
__global__ __launch_bounds__(256) void lookup_kernel(int kind, const rf_vocab_entry* __restrict__ tab, int64_t cap,
                                                     const uint8_t* __restrict__ vb, const int32_t* __restrict__ voff,
                                                     const void* __restrict__ vals, const int32_t* __restrict__ tok_off,
                                                     const int32_t* __restrict__ bag_off, int S, int s, int batch,
                                                     int lmax, int64_t* __restrict__ ids) {
    const int64_t n = (int64_t)batch * lmax;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / lmax), l = (int)(i - (int64_t)b * lmax);
        const int64_t u = (int64_t)b * S + s;
        const int t0 = bag_off[u], len = bag_off[u + 1] - t0;
        int64_t id;
        if (kind == RF_VOCAB_BYTES) {
            const uint8_t* tb = static_cast<const uint8_t*>(vals);
            if (l < len) {
                const int b0 = tok_off[t0 + l];
                id = lookup_bytes(tab, cap, vb, voff, tb + b0, tok_off[t0 + l + 1] - b0);
            } else {
                id = lookup_bytes(tab, cap, vb, voff, tb, 0);  // padding b""
            }
        } else {
            const int64_t* iv = static_cast<const int64_t*>(vals);
            id = lookup_int(tab, cap, l < len ? iv[t0 + l] : 0);  // padding 0
        }
        ids[i] = id;
    }
}

__device__ __forceinline__ int64_t bucketize(const float* __restrict__ bnd, int nb, float x) {
    int lo = 0, hi = nb;  // first boundary with x < bnd[k] (std::upper_bound)
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (x < bnd[mid]) hi = mid; else lo = mid + 1;
    }
    return lo;
}

__global__ __launch_bounds__(256) void bucketize_kernel(const float* __restrict__ vals, const int32_t* __restrict__ bag_off,
                                                        int S, int s, int batch, int lmax, const float* __restrict__ bnd,
                                                        int nb, float pad_value, int64_t* __restrict__ ids) {
    const int64_t n = (int64_t)batch * lmax;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / lmax), l = (int)(i - (int64_t)b * lmax);
        const int64_t u = (int64_t)b * S + s;
        const int t0 = bag_off[u], len = bag_off[u + 1] - t0;
        ids[i] = bucketize(bnd, nb, l < len ? vals[t0 + l] : pad_value);
    }
}

int grid_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 64)); }

}  // namespace

extern "C" int64_t rf_vocab_capacity(int64_t n_vocab) {
    if (n_vocab < 0) return -1;
    int64_t cap = 16;
    while (cap < 2 * n_vocab) cap <<= 1;
    return cap;
}

extern "C" int rf_vocab_build(int32_t kind, const void* values, const int32_t* off, int64_t n_vocab,
                              rf_vocab_entry* table, int64_t cap) {
    RF_REQUIRE(kind == RF_VOCAB_BYTES || kind == RF_VOCAB_INT64, "rf_vocab_build: kind must be RF_VOCAB_BYTES or RF_VOCAB_INT64");
    RF_REQUIRE(n_vocab >= 0 && n_vocab < (1 << 30), "rf_vocab_build: bad vocabulary size");
    RF_REQUIRE(cap >= 2 * n_vocab && cap >= 1 && (cap & (cap - 1)) == 0, "rf_vocab_build: cap must be a power of two >= 2 * n_vocab");
    RF_REQUIRE(table && (n_vocab == 0 || values) && (kind != RF_VOCAB_BYTES || n_vocab == 0 || off), "rf_vocab_build: null pointer");
    for (int64_t h = 0; h < cap; ++h) table[h] = rf_vocab_entry{0, -1, 0};
    const uint8_t* vb = static_cast<const uint8_t*>(values);
    const int64_t* iv = static_cast<const int64_t*>(values);
    for (int64_t i = 0; i < n_vocab; ++i) {
        uint64_t key, h;
        if (kind == RF_VOCAB_BYTES) {
            key = siphash24_host(kVocabK0, kVocabK1, vb + off[i], off[i + 1] - off[i]);
            h = key;
        } else {
            key = (uint64_t)iv[i];
            h = mix64_host(key);
        }
        for (int64_t s = (int64_t)(h & (uint64_t)(cap - 1));; s = (s + 1) & (cap - 1)) {
            rf_vocab_entry& e = table[s];
            if (e.id < 0) {
                e = rf_vocab_entry{key, (int32_t)(i + 1), (int32_t)i};
                break;
            }
            if (e.key != key) continue;
            bool dup = kind == RF_VOCAB_INT64;
            if (!dup) {
                const int32_t a0 = off[e.ref], an = off[e.ref + 1] - a0, b0 = off[i], bn = off[i + 1] - b0;
                dup = an == bn && std::memcmp(vb + a0, vb + b0, (size_t)an) == 0;
            }
            // Keras StringLookup / IntegerLookup reject a vocabulary with repeated entries
            if (dup) return rf_set_error(RF_EINVAL, "rf_vocab_build: the passed vocabulary has at least one repeated term (entry %lld)", (long long)i);
        }
    }
    return RF_OK;
}

extern "C" int rf_lookup_ids(int32_t kind, const rf_vocab_entry* table, int64_t cap, const uint8_t* vocab_bytes,
                             const int32_t* vocab_off, const void* values, const int32_t* tok_off, const int32_t* bag_off,
                             int32_t n_slots, int32_t slot, int32_t batch, int32_t lmax, int64_t* ids, void* stream) {
    RF_REQUIRE(kind == RF_VOCAB_BYTES || kind == RF_VOCAB_INT64, "rf_lookup_ids: bad kind");
    RF_REQUIRE(cap >= 1 && (cap & (cap - 1)) == 0, "rf_lookup_ids: cap must be a power of two");
    RF_REQUIRE(n_slots >= 1 && slot >= 0 && slot < n_slots && batch >= 0 && lmax >= 0, "rf_lookup_ids: bad shape");
    if ((int64_t)batch * lmax == 0) return RF_OK;
    RF_REQUIRE(table && values && bag_off && ids && (kind != RF_VOCAB_BYTES || (tok_off && vocab_bytes && vocab_off)),
               "rf_lookup_ids: null pointer");
    hipLaunchKernelGGL(lookup_kernel, dim3(grid_of((int64_t)batch * lmax)), dim3(256), 0, rf_stream(stream), kind, table, cap,
                       vocab_bytes, vocab_off, values, tok_off, bag_off, n_slots, slot, batch, lmax, ids);
    return rf_check_launch("rf_lookup_ids");
}

extern "C" int rf_bucketize_ids(const float* values, const int32_t* bag_off, int32_t n_slots, int32_t slot, int32_t batch,
                                int32_t lmax, const float* boundaries, int32_t n_boundaries, float pad_value, int64_t* ids,
                                void* stream) {
    RF_REQUIRE(n_slots >= 1 && slot >= 0 && slot < n_slots && batch >= 0 && lmax >= 0 && n_boundaries >= 0,
               "rf_bucketize_ids: bad shape");
    if ((int64_t)batch * lmax == 0) return RF_OK;
    RF_REQUIRE(bag_off && ids && (n_boundaries == 0 || boundaries), "rf_bucketize_ids: null pointer");
    RF_REQUIRE(values || batch == 0, "rf_bucketize_ids: null values");
    hipLaunchKernelGGL(bucketize_kernel, dim3(grid_of((int64_t)batch * lmax)), dim3(256), 0, rf_stream(stream), values,
                       bag_off, n_slots, slot, batch, lmax, boundaries, n_boundaries, pad_value, ids);
    return rf_check_launch("rf_bucketize_ids");
}
