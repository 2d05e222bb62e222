// rf_common.h — shared device/host helpers of librf.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rf_api.h"

// ---------------------------------------------------------------------------------------------
// error state (thread-local message, see rf_last_error)
// ---------------------------------------------------------------------------------------------
int rf_set_error(int code, const char* fmt, ...);
int rf_check_launch(const char* what);  // hipGetLastError -> RF_EHIP with message

#define RF_REQUIRE(cond, ...)                                 \
    do {                                                      \
        if (!(cond)) return rf_set_error(RF_EINVAL, __VA_ARGS__); \
    } while (0)

static inline hipStream_t rf_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// special row ids of the single-token id pass (rf_single_token_ids_fwd) and the ESIM gather staging: the zero row
// (masked empty bag / rows past L) and the NaN row (a slot that does not fit the table, or whose Lmax is not 1)
constexpr uint32_t kRowZero = 0xffffffffu, kRowNaN = 0xfffffffeu;

// ---------------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------------
// Orders this wave's LDS writes before its later LDS reads by other lanes of the same wave.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------------------------
// bf16 <-> f32 (bit exact with oracle/rf_oracle.c)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float bf16_bits_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16_bits(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return ((u >> 16) | 0x40u) & 0xffffu;  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return u >> 16;
}

// ---------------------------------------------------------------------------------------------
// SipHash-2-4 on 64-bit lanes (the compiler splits into 32-bit pairs; rotations -> v_alignbit_b32).
// Reads the token with aligned dword loads: a dword that holds at least one byte of the token never
// crosses a page boundary past the token, so no read faults beyond the caller's buffer.
// ---------------------------------------------------------------------------------------------
// 64-bit rotate by a constant as two v_alignbit_b32 (the shift-or form compiled to a 64-bit shift, two 32-bit
// shifts and two ors per rotate: half of SipHash's VALU)
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int b) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (b == 32) return ((uint64_t)lo << 32) | hi;
    if (b > 32) {
        const uint32_t t = lo;
        lo = hi;
        hi = t;
        b -= 32;
    }
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - b);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - b);
    return ((uint64_t)nhi << 32) | nlo;
}

#define RF_SIPROUND                                                          \
    do {                                                                     \
        v0 += v1; v1 = rotl64(v1, 13); v1 ^= v0; v0 = rotl64(v0, 32);        \
        v2 += v3; v3 = rotl64(v3, 16); v3 ^= v2;                             \
        v0 += v3; v3 = rotl64(v3, 21); v3 ^= v0;                             \
        v2 += v1; v1 = rotl64(v1, 17); v1 ^= v2; v2 = rotl64(v2, 32);        \
    } while (0)

__device__ __forceinline__ uint64_t siphash24_dev(uint64_t k0, uint64_t k1, const uint8_t* p, int n) {
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0;
    uint64_t v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0;
    uint64_t v3 = 0x7465646279746573ULL ^ k1;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a - sh);
    const int nwords = n > 0 ? (int)((sh + (uint32_t)n + 3) >> 2) : 0;  // aligned dwords holding token bytes
    // message dword j = token bytes [4j, 4j+4) = aligned words j, j+1 shifted by sh bytes
    auto msg32 = [&](int j) -> uint32_t {
        uint32_t lo = j < nwords ? w[j] : 0u;
        uint32_t hi = (j + 1) < nwords ? w[j + 1] : 0u;
        return sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    };
    const int nb = n >> 3;
    for (int i = 0; i < nb; ++i) {
        uint64_t m = (uint64_t)msg32(2 * i) | ((uint64_t)msg32(2 * i + 1) << 32);
        v3 ^= m;
        RF_SIPROUND;
        RF_SIPROUND;
        v0 ^= m;
    }
    const int r = n & 7;
    uint64_t tail = 0;
    if (r) {
        tail = (uint64_t)msg32(2 * nb) | ((uint64_t)msg32(2 * nb + 1) << 32);
        tail &= (~0ULL) >> (64 - 8 * r);
    }
    uint64_t bl = ((uint64_t)(uint32_t)n << 56) | tail;
    v3 ^= bl;
    RF_SIPROUND;
    RF_SIPROUND;
    v0 ^= bl;
    v2 ^= 0xff;
    RF_SIPROUND;
    RF_SIPROUND;
    RF_SIPROUND;
    RF_SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

// Keras Hashing bucket (see rf_siphash_bucket in include/rf_api.h)
__device__ __forceinline__ int64_t hash_bucket_dev(uint64_t k0, uint64_t k1, const uint8_t* p, int n,
                                                   int64_t num_bins, int mask_empty) {
    if (mask_empty) {
        if (n == 0) return 0;
        if (num_bins > 1) return 1 + (int64_t)(siphash24_dev(k0, k1, p, n) % (uint64_t)(num_bins - 1));
    }
    return (int64_t)(siphash24_dev(k0, k1, p, n) % (uint64_t)num_bins);
}

// Two SipHash-2-4 states over ONE read of the token: keys (s0,s0) and (s1,s1) — the two Hashing
// layers of DoubleHashingEmbedding (preprocess_layers.py:89-90) hash the same bytes.
__device__ __forceinline__ void siphash24x2_dev(uint64_t s0, uint64_t s1, const uint8_t* p, int n, uint64_t& h0,
                                                uint64_t& h1) {
    uint64_t a0 = 0x736f6d6570736575ULL ^ s0, a1 = 0x646f72616e646f6dULL ^ s0;
    uint64_t a2 = 0x6c7967656e657261ULL ^ s0, a3 = 0x7465646279746573ULL ^ s0;
    uint64_t b0 = 0x736f6d6570736575ULL ^ s1, b1 = 0x646f72616e646f6dULL ^ s1;
    uint64_t b2 = 0x6c7967656e657261ULL ^ s1, b3 = 0x7465646279746573ULL ^ s1;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(a - sh);
    const int nwords = n > 0 ? (int)((sh + (uint32_t)n + 3) >> 2) : 0;
    auto msg32 = [&](int j) -> uint32_t {
        uint32_t lo = j < nwords ? w[j] : 0u;
        uint32_t hi = (j + 1) < nwords ? w[j + 1] : 0u;
        return sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    };
#define RF_SIPROUND2                                                                                 \
    do {                                                                                             \
        uint64_t v0 = a0, v1 = a1, v2 = a2, v3 = a3;                                                 \
        RF_SIPROUND;                                                                                 \
        a0 = v0; a1 = v1; a2 = v2; a3 = v3;                                                          \
        v0 = b0; v1 = b1; v2 = b2; v3 = b3;                                                          \
        RF_SIPROUND;                                                                                 \
        b0 = v0; b1 = v1; b2 = v2; b3 = v3;                                                          \
    } while (0)
    const int nb = n >> 3;
    for (int i = 0; i < nb; ++i) {
        const uint64_t m = (uint64_t)msg32(2 * i) | ((uint64_t)msg32(2 * i + 1) << 32);
        a3 ^= m; b3 ^= m;
        RF_SIPROUND2;
        RF_SIPROUND2;
        a0 ^= m; b0 ^= m;
    }
    const int r = n & 7;
    uint64_t tail = 0;
    if (r) {
        tail = (uint64_t)msg32(2 * nb) | ((uint64_t)msg32(2 * nb + 1) << 32);
        tail &= (~0ULL) >> (64 - 8 * r);
    }
    const uint64_t bl = ((uint64_t)(uint32_t)n << 56) | tail;
    a3 ^= bl; b3 ^= bl;
    RF_SIPROUND2;
    RF_SIPROUND2;
    a0 ^= bl; b0 ^= bl;
    a2 ^= 0xff; b2 ^= 0xff;
    RF_SIPROUND2;
    RF_SIPROUND2;
    RF_SIPROUND2;
    RF_SIPROUND2;
#undef RF_SIPROUND2
    h0 = a0 ^ a1 ^ a2 ^ a3;
    h1 = b0 ^ b1 ^ b2 ^ b3;
}

// siphash24x2_dev over a token whose covering dwords were loaded ahead into registers (so the message reads are not
// round trips inside the rounds): wv[j] = dword j of the aligned window that starts sh = (address & 3) bytes before
// the token, 0 from dword (sh + n + 3) / 4 on; needs sh + n <= 4 kSipRegWords. Same values as siphash24x2_dev.
constexpr int kSipRegWords = 8;
__device__ __forceinline__ void siphash24x2_regs(uint64_t s0, uint64_t s1, const uint32_t (&wv)[kSipRegWords + 1],
                                                 uint32_t sh, int n, uint64_t& h0, uint64_t& h1) {
    uint64_t a0 = 0x736f6d6570736575ULL ^ s0, a1 = 0x646f72616e646f6dULL ^ s0;
    uint64_t a2 = 0x6c7967656e657261ULL ^ s0, a3 = 0x7465646279746573ULL ^ s0;
    uint64_t b0 = 0x736f6d6570736575ULL ^ s1, b1 = 0x646f72616e646f6dULL ^ s1;
    uint64_t b2 = 0x6c7967656e657261ULL ^ s1, b3 = 0x7465646279746573ULL ^ s1;
    auto msg64 = [&](int i) -> uint64_t {  // message word i (bytes 8i .. 8i + 7 of the token); i compile-time
        const uint32_t lo = __builtin_amdgcn_alignbyte(wv[2 * i + 1], wv[2 * i], sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(wv[2 * i + 2], wv[2 * i + 1], sh);
        return (uint64_t)lo | ((uint64_t)hi << 32);
    };
#define RF_SIPROUND2                                                                                 \
    do {                                                                                             \
        uint64_t v0 = a0, v1 = a1, v2 = a2, v3 = a3;                                                 \
        RF_SIPROUND;                                                                                 \
        a0 = v0; a1 = v1; a2 = v2; a3 = v3;                                                          \
        v0 = b0; v1 = b1; v2 = b2; v3 = b3;                                                          \
        RF_SIPROUND;                                                                                 \
        b0 = v0; b1 = v1; b2 = v2; b3 = v3;                                                          \
    } while (0)
    const int nb = n >> 3;
    uint64_t tail = 0;
#pragma unroll
    for (int i = 0; i < kSipRegWords / 2; ++i) {
        const uint64_t m = msg64(i);
        if (i < nb) {
            a3 ^= m; b3 ^= m;
            RF_SIPROUND2;
            RF_SIPROUND2;
            a0 ^= m; b0 ^= m;
        } else if (i == nb) {
            tail = m;
        }
    }
    const int r = n & 7;
    tail = r ? tail & ((~0ULL) >> (64 - 8 * r)) : 0ull;
    const uint64_t bl = ((uint64_t)(uint32_t)n << 56) | tail;
    a3 ^= bl; b3 ^= bl;
    RF_SIPROUND2;
    RF_SIPROUND2;
    a0 ^= bl; b0 ^= bl;
    a2 ^= 0xff; b2 ^= 0xff;
    RF_SIPROUND2;
    RF_SIPROUND2;
    RF_SIPROUND2;
    RF_SIPROUND2;
#undef RF_SIPROUND2
    h0 = a0 ^ a1 ^ a2 ^ a3;
    h1 = b0 ^ b1 ^ b2 ^ b3;
}

__device__ __forceinline__ int64_t bucket_from_hash(uint64_t h, int n, int64_t num_bins, int mask_empty) {
    if (mask_empty) {
        if (n == 0) return 0;
        if (num_bins > 1) return 1 + (int64_t)(h % (uint64_t)(num_bins - 1));
    }
    return (int64_t)(h % (uint64_t)num_bins);
}

// bucket_from_hash with the modulus of a slot prepared once (per item: the slot is wave-uniform there): a
// generic 64-bit unsigned remainder is a long emulated sequence per hash, while with m = floor((2^64 - 1) / d)
// the quotient estimate q = mulhi(h, m) is floor(h / d) or one less (m >= (2^64 - d) / d, h < 2^64), so
// r = h - q d needs at most one correction (two are applied). Exact: bit-identical to bucket_from_hash
// (checked on 44 M (h, d) pairs incl. d = 1, 2^32, 2^63, 2^64 - 1).
struct BucketMod {
    uint64_t d;    // the divisor: num_bins - 1 when mask_empty and num_bins > 1, else num_bins
    uint64_t m;    // floor((2^64 - 1) / d)
    int64_t add;   // 1 when mask_empty and num_bins > 1
    int mask_empty;
};
__device__ __forceinline__ BucketMod bucket_mod_init(int64_t num_bins, int mask_empty) {
    BucketMod b;
    const bool shift = mask_empty && num_bins > 1;
    b.d = (uint64_t)(shift ? num_bins - 1 : num_bins);
    b.m = b.d ? ~0ull / b.d : 0ull;
    b.add = shift ? 1 : 0;
    b.mask_empty = mask_empty;
    return b;
}
__device__ __forceinline__ int64_t bucket_from_hash(uint64_t h, int n, const BucketMod& b) {
    if (b.mask_empty && n == 0) return 0;
    const uint64_t q = __umul64hi(h, b.m);
    uint64_t r = h - q * b.d;
    r = r >= b.d ? r - b.d : r;
    r = r >= b.d ? r - b.d : r;
    return b.add + (int64_t)r;
}

__device__ __forceinline__ uint64_t splitmix64_dev(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}
