// rf_probe.hip — measurement probes that state the ceilings the hot-path kernels are judged against
// (SURVEY §8d "Peak: the measured STREAM-copy bandwidth on the box"). Not on the
// hot path; the bench calls them beside the headline.
//   rf_stream_copy   float4 STREAM copy dst = src (4 variants: lanes' depth, nontemporal, persistent grid; the bench
//                    reports the best): the box's achievable HBM rate for a streaming kernel
//   rf_gather_probe  uniformly random whole-row reads (optionally copied out contiguously): the achievable
//                    rate of the fused encoder's access pattern (random 128-/256-B rows, streaming output)
//                    from a table far larger than the 256 MiB Infinity Cache
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {

typedef float v4f __attribute__((ext_vector_type(4)));

// Every lane moves U float4 per pass, all loads issued before the first store (U * 16 B in flight per lane).
// NT: nontemporal loads / stores (streamed once, no reuse). GRID > 0: a persistent grid of GRID blocks strides
// over the buffer; GRID == 0: one pass per block.
template <int U, bool NT, int GRID>
__global__ __launch_bounds__(256) void stream_copy_kernel(const v4f* __restrict__ src, v4f* __restrict__ dst, int64_t n4) {
    const int64_t step = GRID > 0 ? (int64_t)gridDim.x * 256 * U : 0;
    for (int64_t base = (int64_t)blockIdx.x * (256 * U) + threadIdx.x; base < n4; base += step) {
        if (base + (int64_t)(U - 1) * 256 < n4) {
            v4f v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + base + u * 256) : src[base + u * 256];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (NT) __builtin_nontemporal_store(v[u], dst + base + u * 256);
                else dst[base + u * 256] = v[u];
            }
        } else {
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + u * 256;
                if (i < n4) dst[i] = src[i];
            }
        }
        if (GRID == 0) break;
    }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// A team of LPR lanes reads one row as LPR consecutive 16-byte chunks (the fused encoder's row-load shape);
// each team has G (4, 8 or 16) rows in flight. Row r_i = mulhi(mix64(seed ^ i), rows): uniform over the table, no index
// array to read. COPY: row i is written to out[i] (the encoder's streaming output); else the loaded words
// fold into a register that is stored only if it equals an impossible value (keeps the loads).
template <int LPR, int G, bool COPY>
__global__ __launch_bounds__(256) void gather_probe_kernel(const uint4* __restrict__ table, int64_t rows, int64_t n,
                                                           uint64_t seed, uint4* __restrict__ out,
                                                           uint32_t* __restrict__ sink) {
    constexpr int TEAMS = 256 / LPR;
    const int tl = threadIdx.x % LPR, team = threadIdx.x / LPR;
    const int64_t first = ((int64_t)blockIdx.x * TEAMS + team) * G;
    uint32_t acc = 0;
    int64_t r[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i = first + g;
        r[g] = i < n ? (int64_t)__umul64hi(mix64(seed ^ (uint64_t)i), (uint64_t)rows) : 0;
    }
    uint4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = table[r[g] * LPR + tl];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int64_t i = first + g;
        if (COPY) {
            if (i < n) out[i * LPR + tl] = v[g];
        } else {
            acc ^= v[g].x ^ v[g].y ^ v[g].z ^ v[g].w;
        }
    }
    if (!COPY && acc == 0x7fc0dead) sink[0] = acc;
}

template <int LPR, int G>
int launch_gather(const void* table, int64_t rows, int64_t n, uint64_t seed, void* out, uint32_t* sink,
                  hipStream_t st) {
    const int64_t per_block = (256 / LPR) * G;
    const int64_t blocks = (n + per_block - 1) / per_block;
    if (out)
        hipLaunchKernelGGL((gather_probe_kernel<LPR, G, true>), dim3((unsigned)blocks), dim3(256), 0, st,
                           (const uint4*)table, rows, n, seed, (uint4*)out, sink);
    else
        hipLaunchKernelGGL((gather_probe_kernel<LPR, G, false>), dim3((unsigned)blocks), dim3(256), 0, st,
                           (const uint4*)table, rows, n, seed, (uint4*)nullptr, sink);
    return rf_check_launch("gather_probe_kernel");
}

template <int LPR>
int launch_gather_g(int g, const void* table, int64_t rows, int64_t n, uint64_t seed, void* out, uint32_t* sink,
                    hipStream_t st) {
    switch (g) {
        case 4: return launch_gather<LPR, 4>(table, rows, n, seed, out, sink, st);
        case 8: return launch_gather<LPR, 8>(table, rows, n, seed, out, sink, st);
        default: return launch_gather<LPR, 16>(table, rows, n, seed, out, sink, st);
    }
}

}  // namespace

extern "C" int rf_stream_copy(const void* src, void* dst, int64_t n_bytes, int32_t variant, void* stream) {
    RF_REQUIRE(n_bytes >= 0 && n_bytes % 16 == 0, "rf_stream_copy: n_bytes must be a multiple of 16");
    RF_REQUIRE(variant >= 0 && variant <= 3, "rf_stream_copy: variant must be 0..3");
    if (n_bytes == 0) return RF_OK;
    RF_REQUIRE(src && dst && ((uintptr_t)src % 16 == 0) && ((uintptr_t)dst % 16 == 0),
               "rf_stream_copy: 16-byte aligned src and dst required");
    const int64_t n4 = n_bytes / 16;
    const hipStream_t st = rf_stream(stream);
    const v4f* s4 = (const v4f*)src;
    v4f* d4 = (v4f*)dst;
    auto one_pass = [&](int U) {
        const int64_t b = (n4 + 256 * U - 1) / (256 * U);
        return (unsigned)std::min<int64_t>(b, (int64_t)1 << 30);
    };
    switch (variant) {
        case 0: hipLaunchKernelGGL((stream_copy_kernel<4, false, 0>), dim3(one_pass(4)), dim3(256), 0, st, s4, d4, n4); break;
        case 1: hipLaunchKernelGGL((stream_copy_kernel<8, false, 0>), dim3(one_pass(8)), dim3(256), 0, st, s4, d4, n4); break;
        case 2: hipLaunchKernelGGL((stream_copy_kernel<4, true, 0>), dim3(one_pass(4)), dim3(256), 0, st, s4, d4, n4); break;
        default: hipLaunchKernelGGL((stream_copy_kernel<4, true, 1>), dim3(256 * 8), dim3(256), 0, st, s4, d4, n4); break;
    }
    return rf_check_launch("stream_copy_kernel");
}

extern "C" int rf_gather_probe(const void* table, int64_t rows, int32_t row_bytes, int64_t n, int32_t in_flight,
                               uint64_t seed, void* out, uint32_t* sink, void* stream) {
    RF_REQUIRE(rows > 0 && n >= 0, "rf_gather_probe: rows > 0, n >= 0 required");
    RF_REQUIRE(row_bytes == 64 || row_bytes == 128 || row_bytes == 256 || row_bytes == 512,
               "rf_gather_probe: row_bytes must be 64, 128, 256 or 512");
    RF_REQUIRE(table && sink && (uintptr_t)table % 16 == 0 && (!out || (uintptr_t)out % 16 == 0),
               "rf_gather_probe: 16-byte aligned table / out and a sink word required");
    RF_REQUIRE(in_flight == 4 || in_flight == 8 || in_flight == 16, "rf_gather_probe: in_flight must be 4, 8 or 16");
    if (n == 0) return RF_OK;
    const hipStream_t st = rf_stream(stream);
    switch (row_bytes) {
        case 64: return launch_gather_g<4>(in_flight, table, rows, n, seed, out, sink, st);
        case 128: return launch_gather_g<8>(in_flight, table, rows, n, seed, out, sink, st);
        case 256: return launch_gather_g<16>(in_flight, table, rows, n, seed, out, sink, st);
        default: return launch_gather_g<32>(in_flight, table, rows, n, seed, out, sink, st);
    }
}
