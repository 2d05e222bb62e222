// rf_shard.hip — row-sharded table support (new capability, the reference only mirrors
// whole tables per GPU under MirroredStrategy, backend/utils/gpu_utils.py:13-14).
//   rf_bucketize_owner  owner = g mod P, local = g div P; counts + STABLE owner-major permutation
//   rf_gather_rows      owner-side gather of whole rows for the vector return
//   (rf_route_rows, the dedup'ing alternative to rf_bucketize_owner, is in rf_route.hip)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {
// A tile = kTile consecutive requests. The histogram and the scatter both walk a tile in order, so the
// owner-major permutation is stable (requests keep their relative order within each owner).
constexpr int kTile = 2048;

// pass 1: per-tile owner histogram -> hist[p * tiles + tile] (owner-major, so one flat exclusive scan
// of hist yields every (owner, tile) output base directly)
__global__ __launch_bounds__(256) void owner_hist_kernel(const int64_t* __restrict__ rows, int64_t n, int P,
                                                         int64_t tiles, int32_t* __restrict__ hist) {
    extern __shared__ int32_t s_cnt[];
    for (int p = threadIdx.x; p < P; p += 256) s_cnt[p] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kTile;
    for (int k = threadIdx.x; k < kTile; k += 256) {
        const int64_t i = t0 + k;
        if (i < n) atomicAdd(&s_cnt[(int)(rows[i] % P)], 1);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += 256) hist[(int64_t)p * tiles + blockIdx.x] = s_cnt[p];
}

// pass 2 (one block): exclusive scan of the m = P * tiles histogram entries -> base; counts[P]
__global__ __launch_bounds__(1024) void owner_scan_kernel(const int32_t* __restrict__ hist, int64_t m, int64_t tiles,
                                                          int P, int64_t n, int32_t* __restrict__ base,
                                                          int32_t* __restrict__ counts) {
    constexpr int kPer = 8;
    __shared__ int32_t s_wave[16];
    __shared__ int32_t s_carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    for (int64_t c0 = 0; c0 < m; c0 += 1024 * kPer) {
        const int64_t j0 = c0 + (int64_t)threadIdx.x * kPer;
        int32_t v[kPer], sum = 0;
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            v[e] = j0 + e < m ? hist[j0 + e] : 0;
            sum += v[e];
        }
        int32_t incl = sum;  // wave inclusive scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        int32_t wbase = s_carry;
        for (int w = 0; w < wave; ++w) wbase += s_wave[w];
        int32_t run = wbase + incl - sum;
#pragma unroll
        for (int e = 0; e < kPer; ++e) {
            if (j0 + e < m) base[j0 + e] = run;
            run += v[e];
        }
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = run;
        __syncthreads();
    }
    for (int p = threadIdx.x; p < P; p += 1024)
        counts[p] = (p + 1 < P ? base[(int64_t)(p + 1) * tiles] : (int32_t)n) - base[(int64_t)p * tiles];
}

// pass 3 (one wave per tile): stable scatter. Per 64-request round, lanes with the same owner are ranked
// by a ballot over the round (one iteration per distinct owner present), the round's leader advances the
// owner's running offset in LDS.
__global__ __launch_bounds__(64) void owner_scatter_kernel(const int64_t* __restrict__ rows, int64_t n, int P,
                                                           int64_t tiles, const int32_t* __restrict__ base,
                                                           int32_t* __restrict__ perm, int32_t* __restrict__ inv,
                                                           int64_t* __restrict__ local_rows) {
    extern __shared__ int32_t s_run[];
    const int lane = threadIdx.x;
    for (int p = lane; p < P; p += 64) s_run[p] = base[(int64_t)p * tiles + blockIdx.x];
    __syncthreads();
    const int64_t t0 = (int64_t)blockIdx.x * kTile;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int r = 0; r < kTile; r += 64) {
        const int64_t i = t0 + r + lane;
        if (t0 + r >= n) break;
        const bool valid = i < n;
        const int64_t g = valid ? rows[i] : 0;
        const int own = valid ? (int)(g % P) : -1;
        uint64_t pending = __ballot(valid);
        int32_t pos = 0;
        while (pending) {
            const int leader = __ffsll((long long)pending) - 1;
            const int o = __shfl(own, leader, 64);
            const uint64_t m = __ballot(own == o);
            int32_t b = 0;
            if (lane == leader) {
                b = s_run[o];
                s_run[o] = b + __popcll(m);
            }
            b = __shfl(b, leader, 64);
            if (own == o) pos = b + __popcll(m & lt);
            pending &= ~m;
        }
        if (valid) {
            perm[pos] = (int32_t)i;
            if (inv) inv[i] = pos;
            local_rows[pos] = g / P;
        }
    }
}

__global__ __launch_bounds__(256) void gather_rows_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                          const uint4* __restrict__ table, int64_t table_rows,
                                                          int chunks, uint4* __restrict__ out) {
    const int64_t total = n * chunks;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = x / chunks;
        const int c = (int)(x - i * chunks);
        const int64_t r = rows[i];
        out[x] = (r >= 0 && r < table_rows) ? table[r * chunks + c] : make_uint4(0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u, 0x7fc07fc0u);
    }
}
}  // namespace

extern "C" size_t rf_bucketize_ws_bytes(int64_t n, int32_t nranks) {
    const int64_t tiles = std::max<int64_t>(1, (n + kTile - 1) / kTile);
    return (size_t)(2 * tiles * (int64_t)std::max(nranks, 1) * sizeof(int32_t)) + 256;
}

extern "C" int rf_bucketize_owner(const int64_t* rows, int64_t n, int32_t nranks, int32_t* counts, int32_t* perm,
                                  int32_t* inv_perm, int64_t* local_rows, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096, "rf_bucketize_owner: nranks must be in [1, 4096]");
    RF_REQUIRE(n >= 0 && n < (int64_t)1 << 31, "rf_bucketize_owner: n must be in [0, 2^31)");
    RF_REQUIRE(ws_bytes >= rf_bucketize_ws_bytes(n, nranks), "rf_bucketize_owner: workspace too small");
    RF_REQUIRE(counts && ws, "rf_bucketize_owner: null pointer");
    hipStream_t st = rf_stream(stream);
    if (n == 0) {
        if (hipMemsetAsync(counts, 0, sizeof(int32_t) * nranks, st) != hipSuccess)
            return rf_set_error(RF_EHIP, "rf_bucketize_owner: memset failed");
        return RF_OK;
    }
    RF_REQUIRE(rows && perm && local_rows, "rf_bucketize_owner: null pointer");
    const int64_t tiles = (n + kTile - 1) / kTile;
    int32_t* hist = reinterpret_cast<int32_t*>(ws);
    int32_t* base = hist + tiles * nranks;
    const size_t lds = (size_t)nranks * sizeof(int32_t);
    hipLaunchKernelGGL(owner_hist_kernel, dim3((unsigned)tiles), dim3(256), lds, st, rows, n, nranks, tiles, hist);
    hipLaunchKernelGGL(owner_scan_kernel, dim3(1), dim3(1024), 0, st, hist, tiles * nranks, tiles, nranks, n, base,
                       counts);
    hipLaunchKernelGGL(owner_scatter_kernel, dim3((unsigned)tiles), dim3(64), lds, st, rows, n, nranks, tiles, base,
                       perm, inv_perm, local_rows);
    return rf_check_launch("rf_bucketize_owner");
}

extern "C" int rf_gather_rows(const int64_t* rows, int64_t n, const void* table, int32_t dtype, int64_t table_rows,
                              int32_t dim, void* out, void* stream) {
    RF_REQUIRE(dtype == RF_DTYPE_F32 || dtype == RF_DTYPE_BF16 || dtype == RF_DTYPE_F16, "rf_gather_rows: bad dtype");
    const int esz = dtype == RF_DTYPE_F32 ? 4 : 2;
    RF_REQUIRE(dim > 0 && (dim * esz) % 16 == 0, "rf_gather_rows: row bytes must be a multiple of 16");
    RF_REQUIRE(((uintptr_t)table & 15) == 0 && ((uintptr_t)out & 15) == 0, "rf_gather_rows: table/out must be 16-byte aligned");
    if (n == 0) return RF_OK;
    RF_REQUIRE(rows && table && out, "rf_gather_rows: null pointer");
    const int chunks = dim * esz / 16;
    const int64_t total = n * chunks;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid), dim3(256), 0, rf_stream(stream), rows, n,
                       (const uint4*)table, table_rows, chunks, (uint4*)out);
    return rf_check_launch("gather_rows_kernel");
}

