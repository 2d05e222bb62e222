// rf_shard.hip — row-sharded table support (new capability, the reference only mirrors
// whole tables per GPU under MirroredStrategy, backend/utils/gpu_utils.py:13-14).
//   rf_bucketize_owner  owner = g mod P, local = g div P; counts + STABLE owner-major permutation
//   rf_gather_rows      owner-side gather of whole rows for the vector return
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {
constexpr int kTile = 256;

// pass 1: per-tile owner histogram -> hist[tile][P]
__global__ __launch_bounds__(kTile) void owner_hist_kernel(const int64_t* __restrict__ rows, int64_t n, int P,
                                                           int32_t* __restrict__ hist) {
    extern __shared__ int32_t s_cnt[];
    for (int p = threadIdx.x; p < P; p += kTile) s_cnt[p] = 0;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * kTile + threadIdx.x;
    if (i < n) atomicAdd(&s_cnt[(int)(rows[i] % P)], 1);
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += kTile) hist[(int64_t)blockIdx.x * P + p] = s_cnt[p];
}

// pass 2 (one block): owner-major exclusive scan of hist -> base[tile][P]; counts[P]
__global__ __launch_bounds__(1024) void owner_scan_kernel(const int32_t* __restrict__ hist, int64_t tiles, int P,
                                                          int32_t* __restrict__ base, int32_t* __restrict__ counts) {
    // each thread owns owners p = tid, tid + 1024, ...; serial over tiles (tiles * P is small)
    __shared__ int32_t s_tot[1024];
    __shared__ int32_t s_off[1024];
    for (int p0 = 0; p0 < P; p0 += 1024) {
        const int p = p0 + threadIdx.x;
        int32_t tot = 0;
        if (p < P)
            for (int64_t t = 0; t < tiles; ++t) tot += hist[t * P + p];
        s_tot[threadIdx.x] = tot;
        __syncthreads();
        if (threadIdx.x == 0) {
            int32_t run = p0 == 0 ? 0 : s_off[1023] + s_tot[1023];
            for (int q = 0; q < 1024; ++q) {
                s_off[q] = run;
                run += s_tot[q];
            }
        }
        __syncthreads();
        if (p < P) {
            counts[p] = tot;
            int32_t run = s_off[threadIdx.x];
            for (int64_t t = 0; t < tiles; ++t) {
                base[t * P + p] = run;
                run += hist[t * P + p];
            }
        }
        __syncthreads();
    }
}

// pass 3: stable scatter (rank among equal owners earlier in the same tile)
__global__ __launch_bounds__(kTile) void owner_scatter_kernel(const int64_t* __restrict__ rows, int64_t n, int P,
                                                              const int32_t* __restrict__ base,
                                                              int32_t* __restrict__ perm,
                                                              int64_t* __restrict__ local_rows) {
    __shared__ int32_t s_own[kTile];
    const int64_t i = (int64_t)blockIdx.x * kTile + threadIdx.x;
    const int64_t g = i < n ? rows[i] : 0;
    const int own = i < n ? (int)(g % P) : -1;
    s_own[threadIdx.x] = own;
    __syncthreads();
    if (i < n) {
        int rank = 0;
        for (int j = 0; j < (int)threadIdx.x; ++j) rank += s_own[j] == own;
        const int32_t pos = base[(int64_t)blockIdx.x * P + own] + rank;
        perm[pos] = (int32_t)i;
        local_rows[pos] = g / P;
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
                                  int64_t* local_rows, void* ws, size_t ws_bytes, void* stream) {
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
    hipLaunchKernelGGL(owner_hist_kernel, dim3((unsigned)tiles), dim3(kTile), nranks * sizeof(int32_t), st, rows, n,
                       nranks, hist);
    hipLaunchKernelGGL(owner_scan_kernel, dim3(1), dim3(1024), 0, st, hist, tiles, nranks, base, counts);
    hipLaunchKernelGGL(owner_scatter_kernel, dim3((unsigned)tiles), dim3(kTile), 0, st, rows, n, nranks, base, perm,
                       local_rows);
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
