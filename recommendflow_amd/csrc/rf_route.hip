// rf_route.hip — requester-side routing of one step's row requests with dedup ("per-owner
// dedup"), in owner-major order so that it also replaces rf_bucketize_owner:
//
//   key(g)  = owner(g) * Lp + local(g),  owner = g mod P, local = g div P, Lp = ceil(R / P)
//   sort (key, request index) by key           (hipcub radix sort over the key's significant bits)
//   head[i] = key[i] != key[i-1];  uid = inclusive_scan(head) - 1
//   local_out[uid] = local, row_map[request] = uid, counts[p] = #distinct keys of owner p
//
// The distinct rows come out sorted by (owner, local), i.e. exactly the order of the all-to-all send
// buffer and of the vectors that come back, so row_map indexes the receive buffer directly. Zipf-hot
// rows are requested thousands of times per batch; each one now crosses xGMI once. No atomics on the
// data path (memory-side atomics on MI355X cost ~1 µs each under load, MI355X_MICROARCH.md §Global
// float atomics), the result is deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "rf_common.h"

namespace {

struct RouteLayout {
    int64_t n;
    int end_bit;
    size_t sort_bytes, scan_bytes;
    size_t off_kin, off_kout, off_vin, off_vout, off_scan, off_first, off_tmp, total;
};

int key_bits(uint64_t max_key) {
    int b = 1;
    while (b < 32 && (max_key >> b) != 0) ++b;
    return b;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

RouteLayout route_layout(int64_t n, int32_t nranks, int64_t table_rows) {
    RouteLayout L{};
    L.n = std::max<int64_t>(n, 1);
    const int64_t lp = (table_rows + nranks - 1) / nranks;
    L.end_bit = key_bits((uint64_t)nranks * (uint64_t)lp);  // sentinel key = P * Lp (invalid rows)
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, L.sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)L.n, 0, L.end_bit);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, L.scan_bytes, (const int32_t*)nullptr, (int32_t*)nullptr, (int)L.n);
    size_t o = 0;
    const size_t v = align256((size_t)L.n * 4);
    L.off_kin = o; o += v;
    L.off_kout = o; o += v;
    L.off_vin = o; o += v;
    L.off_vout = o; o += v;
    L.off_scan = o; o += v;
    L.off_first = o; o += align256((size_t)(nranks + 1) * 4);
    L.off_tmp = o; o += align256(std::max(L.sort_bytes, L.scan_bytes));
    L.total = o;
    return L;
}

__global__ __launch_bounds__(256) void route_keys_kernel(const int64_t* __restrict__ rows, int64_t n, int P,
                                                         int64_t lp, int64_t table_rows, uint32_t* __restrict__ keys,
                                                         uint32_t* __restrict__ idx) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = rows[j];
        const bool ok = g >= 0 && g < table_rows;
        keys[j] = ok ? (uint32_t)((g % P) * lp + g / P) : (uint32_t)((int64_t)P * lp);
        idx[j] = (uint32_t)j;
    }
}

__global__ __launch_bounds__(256) void route_heads_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                          int32_t* __restrict__ head) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

__global__ __launch_bounds__(256) void route_emit_kernel(const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ idx,
                                                         const int32_t* __restrict__ scan, int64_t n, int P,
                                                         int64_t lp, int64_t* __restrict__ local_out,
                                                         int32_t* __restrict__ row_map,
                                                         int32_t* __restrict__ first_uid) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t uid = scan[i] - 1;
        const uint32_t k = keys[i];
        row_map[idx[i]] = uid;
        const bool head = i == 0 || k != keys[i - 1];
        if (!head) continue;
        const int64_t owner = std::min<int64_t>((int64_t)(k / (uint64_t)lp), P - 1);  // sentinel -> last owner
        const bool valid = (int64_t)k < (int64_t)P * lp;
        local_out[uid] = valid ? (int64_t)(k % (uint64_t)lp) : (int64_t)-1;  // -1: gathered as NaN
        const bool first = i == 0 || std::min<int64_t>((int64_t)(keys[i - 1] / (uint64_t)lp), P - 1) != owner;
        if (first) first_uid[owner] = uid;
    }
}

// one thread: counts[p] from the first unique id of each owner (owners without requests: 0)
__global__ void route_counts_kernel(const int32_t* __restrict__ first_uid, const int32_t* __restrict__ scan,
                                    int64_t n, int P, int32_t* __restrict__ counts, int32_t* __restrict__ n_uniq) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t end = n > 0 ? scan[n - 1] : 0;
    if (n_uniq) *n_uniq = end;
    for (int p = P - 1; p >= 0; --p) {
        const int32_t f = first_uid[p];
        if (f < 0) {
            counts[p] = 0;
        } else {
            counts[p] = end - f;
            end = f;
        }
    }
}

int grid_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 32)); }

}  // namespace

extern "C" size_t rf_route_ws_bytes(int64_t n, int32_t nranks, int64_t table_rows) {
    if (nranks < 1 || table_rows < 1) return 0;
    return route_layout(n, nranks, table_rows).total;
}

extern "C" int rf_route_rows(const int64_t* rows, int64_t n, int32_t nranks, int64_t table_rows, int32_t* counts,
                             int64_t* local_out, int32_t* row_map, int32_t* n_uniq, void* ws, size_t ws_bytes,
                             void* stream) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096, "rf_route_rows: nranks must be in [1, 4096]");
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 32) - 4096,
               "rf_route_rows: table_rows must be in [1, 2^32 - 4096)");
    RF_REQUIRE(n >= 0 && n < ((int64_t)1 << 31), "rf_route_rows: n must be in [0, 2^31)");
    RF_REQUIRE(counts && ws, "rf_route_rows: null pointer");
    const RouteLayout lay = route_layout(n, nranks, table_rows);
    RF_REQUIRE(ws_bytes >= lay.total, "rf_route_rows: workspace too small (%zu < %zu)", ws_bytes, lay.total);
    hipStream_t st = rf_stream(stream);
    if (n == 0) {
        if (hipMemsetAsync(counts, 0, sizeof(int32_t) * nranks, st) != hipSuccess ||
            (n_uniq && hipMemsetAsync(n_uniq, 0, sizeof(int32_t), st) != hipSuccess))
            return rf_set_error(RF_EHIP, "rf_route_rows: memset failed");
        return RF_OK;
    }
    RF_REQUIRE(rows && local_out && row_map, "rf_route_rows: null pointer");
    char* w = static_cast<char*>(ws);
    auto* kin = reinterpret_cast<uint32_t*>(w + lay.off_kin);
    auto* kout = reinterpret_cast<uint32_t*>(w + lay.off_kout);
    auto* vin = reinterpret_cast<uint32_t*>(w + lay.off_vin);
    auto* vout = reinterpret_cast<uint32_t*>(w + lay.off_vout);
    auto* scan = reinterpret_cast<int32_t*>(w + lay.off_scan);
    auto* first = reinterpret_cast<int32_t*>(w + lay.off_first);
    void* tmp = w + lay.off_tmp;
    const int64_t lp = (table_rows + nranks - 1) / nranks;
    const int g = grid_of(n);
    if (hipMemsetAsync(first, 0xff, sizeof(int32_t) * (nranks + 1), st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_rows: memset failed");
    hipLaunchKernelGGL(route_keys_kernel, dim3(g), dim3(256), 0, st, rows, n, nranks, lp, table_rows, kin, vin);
    size_t sb = lay.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, sb, kin, kout, vin, vout, (int)n, 0, lay.end_bit, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_rows: radix sort failed");
    hipLaunchKernelGGL(route_heads_kernel, dim3(g), dim3(256), 0, st, kout, n, scan);
    size_t cb = lay.scan_bytes;
    if (hipcub::DeviceScan::InclusiveSum(tmp, cb, scan, scan, (int)n, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_rows: scan failed");
    hipLaunchKernelGGL(route_emit_kernel, dim3(g), dim3(256), 0, st, kout, vout, scan, n, nranks, lp, local_out,
                       row_map, first);
    hipLaunchKernelGGL(route_counts_kernel, dim3(1), dim3(64), 0, st, first, scan, n, nranks, counts, n_uniq);
    return rf_check_launch("rf_route_rows");
}
