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
//
// rf_route_hash_build / rf_route_hash_finish (below) produce the same routing with a hash-table dedup
// (one atomic per DISTINCT remote row) and sort only the distinct set; rows the calling rank owns are
// left out of the exchange and read in place by the pooling.
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

// ---------------------------------------------------------------------------------------------
// Hash-table route (rf_route_hash_build / rf_route_hash_finish): each distinct REMOTE key is inserted once
// into an open-addressing table of 32-bit keys (capacity a power of two >= 2 n); a request finds its key
// with a plain load first and only an empty slot is claimed by atomicCAS, so a Zipf-hot row costs one
// atomic in all. Rows this rank owns (rank >= 0) never enter the table: their row_map entry is
// 0x80000000 | local (rf_pool_rows_fwd reads them from the local shard in place). The compacted distinct
// keys are then sorted (radix, key bits only) so the send buffer is owner-major and, within an owner,
// ascending by local row — the same order rf_route_rows produces.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kEmpty = 0xffffffffu;

struct HashLayout {
    int64_t n, cap;
    int log_cap, end_bit;
    size_t sort_bytes;
    size_t off_table, off_slot, off_kin, off_kout, off_vin, off_vout, off_cnt, off_tmp, total;
};

HashLayout hash_layout(int64_t n, int32_t nranks, int64_t table_rows) {
    HashLayout L{};
    L.n = std::max<int64_t>(n, 1);
    L.log_cap = 4;
    while (((int64_t)1 << L.log_cap) < 2 * L.n) ++L.log_cap;
    L.cap = (int64_t)1 << L.log_cap;
    const int64_t lp = (table_rows + nranks - 1) / nranks;
    L.end_bit = key_bits((uint64_t)nranks * (uint64_t)lp);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, L.sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)L.n, 0, L.end_bit);
    size_t o = 0;
    const size_t v = align256((size_t)L.n * 4);
    L.off_table = o; o += align256((size_t)L.cap * 4);
    L.off_slot = o; o += v;
    L.off_kin = o; o += v;
    L.off_kout = o; o += v;
    L.off_vin = o; o += v;
    L.off_vout = o; o += v;
    L.off_cnt = o; o += align256((size_t)(nranks + 2) * 4);  // counts[P] | n_uniq | reserved
    L.off_tmp = o; o += align256(L.sort_bytes);
    L.total = o;
    return L;
}

__device__ __forceinline__ uint32_t key_hash(uint32_t k, int log_cap) {
    return (uint32_t)(((uint64_t)(k * 0x9E3779B1u) * 0x85EBCA77ull) >> (32 - log_cap)) & ((1u << log_cap) - 1u);
}

__global__ __launch_bounds__(256) void rh_insert_kernel(const int64_t* __restrict__ rows, int64_t n, int P, int rank,
                                                        int64_t lp, int64_t table_rows, uint32_t* __restrict__ table,
                                                        int log_cap, uint32_t* __restrict__ slot,
                                                        int32_t* __restrict__ row_map) {
    const uint32_t mask = (1u << log_cap) - 1u;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = rows[j];
        const bool ok = g >= 0 && g < table_rows;
        const int owner = ok ? (int)(g % P) : P - 1;
        if (ok && owner == rank) {  // rank-local: read in place by the pooling, never routed
            row_map[j] = (int32_t)(0x80000000u | (uint32_t)(g / P));
            slot[j] = kEmpty;
            continue;
        }
        const uint32_t key = ok ? (uint32_t)((int64_t)owner * lp + g / P) : (uint32_t)((int64_t)P * lp);
        uint32_t h = key_hash(key, log_cap);
        while (true) {
            uint32_t cur = table[h];
            if (cur == kEmpty) cur = atomicCAS(table + h, kEmpty, key);
            if (cur == kEmpty || cur == key) break;
            h = (h + 1) & mask;
        }
        slot[j] = h;
    }
}

// table slots in order -> (key, slot) pairs; per-owner counts and the distinct total by block-aggregated
// atomics (the pairs' order is fixed by the sort that follows)
__global__ __launch_bounds__(256) void rh_compact_kernel(const uint32_t* __restrict__ table, int64_t cap, int P,
                                                         int64_t lp, uint32_t* __restrict__ kout,
                                                         uint32_t* __restrict__ vout, int32_t* __restrict__ cnt) {
    extern __shared__ int32_t s_own[];
    __shared__ int32_t s_base;
    for (int p = threadIdx.x; p < P; p += 256) s_own[p] = 0;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    const int64_t h = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t k = h < cap ? table[h] : kEmpty;
    const bool live = k != kEmpty;
    const uint64_t m = __ballot(live);
    const int lane = threadIdx.x & 63;
    int wbase = 0;
    if (lane == 0 && m) wbase = atomicAdd(&s_base, __popcll(m));
    wbase = __shfl(wbase, 0, 64);
    if (live) atomicAdd(&s_own[min((int64_t)(k / (uint64_t)lp), (int64_t)P - 1)], 1);
    __syncthreads();
    __shared__ int32_t s_gbase;
    if (threadIdx.x == 0) s_gbase = s_base ? atomicAdd(cnt + P, s_base) : 0;
    for (int p = threadIdx.x; p < P; p += 256)
        if (s_own[p]) atomicAdd(cnt + p, s_own[p]);
    __syncthreads();
    if (live) {
        const int pos = s_gbase + wbase + __popcll(m & ((1ull << lane) - 1ull));
        kout[pos] = k;
        vout[pos] = (uint32_t)h;
    }
}

// sorted distinct keys -> local ids (owner-major send buffer); the table array is reused as slot -> uid
__global__ __launch_bounds__(256) void rh_emit_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ slots,
                                                      int64_t u, int P, int64_t lp, int64_t* __restrict__ local_out,
                                                      uint32_t* __restrict__ uid_of_slot) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < u; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        local_out[i] = (int64_t)k < (int64_t)P * lp ? (int64_t)(k % (uint64_t)lp) : (int64_t)-1;  // -1: gathered as NaN
        uid_of_slot[slots[i]] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void rh_map_kernel(const uint32_t* __restrict__ slot, int64_t n,
                                                     const uint32_t* __restrict__ uid_of_slot, int32_t* __restrict__ row_map) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t sl = slot[j];
        if (sl != kEmpty) row_map[j] = (int32_t)uid_of_slot[sl];
    }
}

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

extern "C" size_t rf_route_hash_ws_bytes(int64_t n, int32_t nranks, int64_t table_rows) {
    if (nranks < 1 || table_rows < 1) return 0;
    return hash_layout(n, nranks, table_rows).total;
}

extern "C" int rf_route_hash_build(const int64_t* rows, int64_t n, int32_t nranks, int32_t rank, int64_t table_rows,
                                   int32_t* row_map, int32_t* counts, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096, "rf_route_hash_build: nranks must be in [1, 4096]");
    RF_REQUIRE(rank >= -1 && rank < nranks, "rf_route_hash_build: rank must be -1 (no local rows) or in [0, nranks)");
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 32) - 4096,
               "rf_route_hash_build: table_rows must be in [1, 2^32 - 4096)");
    RF_REQUIRE((table_rows + nranks - 1) / nranks < ((int64_t)1 << 31), "rf_route_hash_build: shard rows must be < 2^31");
    RF_REQUIRE(n >= 0 && n < ((int64_t)1 << 30), "rf_route_hash_build: n must be in [0, 2^30)");
    RF_REQUIRE(counts && ws, "rf_route_hash_build: null pointer");
    const HashLayout lay = hash_layout(n, nranks, table_rows);
    RF_REQUIRE(ws_bytes >= lay.total, "rf_route_hash_build: workspace too small (%zu < %zu)", ws_bytes, lay.total);
    hipStream_t st = rf_stream(stream);
    char* w = static_cast<char*>(ws);
    int32_t* cnt = reinterpret_cast<int32_t*>(w + lay.off_cnt);
    if (hipMemsetAsync(cnt, 0, sizeof(int32_t) * (nranks + 2), st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_hash_build: memset failed");
    if (n > 0) {
        RF_REQUIRE(rows && row_map, "rf_route_hash_build: null pointer");
        auto* table = reinterpret_cast<uint32_t*>(w + lay.off_table);
        if (hipMemsetAsync(table, 0xff, (size_t)lay.cap * 4, st) != hipSuccess)
            return rf_set_error(RF_EHIP, "rf_route_hash_build: memset failed");
        const int64_t lp = (table_rows + nranks - 1) / nranks;
        hipLaunchKernelGGL(rh_insert_kernel, dim3(grid_of(n)), dim3(256), 0, st, rows, n, nranks, rank, lp, table_rows,
                           table, lay.log_cap, reinterpret_cast<uint32_t*>(w + lay.off_slot), row_map);
        hipLaunchKernelGGL(rh_compact_kernel, dim3((unsigned)((lay.cap + 255) / 256)), dim3(256),
                           (size_t)nranks * sizeof(int32_t), st, table, lay.cap, nranks, lp,
                           reinterpret_cast<uint32_t*>(w + lay.off_kin), reinterpret_cast<uint32_t*>(w + lay.off_vin), cnt);
    }
    if (hipMemcpyAsync(counts, cnt, sizeof(int32_t) * nranks, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_hash_build: copy failed");
    return rf_check_launch("rf_route_hash_build");
}

extern "C" int rf_route_hash_finish(int64_t n, int32_t nranks, int64_t table_rows, int64_t n_uniq, int64_t* local_out,
                                    int32_t* row_map, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096 && table_rows >= 1, "rf_route_hash_finish: bad nranks / table_rows");
    RF_REQUIRE(n >= 0 && n_uniq >= 0 && n_uniq <= n, "rf_route_hash_finish: need 0 <= n_uniq <= n");
    const HashLayout lay = hash_layout(n, nranks, table_rows);
    RF_REQUIRE(ws && ws_bytes >= lay.total, "rf_route_hash_finish: workspace too small");
    if (n == 0 || n_uniq == 0) return RF_OK;
    RF_REQUIRE(local_out && row_map, "rf_route_hash_finish: null pointer");
    hipStream_t st = rf_stream(stream);
    char* w = static_cast<char*>(ws);
    auto* kin = reinterpret_cast<uint32_t*>(w + lay.off_kin);
    auto* kout = reinterpret_cast<uint32_t*>(w + lay.off_kout);
    auto* vin = reinterpret_cast<uint32_t*>(w + lay.off_vin);
    auto* vout = reinterpret_cast<uint32_t*>(w + lay.off_vout);
    auto* table = reinterpret_cast<uint32_t*>(w + lay.off_table);
    size_t sb = lay.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w + lay.off_tmp, sb, kin, kout, vin, vout, (int)n_uniq, 0, lay.end_bit, st) !=
        hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_hash_finish: radix sort failed");
    const int64_t lp = (table_rows + nranks - 1) / nranks;
    hipLaunchKernelGGL(rh_emit_kernel, dim3(grid_of(n_uniq)), dim3(256), 0, st, kout, vout, n_uniq, nranks, lp, local_out,
                       table);
    hipLaunchKernelGGL(rh_map_kernel, dim3(grid_of(n)), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(w + lay.off_slot),
                       n, table, row_map);
    return rf_check_launch("rf_route_hash_finish");
}
