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
        const uint32_t g32 = (uint32_t)g, p32 = (uint32_t)P;  // valid rows < 2^32: 32-bit division
        keys[j] = ok ? (g32 % p32) * (uint32_t)lp + g32 / p32 : (uint32_t)((int64_t)P * lp);
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
        const int64_t owner = std::min<int64_t>((int64_t)(k / (uint32_t)lp), P - 1);  // sentinel -> last owner
        const bool valid = (int64_t)k < (int64_t)P * lp;
        local_out[uid] = valid ? (int64_t)(k % (uint32_t)lp) : (int64_t)-1;  // -1: gathered as NaN
        const bool first = i == 0 || std::min<int64_t>((int64_t)(keys[i - 1] / (uint32_t)lp), P - 1) != owner;
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
// 0x80000000 | local (rf_pool_rows_fwd reads them from the local shard in place). The distinct keys then
// leave the table owner-major:
//   P <= 64 (kOwnerMajorMaxP): rh_count (per-workgroup, per-owner live counts) -> rh_scan_owner (owner-major
//     positions) -> rh_scatter_owner (each key straight to its position, the slot overwritten with it); finish
//     is one launch (local ids + row map). Within an owner the rows come in table-slot order — the same set as
//     rf_route_rows' ascending order; the exchange and the pooled output do not depend on the order within an
//     owner (each distinct row is sent once and the row map follows it). At cfg4 P = 8 this form replaced
//     compact + radix sort + emit (profiles/r04/route_p8_*).
//   P > 64: rh_count -> rh_scan -> rh_scatter compact in slot order, then a radix sort (key bits only) makes the
//     list owner-major and ascending within an owner, the order rf_route_rows produces.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kEmpty = 0xffffffffu;
constexpr int kChunkPerThread = 16;  // table slots per thread of the compaction (rh_count / rh_scatter)
constexpr int kChunk = 256 * kChunkPerThread;
constexpr int kOwnerMajorMaxP = 64;  // P <= this: owner-major scatter, no sort (rh_scan_owner / rh_scatter_owner)

struct HashLayout {
    int64_t n, cap;
    int log_cap, end_bit;
    size_t sort_bytes;
    int64_t n_blk;
    size_t off_table, off_slot, off_kin, off_kout, off_vin, off_vout, off_cnt, off_blk, off_blk_own, off_tmp, total;
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
    L.n_blk = (L.cap + kChunk - 1) / kChunk;
    L.off_blk = o; o += align256((size_t)L.n_blk * 4);
    L.off_blk_own = o; o += nranks <= kOwnerMajorMaxP ? align256((size_t)L.n_blk * nranks * 4) : 0;
    L.off_tmp = o; o += align256(L.sort_bytes);
    L.total = o;
    return L;
}

__device__ __forceinline__ uint32_t key_hash(uint32_t k, int log_cap) {
    return (uint32_t)(((uint64_t)(k * 0x9E3779B1u) * 0x85EBCA77ull) >> (32 - log_cap)) & ((1u << log_cap) - 1u);
}

// kIlp slots per thread per pass in rh_map, their loads issued together. (The same in rh_insert measured
// slower, 144 -> 177 us at cfg4 P = 8: more requests in flight for a Zipf-hot key read its slot empty and
// race on the CAS; its cost is the memory-side atomics, not load latency.)
constexpr int kIlp = 4;

// request j for logical row g: rank-local rows -> row_map (bit 31), others -> the key's table slot (inserted once)
__device__ __forceinline__ void rh_insert_one(int64_t g, int64_t j, int P, int rank, int64_t lp, int64_t table_rows,
                                              uint32_t* __restrict__ table, int log_cap, uint32_t* __restrict__ slot,
                                              int32_t* __restrict__ row_map) {
    const uint32_t mask = (1u << log_cap) - 1u;
    const bool ok = g >= 0 && g < table_rows;
    const uint32_t g32 = (uint32_t)g, p32 = (uint32_t)P;  // valid rows < 2^32: 32-bit division
    const uint32_t gl = g32 / p32;
    const int owner = ok ? (int)(g32 - gl * p32) : P - 1;
    if (ok && owner == rank) {  // rank-local: read in place by the pooling, never routed
        row_map[j] = (int32_t)(0x80000000u | gl);
        slot[j] = kEmpty;
        return;
    }
    const uint32_t key = ok ? (uint32_t)owner * (uint32_t)lp + gl : (uint32_t)((int64_t)P * lp);
    uint32_t h = key_hash(key, log_cap);
    while (true) {
        uint32_t cur = table[h];
        if (cur == kEmpty) cur = atomicCAS(table + h, kEmpty, key);
        if (cur == kEmpty || cur == key) break;
        h = (h + 1) & mask;
    }
    slot[j] = h;
}

__global__ __launch_bounds__(256) void rh_insert_kernel(const int64_t* __restrict__ rows, int64_t n, int P, int rank,
                                                        int64_t lp, int64_t table_rows, uint32_t* __restrict__ table,
                                                        int log_cap, uint32_t* __restrict__ slot,
                                                        int32_t* __restrict__ row_map) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        rh_insert_one(rows[j], j, P, rank, lp, table_rows, table, log_cap, slot, row_map);
}

// rf_hash_rows fused into the insert (rf_route_hash_build_tokens): thread per token of a block's 256 units (its unit by
// binary search over the bag offsets in LDS, as hash_rows_kernel), both hashes, both requests j = 2t, 2t + 1 inserted;
// then the n_tail pre-hashed pad rows as requests 2 n_tok + i. The 16 bytes per token of the [2 n_tok] int64 request
// list are neither written nor read back.
constexpr int kTokUnits = 256;
__global__ __launch_bounds__(kTokUnits) void rh_insert_tok_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                                  const uint8_t* __restrict__ tok_bytes,
                                                                  const int32_t* __restrict__ tok_off,
                                                                  const int32_t* __restrict__ bag_off, int64_t n_units,
                                                                  const int64_t* __restrict__ tail, int n_tail, int64_t n_tok,
                                                                  int P, int rank, int64_t lp, int64_t table_rows,
                                                                  uint32_t* __restrict__ table, int log_cap,
                                                                  uint32_t* __restrict__ slot, int32_t* __restrict__ row_map) {
    __shared__ int32_t s_off[kTokUnits + 1];
    for (int64_t u0 = (int64_t)blockIdx.x * kTokUnits; u0 < n_units; u0 += (int64_t)gridDim.x * kTokUnits) {
        const int nu = (int)min<int64_t>(kTokUnits, n_units - u0);
        __syncthreads();
        for (int j = threadIdx.x; j <= nu; j += kTokUnits) s_off[j] = bag_off[u0 + j];
        __syncthreads();
        const int t0 = s_off[0], t1 = s_off[nu];
        const uint32_t s_first = (uint32_t)(u0 % n_slots);
        for (int t = t0 + (int)threadIdx.x; t < t1; t += kTokUnits) {
            int lo = 0, hi = nu - 1;  // last unit j with s_off[j] <= t
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_off[mid] <= t) lo = mid; else hi = mid - 1;
            }
            const rf_slot_desc* sd = slots + (int)((s_first + (uint32_t)lo) % (uint32_t)n_slots);
            const int b0 = tok_off[t], n = tok_off[t + 1] - b0;
            uint64_t h0, h1;
            siphash24x2_dev(sd->salt[0], sd->salt[1], tok_bytes + b0, n, h0, h1);
            const BucketMod bm = bucket_mod_init(sd->num_bins, sd->mask_empty);
            const int64_t g0 = sd->row_base[0] + bucket_from_hash(h0, n, bm);
            const int64_t g1 = sd->row_base[1] + bucket_from_hash(h1, n, bm);
            rh_insert_one(g0, 2 * (int64_t)t, P, rank, lp, table_rows, table, log_cap, slot, row_map);
            rh_insert_one(g1, 2 * (int64_t)t + 1, P, rank, lp, table_rows, table, log_cap, slot, row_map);
        }
    }
    for (int64_t i = (int64_t)blockIdx.x * kTokUnits + threadIdx.x; i < n_tail; i += (int64_t)gridDim.x * kTokUnits)
        rh_insert_one(tail[i], 2 * n_tok + i, P, rank, lp, table_rows, table, log_cap, slot, row_map);
}

// Compaction of the table's live slots into (key, slot) pairs, in slot order, in three launches with no
// contended atomics: rh_count_kernel (each workgroup owns kChunk consecutive slots: its live count -> blk[b],
// its per-owner counts -> blk_own[b][p] when P <= 64, else one atomic per (workgroup, owner)), rh_scan_kernel
// (exclusive scan of blk -> workgroup bases, the distinct total, and the per-owner sums), rh_scatter_kernel
// (the same slots again, each live one to base + its rank in slot order). The first form (one workgroup per
// 256 slots, a global atomic per workgroup on the total and on every owner: 65,536 workgroups x 9 atomics on
// 9 addresses for the cfg4 P = 8 table of 2^24 slots) measured 1.49 ms per call, serialised on those
// addresses (profiles/r04/route_p8_*).
__global__ __launch_bounds__(256) void rh_count_kernel(const uint32_t* __restrict__ table, int64_t cap, int P,
                                                       int64_t lp, double inv_lp, int32_t* __restrict__ blk,
                                                       int32_t* __restrict__ blk_own, int32_t* __restrict__ cnt) {
    extern __shared__ int32_t s_own[];
    __shared__ int32_t s_wave[4];
    for (int p = threadIdx.x; p < P; p += 256) s_own[p] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * kChunk;
    uint32_t k[kChunkPerThread];
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        const int64_t h = base + i * 256 + threadIdx.x;
        k[i] = h < cap ? table[h] : kEmpty;
    }
    int live = 0;
    const uint32_t lp32 = (uint32_t)lp;
    auto owner_of = [&](uint32_t key) {  // key / lp without the 32-bit division sequence: a double product + fix-up
        uint32_t o = (uint32_t)((double)key * inv_lp);
        if ((uint64_t)o * lp32 > key) --o;
        if ((uint64_t)(o + 1) * lp32 <= key) ++o;
        return min((int)o, P - 1);
    };
    if (P <= 8) {  // per-thread counts packed 8 bits per owner (<= kChunkPerThread each), then a wave sum in 16-bit fields
        uint64_t acc = 0;
#pragma unroll
        for (int i = 0; i < kChunkPerThread; ++i) {
            const bool ok = k[i] != kEmpty;
            live += ok;
            acc += ok ? 1ull << (8 * owner_of(k[i])) : 0ull;
        }
        uint64_t ev = acc & 0x00ff00ff00ff00ffull, od = (acc >> 8) & 0x00ff00ff00ff00ffull;
        for (int off = 32; off; off >>= 1) {
            ev += __shfl_xor(ev, off, 64);
            od += __shfl_xor(od, off, 64);
        }
        if ((threadIdx.x & 63) == 0)
            for (int p = 0; p < P; ++p) {
                const int c = (int)(((p & 1 ? od : ev) >> (16 * (p >> 1))) & 0xffff);
                if (c) atomicAdd(&s_own[p], c);
            }
    } else if (P <= 64) {  // per-owner counts by ballot: lane p of each wave counts owner p, one LDS add per lane
        const int lane = threadIdx.x & 63;
        int mine = 0;
#pragma unroll
        for (int i = 0; i < kChunkPerThread; ++i) {
            const bool ok = k[i] != kEmpty;
            live += ok;
            const int o = ok ? owner_of(k[i]) : -1;
            for (int p = 0; p < P; ++p) {
                const int c = __popcll(__ballot(o == p));
                mine += lane == p ? c : 0;
            }
        }
        if (lane < P && mine) atomicAdd(&s_own[lane], mine);
    } else {
        int run_owner = -1, run = 0;
#pragma unroll
        for (int i = 0; i < kChunkPerThread; ++i) {
            if (k[i] == kEmpty) continue;
            ++live;
            const int o = owner_of(k[i]);
            if (o != run_owner) {  // per-thread run-length of owners before touching LDS
                if (run) atomicAdd(&s_own[run_owner], run);
                run_owner = o;
                run = 0;
            }
            ++run;
        }
        if (run) atomicAdd(&s_own[run_owner], run);
    }
    for (int off = 32; off; off >>= 1) live += __shfl_xor(live, off, 64);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = live;
    __syncthreads();
    if (threadIdx.x == 0) blk[blockIdx.x] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    if (P <= kOwnerMajorMaxP) {  // summed by rh_scan_(owner_)kernel: a global atomic per (workgroup, owner) serialises on P addresses
        for (int p = threadIdx.x; p < P; p += 256) blk_own[(int64_t)blockIdx.x * P + p] = s_own[p];
    } else {
        for (int p = threadIdx.x; p < P; p += 256)
            if (s_own[p]) atomicAdd(cnt + p, s_own[p]);
    }
}

// one workgroup: blk[0..nb) -> exclusive bases in place, cnt[P] = total; P <= 64: cnt[p] = sum_b blk_own[b][p]
__global__ __launch_bounds__(1024) void rh_scan_kernel(int32_t* __restrict__ blk, const int32_t* __restrict__ blk_own,
                                                       int nb, int P, int32_t* __restrict__ cnt) {
    __shared__ int32_t s_part[16];
    __shared__ int32_t s_carry;
    __shared__ int32_t s_own[1024];
    if (P <= 64) {  // 1024 / P readers per owner, fixed order: deterministic
        const int per = 1024 / P, p = threadIdx.x % P, r = threadIdx.x / P;
        int32_t acc = 0;
        if (r < per)
            for (int b = r; b < nb; b += per) acc += blk_own[(int64_t)b * P + p];
        s_own[threadIdx.x] = r < per ? acc : 0;
        __syncthreads();
        if (threadIdx.x < P) {
            int32_t t = 0;
            for (int q = 0; q < per; ++q) t += s_own[q * P + threadIdx.x];
            cnt[threadIdx.x] = t;
        }
    }
    if (threadIdx.x == 0) s_carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int b0 = 0; b0 < nb; b0 += 1024) {
        const int b = b0 + threadIdx.x;
        const int32_t v = b < nb ? blk[b] : 0;
        int32_t x = v;  // inclusive wave scan
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        if (lane == 63) s_part[wave] = x;
        __syncthreads();
        int32_t before = s_carry;
        for (int w = 0; w < wave; ++w) before += s_part[w];
        if (b < nb) blk[b] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) s_carry = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) cnt[P] = s_carry;
}

__global__ __launch_bounds__(256) void rh_scatter_kernel(const uint32_t* __restrict__ table, int64_t cap,
                                                         const int32_t* __restrict__ blk, uint32_t* __restrict__ kout,
                                                         uint32_t* __restrict__ vout) {
    __shared__ int32_t s_cnt[kChunkPerThread * 4];
    const int64_t base = (int64_t)blockIdx.x * kChunk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t k[kChunkPerThread];
    uint64_t m[kChunkPerThread];
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        const int64_t h = base + i * 256 + threadIdx.x;
        k[i] = h < cap ? table[h] : kEmpty;
        m[i] = __ballot(k[i] != kEmpty);
        if (lane == 0) s_cnt[i * 4 + wave] = __popcll(m[i]);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the 64 (row i, wave) counts in slot order
        const int32_t v = s_cnt[threadIdx.x];
        int32_t x = v;
        for (int off = 1; off < 64; off <<= 1) {
            const int32_t y = __shfl_up(x, off, 64);
            if (lane >= off) x += y;
        }
        s_cnt[threadIdx.x] = x - v;
    }
    __syncthreads();
    const int32_t b0 = blk[blockIdx.x];
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        if (k[i] == kEmpty) continue;
        const int pos = b0 + s_cnt[i * 4 + wave] + __popcll(m[i] & below);
        kout[pos] = k[i];
        vout[pos] = (uint32_t)(base + i * 256 + threadIdx.x);
    }
}

// ---- owner-major compaction without the sort (P <= 64, the sharded encoder's case) ----
// rh_scan_owner_kernel: blk_own[b][p] (live slots of owner p in workgroup b's chunk) -> in place, the position of
// that workgroup's first owner-p key in the owner-major key list; cnt[p] = owner totals, cnt[P] = distinct total.
// One workgroup of 1024: thread t = (r, p), p = t % P, owns blocks [r * per_r, (r + 1) * per_r) of owner p.
__global__ __launch_bounds__(1024) void rh_scan_owner_kernel(int32_t* __restrict__ blk_own, int nb, int P,
                                                             int32_t* __restrict__ cnt) {
    __shared__ int32_t s_acc[1024];
    __shared__ int32_t s_base[64];
    const int t = threadIdx.x, p = t % P, r = t / P, R = 1024 / P;
    const int per_r = (nb + R - 1) / R;
    const int b0 = r < R ? r * per_r : nb, b1 = min(nb, b0 + per_r);
    int32_t acc = 0;
    for (int b = b0; b < b1; ++b) acc += blk_own[(int64_t)b * P + p];
    s_acc[t] = acc;
    __syncthreads();
    for (int d = 1; d < R; d <<= 1) {  // inclusive scan over r for each owner (stride P in s_acc)
        const int32_t v = (r < R && r >= d) ? s_acc[t - d * P] : 0;
        __syncthreads();
        if (r < R) s_acc[t] += v;
        __syncthreads();
    }
    if (t == 0) {
        int32_t run = 0;
        for (int q = 0; q < P; ++q) {
            const int32_t tot = s_acc[(R - 1) * P + q];
            s_base[q] = run;
            cnt[q] = tot;
            run += tot;
        }
        cnt[P] = run;
    }
    __syncthreads();
    if (r < R) {
        int32_t run = s_base[p] + s_acc[t] - acc;
        for (int b = b0; b < b1; ++b) {
            const int32_t v = blk_own[(int64_t)b * P + p];
            blk_own[(int64_t)b * P + p] = run;
            run += v;
        }
    }
}

// the chunk's live keys to their owner-major positions (within an owner and workgroup: thread-major order for
// P <= 8, slot order above): keys[pos] = key, and the table slot is overwritten with pos (slot -> distinct id, read by rh_finish_kernel's row map)
__global__ __launch_bounds__(256) void rh_scatter_owner_kernel(uint32_t* table, int64_t cap, int P, int64_t lp,
                                                               double inv_lp, const int32_t* __restrict__ off,
                                                               uint32_t* __restrict__ keys) {
    extern __shared__ int32_t s_c[];  // [kChunkPerThread * 4 entries (i, wave)][P] counts -> exclusive offsets
    __shared__ int32_t s_off[64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kChunk;
    const uint32_t lp32 = (uint32_t)lp;
    if (threadIdx.x < P) s_off[threadIdx.x] = off[(int64_t)blockIdx.x * P + threadIdx.x];
    uint32_t k[kChunkPerThread];
    int o[kChunkPerThread];
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        const int64_t h = base + i * 256 + threadIdx.x;
        k[i] = h < cap ? table[h] : kEmpty;
    }
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        if (k[i] == kEmpty) {
            o[i] = -1;
        } else {
            uint32_t q = (uint32_t)((double)k[i] * inv_lp);
            if ((uint64_t)q * lp32 > k[i]) --q;
            if ((uint64_t)(q + 1) * lp32 <= k[i]) ++q;
            o[i] = min((int)q, P - 1);
        }
    }
    if (P <= 8) {  // thread-major order within (workgroup, owner): packed per-thread counts, one block scan
        __shared__ uint64_t s_w[4][2];
        uint64_t ev = 0, od = 0;  // owner p's count in the 16-bit field p >> 1 of (p & 1 ? od : ev)
#pragma unroll
        for (int i = 0; i < kChunkPerThread; ++i)
            if (o[i] >= 0) {
                const uint64_t one = 1ull << (16 * (o[i] >> 1));
                if (o[i] & 1) od += one; else ev += one;
            }
        uint64_t xe = ev, xo = od;  // inclusive wave scan
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t ye = __shfl_up(xe, d, 64), yo = __shfl_up(xo, d, 64);
            if (lane >= d) { xe += ye; xo += yo; }
        }
        if (lane == 63) { s_w[wave][0] = xe; s_w[wave][1] = xo; }
        __syncthreads();
        uint64_t re = xe - ev, ro = xo - od;  // exclusive, then plus the earlier waves
        for (int w = 0; w < wave; ++w) { re += s_w[w][0]; ro += s_w[w][1]; }
#pragma unroll
        for (int i = 0; i < kChunkPerThread; ++i) {
            if (o[i] < 0) continue;
            const int sh = 16 * (o[i] >> 1);
            uint64_t& r = (o[i] & 1) ? ro : re;
            const int pos = s_off[o[i]] + (int)((r >> sh) & 0xffff);
            r += 1ull << sh;
            keys[pos] = k[i];
            table[base + i * 256 + threadIdx.x] = (uint32_t)pos;
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        int mine = 0;
        for (int p = 0; p < P; ++p) {
            const int c = __popcll(__ballot(o[i] == p));
            mine = lane == p ? c : mine;
        }
        if (lane < P) s_c[(i * 4 + wave) * P + lane] = mine;
    }
    __syncthreads();
    for (int p = wave; p < P; p += 4) {  // exclusive scan over the 64 (i, wave) entries, slot order, per owner
        const int32_t v = s_c[lane * P + p];
        int32_t x = v;
        for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(x, d, 64);
            if (lane >= d) x += y;
        }
        s_c[lane * P + p] = x - v;
    }
    __syncthreads();
    const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
    for (int i = 0; i < kChunkPerThread; ++i) {
        int pos = 0;
        for (int p = 0; p < P; ++p) {
            const uint64_t m = __ballot(o[i] == p);
            if (o[i] == p) pos = s_off[p] + s_c[(i * 4 + wave) * P + p] + __popcll(m & below);
        }
        if (o[i] >= 0) {
            keys[pos] = k[i];
            table[base + i * 256 + threadIdx.x] = (uint32_t)pos;
        }
    }
}

// local_out[i] from the owner-major keys (i < u) and row_map[j] = uid of request j's slot (j < n), one launch
__global__ __launch_bounds__(256) void rh_finish_kernel(const uint32_t* __restrict__ keys, int64_t u, int P, int64_t lp,
                                                        int64_t* __restrict__ local_out, const uint32_t* __restrict__ slot,
                                                        int64_t n, const uint32_t* __restrict__ uid_of_slot,
                                                        int32_t* __restrict__ row_map, const int32_t* __restrict__ u_dev) {
    if (u_dev) u = *u_dev;  // the build's distinct total, read on the device (no host round trip before this launch)
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < u; i += stride) {
        const uint32_t k = keys[i];
        local_out[i] = (int64_t)k < (int64_t)P * lp ? (int64_t)(k % (uint32_t)lp) : (int64_t)-1;  // -1: gathered as NaN
    }
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 < n; j0 += stride * kIlp) {
        uint32_t sl[kIlp], uid[kIlp];
#pragma unroll
        for (int v = 0; v < kIlp; ++v) sl[v] = j0 + v * stride < n ? slot[j0 + v * stride] : kEmpty;
#pragma unroll
        for (int v = 0; v < kIlp; ++v) uid[v] = sl[v] != kEmpty ? uid_of_slot[sl[v]] : 0u;
#pragma unroll
        for (int v = 0; v < kIlp; ++v)
            if (sl[v] != kEmpty) row_map[j0 + v * stride] = (int32_t)uid[v];
    }
}

// sorted distinct keys -> local ids (owner-major send buffer); the table array is reused as slot -> uid
__global__ __launch_bounds__(256) void rh_emit_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ slots,
                                                      int64_t u, int P, int64_t lp, int64_t* __restrict__ local_out,
                                                      uint32_t* __restrict__ uid_of_slot) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < u; i += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t k = keys[i];
        local_out[i] = (int64_t)k < (int64_t)P * lp ? (int64_t)(k % (uint32_t)lp) : (int64_t)-1;  // -1: gathered as NaN
        uid_of_slot[slots[i]] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void rh_map_kernel(const uint32_t* __restrict__ slot, int64_t n,
                                                     const uint32_t* __restrict__ uid_of_slot, int32_t* __restrict__ row_map) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t j0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j0 < n; j0 += stride * kIlp) {
        uint32_t sl[kIlp], uid[kIlp];
#pragma unroll
        for (int u = 0; u < kIlp; ++u) sl[u] = j0 + u * stride < n ? slot[j0 + u * stride] : kEmpty;
#pragma unroll
        for (int u = 0; u < kIlp; ++u) uid[u] = sl[u] != kEmpty ? uid_of_slot[sl[u]] : 0u;
#pragma unroll
        for (int u = 0; u < kIlp; ++u)
            if (sl[u] != kEmpty) row_map[j0 + u * stride] = (int32_t)uid[u];
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

namespace {
// the build after the insert launch (or, tokens form, the fused hash + insert): compaction of the table owner-major
template <typename Insert>
int route_hash_build_impl(const char* name, int64_t n, int32_t nranks, int32_t rank, int64_t table_rows, int32_t* row_map,
                          int32_t* counts, void* ws, size_t ws_bytes, void* stream, Insert&& insert) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096, "%s: nranks must be in [1, 4096]", name);
    RF_REQUIRE(rank >= -1 && rank < nranks, "%s: rank must be -1 (no local rows) or in [0, nranks)", name);
    RF_REQUIRE(table_rows >= 1 && table_rows < ((int64_t)1 << 32) - 4096, "%s: table_rows must be in [1, 2^32 - 4096)", name);
    RF_REQUIRE((table_rows + nranks - 1) / nranks < ((int64_t)1 << 31), "%s: shard rows must be < 2^31", name);
    RF_REQUIRE(n >= 0 && n < ((int64_t)1 << 30), "%s: n must be in [0, 2^30)", name);
    RF_REQUIRE(counts && ws, "%s: null pointer", name);
    const HashLayout lay = hash_layout(n, nranks, table_rows);
    RF_REQUIRE(ws_bytes >= lay.total, "%s: workspace too small (%zu < %zu)", name, ws_bytes, lay.total);
    hipStream_t st = rf_stream(stream);
    char* w = static_cast<char*>(ws);
    int32_t* cnt = reinterpret_cast<int32_t*>(w + lay.off_cnt);
    if (hipMemsetAsync(cnt, 0, sizeof(int32_t) * (nranks + 2), st) != hipSuccess)
        return rf_set_error(RF_EHIP, "%s: memset failed", name);
    if (n > 0) {
        RF_REQUIRE(row_map, "%s: null pointer", name);
        auto* table = reinterpret_cast<uint32_t*>(w + lay.off_table);
        if (hipMemsetAsync(table, 0xff, (size_t)lay.cap * 4, st) != hipSuccess)
            return rf_set_error(RF_EHIP, "%s: memset failed", name);
        const int64_t lp = (table_rows + nranks - 1) / nranks;
        insert(st, lp, table, lay.log_cap, reinterpret_cast<uint32_t*>(w + lay.off_slot));
        auto* blk = reinterpret_cast<int32_t*>(w + lay.off_blk);
        const dim3 gb((unsigned)lay.n_blk);
        auto* blk_own = reinterpret_cast<int32_t*>(w + lay.off_blk_own);
        hipLaunchKernelGGL(rh_count_kernel, gb, dim3(256), (size_t)nranks * sizeof(int32_t), st, table, lay.cap, nranks,
                           lp, 1.0 / (double)lp, blk, blk_own, cnt);
        if (nranks <= kOwnerMajorMaxP) {
            hipLaunchKernelGGL(rh_scan_owner_kernel, dim3(1), dim3(1024), 0, st, blk_own, (int)lay.n_blk, nranks, cnt);
            hipLaunchKernelGGL(rh_scatter_owner_kernel, gb, dim3(256), (size_t)kChunkPerThread * 4 * nranks * sizeof(int32_t),
                               st, table, lay.cap, nranks, lp, 1.0 / (double)lp, blk_own,
                               reinterpret_cast<uint32_t*>(w + lay.off_kin));
        } else {
            hipLaunchKernelGGL(rh_scan_kernel, dim3(1), dim3(1024), 0, st, blk, blk_own, (int)lay.n_blk, nranks, cnt);
            hipLaunchKernelGGL(rh_scatter_kernel, gb, dim3(256), 0, st, table, lay.cap, blk,
                               reinterpret_cast<uint32_t*>(w + lay.off_kin), reinterpret_cast<uint32_t*>(w + lay.off_vin));
        }
    }
    if (hipMemcpyAsync(counts, cnt, sizeof(int32_t) * nranks, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "%s: copy failed", name);
    return rf_check_launch(name);
}
}  // namespace

extern "C" int rf_route_hash_build(const int64_t* rows, int64_t n, int32_t nranks, int32_t rank, int64_t table_rows,
                                   int32_t* row_map, int32_t* counts, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(n == 0 || rows, "rf_route_hash_build: null pointer");
    return route_hash_build_impl("rf_route_hash_build", n, nranks, rank, table_rows, row_map, counts, ws, ws_bytes, stream,
                                 [&](hipStream_t st, int64_t lp, uint32_t* table, int log_cap, uint32_t* slot) {
                                     hipLaunchKernelGGL(rh_insert_kernel, dim3(grid_of(n)), dim3(256), 0, st, rows, n, nranks,
                                                        rank, lp, table_rows, table, log_cap, slot, row_map);
                                 });
}

extern "C" int rf_route_hash_build_tokens(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                          const int32_t* tok_off, const int32_t* bag_off, int32_t batch, int64_t n_tok,
                                          const int64_t* tail, int32_t n_tail, int32_t nranks, int32_t rank,
                                          int64_t table_rows, int32_t* row_map, int32_t* counts, void* ws, size_t ws_bytes,
                                          void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0 && n_tok >= 0 && n_tail >= 0,
               "rf_route_hash_build_tokens: need n_slots >= 1, batch, n_tok, n_tail >= 0");
    RF_REQUIRE(n_tok == 0 || (d_slots && tok_bytes && tok_off && bag_off), "rf_route_hash_build_tokens: null pointer");
    RF_REQUIRE(n_tail == 0 || tail, "rf_route_hash_build_tokens: null tail");
    const int64_t n_units = (int64_t)batch * n_slots;
    const int64_t n = 2 * n_tok + n_tail;
    return route_hash_build_impl(
        "rf_route_hash_build_tokens", n, nranks, rank, table_rows, row_map, counts, ws, ws_bytes, stream,
        [&](hipStream_t st, int64_t lp, uint32_t* table, int log_cap, uint32_t* slot) {
            const int64_t g = std::max<int64_t>((n_units + kTokUnits - 1) / kTokUnits, (n_tail + kTokUnits - 1) / kTokUnits);
            hipLaunchKernelGGL(rh_insert_tok_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 64))),
                               dim3(kTokUnits), 0, st, d_slots, n_slots, tok_bytes, tok_off, bag_off, n_tok ? n_units : 0,
                               tail, n_tail, n_tok, nranks, rank, lp, table_rows, table, log_cap, slot, row_map);
        });
}

extern "C" int rf_route_hash_finish(int64_t n, int32_t nranks, int64_t table_rows, int64_t n_uniq, int64_t* local_out,
                                    int32_t* row_map, void* ws, size_t ws_bytes, void* stream) {
    RF_REQUIRE(nranks >= 1 && nranks <= 4096 && table_rows >= 1, "rf_route_hash_finish: bad nranks / table_rows");
    RF_REQUIRE(n >= 0 && n_uniq >= -1 && n_uniq <= n, "rf_route_hash_finish: need -1 <= n_uniq <= n");
    // n_uniq = -1 (P <= 64 only): the distinct total is read from the workspace on the device, so the launch can be
    // enqueued before the host has read the counts; local_out must then hold n entries (the distinct total's bound)
    RF_REQUIRE(n_uniq >= 0 || nranks <= kOwnerMajorMaxP, "rf_route_hash_finish: n_uniq = -1 needs nranks <= %d", kOwnerMajorMaxP);
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
    const int64_t lp = (table_rows + nranks - 1) / nranks;
    if (nranks <= kOwnerMajorMaxP) {  // keys already owner-major (rh_scatter_owner_kernel), table = slot -> uid
        const int32_t* u_dev = n_uniq < 0 ? reinterpret_cast<const int32_t*>(w + lay.off_cnt) + nranks : nullptr;
        hipLaunchKernelGGL(rh_finish_kernel, dim3(grid_of((n + kIlp - 1) / kIlp)), dim3(256), 0, st, kin, n_uniq < 0 ? n : n_uniq,
                           nranks, lp, local_out, reinterpret_cast<const uint32_t*>(w + lay.off_slot), n, table, row_map,
                           u_dev);
        return rf_check_launch("rf_route_hash_finish");
    }
    size_t sb = lay.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairs(w + lay.off_tmp, sb, kin, kout, vin, vout, (int)n_uniq, 0, lay.end_bit, st) !=
        hipSuccess)
        return rf_set_error(RF_EHIP, "rf_route_hash_finish: radix sort failed");
    hipLaunchKernelGGL(rh_emit_kernel, dim3(grid_of(n_uniq)), dim3(256), 0, st, kout, vout, n_uniq, nranks, lp, local_out,
                       table);
    hipLaunchKernelGGL(rh_map_kernel, dim3(grid_of((n + kIlp - 1) / kIlp)), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(w + lay.off_slot),
                       n, table, row_map);
    return rf_check_launch("rf_route_hash_finish");
}
