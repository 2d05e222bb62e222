// rf_topk.hip — exact top-k over a block of scores, merged with a running top-k (the
// FaissSearcher Flat inner-product search, backend/third_party_components/faiss_searcher.py:141-204, and
// the recall evaluation on top of it, backend/utils/eval_utils.py:85-147).
//
// One 1024-thread workgroup per query row. Every candidate becomes a unique 64-bit key
//   (orderable(score) << 32) | ~index
// so "larger key" = higher score, then smaller index (a deterministic tie order). The row's keys stay in
// registers (IPT per thread, columns t + 1024 j: coalesced loads); a radix select (8 bits a pass, per-wave
// LDS histograms, early exit once the boundary bin holds exactly the missing count) finds the k-th
// largest key, the selected keys and the previous top-k are written to LDS and bitonic-sorted, and the
// best k are the new running top-k. NaN scores are never selected. With a full running top-k that is
// sorted (as this kernel writes it), keys at or below its k-th entry are dropped on load (they cannot
// enter), which skips the radix passes for most rows of a long scan; an unsorted running set gets no floor.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rf_common.h"

namespace {

constexpr int kThreads = 1024;
constexpr int kWavesTopk = kThreads / 64;
constexpr int kMaxK = 1024;

__device__ __forceinline__ uint32_t f2key(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <int IPT>
__global__ __launch_bounds__(kThreads) void topk_kernel(const float* __restrict__ scores, int64_t ld, int cols, int k,
                                                        int64_t col_base, const float* __restrict__ prev_val,
                                                        const int64_t* __restrict__ prev_idx, int k_prev, int64_t prev_ld,
                                                        float* __restrict__ out_val, int64_t* __restrict__ out_idx,
                                                        int64_t out_ld, const uint32_t* __restrict__ col_idx) {
    __shared__ uint32_t hist[kWavesTopk][256];
    __shared__ uint32_t tot[256];
    __shared__ uint64_t cand[2 * kMaxK];
    __shared__ uint64_t pk[kMaxK];  // the running top-k as keys
    __shared__ int s_unsorted;
    __shared__ uint64_t s_prefix, s_mask;
    __shared__ int s_need, s_bin_cnt, s_cnt, s_valid;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int64_t row = blockIdx.x;
    const float* srow = scores + row * ld;
    const uint32_t* irow = col_idx ? col_idx + row * ld : nullptr;  // explicit item indices (rf_topk_merge_idx)

    // previous running top-k as keys (entries with index -1 are empty), and whether it is sorted
    if (t == 0) s_unsorted = 0;
    for (int i = t; i < k_prev; i += kThreads) {
        const int64_t pidx = prev_idx[row * prev_ld + i];
        const float pv = prev_val[row * prev_ld + i];
        const bool ok = pidx >= 0 && !isnan(pv);
        pk[i] = ok ? ((uint64_t)f2key(pv) << 32) | (uint64_t)(~(uint32_t)pidx) : 0ull;
    }
    __syncthreads();
    for (int i = t; i + 1 < k_prev; i += kThreads)
        if (pk[i] < pk[i + 1]) s_unsorted = 1;
    __syncthreads();
    // a full, SORTED running top-k bounds the block: only keys above its k-th entry can enter (keys are
    // unique), so after the first blocks of a scan most rows select a handful of keys and skip the radix
    // passes. An unsorted `prev` (any set, per rf_api.h) has no cheap k-th entry: no floor then.
    const uint64_t floor_key = (k_prev >= k && !s_unsorted) ? pk[k - 1] : 0ull;
    uint64_t key[IPT];
    int nvalid = 0;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const int c = t + kThreads * j;
        const float s = c < cols ? srow[c] : __builtin_nanf("");
        const uint32_t ix = irow ? (c < cols ? irow[c] : 0u) : (uint32_t)(col_base + c);
        uint64_t kv = !isnan(s) ? ((uint64_t)f2key(s) << 32) | (uint64_t)(~ix) : 0ull;
        if (kv <= floor_key) kv = 0ull;
        key[j] = kv;
        nvalid += kv != 0ull;
    }
    // valid count (block reduction)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nvalid += __shfl_xor(nvalid, o, 64);
    if (t == 0) s_valid = 0;
    __syncthreads();
    if (lane == 0) atomicAdd(&s_valid, nvalid);
    if (t == 0) {
        s_prefix = 0;
        s_mask = 0;
        s_cnt = 0;
    }
    __syncthreads();
    const int total = s_valid;
    const int kk = min(k, total);
    if (t == 0) s_need = kk;
    __syncthreads();
    if (kk > 0 && kk < total) {
#pragma unroll 1
        for (int pass = 0; pass < 8; ++pass) {
            const int shift = 56 - 8 * pass;
            for (int i = t; i < kWavesTopk * 256; i += kThreads) (&hist[0][0])[i] = 0;
            __syncthreads();
            const uint64_t prefix = s_prefix, mask = s_mask;
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if (key[j] != 0ull && (key[j] & mask) == prefix) atomicAdd(&hist[wave][(key[j] >> shift) & 255], 1u);
            __syncthreads();
            if (t < 256) {
                uint32_t s = 0;
                for (int w = 0; w < kWavesTopk; ++w) s += hist[w][t];
                tot[t] = s;
            }
            __syncthreads();
            if (wave == 0) {
                // lane owns bins 4*(63-lane) .. +3 (lane 0 the top bins): suffix counts from the top
                uint32_t c[4], loc = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    c[q] = tot[4 * (63 - lane) + (3 - q)];  // descending bin order inside the lane
                    loc += c[q];
                }
                uint32_t incl = loc;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(incl, o, 64);
                    if (lane >= o) incl += y;
                }
                const uint32_t above = incl - loc;  // keys in bins above this lane's bins
                const int need = s_need;
                uint32_t run = above;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (run < (uint32_t)need && run + c[q] >= (uint32_t)need) {
                        const int bin = 4 * (63 - lane) + (3 - q);
                        s_prefix = prefix | ((uint64_t)bin << shift);
                        s_mask = mask | ((uint64_t)0xff << shift);
                        s_need = need - (int)run;
                        s_bin_cnt = (int)c[q];
                    }
                    run += c[q];
                }
            }
            __syncthreads();
            if (s_need == s_bin_cnt) break;  // every key of the boundary bin is selected
            __syncthreads();
        }
    }
    // select: keys whose masked bits are >= the boundary prefix (exactly kk of them)
    const uint64_t prefix = s_prefix, mask = s_mask;
    const bool all = kk >= total;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (key[j] != 0ull && (all || (key[j] & mask) >= prefix)) cand[atomicAdd(&s_cnt, 1)] = key[j];
    }
    __syncthreads();
    const int nsel = s_cnt;
    int p2n = 1;
    while (p2n < nsel) p2n <<= 1;
    for (int i = nsel + t; i < p2n; i += kThreads) cand[i] = 0ull;
    __syncthreads();
    auto emit = [&](int r, uint64_t kv) {
        float v = -INFINITY;
        int64_t idx = -1;
        if (kv != 0ull) {
            v = key2f((uint32_t)(kv >> 32));
            idx = (int64_t)(~(uint32_t)kv);
        }
        out_val[row * out_ld + r] = v;
        out_idx[row * out_ld + r] = idx;
    };
    auto bitonic = [&](uint64_t* a, int n2) {  // descending, n2 a power of two
#pragma unroll 1
        for (int size = 2; size <= n2; size <<= 1) {
#pragma unroll 1
            for (int stride = size >> 1; stride > 0; stride >>= 1) {
                for (int i = t; i < n2 / 2; i += kThreads) {
                    const int lo = 2 * i - (i & (stride - 1));
                    const int hi = lo + stride;
                    const bool desc = (lo & size) == 0;
                    const uint64_t x = a[lo], y = a[hi];
                    if ((x < y) == desc) {
                        a[lo] = y;
                        a[hi] = x;
                    }
                }
                __syncthreads();
            }
        }
    };
    if (!s_unsorted) {
        // the running top-k is sorted (this kernel writes it so): sort only the new keys, then every key's
        // output position is its index plus the number of keys above it in the other list (merge path)
        bitonic(cand, p2n);
        auto above = [](const uint64_t* a, int n, uint64_t x) {  // entries of descending a[0..n) above x
            int lo = 0, hi = n;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (a[mid] > x) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        for (int i = t; i < nsel; i += kThreads) {
            const int r = i + above(pk, k_prev, cand[i]);
            if (r < k) emit(r, cand[i]);
        }
        for (int i = t; i < k_prev; i += kThreads) {
            const int r = i + above(cand, nsel, pk[i]);
            if (r < k) emit(r, pk[i]);
        }
        for (int i = nsel + k_prev + t; i < k; i += kThreads) emit(i, 0ull);
        return;
    }
    // general case: one bitonic sort over the new keys and the running top-k
    const int m = nsel + k_prev;
    for (int i = t; i < k_prev; i += kThreads) cand[nsel + i] = pk[i];
    int p2 = 1;
    while (p2 < m) p2 <<= 1;
    for (int i = m + t; i < p2; i += kThreads) cand[i] = 0ull;
    __syncthreads();
    bitonic(cand, p2);
    for (int i = t; i < k; i += kThreads) emit(i, i < m ? cand[i] : 0ull);
}

}  // namespace

namespace {
// Exact fp32 scores of candidate (query, item) pairs in the k order of gemm_lds_kernel<..., fp32> (rf_linear_fwd's
// LDS-DMA path): per 32-k step kt, per half h, per element e, the four lane groups lg of one
// v_mfma_f32_16x16x4_f32 (k = 32 kt + 16 h + 4 lg + e). ORDER: the order of lg inside one MFMA (0: 0..3, 1: 3..0)
// — the MFMA is an fmaf chain (MI355X_MICROARCH's f32 MFMA row); tests/test_search.py pins which order
// reproduces rf_linear_fwd bit for bit. One 256-thread workgroup per query row, a thread per candidate; a wave
// takes 64 candidates at a time and streams their rows one 128-byte line (32 k) per candidate at a time through a
// double-buffered LDS image filled by LDS-DMA, 8 lanes per line (each line crosses the memory system once, as a
// whole; a lane loading its own row would touch 64 lines per 16-byte load), then each lane runs its candidate's
// fmaf chain from LDS. The LDS reads are inline asm (explicit lgkmcnt waits): hipcc would otherwise drain every
// DMA in flight (vmcnt(0)) in front of their uses.
__device__ __forceinline__ uint32_t rs_lds(const void* p) {
    return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
constexpr int kRescoreLine = 64 * 128;  // one wave's image of one 32-k line per candidate
typedef float rs_f4 __attribute__((ext_vector_type(4)));
template <int ORDER>
__global__ __launch_bounds__(256) void ip_rescore_kernel(const float* __restrict__ q, int64_t ldq, const float* __restrict__ items,
                                                         int K, const int32_t* __restrict__ count, int cap,
                                                         float* __restrict__ cval, const uint32_t* __restrict__ cidx) {
    extern __shared__ __attribute__((aligned(16))) char rs_smem[];
    float* qs = reinterpret_cast<float*>(rs_smem);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char* wbuf = rs_smem + (size_t)K * 4 + wave * 2 * kRescoreLine;
    const int64_t row = blockIdx.x;
    for (int k = threadIdx.x; k < K; k += 256) qs[k] = q[row * ldq + k];
    const int n = min(count[row], cap);
    float* cv = cval + row * (int64_t)cap;
    const uint32_t* ci = cidx + row * (int64_t)cap;
    __syncthreads();
    const int nkt = K / 32;
    const uint32_t qsl = rs_lds(qs);
    for (int g0 = wave * 64; g0 < n; g0 += 256) {  // wave-uniform
        const int c = g0 + lane;
        uint32_t my = ci[c < n ? c : g0];  // past n: any listed row (never stored)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("" : "+v"(my));
        // the line kt of the wave's 64 candidate rows into buffer b: wave-instruction g copies candidates
        // 8 g .. 8 g + 7, 8 lanes x 16 bytes each, chunk p of candidate r stored at chunk p ^ (r & 7)
        auto dma = [&](int kt, int b) __attribute__((always_inline)) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const int r = 8 * g + (lane >> 3), p = lane & 7;
                const uint32_t ix = (uint32_t)__shfl((int)my, r);
                const float* src = items + (int64_t)ix * K + kt * 32 + ((p ^ (r & 7)) << 2);
                __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(wbuf + b * kRescoreLine + g * 1024),
                                                 16, 0, 0);
            }
        };
        dma(0, 0);
        float acc = 0.f;
        for (int kt = 0; kt < nkt; ++kt) {
            if (kt + 1 < nkt) {
                dma(kt + 1, (kt + 1) & 1);  // buffer (kt + 1) & 1 was last read at kt - 1 (its reads waited for)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t vl = rs_lds(wbuf + (kt & 1) * kRescoreLine) + lane * 128;
            rs_f4 ch[8], qc[8];
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                asm volatile("ds_read_b128 %0, %1" : "=v"(ch[p]) : "v"(vl + ((p ^ (lane & 7)) << 4)));
                asm volatile("ds_read_b128 %0, %1" : "=v"(qc[p]) : "v"(qsl + kt * 128 + p * 16));
            }
            asm volatile("s_waitcnt lgkmcnt(0)");
#pragma unroll
            for (int p = 0; p < 8; ++p) asm volatile("" : "+v"(ch[p]), "+v"(qc[p]));
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int lg = ORDER ? 3 - t : t;
                        acc = __builtin_fmaf(qc[4 * h + lg][e], ch[4 * h + lg][e], acc);
                    }
        }
        if (c < n) cv[c] = acc;
    }
}
}  // namespace

extern "C" int rf_ip_rescore_f32(const float* q, int64_t ldq, int32_t M, const float* items, int32_t K,
                                 const int32_t* count, int32_t cap, float* cand_val, const uint32_t* cand_idx, int32_t order,
                                 void* stream) {
    RF_REQUIRE(M >= 0 && K >= 32 && K % 32 == 0 && K <= 8192 && ldq >= K && cap >= 1 && (order == 0 || order == 1),
               "rf_ip_rescore_f32: needs K %% 32 == 0, 32 <= K <= 8192, cap >= 1, order 0 or 1");
    if (M == 0) return RF_OK;
    RF_REQUIRE(q && items && count && cand_val && cand_idx, "rf_ip_rescore_f32: null pointer");
    RF_REQUIRE(((uintptr_t)items & 15) == 0, "rf_ip_rescore_f32: items must be 16-byte aligned");
    hipStream_t st = rf_stream(stream);
    const size_t lds = (size_t)K * sizeof(float) + 4 * 2 * kRescoreLine;
    const hipError_t e = order ? hipFuncSetAttribute(reinterpret_cast<const void*>(ip_rescore_kernel<1>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)
                               : hipFuncSetAttribute(reinterpret_cast<const void*>(ip_rescore_kernel<0>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return rf_set_error(RF_EHIP, "ip_rescore_kernel: %s", hipGetErrorString(e));
    if (order) hipLaunchKernelGGL(ip_rescore_kernel<1>, dim3((unsigned)M), dim3(256), lds, st, q, ldq, items, K, count, cap, cand_val, cand_idx);
    else hipLaunchKernelGGL(ip_rescore_kernel<0>, dim3((unsigned)M), dim3(256), lds, st, q, ldq, items, K, count, cap, cand_val, cand_idx);
    return rf_check_launch("ip_rescore_kernel");
}

namespace {
int topk_launch(const float* scores, const uint32_t* col_idx, int64_t ld, int32_t rows, int32_t cols, int32_t k,
                int64_t col_base, const float* prev_val, const int64_t* prev_idx, int32_t k_prev, int64_t prev_ld,
                float* out_val, int64_t* out_idx, int64_t out_ld, void* stream) {
    RF_REQUIRE(rows >= 0 && cols >= 0 && cols <= 32 * kThreads, "rf_topk_merge: cols must be in [0, 32768]");
    RF_REQUIRE(k >= 1 && k <= kMaxK && k_prev >= 0 && k_prev <= kMaxK, "rf_topk_merge: k and k_prev must be in [1, 1024]");
    RF_REQUIRE(ld >= cols && out_ld >= k && (k_prev == 0 || prev_ld >= k_prev), "rf_topk_merge: bad leading dimension");
    RF_REQUIRE(col_base >= 0 && col_base + cols <= ((int64_t)1 << 32) - 1, "rf_topk_merge: item index must fit 32 bits");
    if (rows == 0) return RF_OK;
    RF_REQUIRE((cols == 0 || scores) && out_val && out_idx && (k_prev == 0 || (prev_val && prev_idx)),
               "rf_topk_merge: null pointer");
    const int ipt = std::max(1, (cols + kThreads - 1) / kThreads);
    hipStream_t st = rf_stream(stream);
#define RF_TOPK(N)                                                                                                  \
    hipLaunchKernelGGL(topk_kernel<N>, dim3(rows), dim3(kThreads), 0, st, scores, ld, cols, k, col_base, prev_val, \
                       prev_idx, k_prev, prev_ld, out_val, out_idx, out_ld, col_idx)
    if (ipt <= 1) RF_TOPK(1);
    else if (ipt <= 2) RF_TOPK(2);
    else if (ipt <= 4) RF_TOPK(4);
    else if (ipt <= 8) RF_TOPK(8);
    else if (ipt <= 16) RF_TOPK(16);
    else RF_TOPK(32);
#undef RF_TOPK
    return rf_check_launch("rf_topk_merge");
}
}  // namespace

extern "C" int rf_topk_merge(const float* scores, int64_t ld, int32_t rows, int32_t cols, int32_t k, int64_t col_base,
                             const float* prev_val, const int64_t* prev_idx, int32_t k_prev, int64_t prev_ld,
                             float* out_val, int64_t* out_idx, int64_t out_ld, void* stream) {
    return topk_launch(scores, nullptr, ld, rows, cols, k, col_base, prev_val, prev_idx, k_prev, prev_ld, out_val, out_idx,
                       out_ld, stream);
}

extern "C" int rf_topk_merge_idx(const float* scores, const uint32_t* col_idx, int64_t ld, int32_t rows, int32_t cols,
                                 int32_t k, const float* prev_val, const int64_t* prev_idx, int32_t k_prev, int64_t prev_ld,
                                 float* out_val, int64_t* out_idx, int64_t out_ld, void* stream) {
    RF_REQUIRE(cols == 0 || col_idx, "rf_topk_merge_idx: null col_idx");
    return topk_launch(scores, col_idx, ld, rows, cols, k, 0, prev_val, prev_idx, k_prev, prev_ld, out_val, out_idx, out_ld,
                       stream);
}
