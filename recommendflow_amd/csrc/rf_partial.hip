// rf_partial.hip — owner-side partial pooling, the alternative exchange of the row-sharded lookup (SURVEY §8e:
// "pool partial sums at the owner and return pooled partials instead"). The default exchange ships every
// distinct row to its requester once (rf_route_hash_*); here the requester ships, for every (example, slot,
// table) unit, its positions' local rows to their owners, each owner pools the positions it owns per unit, and
// one partial vector per (unit, owner) travels back:
//
//   rf_pp_plan        requester: the unit's pooling entries in position order — (global row, unit, multiplicity);
//                     the padding positions of a unit collapse into ONE entry of multiplicity Lmax - len
//   (rf_bucketize_owner then orders them owner-major, stably, so each owner's entries stay in unit order)
//   rf_pp_heads       requester: segment heads (a new unit, or a new owner chunk) of the owner-major entries,
//                     their global segment index (= the index of the partial that comes back) and per-owner
//                     segment counts (sent with the entry counts, so one host read sizes both all-to-alls)
//   rf_pp_owner_pool  owner: one partial per segment: sum (fp32, position order, multiplicity repeats) / max /
//                     min over the segment's rows; first / last: the one row
//   rf_pp_combine     requester: per unit, the partials of owners 0 .. P-1 in that order -> the pooled output
//
// Semantics are the reference pooling (preprocess_layers.py:44-64, padding as rf_fused_hash_embed_fwd). max /
// min / first / last are exact at any P; sum / avg add each owner's partial in owner order (deviation
// D-partial-pool-order), which at P = 1 is the sequential order: bit-identical to the unsharded kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <hipcub/hipcub.hpp>

#include "rf_fused.h"

namespace {
using namespace rf;

__device__ __forceinline__ int unit_len(int comb, int len, int lm, bool mask_pad) {
    return mask_pad ? len : max(lm, len);  // positions the combiner sees (the reference pads to the batch max)
}

// number of pooling entries of a unit (no row is read: the count pass must not touch rows)
__device__ __forceinline__ int unit_count(int comb, int len, int L) {
    if (L == 0) return 0;
    if (comb == RF_COMB_FIRST || comb == RF_COMB_LAST) return 1;
    return len + (L > len ? 1 : 0);
}

// the entries of unit (b, s, k) in position order (padding collapsed into one entry of multiplicity L - len)
__device__ __forceinline__ int unit_emit(int comb, int len, int L, int t0, int k, int64_t pad_row,
                                         const int64_t* __restrict__ rows, int64_t* __restrict__ er,
                                         int32_t* __restrict__ em) {
    if (L == 0) return 0;
    if (comb == RF_COMB_FIRST || comb == RF_COMB_LAST) {
        const bool tok = comb == RF_COMB_FIRST ? len > 0 : len >= L;
        const int l = comb == RF_COMB_FIRST ? 0 : L - 1;
        er[0] = tok ? rows[2 * (int64_t)(t0 + l) + k] : pad_row;
        em[0] = 1;
        return 1;
    }
    for (int l = 0; l < len; ++l) {
        er[l] = rows[2 * (int64_t)(t0 + l) + k];
        em[l] = 1;
    }
    if (L > len) {
        er[len] = pad_row;
        em[len] = L - len;
        return len + 1;
    }
    return len;
}

__global__ __launch_bounds__(256) void pp_count_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                       const int32_t* __restrict__ bag_off,
                                                       const int32_t* __restrict__ lmax, int batch, int flags,
                                                       int32_t* __restrict__ cnt) {
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const int64_t n_units = 2 * (int64_t)batch * n_slots;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_units; u += (int64_t)gridDim.x * blockDim.x) {
        const int64_t bs = u >> 1;
        const int s = (int)(bs % n_slots);
        const int t0 = bag_off[bs], len = bag_off[bs + 1] - t0;
        const int comb = slots[s].combiner;
        const int L = unit_len(comb, len, lmax[s], mask_pad);
        cnt[u] = unit_count(comb, len, L);
    }
}

__global__ __launch_bounds__(256) void pp_emit_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                      const int32_t* __restrict__ bag_off,
                                                      const int32_t* __restrict__ lmax, int batch, int64_t n_tok,
                                                      int flags, const int64_t* __restrict__ rows,
                                                      const int32_t* __restrict__ off, int64_t* __restrict__ ent_row,
                                                      int32_t* __restrict__ ent_unit, int32_t* __restrict__ ent_mult) {
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const int64_t n_units = 2 * (int64_t)batch * n_slots;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n_units; u += (int64_t)gridDim.x * blockDim.x) {
        const int64_t bs = u >> 1;
        const int k = (int)(u & 1);
        const int s = (int)(bs % n_slots);
        const int t0 = bag_off[bs], len = bag_off[bs + 1] - t0;
        const int comb = slots[s].combiner;
        const int L = unit_len(comb, len, lmax[s], mask_pad);
        const int64_t pad = rows[2 * n_tok + 2 * (int64_t)s + k];
        const int32_t o = off[u];
        const int n = unit_emit(comb, len, L, t0, k, pad, rows, ent_row + o, ent_mult + o);
        for (int i = 0; i < n; ++i) ent_unit[o + i] = (int32_t)u;
    }
}

// segment heads over the owner-major entries: a head where the unit changes or an owner chunk starts
__global__ __launch_bounds__(256) void pp_heads_kernel(const int32_t* __restrict__ unit, int64_t n,
                                                       const int32_t* __restrict__ counts, int P,
                                                       int32_t* __restrict__ head) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        bool h = i == 0 || unit[i] != unit[i - 1];
        if (!h) {  // a chunk boundary between owners (P is small: walk the counts)
            int64_t c = 0;
            for (int p = 0; p < P && c <= i; ++p) {
                if (c == i) h = true;
                c += counts[p];
            }
        }
        head[i] = h ? 1 : 0;
    }
}

// from the inclusive scan of the heads: the segment index of each head, per-owner segment counts, and (requester)
// seg_of[unit * P + owner]; (owner) seg_start[segment]
__global__ __launch_bounds__(256) void pp_seg_kernel(const int32_t* __restrict__ unit, const int32_t* __restrict__ head,
                                                     const int32_t* __restrict__ scan, int64_t n,
                                                     const int32_t* __restrict__ counts, int P,
                                                     int32_t* __restrict__ seg_counts, int32_t* __restrict__ seg_of,
                                                     int32_t* __restrict__ seg_start) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (!head[i]) continue;
        const int seg = scan[i] - 1;
        int owner = 0;
        int64_t c = counts[0];
        while (owner + 1 < P && i >= c) c += counts[++owner];
        if (seg_of) seg_of[(int64_t)unit[i] * P + owner] = seg;
        if (seg_start) seg_start[seg] = (int32_t)i;
    }
}

// segments per owner chunk from the inclusive head scan at the chunk edges (no atomics: a counter shared by
// millions of heads serialises at the memory side)
__global__ void pp_segcount_kernel(const int32_t* __restrict__ scan, const int32_t* __restrict__ counts, int P,
                                   int32_t* __restrict__ seg_counts) {
    for (int o = threadIdx.x; o < P; o += blockDim.x) {
        int64_t start = 0;
        for (int p = 0; p < o; ++p) start += counts[p];
        const int64_t end = start + counts[o];
        seg_counts[o] = end > start ? scan[end - 1] - (start > 0 ? scan[start - 1] : 0) : 0;
    }
}

// owner: one team of LPR lanes per segment, a 16-byte chunk per lane, fp32 accumulation in entry order
template <int LPR, typename TT>
__global__ __launch_bounds__(256) void pp_owner_pool_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                            const int32_t* __restrict__ ent,  // [n][3]: local, unit, mult
                                                            int64_t n, const int32_t* __restrict__ seg_start,
                                                            int64_t n_seg, const TT* __restrict__ shard,
                                                            int64_t shard_rows, int dim, float* __restrict__ part) {
    constexpr int EPV = Elem<TT>::EPV;
    constexpr int TEAMS = 256 / LPR;
    const int team = threadIdx.x / LPR, tl = threadIdx.x % LPR;
    const int nch = dim / EPV;
    for (int64_t g = (int64_t)blockIdx.x * TEAMS + team; g < n_seg; g += (int64_t)gridDim.x * TEAMS) {
        const int64_t a = seg_start[g], e = g + 1 < n_seg ? seg_start[g + 1] : n;
        const int unit = ent[3 * a + 1];
        const int s = (int)((unit >> 1) % n_slots);
        const int comb = slots[s].combiner;
        for (int c = tl; c < nch; c += LPR) {
            float acc[EPV];
            const float init = comb == RF_COMB_MAX ? -INFINITY : comb == RF_COMB_MIN ? INFINITY : 0.0f;
#pragma unroll
            for (int q = 0; q < EPV; ++q) acc[q] = init;
            for (int64_t i = a; i < e; ++i) {
                const int64_t r = ent[3 * i];
                const int m = ent[3 * i + 2];
                float f[EPV];
                if (r >= 0 && r < shard_rows) {
                    unpack16<TT>(*reinterpret_cast<const uint4*>(shard + r * dim + (int64_t)c * EPV), f);
                } else {
#pragma unroll
                    for (int q = 0; q < EPV; ++q) f[q] = __builtin_nanf("");
                }
                if (comb == RF_COMB_SUM || comb == RF_COMB_AVG) {
                    for (int rep = 0; rep < m; ++rep)
#pragma unroll
                        for (int q = 0; q < EPV; ++q) acc[q] = __fadd_rn(acc[q], f[q]);
                } else if (comb == RF_COMB_MAX) {
#pragma unroll
                    for (int q = 0; q < EPV; ++q) acc[q] = f[q] > acc[q] ? f[q] : acc[q];
                } else if (comb == RF_COMB_MIN) {
#pragma unroll
                    for (int q = 0; q < EPV; ++q) acc[q] = f[q] < acc[q] ? f[q] : acc[q];
                } else {
#pragma unroll
                    for (int q = 0; q < EPV; ++q) acc[q] = f[q];
                }
            }
            float* dst = part + g * (int64_t)dim + (int64_t)c * EPV;
#pragma unroll
            for (int q = 0; q < EPV; ++q) dst[q] = acc[q];
        }
    }
}

// requester: unit u's partials in owner order -> out[b][out_off + k * dim]
template <typename OT>
__global__ __launch_bounds__(256) void pp_combine_kernel(const rf_slot_desc* __restrict__ slots, int n_slots,
                                                         const int32_t* __restrict__ bag_off,
                                                         const int32_t* __restrict__ lmax, int batch, int flags, int P,
                                                         const int32_t* __restrict__ seg_of,
                                                         const float* __restrict__ part, int dim, OT* __restrict__ out,
                                                         int64_t out_stride) {
    const bool mask_pad = (flags & RF_FLAG_MASK_PADDING) != 0;
    const int64_t total = 2 * (int64_t)batch * n_slots * (dim / 4);
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = x / (dim / 4);
        const int c4 = (int)(x - u * (dim / 4));
        const int64_t bs = u >> 1;
        const int k = (int)(u & 1);
        const int b = (int)(bs / n_slots), s = (int)(bs % n_slots);
        const int comb = slots[s].combiner;
        const int len = bag_off[bs + 1] - bag_off[bs];
        const int L = unit_len(comb, len, lmax[s], mask_pad);
        float a[4];
        const float init = comb == RF_COMB_MAX ? -INFINITY : comb == RF_COMB_MIN ? INFINITY : 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = init;
        for (int o = 0; o < P; ++o) {
            const int sg = seg_of[u * P + o];
            if (sg < 0) continue;
            const float4 p = *reinterpret_cast<const float4*>(part + (int64_t)sg * dim + 4 * c4);
            const float pv[4] = {p.x, p.y, p.z, p.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (comb == RF_COMB_SUM || comb == RF_COMB_AVG) a[q] = __fadd_rn(a[q], pv[q]);
                else if (comb == RF_COMB_MAX) a[q] = pv[q] > a[q] ? pv[q] : a[q];
                else if (comb == RF_COMB_MIN) a[q] = pv[q] < a[q] ? pv[q] : a[q];
                else a[q] = pv[q];
            }
        }
        if (comb == RF_COMB_AVG)
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = L == 0 ? kMeanOfNothing : a[q] / (float)L;
        if (L == 0 && mask_pad)
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = 0.0f;
        OT* dst = out + (int64_t)b * out_stride + slots[s].out_off + (int64_t)k * dim + 4 * c4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (sizeof(OT) == 4) dst[q] = a[q];
            else dst[q] = (OT)f32_to_bf16_bits(a[q]);
        }
    }
}

int grid_pp(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 32)); }

}  // namespace

extern "C" int rf_pp_plan(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                          int32_t batch, int64_t n_tok, const int64_t* rows, int32_t flags, int32_t* ent_off,
                          int64_t* ent_row, int32_t* ent_unit, int32_t* ent_mult, int32_t* n_ent, void* ws,
                          size_t ws_bytes, void* stream) {
    RF_REQUIRE(n_slots >= 1 && batch >= 0 && n_tok >= 0, "rf_pp_plan: bad sizes");
    RF_REQUIRE((flags & ~RF_FLAG_MASK_PADDING) == 0, "rf_pp_plan: only RF_FLAG_MASK_PADDING is accepted");
    const int64_t n_units = 2 * (int64_t)batch * n_slots;
    RF_REQUIRE(n_units < ((int64_t)1 << 31), "rf_pp_plan: too many units");
    hipStream_t st = rf_stream(stream);
    if (n_units == 0) {
        if (hipMemsetAsync(n_ent, 0, 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_pp_plan: memset failed");
        return RF_OK;
    }
    RF_REQUIRE(d_slots && bag_off && lmax && rows && ent_off && ent_row && ent_unit && ent_mult && n_ent && ws,
               "rf_pp_plan: null pointer");
    size_t sb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n_units + 1);
    RF_REQUIRE(ws_bytes >= sb + (size_t)(n_units + 1) * 4 + 256, "rf_pp_plan: workspace too small");
    int32_t* cnt = reinterpret_cast<int32_t*>(ws);
    void* tmp = static_cast<char*>(ws) + (((size_t)(n_units + 1) * 4 + 255) & ~(size_t)255);
    if (hipMemsetAsync(cnt + n_units, 0, 4, st) != hipSuccess) return rf_set_error(RF_EHIP, "rf_pp_plan: memset failed");
    hipLaunchKernelGGL(pp_count_kernel, dim3(grid_pp(n_units)), dim3(256), 0, st, d_slots, n_slots, bag_off, lmax, batch,
                       flags, cnt);
    if (hipcub::DeviceScan::ExclusiveSum(tmp, sb, cnt, ent_off, (int)n_units + 1, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_pp_plan: scan failed");
    if (hipMemcpyAsync(n_ent, ent_off + n_units, 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_pp_plan: copy failed");
    hipLaunchKernelGGL(pp_emit_kernel, dim3(grid_pp(n_units)), dim3(256), 0, st, d_slots, n_slots, bag_off, lmax, batch,
                       n_tok, flags, rows, ent_off, ent_row, ent_unit, ent_mult);
    return rf_check_launch("rf_pp_plan");
}

extern "C" size_t rf_pp_ws_bytes(int64_t n) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const int32_t*)nullptr, (int32_t*)nullptr, (int)std::max<int64_t>(n, 1) + 1);
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr, (int)std::max<int64_t>(n, 1));
    return std::max(a, b) + (size_t)(std::max<int64_t>(n, 1) + 1) * 8 + 512;
}

extern "C" int rf_pp_heads(const int32_t* unit, int64_t n, const int32_t* counts, int32_t nranks, int32_t* seg_counts,
                           int32_t* seg_of, int64_t n_units, int32_t* seg_start, void* ws, size_t ws_bytes,
                           void* stream) {
    RF_REQUIRE(nranks >= 1 && n >= 0, "rf_pp_heads: bad sizes");
    RF_REQUIRE(ws && ws_bytes >= rf_pp_ws_bytes(n) && counts && seg_counts, "rf_pp_heads: workspace / pointers");
    hipStream_t st = rf_stream(stream);
    if (hipMemsetAsync(seg_counts, 0, sizeof(int32_t) * nranks, st) != hipSuccess ||
        (seg_of && hipMemsetAsync(seg_of, 0xff, sizeof(int32_t) * (size_t)n_units * nranks, st) != hipSuccess))
        return rf_set_error(RF_EHIP, "rf_pp_heads: memset failed");
    if (n == 0) return RF_OK;
    RF_REQUIRE(unit, "rf_pp_heads: null pointer");
    int32_t* head = reinterpret_cast<int32_t*>(ws);
    int32_t* scan = head + ((n + 63) & ~(int64_t)63);
    void* tmp = reinterpret_cast<char*>(scan + ((n + 63) & ~(int64_t)63));
    size_t sb = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, sb, head, scan, (int)n);
    hipLaunchKernelGGL(pp_heads_kernel, dim3(grid_pp(n)), dim3(256), 0, st, unit, n, counts, nranks, head);
    if (hipcub::DeviceScan::InclusiveSum(tmp, sb, head, scan, (int)n, st) != hipSuccess)
        return rf_set_error(RF_EHIP, "rf_pp_heads: scan failed");
    hipLaunchKernelGGL(pp_seg_kernel, dim3(grid_pp(n)), dim3(256), 0, st, unit, head, scan, n, counts, nranks, seg_counts,
                       seg_of, seg_start);
    hipLaunchKernelGGL(pp_segcount_kernel, dim3(1), dim3(256), 0, st, scan, counts, nranks, seg_counts);
    return rf_check_launch("rf_pp_heads");
}

extern "C" int rf_pp_owner_pool(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* ent, int64_t n,
                                const int32_t* seg_start, int64_t n_seg, const void* shard, int32_t dtype,
                                int64_t shard_rows, int32_t dim, float* part, void* stream) {
    RF_REQUIRE(dtype == RF_DTYPE_F32 || dtype == RF_DTYPE_BF16, "rf_pp_owner_pool: dtype must be F32 or BF16");
    const int epv = dtype == RF_DTYPE_F32 ? 4 : 8;
    RF_REQUIRE(dim > 0 && dim % 8 == 0 && dim % epv == 0, "rf_pp_owner_pool: dim must be a multiple of 8");
    if (n_seg == 0) return RF_OK;
    RF_REQUIRE(d_slots && ent && seg_start && shard && part, "rf_pp_owner_pool: null pointer");
    hipStream_t st = rf_stream(stream);
    const int nch = dim / epv;
    const int lpr = nch >= 16 ? 16 : nch >= 8 ? 8 : nch >= 4 ? 4 : nch >= 2 ? 2 : 1;
    const int grid = grid_pp(n_seg * lpr);
#define RF_PP(L, T) hipLaunchKernelGGL((pp_owner_pool_kernel<L, T>), dim3(grid), dim3(256), 0, st, d_slots, n_slots, ent, n, \
                                       seg_start, n_seg, (const T*)shard, shard_rows, dim, part)
#define RF_PP_T(T) \
    switch (lpr) { case 16: RF_PP(16, T); break; case 8: RF_PP(8, T); break; case 4: RF_PP(4, T); break; \
                   case 2: RF_PP(2, T); break; default: RF_PP(1, T); break; }
    if (dtype == RF_DTYPE_F32) { RF_PP_T(float) } else { RF_PP_T(uint16_t) }
#undef RF_PP_T
#undef RF_PP
    return rf_check_launch("pp_owner_pool_kernel");
}

extern "C" int rf_pp_combine(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                             int32_t batch, int32_t flags, int32_t nranks, const int32_t* seg_of, const float* part,
                             int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, void* stream) {
    RF_REQUIRE(out_dtype == RF_DTYPE_F32 || out_dtype == RF_DTYPE_BF16, "rf_pp_combine: out dtype must be F32 or BF16");
    RF_REQUIRE(dim > 0 && dim % 4 == 0 && ((uintptr_t)part & 15) == 0, "rf_pp_combine: dim % 4 == 0, aligned partials");
    const int64_t total = 2 * (int64_t)batch * n_slots * (dim / 4);
    if (total == 0) return RF_OK;
    RF_REQUIRE(d_slots && bag_off && lmax && seg_of && out, "rf_pp_combine: null pointer");
    hipStream_t st = rf_stream(stream);
    if (out_dtype == RF_DTYPE_F32)
        hipLaunchKernelGGL(pp_combine_kernel<float>, dim3(grid_pp(total)), dim3(256), 0, st, d_slots, n_slots, bag_off,
                           lmax, batch, flags, nranks, seg_of, part, dim, (float*)out, out_stride);
    else
        hipLaunchKernelGGL(pp_combine_kernel<uint16_t>, dim3(grid_pp(total)), dim3(256), 0, st, d_slots, n_slots, bag_off,
                           lmax, batch, flags, nranks, seg_of, part, dim, (uint16_t*)out, out_stride);
    return rf_check_launch("pp_combine_kernel");
}
