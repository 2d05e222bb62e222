// rf_fused_bf16.hip — instantiations of the fused kernel (rf_fused.h) for uint16_t tables.
#include "rf_fused.h"

namespace rf {

int launch_fused_bf16(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
        const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int64_t n_units, const void* table,
        int64_t table_rows, int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags,
        int64_t* idx_out, int max_lpr, int grid, hipStream_t st) {
    constexpr int epv = Elem<uint16_t>::EPV;
    return dispatch_fused(dim / epv, max_lpr, [&](auto lpr, auto cpl) -> int {
        constexpr int LPR = decltype(lpr)::value, CPL = decltype(cpl)::value;
        const bool full = dim / epv == LPR * CPL;
#define RF_FUSED_LAUNCH(FULL, OT)                                                                                  \
    hipLaunchKernelGGL((fused_hash_embed_kernel<LPR, CPL, FULL, uint16_t, OT>), dim3(grid), dim3(kWaves * 64), 0, st,  \
                       d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, (const uint16_t*)table, table_rows,    \
                       dim, (OT*)out, out_stride, flags, idx_out)
        if (out_dtype == RF_DTYPE_F32) {
            if (full) RF_FUSED_LAUNCH(true, float); else RF_FUSED_LAUNCH(false, float);
        } else {
            if (full) RF_FUSED_LAUNCH(true, uint16_t); else RF_FUSED_LAUNCH(false, uint16_t);
        }
#undef RF_FUSED_LAUNCH
        return rf_check_launch("fused_hash_embed_kernel");
    });
}

}  // namespace rf
