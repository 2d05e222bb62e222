// rf_single.hip — the single-token fused kernel (rf_fused.h, RF_FLAG_SINGLE_TOKEN) for every (table dtype,
// output dtype) pair, in its own translation unit (parallel build).
#include "rf_fused.h"

namespace rf {

int launch_single_token_any(int32_t table_dtype, int32_t out_dtype, const rf_slot_desc* d_slots, int32_t n_slots,
                            const uint8_t* tok_bytes, const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                            int64_t n_units, const void* table, int64_t table_rows, int32_t dim, void* out,
                            int64_t out_stride, int32_t flags, int grid, hipStream_t st) {
    const bool tf = table_dtype == RF_DTYPE_F32, of = out_dtype == RF_DTYPE_F32;
    auto* fn = tf ? (of ? launch_single_token<float, float> : launch_single_token<float, uint16_t>)
                  : (of ? launch_single_token<uint16_t, float> : launch_single_token<uint16_t, uint16_t>);
    return fn(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table, table_rows, dim, out, out_stride, flags,
              grid, st);
}

}  // namespace rf
