// rf_pool_bf16_of32.hip — pre-gathered (rf_pool_rows_fwd) instantiations of the fused kernel (rf_fused.h): uint16_t table, float output.
#include "rf_fused.h"

namespace rf {

RF_FUSED_LAUNCH_DECL(launch_pool_bf16_of32) {
    return launch_fused_impl<uint16_t, true, float>(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table,
                                             table_rows, dim, out, out_stride, flags, idx_out, grid, st);
}

}  // namespace rf
