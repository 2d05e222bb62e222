// rf_fused_bf16_of32.hip — hashing instantiations of the fused kernel (rf_fused.h): uint16_t table, float output.
#include "rf_fused.h"

namespace rf {

RF_FUSED_LAUNCH_DECL(launch_fused_bf16_of32) {
    return launch_fused_impl<uint16_t, false, float>(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table,
                                             table_rows, dim, out, out_stride, flags, idx_out, grid, st);
}

}  // namespace rf
