// rf_pool_bf16.hip — pre-gathered (rf_pool_rows_fwd) instantiations of the fused kernel (rf_fused.h) for uint16_t tables.
#include "rf_fused.h"

namespace rf {

RF_FUSED_LAUNCH_DECL(launch_pool_bf16) {
    return launch_fused_impl<uint16_t, true>(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table, table_rows,
                                        dim, out, out_dtype, out_stride, flags, idx_out, max_lpr, grid, st);
}

}  // namespace rf
