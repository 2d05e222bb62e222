// rf_pool_f32.hip — pre-gathered (rf_pool_rows_fwd) instantiations of the fused kernel (rf_fused.h) for float tables.
#include "rf_fused.h"

namespace rf {

RF_FUSED_LAUNCH_DECL(launch_pool_f32) {
    return launch_fused_impl<float, true>(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table, table_rows,
                                        dim, out, out_dtype, out_stride, flags, idx_out, max_lpr, grid, st);
}

}  // namespace rf
