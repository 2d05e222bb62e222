// rf_fused_f32.hip — hashing instantiations of the fused kernel (rf_fused.h) for float tables.
#include "rf_fused.h"

namespace rf {

RF_FUSED_LAUNCH_DECL(launch_fused_f32) {
    return launch_fused_impl<float, false>(d_slots, n_slots, tok_bytes, tok_off, bag_off, lmax, n_units, table, table_rows,
                                        dim, out, out_dtype, out_stride, flags, idx_out, max_lpr, grid, st);
}

}  // namespace rf
