/*
 * rf_diag.h — diagnostic entry points of librf.so for tools/ (ablation microbenchmarks). NOT part of the
 * production ABI (rf_api.h): a caller of the reference path never needs these, and they can return
 * results that differ from the reference on purpose.
 */
#ifndef RF_DIAG_H
#define RF_DIAG_H

#include "rf_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Ablation bits accepted ONLY here (they change results):
 *   RF_DIAG_NO_HASH  (bit 12) rows come from a synthetic index instead of SipHash (gather/pool cost alone)
 *   RF_DIAG_NO_POOL  (bit 13) hash + bucket only, no row loads (hash cost alone)
 *   RF_DIAG_NO_PAD   (bit 14) padded positions are skipped (padding cost)                             */
#define RF_DIAG_NO_HASH 0x1000
#define RF_DIAG_NO_POOL 0x2000
#define RF_DIAG_NO_PAD 0x4000

/* Same arguments and conventions as rf_fused_hash_embed_fwd (rf_api.h), flags additionally 0x1000-0x4000. */
int rf_diag_fused_hash_embed_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                 const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                                 const void* table, int32_t table_dtype, int64_t table_rows, int32_t dim, void* out,
                                 int32_t out_dtype, int64_t out_stride, int32_t flags, int64_t* idx_out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RF_DIAG_H */
