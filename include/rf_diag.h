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

/* rf_esim_gather_fwd (rf_api.h) with per-phase shader-clock stamps (d = 128, 97 <= L <= 112 only): for every
 * workgroup g, wave w < 4 and the workgroup's k-th example (k < stamp_ex; later ones overwrite the last slot),
 * stamps[((g * 4 + w) * stamp_ex + k) * 10 + p] = low 32 bits of s_memtime at point p:
 *   0 loop top, 1 next rows' loads issued, 7 scores done, 8 softmax done, 9 side 0 done, 2 compute done,
 *   3 after the compute barrier, 4 next images written, 5 pooled features reduced, 6 after the second barrier.
 * The grid is min(batch, 2 x CUs) workgroups: size stamps for that. Same results as rf_esim_gather_fwd. */
int rf_diag_esim_gather_stamped(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows,
                                const void* a_table, int64_t a_rows, int32_t dtype, int32_t batch, int32_t L, int32_t d,
                                float* out, int64_t out_stride, int64_t out_off, uint32_t* stamps, int32_t stamp_ex,
                                void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RF_DIAG_H */
