// rf_tfr_blob.h — layout of the device schema blob (rf_tfr_schema_blob, include/rf_io.h), shared by the
// host builder (rf_io.cpp, g++) and the parse kernels (rf_tfr.hip). Plain C++: no HIP types here.
//
//   TfrBlobHdr | TfrBlobFeat[F] | int32 htab[hmask + 1] | key bytes
//
// htab is open addressing (linear probing) on tfr_key_hash(key) & hmask; a slot holds the schema index
// or -1. hmask + 1 is a power of two >= 2F, so every probe sequence reaches an empty slot.
#ifndef RF_TFR_BLOB_H
#define RF_TFR_BLOB_H

#include <stdint.h>

struct TfrBlobHdr {
    int32_t F, Sb, Si, Sf, Ni, Nf;  // features; BYTES / INT64-SEQ / FLOAT-SEQ / INT64-SCALAR / FLOAT-SCALAR counts
    int32_t hmask;                  // hash table size - 1
    int32_t names_off;              // byte offset of the key bytes from the blob start
    int64_t total_bytes;            // blob size
};

struct TfrBlobFeat {
    int32_t kind, shape, gpos;  // RF_TFR_* kind and shape, position within the feature's output group
    int32_t name_off, name_len; // key bytes at names_off + name_off
    int32_t pad;
    int64_t def_i;  // SCALAR INT64 default
    float def_f;    // SCALAR FLOAT default (as the CPU reader rounds it)
    int32_t pad2;
};

static_assert(sizeof(TfrBlobHdr) == 40, "blob header layout");
static_assert(sizeof(TfrBlobFeat) == 40, "blob feature layout");

// FNV-1a, 32 bit.
inline uint32_t tfr_key_hash_host(const uint8_t* p, uint32_t n) {
    uint32_t h = 2166136261u;
    for (uint32_t i = 0; i < n; ++i) h = (h ^ p[i]) * 16777619u;
    return h;
}

// Worst-case element counts of a batch of B records holding n_rec_bytes payload bytes (rf_io.h).
inline int64_t tfr_cap_tok(int64_t n_rec_bytes, int64_t B, int64_t Sb) { return n_rec_bytes / 2 + B * Sb; }
inline int64_t tfr_cap_ival(int64_t n_rec_bytes) { return n_rec_bytes; }
inline int64_t tfr_cap_fval(int64_t n_rec_bytes) { return n_rec_bytes / 4; }

#endif  // RF_TFR_BLOB_H
