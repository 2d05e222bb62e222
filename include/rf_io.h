/*
 * rf_io.h — host-side feature pipe of librf.so: TFRecord(GZIP) files <-> batched CSR.
 *
 * Replaces the reference's input pipeline for the hot path:
 *   writer  utils/make_tfrecord.py:26-41 (tf.train.Feature builders), :108-119 (tf.train.Example),
 *           :139-144 (tf.io.TFRecordWriter(out_file, "GZIP"))
 *   reader  backend/core/dataloader.py:23-44 (build_feature_description), :77-89 (parse_example),
 *           :541-578 (TFRecordDataset(compression_type, num_parallel_reads=thread_num).batch(B))
 *
 * The reader yields exactly what parse_example hands the model, minus the padding: every
 * FixedLenSequenceFeature(allow_missing=True) becomes a batched-CSR slot whose padded width
 * (the batch max list length, dataloader.py:32-33) is lmax[s]; FixedLenFeature(()) becomes a
 * dense [B][n] column block with the feature's default where the key is missing. The bytes
 * CSR is byte-for-byte the input of rf_fused_hash_embed_fwd (rf_api.h).
 *
 * Conventions (as rf_api.h): caller-owned buffers (here HOST buffers — pinned ones, so the
 * caller can stream them to HBM on a side HIP stream), RF_OK or a negative RF_E* code,
 * rf_last_error() for the message, no C++ exceptions across the boundary. Reader/writer
 * handles are opaque and owned by the caller (close them); a handle is not thread-safe,
 * distinct handles are. The reader uses its own worker threads (decompression per open file,
 * parsing per example range).
 */
#ifndef RF_IO_H
#define RF_IO_H

#include <stddef.h>
#include <stdint.h>

#include "rf_api.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RF_EDATA (-4)  /* corrupt or truncated TFRecord / malformed tf.train.Example (TF: DataLossError) */
#define RF_ENOSPC (-5) /* an output capacity is too small; the needed sizes are in rf_tfr_columns.n_*;
                          rf_tfr_next_batch keeps the batch pending so a retry with larger buffers
                          returns the same examples */
#define RF_EIO (-6)    /* open/read/write of a file failed */

/* compression_type of TFRecordDataset / TFRecordWriter */
#define RF_TFR_NONE 0
#define RF_TFR_GZIP 1

/* tf.train.Feature kinds (feature.proto: bytes_list = 1, float_list = 2, int64_list = 3) */
#define RF_TFR_BYTES 0
#define RF_TFR_INT64 1
#define RF_TFR_FLOAT 2

/* parse shapes (dataloader.py:29-43) */
#define RF_TFR_SEQ 0    /* FixedLenSequenceFeature(shape=(), allow_missing=True): list, missing -> [] */
#define RF_TFR_SCALAR 1 /* FixedLenFeature(shape=()): exactly one value, missing -> default */

/* One entry of the feature description (build_feature_description, dataloader.py:23-44). */
typedef struct rf_tfr_feature {
    const char* name; /* tf.train.Features map key (NUL-terminated) */
    int32_t kind;     /* RF_TFR_BYTES / INT64 / FLOAT */
    int32_t shape;    /* RF_TFR_SEQ / RF_TFR_SCALAR */
    int64_t default_i; /* SCALAR INT64 default (DEFAULT_MAP, config_proto.py:42: 0) */
    double default_f;  /* SCALAR FLOAT default (0.0); SCALAR BYTES default is always b"" */
} rf_tfr_feature;      /* 32 bytes */

/*
 * Column buffers of one batch (host memory). Features are grouped by kind, each group in
 * schema order:
 *   BYTES (SEQ and SCALAR; a SCALAR bytes feature is a slot with exactly one token):
 *       tok_bytes/tok_off/bag_off[B*Sb+1]/lmax[Sb]  — example-major batched CSR (runtime/batch.py)
 *   INT64 SEQ:   ival / ibag_off[B*Si+1] / ilmax[Si]
 *   FLOAT SEQ:   fval / fbag_off[B*Sf+1] / flmax[Sf]
 *   INT64 SCALAR iscalar[B][Ni], FLOAT SCALAR fscalar[B][Nf]
 * Pointers of an empty group may be NULL. *_cap are element capacities (inputs); n_* are the
 * element counts written (outputs; on RF_ENOSPC the counts needed).
 */
typedef struct rf_tfr_columns {
    uint8_t* tok_bytes;
    int32_t* tok_off;
    int32_t* bag_off;
    int32_t* lmax;
    int64_t* ival;
    int32_t* ibag_off;
    int32_t* ilmax;
    float* fval;
    int32_t* fbag_off;
    int32_t* flmax;
    int64_t* iscalar;
    float* fscalar;
    int64_t tok_bytes_cap, tok_cap, ival_cap, fval_cap;
    int64_t n_tok_bytes, n_tok, n_ival, n_fval;
    int32_t batch;    /* examples in this batch (output of rf_tfr_next_batch; input of encode) */
    int32_t reserved; /* must be 0 */
} rf_tfr_columns;

/* ---- checksums (TFRecord framing uses CRC-32C, masked) ------------------------------ */
/* CRC-32C (Castagnoli, reflected 0x82F63B78) of data, continuing from crc (0 to start). */
uint32_t rf_crc32c(uint32_t crc, const void* data, size_t n);
/* TFRecord mask: ((c >> 15) | (c << 17)) + 0xa282ead8 of c = crc32c(data). */
uint32_t rf_crc32c_masked(const void* data, size_t n);

/* ---- writer: tf.io.TFRecordWriter(path, compression) (make_tfrecord.py:142) ---------- */
/* level: zlib level 0-9 or -1 for the default; ignored for RF_TFR_NONE. */
int rf_tfw_open(const char* path, int32_t compression, int32_t level, void** out_writer);
/* Frames one record: u64 length, masked crc32c(length), payload, masked crc32c(payload). */
int rf_tfw_write(void* writer, const void* record, int64_t len);
/* Flushes (finishes the gzip member) and frees the handle; RF_EIO if any write failed. */
int rf_tfw_close(void* writer);

/*
 * Serialises cols.batch examples as tf.train.Example records (build_tfrecord,
 * make_tfrecord.py:94-119): one Features map entry per schema feature, in schema order; SEQ
 * features whose list is empty are written as an empty list of their kind (the writer's
 * "-1" -> [b""] rule for strings is applied above this call, by the Python builder).
 * Records are concatenated into out[0..*needed) with record i at [rec_off[i], rec_off[i+1]).
 */
int rf_tfr_encode_examples(const rf_tfr_feature* feats, int32_t n_feats, const rf_tfr_columns* cols,
                           uint8_t* out, int64_t out_cap, int64_t* rec_off, int64_t* needed);

/* ---- reader: TFRecordDataset(...).batch(B).map(parse_example) (dataloader.py:541-578) ---- */
/*
 * Opens n_paths files. Records are interleaved like tf.data's deterministic parallel interleave
 * with cycle_length = min(n_threads, n_paths) and block_length = 1: one record from each open
 * file in turn; an exhausted file is replaced, in its cycle position, by the next unopened path.
 * n_threads also sizes the parse pool. n_threads = 1 reads the files back to back.
 */
int rf_tfr_open(const char* const* paths, int32_t n_paths, int32_t compression, int32_t n_threads,
                void** out_reader);
/*
 * Reads up to `batch` records and parses them into `cols` (drop_remainder=False: the last batch
 * may be short; cols->batch = 0 at end of data). Parse errors (type mismatch, a SCALAR with
 * other than one value, malformed protobuf) return RF_EDATA naming the record and key.
 */
int rf_tfr_next_batch(void* reader, const rf_tfr_feature* feats, int32_t n_feats, int32_t batch,
                      rf_tfr_columns* cols);
/* Records handed out so far (for diagnostics and tests). */
int64_t rf_tfr_records_read(void* reader);
int rf_tfr_close(void* reader);

/* ---- device parse: the same batch, parsed on the GPU ------------------------------------------ */
/*
 * Host half. Frames (and CRC-checks) the next `batch` records in the same interleave order as
 * rf_tfr_next_batch and packs their serialized tf.train.Example payloads back to back into `out`
 * (a pinned host buffer, so it can be streamed to HBM): record i = out[rec_off[i], rec_off[i+1]),
 * rec_off has batch+1 entries. *n_records = records packed (0 at end of data), *n_bytes =
 * rec_off[*n_records]. RF_ENOSPC if out_cap < the payload bytes (*n_bytes = bytes needed; the
 * records stay pending, so a retry with a larger buffer returns them).
 */
int rf_tfr_next_records(void* reader, int32_t batch, uint8_t* out, int64_t out_cap, int64_t* rec_off,
                        int32_t* n_records, int64_t* n_bytes);

/*
 * Device schema: the feature description compiled into one flat blob (names, kinds, group
 * positions, defaults and an open-addressing hash of the keys) that the parse kernels read from
 * HBM. rf_tfr_schema_blob writes it to a host buffer (the caller copies it to device memory once);
 * *needed = its size. RF_EINVAL for a schema the CPU reader also rejects (bad kind/shape,
 * duplicate name).
 */
int rf_tfr_schema_blob(const rf_tfr_feature* feats, int32_t n_feats, void* out, int64_t out_cap, int64_t* needed);

/* Written by rf_tfr_parse_device (device memory), read back by the host (rf_tfr_device_check). */
typedef struct rf_tfr_dev_stats {
    int64_t n_tok_bytes, n_tok, n_ival, n_fval; /* as rf_tfr_columns.n_* */
    int32_t err_b;    /* first failing batch position, or INT32_MAX when the batch parsed */
    int32_t err_type; /* 1 malformed Example, 2 kind mismatch, 3 malformed list, 4 SCALAR value count */
    int32_t err_feat; /* schema index of the failing key (types 2-4) */
    int32_t err_kind; /* type 2: the kind found */
    int64_t err_count; /* type 4: the value count found */
    int64_t reserved;
} rf_tfr_dev_stats; /* 64 bytes */

/* Device scratch rf_tfr_parse_device needs for a batch of B examples (bytes). */
int64_t rf_tfr_device_workspace_bytes(const void* schema_blob_host, int32_t batch);

/*
 * Device half: parses B packed records (`rec`, `rec_off[B+1]`, both DEVICE memory; `rec` readable
 * up to rec_off[B] + 16 bytes) into `cols`, whose pointers are DEVICE buffers with the layout of
 * rf_tfr_columns — the same values, offsets and lmax as rf_tfr_next_batch on the same records.
 * n_rec_bytes = rec_off[B] and max_rec_bytes = the longest record (host copies; the latter sizes the
 * per-record LDS staging, records that do not fit are parsed straight from HBM). Capacities must cover the worst case those bytes allow:
 * tok_bytes_cap >= n_rec_bytes, tok_cap >= n_rec_bytes / 2 + B * Sb, ival_cap >= n_rec_bytes,
 * fval_cap >= n_rec_bytes / 4 (RF_ENOSPC otherwise); tok_off needs tok_cap + 1 entries.
 * Stream-ordered and asynchronous: totals, lmax and the first parse error land in `stats` and
 * `cols->lmax/ilmax/flmax` (device); nothing else is written when the batch has an error. cols->n_*
 * and cols->batch are not written (read them from stats after the stream reaches this point).
 */
int rf_tfr_parse_device(const void* schema_blob_dev, const void* schema_blob_host, const uint8_t* rec,
                        const int64_t* rec_off, int32_t batch, int64_t n_rec_bytes, int64_t max_rec_bytes,
                        const rf_tfr_columns* cols,
                        rf_tfr_dev_stats* stats, void* workspace, int64_t workspace_bytes, void* stream);

/*
 * RF_OK when the stats (copied to the host) report no error; otherwise RF_EDATA with the message
 * rf_tfr_next_batch gives for the same record (first_record = records handed out before this batch).
 */
int rf_tfr_device_check(const rf_tfr_dev_stats* stats, const rf_tfr_feature* feats, int32_t n_feats,
                        int64_t first_record);

#ifdef __cplusplus
}
#endif
#endif /* RF_IO_H */
