/*
 * rf_api.h — C ABI of the MI355X-native RecommendFlow hot path (librf.so).
 *
 * The reference (mechsihao/RecommendFlow) has no native boundary: its hot path is
 * Keras operators. Each entry point below replaces one reference operator; the
 * operator it replaces is cited next to it (paths relative to the reference root).
 * The Python mirror of the reference operator API (recommendflow_amd/backend/...)
 * is the only in-tree caller; INTEGRATION.md shows the ctypes binding.
 *
 * Conventions
 *  - All data pointers are caller-owned DEVICE buffers (hipMalloc / torch CUDA
 *    tensors). The library allocates nothing, frees nothing, never synchronises.
 *  - `stream` is a hipStream_t passed as void* (0 = default stream). All work is
 *    stream-ordered and asynchronous; entry points are reentrant.
 *  - Return value: RF_OK (0) or a negative RF_E* code; rf_last_error() returns a
 *    thread-local message for the last failing call on this thread.
 *  - Table rows are row-major [rows][dim], element type RF_DTYPE_*.
 *  - No C++ exceptions cross this boundary.
 */
#ifndef RF_API_H
#define RF_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RF_ABI_VERSION 1

/* error codes */
#define RF_OK 0
#define RF_EINVAL (-1) /* bad argument (shape, dtype, combiner, alignment) */
#define RF_EHIP (-2)   /* a HIP runtime call failed (launch error) */
#define RF_EOOB (-3)   /* a computed row index falls outside the table */

/* element types */
#define RF_DTYPE_F32 0
#define RF_DTYPE_BF16 1
#define RF_DTYPE_F16 2

/* pooling combiners, EmbeddingBag.get_combiner (backend/layers/preprocess_layers.py:44-64) */
#define RF_COMB_SUM 0
#define RF_COMB_AVG 1
#define RF_COMB_MAX 2
#define RF_COMB_MIN 3
#define RF_COMB_FIRST 4 /* position 0 of each example (deviation D-first-last; `cls` aliases it) */
#define RF_COMB_LAST 5  /* position Lmax-1 of each example (deviation D-first-last) */
#define RF_COMB_NULL 6  /* no pooling: [Lmax, D] per table, concatenated along the sequence axis */

/* flags for rf_fused_hash_embed_fwd */
#define RF_FLAG_MASK_PADDING 0x1 /* exclude padding positions (mask_zero intent); default OFF = reference parity:
                                    padded positions gather row 0 and count in sum/avg/max/min
                                    (dataloader.py:32-33 pads with b"" which Hashing maps to bin 0) */
#define RF_FLAG_EMIT_IDX 0x2     /* also write the two bucket ids of every token to idx_out[2*t + k] */
#define RF_FLAG_SINGLE_TOKEN 0x4 /* the caller knows every slot's batch Lmax is <= 1 (single-valued slots, e.g.
                                    cfg3): a low-register single-token kernel runs (same values); a slot whose
                                    lmax is > 1 is then written as NaN. Not with RF_FLAG_EMIT_IDX. */
#define RF_FLAG_TREE_REDUCE 0x10  /* embedding backward only (rf_fused_hash_embed_bwd / _bwd_reduce): rows with more than
                                    256 positions are summed as fixed-order partials + a pairwise tree (deterministic,
                                    within SURVEY 8d's |d| <= L 2^-23 sum|x|) instead of the reference's CPU order */
#define RF_FLAG_SPEC_ROWS 0x20  /* rf_single_token_ids_fwd / _multi_fwd only: the NaN row is id table_rows and the zero
                                   row table_rows + 1 (rows the caller keeps right after the table, as rf_esim_gather_fwd
                                   reads them) instead of 0xfffffffe / 0xffffffff */
#define RF_FLAG_DIAG_XCD_ORDER 0x0800      /* A/B switch: slot-interleaved XCD item order (measured slower); results identical */
#define RF_FLAG_DIAG_GENERAL_PHASE2 0x8000 /* A/B switch: force the general pooling path for Lmax = 1 slots; results identical */
/* Only these two result-preserving switches are accepted here; any other bit returns RF_EINVAL. Bits 12-14
   are ablations that CHANGE results (synthetic rows instead of the hash, no pooling, no padding) and are
   accepted only by rf_diag_fused_hash_embed_fwd (include/rf_diag.h, tools only, not part of this ABI). */

/*
 * One hashed feature ("slot") of a fused multi-slot table.
 * Reference: DoubleHashingEmbedding.__init__ (backend/layers/preprocess_layers.py:82-92) builds
 * two Keras Hashing layers (salt seeds[0], seeds[1]) and two Embedding tables of num_bins rows;
 * here the two tables are two segments [row_base[k], row_base[k] + num_bins) of ONE fused table.
 */
typedef struct rf_slot_desc {
    int64_t row_base[2]; /* first fused-table row of table k (k = 0: seeds[0], k = 1: seeds[1]) */
    int64_t num_bins;    /* Keras Hashing num_bins (>= 1) */
    uint64_t salt[2];    /* SipHash key for table k is (salt[k], salt[k]) (Keras Hashing int salt) */
    int64_t out_off;     /* element offset of this slot's [2*D] (or [2*Lmax*D] for NULL) in an output row */
    int32_t dim;         /* embedding dim D (must equal the launch's dim) */
    int32_t combiner;    /* RF_COMB_* */
    int32_t mask_empty;  /* 1: Hashing(mask_value="") — b"" -> bin 0, others 1 + h mod (N-1) */
    int32_t reserved;    /* must be 0 */
} rf_slot_desc;          /* 64 bytes */

/* ---- version / errors ------------------------------------------------------------- */
int32_t rf_abi_version(void);
const char* rf_last_error(void);

/*
 * Keras Hashing(num_bins, mask_value="" | None, salt=s) over a batch of byte strings.
 * Replaces: tf.keras.layers.Hashing -> tf.strings.to_hash_bucket_strong, called at
 * backend/layers/preprocess_layers.py:89-90,95.
 * tokens: tok_bytes[tok_off[t] .. tok_off[t+1]) for t in [0, n_tok); out: int64 [n_tok].
 * bucket = mask_empty && len == 0 ? 0
 *        : mask_empty && num_bins > 1 ? 1 + SipHash24((k0,k1), tok) mod (num_bins - 1)
 *        : SipHash24((k0,k1), tok) mod num_bins
 */
int rf_siphash_bucket(const uint8_t* tok_bytes, const int32_t* tok_off, int64_t n_tok, uint64_t k0,
                      uint64_t k1, int64_t num_bins, int32_t mask_empty, int64_t* out, void* stream);

/*
 * Fused multi-slot  hash -> gather -> pool -> concat  (one launch for every slot of a tower).
 * Replaces, per hashing feature f of get_preprocess_layers (backend/utils/preprocess_utils.py:7-20):
 *   DoubleHashingEmbedding.call (preprocess_layers.py:94-97) = Hashing x2 -> EmbeddingBag x2
 *   (Embedding gather :67 + combiner :44-64) -> tf.concat(axis=1) :97,
 * over the padded [B, Lmax_f] string tensor produced by parse_example (dataloader.py:32-33,86).
 *
 * Input batch (CSR, example-major):
 *   bag_off[b*n_slots + s] .. bag_off[b*n_slots + s + 1]  token range of (example b, slot s)
 *   tok_off[t] .. tok_off[t+1]                             byte range of token t in tok_bytes
 *   lmax[s]                                                batch max list length of slot s (Lmax_f)
 * d_slots: DEVICE array of n_slots rf_slot_desc, all with .dim == dim.
 * table: fused [table_rows][dim] (table_dtype F32 or BF16).
 * out: [batch][out_stride] (out_dtype F32 or BF16); slot s writes
 *   out[b, out_off + k*dim + d]          (k = 0,1; pooled combiners)
 *   out[b, out_off + (k*Lmax + l)*dim + d] (RF_COMB_NULL)
 * Accumulation is fp32, sequential over positions l = 0 .. Lmax-1 (deterministic).
 * idx_out (optional, RF_FLAG_EMIT_IDX): int64 [n_tok][2] bucket ids (before row_base).
 */
int rf_fused_hash_embed_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                            const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax,
                            int32_t batch, const void* table, int32_t table_dtype, int64_t table_rows,
                            int32_t dim, void* out, int32_t out_dtype, int64_t out_stride, int32_t flags,
                            int64_t* idx_out, void* stream);

/*
 * EmbeddingBag over dense integer ids [batch][len] (every position pooled, as Keras does).
 * Replaces: EmbeddingBag.call (backend/layers/preprocess_layers.py:66-68) when its input ids come
 * from StringLookup/IntegerLookup/Discretization (LookupEmbedding :157-160, DiscreteEmbedding :189-191).
 * ids are rows of `table` (row_base added); out [batch][out_stride] at out_off (pooled: D
 * elements; NULL: len*D elements).
 */
int rf_embedding_bag_fwd(const int64_t* ids, int32_t batch, int32_t len, int64_t row_base,
                         const void* table, int32_t table_dtype, int64_t table_rows, int32_t dim,
                         int32_t combiner, void* out, int32_t out_dtype, int64_t out_stride,
                         int64_t out_off, void* stream);

/*
 * Counter-based table init, identical for any sharding: fused global row g = row0 + r*row_stride
 *   T[r][d] = lo + (hi - lo) * ((splitmix64(seed ^ (g*dim + d)) >> 40) * 2^-24)
 * (Keras Embedding 'uniform' initializer is U(-0.05, 0.05), preprocess_layers.py:24,31-39).
 */
int rf_table_init_uniform(void* table, int32_t dtype, int64_t rows, int32_t dim, int64_t row0,
                          int64_t row_stride, uint64_t seed, float lo, float hi, void* stream);

/*
 * ESIM local inference + composition pooling, one fused launch.
 * Replaces: SoftAttention.__call__ (backend/layers/attention_layers.py:15-30, _attention :33-47,
 * _soft_alignment :56-74) followed by the Esim.call combine (models/ranking/esim.py:79-84):
 *   E[i,j]   = sum_k a[i,k] q[j,k]           (x0 = q, x1 = a; [L1, L0])
 *   S        = softmax_j(E)                  (max-subtracted, fp32)
 *   att_q    = S @ q,  att_a = S @ a         (L0 == L1 == L)
 *   m_q      = [q; att_q; q-att_q; q*att_q] (4L rows), m_a likewise
 *   pooled   = [avg(m_q), max(m_q), avg(m_a), max(m_a), avg_q-avg_a, max_q-max_a]   [6d]
 * q, a: [batch][L][d] (dtype BF16 or F16), row stride ld (elements) between positions, example
 * stride ex_stride (elements). out: F32 [batch][out_stride], pooled written at out_off.
 * Optional att_out (F32 [batch][2][L][d], may be NULL): att_q then att_a, for tests.
 * Constraints: 1 <= L <= 128, d in {64, 128}.
 * The max statistic uses IEEE maximum (a NaN element propagates; DESIGN D-esim-max-nan). Without att_out
 * the 4-wave two-per-CU kernel runs; with it, the 8-wave one.
 */
int rf_esim_soft_attention_fwd(const void* q, const void* a, int32_t dtype, int32_t batch, int32_t L,
                               int32_t d, int64_t ex_stride, int64_t ld, float* out, int64_t out_stride,
                               int64_t out_off, float* att_out, void* stream);
/* rf_esim_soft_attention_fwd over pairs built by index instead of copies (the cascade's rank stage, cfg5): pair e
 * reads its q sequence at q + (e / q_rep) * q_stride (one user's sequence for q_rep consecutive candidates) and its
 * a sequence at a + a_rows[e] * a_stride (a candidate item's row of a catalog of encoded sequences); rows ld apart
 * inside an example. Same pooled values as expanding / gathering q and a first. a_count = the catalog's row count:
 * a_rows[e] outside [0, a_count) is checked on the device, reads nothing and gives pair e NaN features. */
int rf_esim_soft_attention_idx_fwd(const void* q, int32_t q_rep, const void* a, const int64_t* a_rows, int64_t a_count,
                                   int64_t a_stride,
                                   int32_t dtype, int32_t batch, int32_t L, int32_t d, int64_t q_stride, int64_t ld,
                                   float* out, int64_t out_stride, int64_t out_off, void* stream);

/*
 * Exact-fp32 GEMM of the DSSM towers, forward and training step (models/matching/dssm.py:25-26 create_mlp(...,
 * "selu", BatchNormalization) -> backend/blocks/mlp.py:4-15 Dense; its gradients under model.fit,
 * example/ranking_search/train.py:96-104): C[m][n] = act(sum_k A(m, k) B(k, n) + bias[n]), f32 products and f32
 * accumulation (v_mfma_f32_16x16x4_f32), every operand layout the towers need:
 *   a_kc = 1: A(m, k) = A[m lda + k] (k contiguous)      a_kc = 0: A(m, k) = A[k lda + m]
 *   b_kc = 1: B(k, n) = B[n ldb + k] (k contiguous)      b_kc = 0: B(k, n) = B[k ldb + n]
 * forward y = x W^T: (a_kc, b_kc) = (1, 1); weight gradient G = dpre^T h: (0, 0); input gradient dz = dpre W: (1, 0).
 * bias may be NULL; act an elementwise RF_ACT_*. Requirements: K, lda, ldb multiples of 4, A and B 16-byte
 * aligned, a k-contiguous operand's 128-row block and an m/n-contiguous operand's K + 64 rows below 2 GiB.
 * Stream-K over one persistent workgroup per CU: a 128 x 128 tile cut between workgroups is summed by the last to
 * finish in k order, so the result is the same bits every launch. ws: rf_gemm_f32_ws_bytes(M, N, K) bytes; its
 * first 4 ceil(M / 128) ceil(N / 128) bytes (rounded up to 256) are per-tile counters that must be ZERO before the
 * first call on a ws; every call leaves them zero. One zeroed ws serves calls of every shape it is large enough for
 * (the partial tiles sit at its far end); one stream at a time. Replaces the tower Dense's MatMul / BiasAdd / Selu
 * and the two MatMuls of its gradient.
 */
size_t rf_gemm_f32_ws_bytes(int64_t M, int64_t N, int64_t K);
int rf_gemm_f32(const float* A, int64_t lda, int32_t a_kc, const float* B, int64_t ldb, int32_t b_kc, int64_t M, int64_t N,
                int64_t K, const float* bias, int32_t act, float* C, int64_t ldc, void* ws, size_t ws_bytes, void* stream);
/* rf_gemm_f32_grouped: 1..4 independent GEMMs of one operand layout in ONE launch (the same layer of both DSSM
 * towers: their tiles share the stream-K grid, so two small GEMMs fill the chip that one would leave idle). probs is
 * a HOST array; per problem the rf_gemm_f32 fields and requirements; ws: rf_gemm_f32_grouped_ws_bytes(probs, n). */
typedef struct rf_gemm_f32_problem {
    const float* A;
    int64_t lda;
    const float* B;
    int64_t ldb;
    float* C;
    int64_t ldc;
    const float* bias;
    int64_t M, N, K;
    int32_t act;
    int32_t reserved; /* 0 */
} rf_gemm_f32_problem;
size_t rf_gemm_f32_grouped_ws_bytes(const rf_gemm_f32_problem* probs, int32_t n);
int rf_gemm_f32_grouped(const rf_gemm_f32_problem* probs, int32_t n, int32_t a_kc, int32_t b_kc, void* ws, size_t ws_bytes,
                        void* stream);

/*
 * DSSM tower training (models/matching/dssm.py:25-26: create_mlp([1024, 512, 256], 0.3, "selu",
 * BatchNormalization(1e-6)) per tower, trained by model.fit, example/ranking_search/train.py:96-104). All F32.
 * A layer's BatchNormalization in training mode (batch statistics; Keras tf.nn.moments, biased variance) folds
 * into its Dense: W' = W diag(a), b' = b + W c, a = gamma / sqrt(var + eps), c = beta - mean a, so the forward
 * GEMM (rf_linear_fwd / rf_linear_splitk_fwd with RF_ACT_SELU) reads the raw activations.
 *   rf_col_stats         mean[K], var[K] of x [M][K] over the M rows (deterministic: fixed row chunks, per-chunk
 *                        pivot, Chan's combine in chunk order)
 *   rf_bn_fold           W' [N][K], b' [N] as above (b may be NULL)
 *   rf_dropout_fwd       y = x / (1 - rate) where kept, 0 elsewhere; keep(r, c) = top 24 bits of
 *                        splitmix64(seed ^ (r * N + c)) / 2^24 >= rate (Keras Dropout(rate) in training; the mask
 *                        is recomputed in the backward, never stored); y may alias x (same strides)
 *   rf_selu_dropout_bwd  dpre = dh * keep / (1 - rate) * SeluGrad(y) with y = h (1 - rate) the activation
 *                        (h = the layer's dropout output), db[N] = column sums of dpre
 *   rf_bn_fold_grad      dW = G diag(a) + db c^T for G = dpre^T x (the Dense weight's gradient)
 *   rf_bn_bwd            dgamma = sum(dz xhat), dbeta = sum(dz), dx = gamma rstd (dz - dbeta / M - xhat dgamma / M)
 * Column sums reduce fixed row chunks in chunk order (replay-deterministic). ws: rf_tower_ws_bytes(M, K) bytes
 * (K = the reduced width). M <= 65535.
 */
size_t rf_tower_ws_bytes(int64_t M, int32_t K);
int rf_col_stats(const float* x, int64_t M, int32_t K, int64_t ldx, float* mean, float* var, void* ws, size_t ws_bytes,
                 void* stream);
int rf_bn_fold(const float* W, int32_t N, int32_t K, const float* b, const float* gamma, const float* beta,
               const float* mean, const float* var, float eps, float* W_out, float* b_out, void* stream);
int rf_dropout_fwd(const float* x, int64_t M, int32_t N, int64_t ldx, float rate, uint64_t seed, float* y, int64_t ldy,
                   void* stream);
int rf_selu_dropout_bwd(const float* dh, int64_t lddh, const float* h, int64_t ldh, int64_t M, int32_t N, float rate,
                        uint64_t seed, float* dpre, int64_t ldd, float* db, void* ws, size_t ws_bytes, void* stream);
int rf_bn_fold_grad(const float* G, int32_t N, int32_t K, const float* db, const float* gamma, const float* beta,
                    const float* mean, const float* var, float eps, float* dW, void* stream);
int rf_bn_bwd(const float* dz, int64_t lddz, const float* x, int64_t ldx, int64_t M, int32_t K, const float* mean,
              const float* var, const float* gamma, float eps, float* dx, int64_t lddx, float* dgamma, float* dbeta,
              void* ws, size_t ws_bytes, void* stream);

/* activations for rf_linear_fwd */
#define RF_ACT_NONE 0
#define RF_ACT_GELU 1 /* exact erf gelu (tf.keras.activations.gelu, approximate=False) */
#define RF_ACT_RELU 2
#define RF_ACT_SELU 3
#define RF_ACT_SOFTMAX 4 /* row softmax over the N outputs (Dense(units, activation='softmax')) */

/*
 * Row normalisation feeding a Dense layer (the `normalization_layer` of create_mlp,
 * backend/blocks/mlp.py:4-15):
 *   mode 0 LayerNormalization(eps): y = (x - mean) / sqrt(var + eps) * gamma + beta
 *   mode 1 BatchNormalization(eps), inference: y = (x - mean[c]) / sqrt(var[c] + eps) * gamma + beta
 * x: F32 [rows][cols] (row stride ldx); y: [rows][cols] in y_dtype (BF16 or F32), row stride ldy.
 * mode 1 reads running mean/var from `mean`/`var` (per column); mode 0 ignores them.
 */
int rf_norm_fwd(const float* x, int64_t rows, int32_t cols, int64_t ldx, int32_t mode, float eps,
                const float* gamma, const float* beta, const float* mean, const float* var, void* y,
                int32_t y_dtype, int64_t ldy, void* stream);

/*
 * Dense layer  y = act(x @ W + b)  (tf.keras.layers.Dense, mlp.py:12; esim.py:53,88; dssm.py:25-26).
 * x: [M][K] (x_dtype BF16 -> bf16 MFMA, or F32 -> exact-fp32 MFMA), row stride ldx.
 * W: [N][K] row-major (i.e. the Keras kernel transposed), same dtype as x. b: F32 [N] (may be NULL).
 * y: F32 [M][N] with row stride ldy. fp32 accumulate. RF_ACT_SOFTMAX requires N <= 64.
 */
int rf_linear_fwd(const void* x, int32_t x_dtype, int64_t M, int32_t K, int64_t ldx, const void* W,
                  int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* stream);

/*
 * rf_linear_fwd with split-K for fp32 layers whose 128-tile grid leaves CUs half-occupied at deep K (the DSSM
 * towers, K = 8704 / 20480 at B = 4096): S K-ranges as S workgroups per tile writing fp32 partials to ws, then
 * y = act(sum_{s = 0..S-1} partial_s + b) in that fixed order (deterministic; not the unsplit fmaf chain).
 * rf_linear_splitk_ws_bytes: the ws it needs (0 = no split for this shape); with a smaller ws (or none) it is
 * exactly rf_linear_fwd. ws, x, W, b 16-byte aligned.
 */
size_t rf_linear_splitk_ws_bytes(int32_t x_dtype, int64_t M, int32_t K, int32_t N);
int rf_linear_splitk_fwd(const void* x, int32_t x_dtype, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t N,
                         const float* b, int32_t act, float* y, int64_t ldy, void* ws, size_t ws_bytes, void* stream);

/*
 * A two-layer create_mlp on a narrow input in ONE launch (the ESIM input_mlp [256, 512] over the dense
 * features, esim.py:45-48; mlp.py:4-15 with LayerNormalization):
 *   out = act(LN1(act(LN0(x) W0^T + b0)) W1^T + b1)
 * x: F32 [M][K0] (K0 <= 32), row stride ldx. LN0/LN1: gamma/beta F32 [K0] / [H], epsilon eps.
 * W0: BF16 [H][K0], W1: BF16 [O][H] (16-byte aligned), b0 [H] / b1 [O] F32 (may be NULL). H = 128 or 256.
 * LN outputs are rounded once to bf16 (the MFMA operands), as the rf_norm_fwd -> rf_linear_fwd chain.
 * out: F32 [M][O], row stride ldo (e.g. the first O columns of the pooled [B, 512 + 6d] tensor).
 * act: an elementwise RF_ACT_* (not SOFTMAX).
 */
int rf_mlp2_small_fwd(const float* x, int64_t M, int32_t K0, int64_t ldx, float eps, const float* ln0_gamma,
                      const float* ln0_beta, const void* W0, const float* b0, int32_t H, const float* ln1_gamma,
                      const float* ln1_beta, const void* W1, const float* b1, int32_t O, int32_t act, float* out,
                      int64_t ldo, void* stream);
/*
 * rf_mlp2_small_fwd with out as BF16 [M][O] (row stride ldo) plus, per row and 32-column slice s of it, the pair
 * (sum, squared deviations from the slice mean) of the fp32 values in stats[row][stats_p0 + s] (stats_P pairs per
 * row): the producer half of an LN-folded consumer (rf_linear_lnfold_stats_fwd), as rf_linear_stats_fwd's row_stats.
 */
int rf_mlp2_small_stats_fwd(const float* x, int64_t M, int32_t K0, int64_t ldx, float eps, const float* ln0_gamma,
                            const float* ln0_beta, const void* W0, const float* b0, int32_t H, const float* ln1_gamma,
                            const float* ln1_beta, const void* W1, const float* b1, int32_t O, int32_t act,
                            void* out_bf16, int64_t ldo, float* stats, int32_t stats_P, int32_t stats_p0, void* stream);

/*
 * A create_mlp layer pair with the second layer's LayerNormalization folded across the GEMMs (mlp.py:10-13:
 * Norm -> Dense(act) per hidden size; the reference normalises between the two Dense layers):
 *   rf_linear_stats_fwd   y = act(x W^T + b) stored as BF16 [M][N] (row stride ldy), and row_stats
 *                         [M][P][2], P = 4 * ceil(N / 128): for each 32-column slice p of a row (columns
 *                         32p .. 32p + 31 below N, n_p of them) the pair (S_p, M2_p) of its fp32 values — their
 *                         sum and their squared deviations from the slice mean S_p / n_p — written by the
 *                         GEMM's epilogue (no pass over y, no atomics: fixed reduction order, deterministic).
 *   rf_linear_lnfold_fwd  y = act(rstd_r (x Wg^T - mu_r s) + t) = act(LN(x) W^T + b) for the raw BF16 x of
 *                         the previous call, with Wg = W diag(gamma) (BF16 [N][K]), s[c] = sum_k Wg[c][k],
 *                         t[c] = sum_k W[c][k] beta[k] + b[c] (F32 [N]), mu_r = sum_p S_p / K and
 *                         rstd_r = 1 / sqrt(var_r + eps), var_r = sum_p (M2_p + (S_p - n_p mu_r)^2 / n_p) / K
 *                         (Chan's pairwise combine; the stats call's N is this call's K).
 * Both: x BF16 [M][K] (16-byte aligned, ldx % 8 == 0), K >= 512 and K % 64 == 0 (the LDS-DMA GEMM),
 * elementwise activations only. The pair replaces rf_norm_fwd -> rf_linear_fwd for the second layer.
 */
int rf_linear_stats_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t N, const float* b,
                        int32_t act, void* y_bf16, int64_t ldy, float* row_stats, void* stream);
int rf_linear_lnfold_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N, const float* s,
                         const float* t, const float* row_stats, float eps, int32_t act, float* y, int64_t ldy,
                         void* stream);
/*
 * An LN-folded chain of create_mlp layers whose FIRST LayerNormalization is folded too (cfg3's output_mlp behind
 * the pooled row, esim.py:84-88; mlp.py:10-13): the producers of x (rf_mlp2_small_stats_fwd, rf_esim_gather_stats_fwd)
 * wrote it as BF16 with its slice partials, so no normalisation pass runs anywhere in the chain.
 *   rf_linear_lnfold_stats_fwd  rf_linear_lnfold_fwd's y, written as rf_linear_stats_fwd writes its output: BF16
 *                               y_bf16 [M][N] plus out_stats [M][4 ceil(N / 128)][2] (the next layer's input)
 *   rf_linear_lnfold_head_fwd   rf_linear_lnfold_fwd's y (stored only when y is not NULL) and a Dense(head_n, head_act)
 *                               head on it: out[r][h] = head_act(sum_c y[r][c] head_w[h][c] + head_b[h]), head_w
 *                               BF16 [head_n][N], head_n = 2 (esim.py:53,88 Dense(2, 'softmax')); the per-row
 *                               partial logits of each 128-column tile (fp32, fixed order) go through ws
 *                               (rf_linear_lnfold_head_ws_bytes(M, N) bytes); the last tile of each 64-row block
 *                               to finish adds them in tile order and writes the softmax. ws STARTS with one
 *                               counter per 64-row block (the partials sit at its far end): the counters must be
 *                               ZERO before the first call on a ws, and every call leaves them zero. One zeroed ws
 *                               serves calls of any M <= the M it was sized for, with the same N (one stream at a
 *                               time).
 */
int rf_linear_lnfold_stats_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N,
                               const float* s, const float* t, const float* row_stats, float eps, int32_t act,
                               void* y_bf16, int64_t ldy, float* out_stats, void* stream);
size_t rf_linear_lnfold_head_ws_bytes(int64_t M, int32_t N);
int rf_linear_lnfold_head_fwd(const void* x, int64_t M, int32_t K, int64_t ldx, const void* Wg, int32_t N,
                              const float* s, const float* t, const float* row_stats, float eps, int32_t act, float* y,
                              int64_t ldy, const void* head_w, int32_t head_n, const float* head_b, int32_t head_act,
                              float* out, int64_t ldo, void* ws, size_t ws_bytes, void* stream);

/*
 * Small Dense head on fp32 activations  y = act(x @ W + b),  N <= 64 outputs (the ESIM scorer's
 * Dense(2, 'softmax'), esim.py:53,88): replaces rf_linear_fwd's small-N path when the activations are the
 * fp32 output of the previous layer (no bf16 round trip of x). x: F32 [M][K], row stride ldx, 16-byte
 * aligned rows, K % 4 == 0. W: [N][K] in w_dtype (BF16 widened to fp32, or F32). b: F32 [N] or NULL.
 * y: F32 [M][N], row stride ldy. One wave per row, fp32 products and sums.
 */
int rf_dense_head_fwd(const float* x, int64_t M, int32_t K, int64_t ldx, const void* W, int32_t w_dtype,
                      int32_t N, const float* b, int32_t act, float* y, int64_t ldy, void* stream);

/*
 * The ESIM forward without the encoders' [B, L, 2D] outputs (cfg3; esim.py:78-84 over the DoubleHashingEmbedding
 * tokens, preprocess_layers.py:82-97): rf_single_token_ids_fwd writes, for every unit u = b * n_slots + s of a
 * batch whose slots all have batch Lmax == 1, ids[u][k] = the fused-table row of hash k of the bag's token (the
 * index half of rf_fused_hash_embed_fwd with RF_FLAG_SINGLE_TOKEN; an empty bag: the slot's pad rows, or
 * 0xffffffff = the zero row under RF_FLAG_MASK_PADDING; a slot whose Lmax is not 1 or that does not fit the
 * table: 0xfffffffe = the NaN row; with RF_FLAG_SPEC_ROWS those two are table_rows + 1 and table_rows).
 * rf_esim_gather_fwd then runs rf_esim_soft_attention_fwd's kernel with each example's q / a images gathered from
 * q_table / a_table (BF16 [rows + 2][d / 2]: the table's q_rows / a_rows rows, then a NaN row and a zero row) by
 * ids made with RF_FLAG_SPEC_ROWS. Same pooled outputs as encoders + rf_esim_soft_attention_fwd (x enters the
 * statistics through the selector MFMA, so a -0 in a table row gives the +0 the encoder writes).
 */
int rf_single_token_ids_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                            const int32_t* bag_off, const int32_t* lmax, int32_t batch, int64_t table_rows, uint32_t* ids,
                            int32_t flags, void* stream);
/*
 * rf_single_token_ids_fwd for up to 4 batches (towers) in ONE launch (the ESIM forward's user and ad sides: both
 * DoubleHashingEmbedding index passes, preprocess_layers.py:82-97 per tower): tasks is a HOST array of n_tasks
 * (1..4) descriptions; each task's ids are exactly what rf_single_token_ids_fwd writes for it.
 */
typedef struct rf_ids_task {
    const rf_slot_desc* slots; /* device */
    const uint8_t* tok_bytes;
    const int32_t* tok_off;
    const int32_t* bag_off;
    const int32_t* lmax;
    uint32_t* ids;             /* [batch * n_slots][2], 8-byte aligned */
    int64_t table_rows;
    int32_t n_slots;
    int32_t batch;
    int32_t flags;             /* 0, RF_FLAG_MASK_PADDING, RF_FLAG_SPEC_ROWS */
    int32_t reserved;          /* must be 0 */
} rf_ids_task;
int rf_single_token_ids_multi_fwd(const rf_ids_task* tasks, int32_t n_tasks, void* stream);
int rf_esim_gather_fwd(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows,
                       const void* a_table, int64_t a_rows, int32_t dtype, int32_t batch, int32_t L, int32_t d, float* out,
                       int64_t out_stride, int64_t out_off, void* stream);
/*
 * rf_esim_gather_fwd with the 6 d pooled features written as BF16 (out_bf16 + row * out_stride + out_off, elements)
 * and, per 32-column slice s of them (s = 0 .. 6 d / 32 - 1), the (sum, squared deviations from the slice mean) pair
 * of their fp32 values in stats[row][stats_p0 + s] (stats_P pairs per row): the attention's half of the pooled row
 * for rf_linear_lnfold_stats_fwd (cfg3: out_off = 32 stats_p0 = d_emb).
 */
int rf_esim_gather_stats_fwd(const uint32_t* q_ids, const uint32_t* a_ids, const void* q_table, int64_t q_rows,
                             const void* a_table, int64_t a_rows, int32_t dtype, int32_t batch, int32_t L, int32_t d,
                             void* out_bf16, int64_t out_stride, int64_t out_off, float* stats, int32_t stats_P,
                             int32_t stats_p0, void* stream);

/*
 * Masked scaled-dot-product attention over heads (backend/layers/layer_utils.py:4-24, with the
 * split_heads / merge transposes of MultiHeadAttention.call, attention_layers.py:159-167, folded
 * into the addressing):
 *   logits = q k^T / sqrt(depth); logits[i, :] = -4294967295 where mask[b, i] == 0 (QUERY rows, as
 *   the reference's [..., Lq, 1] mask broadcasts over keys); softmax over keys (fp32); out = P v.
 * q: [batch][Lq][heads*depth], k, v: [batch][Lk][heads*depth] (dtype F16 or BF16, contiguous; head h
 * owns columns [h*depth, (h+1)*depth)); mask: F32 [batch][Lq] (NULL = no mask).
 * out: F32 [batch][Lq][heads*depth]. Constraints: 1 <= Lq, Lk <= 256, depth in {32, 64, 128}.
 */
int rf_sdpa_fwd(const void* q, const void* k, const void* v, int32_t dtype, int32_t batch, int32_t heads,
                int32_t Lq, int32_t Lk, int32_t depth, const float* mask, float* out, void* stream);

/*
 * Row-sharded tables: route fused-table rows to their owner rank (owner = g mod P, local = g div P).
 * Stage 1 of the sharded lookup: for n global rows, write counts[P] (int32) and a
 * stable owner-major permutation perm[n] (int32; perm[pos] = source index) with local_rows[n] (int64)
 * in permuted order, and (if inv_perm != NULL) its inverse inv_perm[i] = pos.
 * ws must hold rf_bucketize_ws_bytes(n, P) bytes.
 */
size_t rf_bucketize_ws_bytes(int64_t n, int32_t nranks);
int rf_bucketize_owner(const int64_t* rows, int64_t n, int32_t nranks, int32_t* counts, int32_t* perm,
                       int32_t* inv_perm, int64_t* local_rows, void* ws, size_t ws_bytes, void* stream);

/*
 * Global fused-table rows of every token, both tables: rows_out[2*t + k] = row_base[k] + bucket_k(token t)
 * (the index half of rf_fused_hash_embed_fwd; the requester side of the sharded lookup).
 */
int rf_hash_rows(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes, const int32_t* tok_off,
                 const int32_t* bag_off, int32_t batch, int64_t* rows_out, void* stream);

/*
 * Pool pre-gathered rows with exactly the semantics and accumulation order of rf_fused_hash_embed_fwd
 * (so a sharded lookup is bit-identical to the single-GPU one). `gathered` holds [2*n_tok + 2*n_slots][dim]:
 * row 2*t + k = the table-k row of token t, row 2*n_tok + 2*s + k = the padding row of slot s, table k
 * (bin 0 of the segment, or the bin of b"" when mask_empty == 0). Descriptors supply combiner, out_off, dim.
 * row_map (int32 [2*n_tok + 2*n_slots], may be NULL = identity): logical row j is read from gathered row
 * row_map[j] — pass rf_bucketize_owner's inv_perm to pool straight from the all-to-all receive buffer.
 * local_table (may be NULL; same dtype/dim): a row_map entry with bit 31 set reads row (entry & 0x7fffffff) of
 * local_table instead — the rank's own shard, so rows it owns are pooled in place (rf_route_hash_build).
 */
int rf_pool_rows_fwd(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                     int32_t batch, int64_t n_tok, const void* gathered, const int32_t* row_map,
                     const void* local_table, int32_t dtype, int32_t dim, void* out, int32_t out_dtype,
                     int64_t out_stride, int32_t flags, void* stream);

/*
 * Route one step's row requests WITH dedup (the default requester stage of the sharded lookup; SURVEY
 * §8e "per-owner dedup"). For n global rows g < table_rows and P ranks (owner = g mod P, local = g div P):
 *   every distinct row once, sorted by (owner, local): local_out[0 .. n_uniq) (int64; -1 for a row outside
 *   [0, table_rows), which rf_gather_rows returns as NaN), counts[P] = distinct rows per owner (int32),
 *   row_map[j] = position of request j's row in that order (int32) — i.e. in the all-to-all receive
 *   buffer, so rf_pool_rows_fwd can take it as its row_map. n_uniq: DEVICE int32 (may be NULL).
 * Deterministic (radix sort, no atomics). ws: rf_route_ws_bytes(n, P, table_rows) bytes, 256-B aligned.
 */
size_t rf_route_ws_bytes(int64_t n, int32_t nranks, int64_t table_rows);
/*
 * The same routing by a hash-table dedup, in two calls around the host's read of the counts (the split sizes of
 * the all-to-alls): rf_route_hash_build inserts every request's owner-major key into an open-addressing table
 * (one atomicCAS per DISTINCT row; repeats find their key with a plain load) and writes counts[P] (distinct rows
 * per owner, DEVICE int32). With rank >= 0 the rows that rank owns are NOT routed: row_map[j] = 0x80000000 |
 * local for them (rf_pool_rows_fwd reads them from its local_table), counts[rank] = 0. rf_route_hash_finish
 * (n_uniq = the sum of counts, from the host) sorts the distinct keys (radix over the key bits of the distinct
 * set only) and writes local_out[0 .. n_uniq) in (owner, local) order and the remaining row_map entries, exactly
 * as rf_route_rows would for the routed rows. Same ws for both calls: rf_route_hash_ws_bytes(n, P, table_rows).
 * n_uniq = -1 (P <= 64): the distinct total is read from the workspace on the device, so the finish can be enqueued
 * before the host has read the counts (local_out then needs n entries; its first sum(counts) are the rows).
 */
size_t rf_route_hash_ws_bytes(int64_t n, int32_t nranks, int64_t table_rows);
int rf_route_hash_build(const int64_t* rows, int64_t n, int32_t nranks, int32_t rank, int64_t table_rows,
                        int32_t* row_map, int32_t* counts, void* ws, size_t ws_bytes, void* stream);
int rf_route_hash_finish(int64_t n, int32_t nranks, int64_t table_rows, int64_t n_uniq, int64_t* local_out,
                         int32_t* row_map, void* ws, size_t ws_bytes, void* stream);
/*
 * rf_hash_rows fused into rf_route_hash_build: the requests are the two hashed rows of every token (j = 2 t + k, the
 * rows rf_hash_rows would write) followed by the n_tail rows of `tail` (j = 2 n_tok + i: the slots' padding rows),
 * hashed and inserted in one launch, with no [2 n_tok] request list in HBM. The same table, counts, row_map and
 * workspace as rf_route_hash_build over that list (n = 2 n_tok + n_tail); rf_route_hash_finish follows unchanged.
 * Replaces rf_hash_rows + rf_route_hash_build in the row-sharded lookup (new capability: the reference mirrors every
 * table, gpu_utils.py:13-14). The hashing is rf_hash_rows' (preprocess_layers.py:86-97).
 */
int rf_route_hash_build_tokens(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                               const int32_t* tok_off, const int32_t* bag_off, int32_t batch, int64_t n_tok,
                               const int64_t* tail, int32_t n_tail, int32_t nranks, int32_t rank, int64_t table_rows,
                               int32_t* row_map, int32_t* counts, void* ws, size_t ws_bytes, void* stream);
/*
 * Owner-side partial pooling, the alternative exchange of the sharded lookup (SURVEY §8e "pool partial sums at
 * the owner"; deviation D-partial-pool-order: sum / avg add the owners' partials in owner order, exact at P = 1).
 * rf_pp_plan (requester): rows = rf_hash_rows + the 2*n_slots pad rows; for every unit u = 2*(b*n_slots + s) + k
 *   its pooling entries in position order: (ent_row global row, ent_unit u, ent_mult multiplicity; the padding
 *   positions of a unit are ONE entry of multiplicity Lmax - len; first / last: the one position). ent_off
 *   int32 [2*batch*n_slots + 1] (exclusive scan of the entry counts), n_ent DEVICE int32. Capacity of the entry
 *   arrays: 2*n_tok + 2*batch*n_slots. ws: rf_pp_ws_bytes(2*batch*n_slots).
 * rf_pp_heads: over owner-major entries (rf_bucketize_owner order) with per-owner entry counts (DEVICE int32[P]):
 *   seg_counts[P] (segments = runs of one unit inside an owner's chunk), and seg_of [n_units][P] (requester:
 *   the global index of unit u's segment at owner o, or -1) and/or seg_start [n_seg] (owner: first entry of
 *   each segment). ws: rf_pp_ws_bytes(n).
 * rf_pp_owner_pool (owner): ent = int32 [n][3] (local row, unit, multiplicity) as received, segments from
 *   rf_pp_heads -> part fp32 [n_seg][dim]: sum (fp32, entry order, multiplicity repeats) / max / min / the row.
 * rf_pp_combine (requester): per unit the partials part[seg_of[u][o]] for o = 0 .. P-1 -> out (avg: / Lmax).
 */
size_t rf_pp_ws_bytes(int64_t n);
int rf_pp_plan(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
               int64_t n_tok, const int64_t* rows, int32_t flags, int32_t* ent_off, int64_t* ent_row, int32_t* ent_unit,
               int32_t* ent_mult, int32_t* n_ent, void* ws, size_t ws_bytes, void* stream);
int rf_pp_heads(const int32_t* unit, int64_t n, const int32_t* counts, int32_t nranks, int32_t* seg_counts,
                int32_t* seg_of, int64_t n_units, int32_t* seg_start, void* ws, size_t ws_bytes, void* stream);
int rf_pp_owner_pool(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* ent, int64_t n, const int32_t* seg_start,
                     int64_t n_seg, const void* shard, int32_t dtype, int64_t shard_rows, int32_t dim, float* part,
                     void* stream);
int rf_pp_combine(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                  int32_t batch, int32_t flags, int32_t nranks, const int32_t* seg_of, const float* part, int32_t dim,
                  void* out, int32_t out_dtype, int64_t out_stride, void* stream);
int rf_route_rows(const int64_t* rows, int64_t n, int32_t nranks, int64_t table_rows, int32_t* counts,
                  int64_t* local_out, int32_t* row_map, int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream);

/* Gather whole rows: out[i] = table[rows[i]] (owner side of the sharded lookup). */
int rf_gather_rows(const int64_t* rows, int64_t n, const void* table, int32_t dtype, int64_t table_rows,
                   int32_t dim, void* out, void* stream);

/* ---- training backward of the sparse path (rf_train.hip) ------------------------ */
/*
 * Backward of rf_fused_hash_embed_fwd for an fp32 table and fp32 output/gradient: the deduplicated
 * sparse gradient Keras hands its optimizer. Reference: the Embedding gather gradient is an
 * IndexedSlices over every position of the padded [B, Lmax] ids (preprocess_layers.py:67; padding
 * positions gather bin 0, dataloader.py:32-33) shaped by the combiner's gradient (:44-64:
 * reduce_sum -> g, reduce_mean -> g / L, reduce_max/min -> (x == y) / num_selected * g, first/last ->
 * g at that position and 0 elsewhere); OptimizerV2._deduplicate_indexed_slices sums it per row
 * (unsorted_segment_sum, (b, l) order on CPU). Outputs: uniq_rows[u] ascending distinct fused-table rows,
 * uniq_grad[u][dim] their summed gradients (same order of additions as the reference, bit-exact),
 * *n_uniq (DEVICE int32) = number of distinct rows, or -(error bits) for an invalid batch (1: a row
 * outside the table, 2: n_positions wrong, 4: a bag longer than lmax). Rows beyond uniq_cap are dropped
 * (n_uniq > uniq_cap tells the caller). n_positions = batch * sum_s 2 * lmax[s] (host-known).
 * out (the forward output) and minmax_count (int32 scratch shaped like out) are needed iff a slot pools
 * max/min, else may be NULL. dout and out share out_stride. ws: rf_embed_bwd_ws_bytes bytes.
 */
size_t rf_embed_bwd_ws_bytes(int64_t n_positions, int32_t n_slots, int64_t table_rows);
int rf_fused_hash_embed_bwd(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                            const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                            int64_t n_positions, const float* table, int64_t table_rows, int32_t dim,
                            const float* out, const float* dout, int64_t out_stride, int32_t flags,
                            int32_t* minmax_count, int64_t* uniq_rows, float* uniq_grad, int64_t uniq_cap,
                            int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream);

/*
 * rf_fused_hash_embed_bwd in two halves on one workspace: _plan (enumerate, sort, segment: the batch alone
 * decides it) writes uniq_rows / n_uniq and keeps the plan in ws; _reduce (the same ws, untouched in between)
 * reads dout and writes uniq_grad. plan + reduce == rf_fused_hash_embed_bwd, bit for bit. The plan can run
 * while the dense layers still compute dout (the DSSM train step runs it, and rf_adam_untouched, on a side stream).
 */
int rf_fused_hash_embed_bwd_plan(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                 const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                                 int64_t n_positions, int64_t table_rows, int32_t dim, int64_t out_stride, int32_t flags,
                                 int64_t* uniq_rows, int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes,
                                 void* stream);
int rf_fused_hash_embed_bwd_reduce(const rf_slot_desc* d_slots, int32_t n_slots, const uint8_t* tok_bytes,
                                   const int32_t* tok_off, const int32_t* bag_off, const int32_t* lmax, int32_t batch,
                                   int64_t n_positions, const float* table, int64_t table_rows, int32_t dim,
                                   const float* out, const float* dout, int64_t out_stride, int32_t flags,
                                   int32_t* minmax_count, int64_t* uniq_rows, float* uniq_grad, int64_t uniq_cap,
                                   int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream);

/*
 * Backward of rf_pool_rows_fwd (the requester side of the sharded lookup): the same
 * per-position gradients and (b, l) summation order as rf_fused_hash_embed_bwd, keyed by the distinct
 * gathered row each logical row maps to (row_map, as in the forward; n_rows = number of gathered rows).
 * uniq_rows are gathered-row indices, i.e. positions in the all-to-all receive buffer = the request order.
 * gathered (the received rows) is read for max/min only.
 */
int rf_pool_rows_bwd(const rf_slot_desc* d_slots, int32_t n_slots, const int32_t* bag_off, const int32_t* lmax,
                     int32_t batch, int64_t n_tok, int64_t n_positions, const int32_t* row_map, const float* gathered,
                     int64_t n_rows, int32_t dim, const float* out, const float* dout, int64_t out_stride, int32_t flags,
                     int32_t* minmax_count, int64_t* uniq_rows, float* uniq_grad, int64_t uniq_cap, int32_t* n_uniq,
                     void* ws, size_t ws_bytes, void* stream);
/*
 * Owner side of the sharded backward: rows vals[i] (f32 [n][dim]) with ids[i] in [0, id_range) are summed
 * per id in input order (the concatenation of the requesters' gradients in rank order): uniq_ids ascending,
 * uniq_vals their sums (acc = 0; acc += v in order). Ids outside the range are dropped. n_uniq: DEVICE int32.
 * ws: rf_segment_sum_ws_bytes(n, id_range).
 */
size_t rf_segment_sum_ws_bytes(int64_t n, int64_t id_range);
int rf_segment_sum_rows(const int64_t* ids, const float* vals, int64_t n, int32_t dim, int64_t id_range, int64_t* uniq_ids,
                        float* uniq_vals, int64_t uniq_cap, int32_t* n_uniq, void* ws, size_t ws_bytes, void* stream);

/*
 * One tf.keras.optimizers.Adam step on an fp32 table from a deduplicated sparse gradient
 * (Adam._resource_apply_sparse, example/ranking_search/train.py:97):
 *   m = m * beta1 (every row); m[r] += g_r * (1 - beta1) (listed rows); v likewise with g_r * g_r * (1 - beta2);
 *   table -= lr * m / (sqrt(v) + epsilon) (every row).
 * lr must already carry Keras' bias correction: lr_t * sqrt(1 - beta2^t) / (1 - beta1^t) (fp32).
 * lazy != 0: only the listed rows are decayed and updated (TF-Addons LazyAdam semantics; a deviation,
 * much less HBM traffic). n_uniq is the DEVICE count written by rf_fused_hash_embed_bwd.
 * ws: rf_adam_ws_bytes(table_rows, lazy) bytes (dense mode: a row -> gradient map).
 */
size_t rf_adam_ws_bytes(int64_t table_rows, int32_t lazy);
/* Keras Adam on a dense fp32 variable of n elements (the towers' weights; Adam._resource_apply_dense ->
 * ResourceApplyAdam): m += (g - m)(1 - beta1); v += (g^2 - v)(1 - beta2); w -= m lr / (sqrt(v) + epsilon), with lr
 * the bias-corrected step size lr * sqrt(1 - beta2^t) / (1 - beta1^t) in fp32. In place, one launch.
 */
int rf_adam_dense(float* w, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float epsilon,
                  void* stream);
/* rf_adam_dense over a list of variables in one launch. tensors: a DEVICE array of n_tensors descriptors
 * (every n <= max_n); the same update, bit for bit, as one rf_adam_dense per entry. */
typedef struct rf_adam_tensor {
    float* w;
    const float* g;
    float* m;
    float* v;
    int64_t n;
} rf_adam_tensor;
int rf_adam_dense_multi(const rf_adam_tensor* tensors, int32_t n_tensors, int64_t max_n, float lr, float beta1, float beta2,
                        float epsilon, void* stream);

/*
 * The dense step split in time: rf_adam_untouched updates every row NOT listed in uniq_rows[:n_uniq] (their
 * Keras update needs no gradient: m, v decay, var moves by lr m / (sqrt(v) + eps)), so it can run as soon as
 * the row set is known (rf_fused_hash_embed_bwd_plan); rf_adam_apply(lazy = 1) on the gradient then updates
 * the listed rows with the same lr. Together: rf_adam_apply(lazy = 0), bit for bit.
 * ws: rf_adam_ws_bytes(table_rows, 0).
 */
int rf_adam_untouched(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                      const int32_t* n_uniq, int64_t uniq_cap, float lr, float beta1, float beta2, float epsilon, void* ws,
                      size_t ws_bytes, void* stream);
int rf_adam_apply(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                  const float* uniq_grad, const int32_t* n_uniq, int64_t uniq_cap, float lr, float beta1,
                  float beta2, float epsilon, int32_t lazy, void* ws, size_t ws_bytes, void* stream);
/*
 * The dense step deferred, exactly: last[r] (int32, one per row) = the step through which row r's var / m / v
 * are current. rf_adam_replay brings every row of uniq_rows[:n_uniq] (all rows when uniq_rows is NULL) from
 * last[r] to t_now by applying the untouched-row update of each step s in last[r] + 1 .. t_now with lr_log[s]
 * (f32, the step's bias-corrected lr, index = step), then sets last[r] = t_set (t_now, or t_now + 1 when the
 * caller's rf_adam_apply(lazy = 1) for step t_now + 1 follows on the same stream). n_uniq NULL: all uniq_cap
 * listed rows. A row may be listed more than once (it is replayed once: the first team to swap last[r] owns it);
 * rows outside [0, table_rows) are skipped. The same fp32 expressions in
 * the same order as rf_adam_untouched step by step: bit-identical var / m / v whenever a row is read. The DSSM
 * train step replays the batch's rows (rf_fused_hash_embed_bwd_plan) before its forward and the gradient's rows
 * before the touched update; a full replay (materialize) precedes any other read of the table. n_uniq < 0 (the
 * plan's invalid-batch flag): nothing moves. Same Keras reference as rf_adam_apply.
 */
int rf_adam_replay(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                   const int32_t* n_uniq, int64_t uniq_cap, int32_t* last, int32_t t_now, int32_t t_set,
                   const float* lr_log, float beta1, float beta2, float epsilon, void* stream);
/*
 * The touched half of the deferred step when every listed row is already current through t_set - 1 (the caller
 * replayed exactly these rows for this step, e.g. the DSSM step's plan rows): rf_adam_apply(lazy = 1) on
 * uniq_rows[:n_uniq] plus last[r] = t_set, in one pass (no separate marking replay). Rows must be distinct.
 */
int rf_adam_apply_current(float* table, float* m, float* v, int64_t table_rows, int32_t dim, const int64_t* uniq_rows,
                          const float* uniq_grad, const int32_t* n_uniq, int64_t uniq_cap, float lr, float beta1,
                          float beta2, float epsilon, int32_t* last, int32_t t_set, void* stream);

/* ---- two-tower training losses (rf_loss.hip), forward + gradient ---------------- */
/*
 * The DSSM score ahead of cosent_loss (dssm.py:35-36 K.l2_normalize of both towers, match_losses.py:46 row dot):
 * score[i] = <a_i / max(|a_i|, eps), b_i / max(|b_i|, eps)> for a, b [batch, n] fp32 (row strides lda / ldb);
 * norms[2i], norms[2i+1] = |a_i|, |b_i| (unclamped, for the backward). The backward writes
 * da_i = g ds_i (v_i - s_i u_i) / |a_i| (v_i / eps where |a_i| <= eps) and db likewise, g = *gscale (device
 * scalar, NULL = 1): the upstream gradient of the loss folded in, so the cosent dscore feeds it directly.
 */
int rf_cosine_rows_fwd(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t batch, int32_t n, float eps,
                       float* score, float* norms, void* stream);
int rf_cosine_rows_bwd(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t batch, int32_t n, float eps,
                       const float* score, const float* norms, const float* dscore, const float* gscale, float* da,
                       int64_t ldda, float* db, int64_t lddb, void* stream);
/* Workspace of both loss entry points (bytes). */
size_t rf_loss_ws_bytes(int32_t batch);
/*
 * cosent_loss (backend/losses/match_losses.py:42-56) on precomputed scores s_i = <query_i, doc_i>:
 * *loss (device f32) = logsumexp([0] ++ [scale * (s_i - s_j) for y_i < y_j]); dscore[i] = dloss/ds_i
 * (may be NULL).
 */
int rf_cosent_loss(const float* score, const float* label, int32_t batch, float scale, float* loss, float* dscore,
                   void* ws, size_t ws_bytes, void* stream);
/*
 * batch_neg_sample_scaled_multi_class_ce_loss (match_losses.py:150-165) on logits P = query . doc^T
 * ([batch][ld], a library GEMM): *loss = mean_i(-log softmax(scale * P_i.)_i * y_i);
 * dlogits[i][j] = dloss/dP_ij (may be NULL).
 */
int rf_inbatch_ce_loss(const float* logits, int64_t ld, const float* label, int32_t batch, float scale, float* loss,
                       float* dlogits, int64_t ldd, void* ws, size_t ws_bytes, void* stream);
/*
 * The ESIM click head's loss (esim.py:53,88 Dense(2, 'softmax') trained by model.fit, example/ranking_search/train.py:96-104):
 * sparse categorical cross-entropy of the softmax, computed from its logits as Keras does. logits [batch][ld] F32,
 * label int32 [batch] in [0, n_classes): *loss = mean_b(logsumexp(z_b) - z_b[y_b]); prob (may be NULL) = softmax(z);
 * dlogits (may be NULL) = (prob - onehot(y)) / batch. A label out of range makes that row NaN. ws: rf_loss_ws_bytes.
 */
int rf_softmax_ce_loss(const float* logits, int64_t ld, const int32_t* label, int32_t batch, int32_t n_classes, float* loss,
                       float* prob, int64_t ldp, float* dlogits, int64_t ldd, void* ws, size_t ws_bytes, void* stream);

/* ---- ESIM ranking-model training (SURVEY §8f.1 for models/ranking: esim.py:45-53,69-89 under model.fit) -------
 * The exact-fp32 training path of the ranker: Keras builds the model in float32, so every stage here computes in
 * fp32 (the inference path above runs bf16 MFMA).
 *
 * rf_esim_train_fwd_f32: the ESIM attention block on fp32 q, a (example e at q + e * ex_stride, rows ld apart,
 *   16-byte aligned; 1 <= L <= 128, d in {64, 128}): out[e][out_off ..] = [avg_q, max_q, avg_a, max_a,
 *   avg_q - avg_a, max_q - max_a] (6d floats) and aux[e][2][d] = how many of the 4L pooled candidates equal each
 *   max (TF's reduce_max gradient splits evenly over ties). v_mfma_f32_16x16x4_f32 products (exact fp32).
 * rf_esim_train_bwd_f32: given the forward's pooled output and aux and dpooled (the gradient of those 6d columns),
 *   writes dq, da (example stride g_ex_stride, rows ldg apart; every row < L overwritten). ws:
 *   rf_esim_train_ws_bytes(batch, L, d) (per example S^T, dE^T [Lp][Lp] and G_q^T, G_a^T [d][Lp] fp32, Lp = L
 *   rounded up to 16). Deterministic.
 */
size_t rf_esim_train_ws_bytes(int32_t batch, int32_t L, int32_t d);
int rf_esim_train_fwd_f32(const float* q, const float* a, int32_t batch, int32_t L, int32_t d, int64_t ex_stride, int64_t ld,
                          float* out, int64_t out_stride, int64_t out_off, float* aux, void* stream);
int rf_esim_train_bwd_f32(const float* q, const float* a, int32_t batch, int32_t L, int32_t d, int64_t ex_stride, int64_t ld,
                          const float* pooled, int64_t p_stride, int64_t p_off, const float* dpooled, int64_t dp_stride,
                          int64_t dp_off, const float* aux, float* dq, float* da, int64_t g_ex_stride, int64_t ldg, void* ws,
                          size_t ws_bytes, void* stream);
/*
 * create_mlp(units, rate, gelu, LayerNormalization(1e-6)) training stages (mlp.py:4-15; the ESIM input / output MLPs):
 * rf_act_dropout_fwd   h = Dropout(rate)(act(pre)) with rf_dropout_fwd's keep mask (rate 0: no mask); act elementwise
 * rf_act_dropout_bwd   dpre = dh keep / (1 - rate) act'(pre), db[N] = column sums of dpre (ws: rf_tower_ws_bytes(M, N))
 * rf_layernorm_bwd     LayerNormalization(eps) backward over the last axis from its input x: dx, dgamma = sum(dy xhat),
 *                      dbeta = sum(dy) (tf.nn.moments statistics; ws: rf_layernorm_bwd_ws_bytes(M, K))
 * Column sums reduce fixed row chunks in chunk order (replay-deterministic). The forward LayerNorm is rf_norm_fwd
 * (mode 0, F32 out) and the Dense products rf_gemm_f32.
 */
int rf_act_dropout_fwd(const float* pre, int64_t ldp, int64_t M, int32_t N, int32_t act, float rate, uint64_t seed, float* h,
                       int64_t ldh, void* stream);
int rf_act_dropout_bwd(const float* dh, int64_t lddh, const float* pre, int64_t ldp, int64_t M, int32_t N, int32_t act,
                       float rate, uint64_t seed, float* dpre, int64_t ldd, float* db, void* ws, size_t ws_bytes, void* stream);
size_t rf_layernorm_bwd_ws_bytes(int64_t M, int32_t K);
int rf_layernorm_bwd(const float* dy, int64_t lddy, const float* x, int64_t ldx, int64_t M, int32_t K, const float* gamma,
                     float eps, float* dx, int64_t lddx, float* dgamma, float* dbeta, void* ws, size_t ws_bytes, void* stream);

/* ---- Lookup / Discrete embeddings: GPU index producers (rf_lookup.hip) ----------- */
/*
 * StringLookup / IntegerLookup (backend/layers/preprocess_layers.py:135-169, Keras TF >= 2.6 defaults:
 * num_oov_indices = 1, mask_token = None): vocab[i] -> i + 1, any other value -> 0. The vocabulary is an
 * open-addressing table (linear probing) of `cap` entries, cap a power of two >= 2 * n_vocab
 * (rf_vocab_capacity); string keys are a SipHash-2-4 of the bytes (hits are verified against the
 * vocabulary bytes), integer keys the value itself.
 */
#define RF_VOCAB_BYTES 0
#define RF_VOCAB_INT64 1
typedef struct rf_vocab_entry {
    uint64_t key; /* SipHash of the term (bytes) or the term (int64) */
    int32_t id;   /* i + 1 for vocabulary entry i; -1 = empty slot */
    int32_t ref;  /* vocabulary index i (bytes: for the byte-for-byte check) */
} rf_vocab_entry; /* 16 bytes */
int64_t rf_vocab_capacity(int64_t n_vocab);
/* HOST function: fills a HOST table (copy it to the device). values: bytes + off[n_vocab + 1] for
 * RF_VOCAB_BYTES, int64[n_vocab] for RF_VOCAB_INT64. A repeated term -> RF_EINVAL (Keras raises too). */
int rf_vocab_build(int32_t kind, const void* values, const int32_t* off, int64_t n_vocab, rf_vocab_entry* table,
                   int64_t cap);
/*
 * Padded ids of one slot of a batched CSR group (bag_off[B * n_slots + 1], example-major):
 * ids[b][l] (int64, [batch][lmax]) = lookup(value l of bag (b, slot)) for l < len, lookup(default) for
 * padding (b"" / 0: the value parse_example pads with, dataloader.py:32-33). values = token bytes (+ tok_off)
 * for RF_VOCAB_BYTES, int64 values for RF_VOCAB_INT64. Feed ids to rf_embedding_bag_fwd.
 */
int rf_lookup_ids(int32_t kind, const rf_vocab_entry* table, int64_t cap, const uint8_t* vocab_bytes,
                  const int32_t* vocab_off, const void* values, const int32_t* tok_off, const int32_t* bag_off,
                  int32_t n_slots, int32_t slot, int32_t batch, int32_t lmax, int64_t* ids, void* stream);
/*
 * Discretization(bin_boundaries) (preprocess_layers.py:172-200) = tf Bucketize: ids[b][l] = number of
 * boundaries <= x (upper bound; NaN -> n_boundaries), padding x = pad_value (the float default 0.0).
 */
int rf_bucketize_ids(const float* values, const int32_t* bag_off, int32_t n_slots, int32_t slot, int32_t batch,
                     int32_t lmax, const float* boundaries, int32_t n_boundaries, float pad_value, int64_t* ids,
                     void* stream);

/* ---- recall search: exact top-k (rf_topk.hip) ------------------------------------ */
/*
 * FaissSearcher Flat search (faiss_searcher.py:141-204) in blocks of items: for each of `rows` queries,
 * the best k of { scores[row][0 .. cols) with item index col_base + c } U { prev_val/prev_idx[row][0 .. k_prev) }
 * -> out_val/out_idx[row][0 .. k), sorted by score descending, ties by smaller item index; NaN scores
 * never selected; missing entries are (-inf, -1). Chain calls over item blocks (scores of a block =
 * rf_linear_fwd(queries, items_block)) with out as the next call's prev (double-buffered).
 * cols <= 32768, 1 <= k <= 1024, k_prev <= 1024, item indices < 2^32. out must not alias prev.
 */
int rf_topk_merge(const float* scores, int64_t ld, int32_t rows, int32_t cols, int32_t k, int64_t col_base,
                  const float* prev_val, const int64_t* prev_idx, int32_t k_prev, int64_t prev_ld, float* out_val,
                  int64_t* out_idx, int64_t out_ld, void* stream);
/* rf_topk_merge with the block's item indices given per entry (col_idx[row][c], same ld as scores) instead of
 * col_base + c: the candidate lists of rf_ip_candidates_f32 (entries past a row's count hold NaN scores). */
int rf_topk_merge_idx(const float* scores, const uint32_t* col_idx, int64_t ld, int32_t rows, int32_t cols, int32_t k,
                      const float* prev_val, const int64_t* prev_idx, int32_t k_prev, int64_t prev_ld, float* out_val,
                      int64_t* out_idx, int64_t out_ld, void* stream);
/*
 * FaissSearcher Flat's screen (faiss_searcher.py:141-204, exact): for M queries q [M][K] (row stride ldq) against N
 * items [N][K] (contiguous rows), every pair with score <q_m, item_n> >= thr[m] is appended, in no particular order,
 * to row m's list: cand_val[m][0 .. cap) and cand_idx[m][0 .. cap) (item index col_base + n); count[m] (zero
 * before the call) counts every such pair, so count[m] > cap means entries were dropped. The scores are bit for bit
 * those of rf_linear_fwd (fp32, the LDS-DMA MFMA kernel), and no score matrix is written. With thr[m] = the k-th best
 * score of any subset of the items, the lists hold every item of the exact top-k (the k-th best over all items is
 * at least thr[m]). K >= 256, K % 32 == 0, 16-byte aligned q and items.
 */
int rf_ip_candidates_f32(const float* q, int64_t ldq, int32_t M, const float* items, int32_t N, int32_t K,
                         const float* thr, int32_t cap, int32_t* count, float* cand_val, uint32_t* cand_idx,
                         int64_t col_base, void* stream);
/* The same screen on bf16 copies of q and the items (rows of K % 64 == 0 bf16, ldq % 8 == 0): a pair is kept when its
 * bf16 score (fp32 accumulation) is >= thr[m] - qbound[m] * vnorm[n], with qbound = C ||q_m|| and vnorm the items'
 * fp32 norms; C >= (2u + u^2 + 2 gamma_K (1 + u)^2) (u = 2^-8, gamma_K = K 2^-24 / (1 - K 2^-24)) bounds the distance
 * between a bf16 score and the fp32 one, so every pair whose fp32 score reaches thr[m] is kept (finite inputs). The
 * kept scores are bf16 ones: rf_ip_rescore_f32 replaces them by the exact fp32 scores. */
int rf_ip_candidates_bf16(const void* q, int64_t ldq, int32_t M, const void* items, int32_t N, int32_t K, const float* thr,
                          const float* qbound, const float* vnorm, int32_t cap, int32_t* count, float* cand_val,
                          uint32_t* cand_idx, int64_t col_base, void* stream);
/* cand_val[m][c] = the fp32 score <q_m, items[cand_idx[m][c]]> for c < min(count[m], cap), computed in the k order
 * of rf_linear_fwd's fp32 MFMA kernel (per 32-k step, half, element, lane group ascending: an fmaf chain), i.e.
 * the same bits as rf_linear_fwd (order = 0; 1 = lane groups descending, a diagnostic). K % 32 == 0, K <= 8192. */
int rf_ip_rescore_f32(const float* q, int64_t ldq, int32_t M, const float* items, int32_t K, const int32_t* count,
                      int32_t cap, float* cand_val, const uint32_t* cand_idx, int32_t order, void* stream);

/*
 * Que2Search AttentionFusion forward (backend/layers/fusion_layers.py:35-46), fp32:
 * x: [batch][channels * dim] (the K.concatenate of the channel inputs, row stride ldx); W: [channels*dim][channels]
 * (Keras layout). att = softmax(x @ W); out[b] = sum_c att[b][c] * x_c[b] (l2-normalised if is_norm,
 * tf.nn.l2_normalize eps 1e-12) -> out [batch][dim] (stride ldo); att_out [batch][channels] optional.
 */
int rf_attention_fusion_fwd(const float* x, int32_t batch, int32_t channels, int32_t dim, int64_t ldx, const float* W,
                            int32_t is_norm, float* out, int64_t ldo, float* att_out, void* stream);

/*
 * Measurement probes (not a reference operator: the ceilings SURVEY §8d states the hot path against).
 * rf_stream_copy: dst = src, n_bytes % 16 == 0, 16-byte aligned; float4 STREAM copy (2 * n_bytes of HBM traffic);
 * variant 0: 4 float4 per lane, one pass per block; 1: 8 per lane; 2: as 0 with nontemporal loads/stores;
 * 3: nontemporal, persistent grid of 2048 blocks.
 * rf_gather_probe: n uniformly random rows (row r_i = mulhi(splitmix64(seed ^ i), rows), no index array) of
 * row_bytes (64/128/256/512) from table [rows][row_bytes], in_flight (4/8/16) rows per team of row_bytes/16
 * lanes; out != NULL: row i is copied to out[i] (the fused encoder's read-random / write-streaming shape),
 * else only read (sink: one device word, written only on an impossible value).
 */
int rf_stream_copy(const void* src, void* dst, int64_t n_bytes, int32_t variant, void* stream);
int rf_gather_probe(const void* table, int64_t rows, int32_t row_bytes, int64_t n, int32_t in_flight, uint64_t seed,
                    void* out, uint32_t* sink, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RF_API_H */
