// rf_gemm32.hip — the exact-fp32 GEMMs of the DSSM towers (models/matching/dssm.py:25-26:
// create_mlp([1024, 512, 256], 0.3, "selu", BatchNormalization(1e-6)), backend/blocks/mlp.py:4-15), forward and
// training step (example/ranking_search/train.py:96-104, model.fit with Adam):
//   forward        y  = act(x W'^T + b')   A = x    [M][K]    (k contiguous),   B = W'  [N][K] (k contiguous)
//   weight grad    G  = dpre^T h           A = dpre [K][M]    (m contiguous),   B = h   [K][N] (n contiguous)
//   input grad     dz = dpre W             A = dpre [M][K]    (k contiguous),   B = W   [K][N] (n contiguous)
// C[m][n] = sum_k A(m, k) B(k, n) on v_mfma_f32_16x16x4_f32 (f32 products, f32 accumulation; gfx950 has no xf32).
//
// Schedule (one 128 x 128 output tile per workgroup at a time, 4 waves of 64 x 64, one workgroup per CU):
//   * stream-K: the (tile, 64-k step) iterations of the whole GEMM are cut into G equal ranges, one per persistent
//     workgroup (G = the CU count), so every workgroup does the same MFMA work whatever the tile count; ranges are
//     laid out XCD-major (the workgroups of one XCD take consecutive tiles: their A rows / B columns share its L2);
//   * a tile cut between workgroups: each stores its raw partial tile (write-through sc1 stores), one agent-scope
//     ticket per workgroup, and the LAST to arrive adds every segment in k order (fixed: the result does not depend
//     on arrival order) and runs the epilogue (MI355X_MICROARCH.md, inter-workgroup hand-off: sc1 payload,
//     vmcnt(0), barrier, one relaxed agent-scope add whose return value names the last arriver, sc1 loads);
//   * per 64-k step (256 MFMAs per wave, in four quarters of 64): the next step's 64 KB sit in registers (buffer
//     loads, 8 x 16 B per thread and operand, issued one step ahead) and are copied into the other half of a
//     double-buffered LDS ring, one (copy, reload) pair per 12 MFMAs over the first three quarters; each quarter
//     reads the next quarter's fragments; one barrier per step, 16 MFMAs into the last quarter. Measured on the
//     tower shapes (tools/gemm32_cmp.sh): bursts of copies or loads between consecutive MFMAs starve the MFMA pipe
//     (clustered: 0.87 of peak; one pair per 5 MFMAs: 0.90; per 12: 0.91-0.92);
//   * LDS formats: a k-contiguous operand keeps 256-byte rows (64 k), 16-byte chunk c of row r at c ^ (r & 15)
//     (the 16 rows of one ds_read_b128 quarter-wave hit 16 distinct bank groups); an m/n-contiguous operand keeps
//     64 k-rows of 512 bytes, chunk c of k-row kk at c ^ (((kk >> 2) & 3) << 2) (the four lane groups of an MFMA
//     read four k-rows: distinct banks), read as ds_read_b32 (pairs of k-rows 512 B apart: ds_read2_b32);
//   * both layouts feed the MFMA in one permuted k order: in quarter q, MFMA e takes k = 16 q + 4 lg + e in lane
//     group lg.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "rf_act.h"
#include "rf_common.h"

namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 128, kBN = 128, kBK = 64, kThreads = 256;
constexpr int kStage = (kBM + kBN) * kBK;  // floats per LDS stage (64 KB)
constexpr int kSlot = kBM * kBN;           // floats per partial tile (64 KB)
constexpr int kMinIters = 2;               // 64-k steps per workgroup at least (small GEMMs take fewer workgroups)
constexpr int kWgPerCu = 1;                // one 4-wave workgroup per CU: one wave per SIMD, registers to spare
constexpr uint32_t kOOB = 0x80000000u;            // a buffer offset past every extent: the load returns zeros
constexpr int kLdsBytes = 2 * kStage * 4 + 16;     // two stages + the last-arriver flag

// One GEMM of a launch (a launch runs up to kMaxProbs of them, same operand layouts: e.g. the same layer of both
// DSSM towers); its tiles and 64-k steps continue the previous problem's in the stream-K numbering.
struct Prob {
    const float* A;
    const float* B;
    float* C;
    const float* bias;
    int64_t lda, ldb, ldc;
    int M, N, K;
    int act;
    int tiles_n, nk;
    int64_t unit0;  // first stream-K unit (tile-major, 64-k steps minor) of this problem
    int tile0;      // first global tile (arrival counter index)
    int pad_;
};
constexpr int kMaxProbs = 4;

struct GemmArgs {
    Prob p[kMaxProbs];
    int np;
    int one;        // 1 (a branch condition the compiler cannot fold)
    int64_t units;  // all problems' units
    int* cnt;       // one arrival counter per global tile (zero between launches)
    float* slots;   // 2 G partial tiles
    int defer;      // cut tiles: partials only, gemm32_fixup_kernel combines them (many segments per tile)
};

__device__ __forceinline__ int64_t seg_lo(int64_t v, int64_t U, int G) { return v * U / G; }

__device__ __forceinline__ int prob_of(const GemmArgs& g, int64_t x) {
    int q = 0;
    while (q + 1 < g.np && x >= g.p[q + 1].unit0) ++q;
    return q;
}

// the global tile holding stream-K unit x
__device__ __forceinline__ int gtile_of(const GemmArgs& g, int64_t x) {
    const int q = prob_of(g, x);
    return g.p[q].tile0 + (int)((x - g.p[q].unit0) / g.p[q].nk);
}

// the workgroup (virtual index) whose range holds iteration x
__device__ __forceinline__ int seg_owner(int64_t x, int64_t U, int G) {
    int v = (int)(x * G / U);
    while (v + 1 < G && seg_lo(v + 1, U, G) <= x) ++v;
    while (v > 0 && seg_lo(v, U, G) > x) --v;
    return v;
}

__device__ __forceinline__ f4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// extents are < 2^31 (rf_gemm_f32 checks): kOOB is past every one
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, bytes <= 0 ? 0u : (uint32_t)bytes, 0x00020000);
}

// One operand of the tile: where this thread's four 16-byte chunks per 32-k step come from and go to. KC: k-contiguous
// rows (tile dim = rows); else k-rows with the tile dim contiguous. One buffer resource per segment whose extent ends
// at the matrix's last byte (k-rows past K and the last row's k tail read zeros); the step's k offset rides in the
// per-lane offset (the range check covers it).
template <bool KC>
struct Operand {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t voff[8];  // per chunk, at k = 0
    uint32_t kstep;    // bytes per 64-k step
    int kcol;          // KC: this thread's k offset in a step (the K tail masks it)
    uint32_t loff[8];  // LDS float offsets of the chunks

    __device__ __forceinline__ void init(const float* p, int64_t ld, int rows, int row0, int K, int tid) {
        if constexpr (KC) {
            // 256-byte rows (64 k) = 16 chunks; 16 threads per row; chunk c of row r at c ^ (r & 15)
            const int ch = tid & 15;
            kcol = ch * 4;
            const int last = rows - 1 - row0;
            rs = rsrc(p + (int64_t)row0 * ld, (int64_t)last * ld * 4 + (int64_t)K * 4);
            kstep = kBK * 4;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int r = (tid >> 4) + 16 * c;
                voff[c] = (uint32_t)(((int64_t)min(r, last) * ld + ch * 4) * 4);
                loff[c] = r * 64 + ((ch ^ (r & 15)) << 2);
            }
        } else {
            const int c32 = tid & 31;
            kcol = 0;
            // the extent ends at the view's last column of its last k-row (rows, not ld: a trailing-column view's
            // last k-row may end where the parent allocation does)
            rs = rsrc(p + row0, ((int64_t)(K - 1) * ld + (rows - row0)) * 4);
            kstep = (uint32_t)(kBK * ld * 4);
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int kk = (tid >> 5) + 8 * c;
                voff[c] = (uint32_t)(((int64_t)kk * ld + c32 * 4) * 4);
                loff[c] = kk * 128 + ((c32 ^ (((kk >> 2) & 3) << 2)) << 2);
            }
        }
    }

    __device__ __forceinline__ void load1(f4& r, int c, int kt, int K) const {
        const uint32_t ko = (uint32_t)kt * kstep;
        if constexpr (KC) {
            const bool ok = kt * kBK + kcol < K;
            r = bload(rs, ok ? voff[c] + ko : kOOB);
        } else {
            r = bload(rs, voff[c] + ko);
        }
    }
    __device__ __forceinline__ void store1(const f4& r, int c, float* st) const {
        *reinterpret_cast<f4*>(st + loff[c]) = r;
    }
};

// fragments of k-chunk q (16 k): f[i][e] = X(k = 16 q + 4 lg + e, tile index t0 + 16 i + lr)
template <bool KC>
__device__ __forceinline__ void read_frag(f4 (&f)[4], const float* st, int t0, int q, int lr, int lg) {
    if constexpr (KC) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
            f[i] = *reinterpret_cast<const f4*>(st + (t0 + 16 * i + lr) * 64 + (((4 * q + lg) ^ lr) << 2));
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int col = t0 + 16 * i + lr;
            const float* p = st + (((col >> 2) ^ (lg << 2)) << 2) + (col & 3) + (16 * q + 4 * lg) * 128;
#pragma unroll
            for (int e = 0; e < 4; ++e) f[i][e] = p[e * 128];
        }
    }
}

template <int E0 = 0, int E1 = 4>
__device__ __forceinline__ void mfma_quarter(f4 (&acc)[4][4], const f4 (&a)[4], const f4 (&b)[4]) {
#pragma unroll
    for (int e = E0; e < E1; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
}

template <bool AKC, bool BKC>
__global__ __launch_bounds__(kThreads, 1) void gemm32_kernel(GemmArgs g) {
    // DS read instructions per quarter-step for both operands: 4 ds_read_b128 (k-contiguous) or 8 ds_read2_b32 (else)
    constexpr int kFragReads = (AKC ? 4 : 8) + (BKC ? 4 : 8);
    extern __shared__ __attribute__((aligned(16))) float lds[];  // 2 stages + the last-arriver flag
    int& s_last = *reinterpret_cast<int*>(lds + 2 * kStage);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    const int G = gridDim.x;
    // XCD-major virtual index (block b runs on XCD b % 8): one XCD's workgroups take consecutive ranges
    const int q8 = G / 8, r8 = G % 8, xcd = blockIdx.x % 8;
    const int v = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int64_t U = g.units;
    const int64_t lo = seg_lo(v, U, G), hi = seg_lo(v + 1, U, G);
    const int lo_tile = gtile_of(g, lo);

    for (int64_t u = lo; u < hi;) {
        const Prob& P = g.p[prob_of(g, u)];
        const int K = P.K;
        const int tile = (int)((u - P.unit0) / P.nk);
        const int64_t t_unit0 = P.unit0 + (int64_t)tile * P.nk;  // the tile's first unit
        const int k_lo = (int)(u - t_unit0);
        const int k_hi = (int)min<int64_t>(P.nk, hi - t_unit0);
        u = t_unit0 + k_hi;
        const int gt = P.tile0 + tile;
#if RF_G32_MFAST
        const int tiles_m = (P.M + kBM - 1) / kBM;
        const int m0 = (tile % tiles_m) * kBM, n0 = (tile / tiles_m) * kBN;
#else
        const int m0 = (tile / P.tiles_n) * kBM, n0 = (tile % P.tiles_n) * kBN;
#endif

        Operand<AKC> oa;
        Operand<BKC> ob;
        oa.init(P.A, P.lda, P.M, m0, K, tid);
        ob.init(P.B, P.ldb, P.N, n0, K, tid);
        float bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bv[j] = P.bias ? P.bias[min(n0 + wn * 64 + 16 * j + lr, P.N - 1)] : 0.f;

        f4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

        __syncthreads();  // the previous segment's LDS reads and s_last are done
        // one register set: step kt's data is loaded during step kt - 2 ... written during step kt - 1
        f4 ra[8], rb[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) { oa.load1(ra[c], c, k_lo, K); ob.load1(rb[c], c, k_lo, K); }
#pragma unroll
        for (int c = 0; c < 8; ++c) { oa.store1(ra[c], c, lds); ob.store1(rb[c], c, lds + kBM * kBK); }
#pragma unroll
        for (int c = 0; c < 8; ++c) { oa.load1(ra[c], c, k_lo + 1, K); ob.load1(rb[c], c, k_lo + 1, K); }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
        f4 fa[2][4], fb[2][4];
        read_frag<AKC>(fa[0], lds, wm * 64, 0, lr, lg);
        read_frag<BKC>(fb[0], lds + kBM * kBK, wn * 64, 0, lr, lg);

        constexpr int G1 = kFragReads >= 16 ? 1 : 24 / kFragReads;  // reads G1 MFMAs apart
        // One step (64 k) in four quarters of 64 MFMAs, each in a block of its own (behind branches the compiler
        // cannot fold: MFMAs carry no chain, instruction selection would order them past the barrier):
        //   Q0: MFMAs of chunk 0 | reads of chunk 1 | copies 0..7 of the next tile (A), loads of the tile after
        //   Q1: MFMAs of chunk 1 | reads of chunk 2 | copies 0..7 (B), loads
        //   Q2: MFMAs of chunk 2 | reads of chunk 3            then barrier (the next tile written, this read)
        //   Q3: MFMAs of chunk 3 | reads of the next tile's chunk 0
        // One step (64 k) in four quarters of 64 MFMAs, each in a block of its own (behind branches the compiler
        // cannot fold: MFMAs carry no chain, instruction selection would order them past the barrier). The 16
        // (copy, load) pairs of the next tile are spread over Q0..Q2 (6, 5, 5: one per 12 MFMAs); the barrier sits
        // 16 MFMAs into Q3.
#define RF_Q(ID, NP, PG)                                                                  \
        do {                                                                              \
            _Pragma("unroll") for (int q = 0; q < kFragReads; ++q) {                      \
                __builtin_amdgcn_sched_group_barrier(0x008, G1, ID);                      \
                __builtin_amdgcn_sched_group_barrier(0x100, 1, ID);                       \
            }                                                                             \
            _Pragma("unroll") for (int q = 0; q < NP; ++q) {                              \
                __builtin_amdgcn_sched_group_barrier(0x200, 1, ID);                       \
                __builtin_amdgcn_sched_group_barrier(0x008, PG / 2, ID);                  \
                __builtin_amdgcn_sched_group_barrier(0x020, 1, ID);                       \
                __builtin_amdgcn_sched_group_barrier(0x008, PG - PG / 2, ID);             \
            }                                                                             \
            __builtin_amdgcn_sched_group_barrier(0x008, 64 - G1 * kFragReads - NP * PG, ID); \
        } while (0)
#define RF_SEP()                                         \
        do {                                             \
            __builtin_amdgcn_sched_barrier(0);           \
            if (g.one) asm volatile("" ::: "memory");    \
            __builtin_amdgcn_sched_barrier(0);           \
        } while (0)
        auto step = [&](int kt, const float* cur, float* nxt) {
            // Q0: chunk 0's MFMAs | chunk 1's fragments | A chunks 0..5 of the next tile (copy, then reload)
            read_frag<AKC>(fa[1], cur, wm * 64, 1, lr, lg);
            read_frag<BKC>(fb[1], cur + kBM * kBK, wn * 64, 1, lr, lg);
#pragma unroll
            for (int c = 0; c < 6; ++c) { oa.store1(ra[c], c, nxt); oa.load1(ra[c], c, kt + 2, K); }
            mfma_quarter(acc, fa[0], fb[0]);
            RF_Q(0, 6, 6);
            RF_SEP();
            // Q1: chunk 1 | chunk 2's fragments | A chunks 6, 7, B chunks 0..2
            read_frag<AKC>(fa[0], cur, wm * 64, 2, lr, lg);
            read_frag<BKC>(fb[0], cur + kBM * kBK, wn * 64, 2, lr, lg);
#pragma unroll
            for (int c = 6; c < 8; ++c) { oa.store1(ra[c], c, nxt); oa.load1(ra[c], c, kt + 2, K); }
#pragma unroll
            for (int c = 0; c < 3; ++c) { ob.store1(rb[c], c, nxt + kBM * kBK); ob.load1(rb[c], c, kt + 2, K); }
            mfma_quarter(acc, fa[1], fb[1]);
            RF_Q(1, 5, 7);
            RF_SEP();
            // Q2: chunk 2 | chunk 3's fragments | B chunks 3..7
            read_frag<AKC>(fa[1], cur, wm * 64, 3, lr, lg);
            read_frag<BKC>(fb[1], cur + kBM * kBK, wn * 64, 3, lr, lg);
#pragma unroll
            for (int c = 3; c < 8; ++c) { ob.store1(rb[c], c, nxt + kBM * kBK); ob.load1(rb[c], c, kt + 2, K); }
            mfma_quarter(acc, fa[0], fb[0]);
            RF_Q(2, 5, 7);
            RF_SEP();
            // Q3: 16 MFMAs of chunk 3, the barrier, its other 48 under the next tile's chunk-0 fragments
            mfma_quarter<0, 1>(acc, fa[1], fb[1]);
            __builtin_amdgcn_sched_barrier(0);
            if (g.one) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();  // the next tile is written; every wave is done reading this one
            }
            __builtin_amdgcn_sched_barrier(0);
            read_frag<AKC>(fa[0], nxt, wm * 64, 0, lr, lg);
            read_frag<BKC>(fb[0], nxt + kBM * kBK, wn * 64, 0, lr, lg);
            mfma_quarter<1, 4>(acc, fa[1], fb[1]);
#pragma unroll
            for (int q = 0; q < kFragReads; ++q) {
                __builtin_amdgcn_sched_group_barrier(0x008, G1 / 2 > 0 ? G1 / 2 : 1, 3);
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 3);
            }
            __builtin_amdgcn_sched_barrier(0);
        };
        int kt = k_lo;
        for (; kt + 1 < k_hi; kt += 2) {
            step(kt, lds, lds + kStage);
            step(kt + 1, lds + kStage, lds);
        }
        if (kt < k_hi) step(kt, lds, lds + kStage);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

        const bool full = k_lo == 0 && k_hi == P.nk;
        if (!full) {
            // a cut tile: this segment's raw partial into its slot, one ticket; the last arriver combines in k order
            const int slot_id = gt == lo_tile ? 2 * v : 2 * v + 1;
            float* slot = g.slots + (size_t)slot_id * kSlot;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        __hip_atomic_store(slot + ((wave * 64 + (i * 4 + j) * 4 + r) * 64 + lane), acc[i][j][r],
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (g.defer) continue;  // gemm32_fixup_kernel adds the segments (same order) after this launch
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            const int v_first = seg_owner(t_unit0, U, G);
            const int v_last = seg_owner(t_unit0 + P.nk - 1, U, G);
            if (tid == 0) {
                const int old = __hip_atomic_fetch_add(g.cnt + gt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s_last = old == v_last - v_first;
            }
            __syncthreads();
            if (!s_last) continue;
            // The hand-off: every segment's slot stores are agent-scope atomics (gfx950 emits them with sc1, written
            // through past this XCD's L2) retired by vmcnt(0) before its ticket; the last arriver's acquire fence
            // (one L2 invalidate per cut tile, not per ticket) orders its slot loads after the ticket it read
            // (the HIP model's happens-before edge, at the cost of one buffer_inv)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (tid == 0) __hip_atomic_store(g.cnt + gt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int w = v_first; w <= v_last; ++w) {
                const int sid = gt == gtile_of(g, seg_lo(w, U, G)) ? 2 * w : 2 * w + 1;
                const float* p = g.slots + (size_t)sid * kSlot;
                float t[4][4][4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            t[i][j][r] = __hip_atomic_load(p + ((wave * 64 + (i * 4 + j) * 4 + r) * 64 + lane),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = w == v_first ? t[i][j][r] : acc[i][j][r] + t[i][j][r];
            }
        }
        // epilogue: bias + activation, values first, stores after (unguarded on interior tiles)
        rf_act::with_act(P.act, [&](auto F) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[i][j][r] = F(acc[i][j][r] + bv[j]);
        });
        const int rbase = m0 + wm * 64 + lg * 4, cbase = n0 + wn * 64 + lr;
        if (m0 + kBM <= P.M && n0 + kBN <= P.N) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float* yr = P.C + (int64_t)(rbase + 16 * i + r) * P.ldc + cbase;
#pragma unroll
                    for (int j = 0; j < 4; ++j) yr[16 * j] = acc[i][j][r];
                }
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = rbase + 16 * i + r;
                    if (row >= P.M) continue;
                    float* yr = P.C + (int64_t)row * P.ldc + cbase;
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (cbase + 16 * j < P.N) yr[16 * j] = acc[i][j][r];
                }
        }
    }
}

// The cut tiles' combine as a launch of its own (GemmArgs::defer: a few tiles over a long K, e.g. a weight gradient
// [4 x 512] or [256 x 16] over K = 4096, cut into 32 segments each). The in-kernel last arriver reads its tile's
// segments one after the other (32 dependent 64 KB rounds: 59-66 us for those shapes); here kFixParts workgroups
// per tile each take 1024 of its elements and issue every segment's loads together. The sum runs in the same order
// (segment v_first, + v_first + 1, ...) and the epilogue is the same, so the result is bit-identical to the
// in-kernel hand-off.
constexpr int kFixParts = 32, kFixPer = kSlot / kFixParts / kThreads;  // 2 elements per thread
constexpr int kFixBatch = 8;                                             // segments whose loads are issued together
__global__ __launch_bounds__(kThreads) void gemm32_fixup_kernel(GemmArgs g, int G) {
    const int b = blockIdx.x, part = b % kFixParts;
    const int gt = b / kFixParts;
    int q = 0;
    while (q + 1 < g.np && gt >= g.p[q + 1].tile0) ++q;
    const Prob& P = g.p[q];
    const int tile = gt - P.tile0;
    const int64_t U = g.units, t_unit0 = P.unit0 + (int64_t)tile * P.nk;
    const int v_first = seg_owner(t_unit0, U, G), v_last = seg_owner(t_unit0 + P.nk - 1, U, G);
    if (v_first == v_last) return;  // a whole tile: the GEMM launch stored it
#if RF_G32_MFAST
    const int tiles_m = (P.M + kBM - 1) / kBM;
    const int m0 = (tile % tiles_m) * kBM, n0 = (tile / tiles_m) * kBN;
#else
    const int m0 = (tile / P.tiles_n) * kBM, n0 = (tile % P.tiles_n) * kBN;
#endif
    float acc[kFixPer];
    int row[kFixPer], col[kFixPer];
    int e0 = part * (kSlot / kFixParts) + threadIdx.x;
#pragma unroll
    for (int s = 0; s < kFixPer; ++s) {
        const int e = e0 + s * kThreads;  // = ((wave * 64 + (i * 4 + j) * 4 + r) * 64 + lane), as the slot stores
        const int wave = e >> 12, ijr = (e >> 6) & 63, lane = e & 63;
        const int i = ijr >> 4, j = (ijr >> 2) & 3, r = ijr & 3;
        row[s] = m0 + (wave >> 1) * 64 + (lane >> 4) * 4 + 16 * i + r;
        col[s] = n0 + (wave & 1) * 64 + (lane & 15) + 16 * j;
    }
    for (int w0 = v_first; w0 <= v_last; w0 += kFixBatch) {
        float t[kFixBatch][kFixPer];
#pragma unroll
        for (int b = 0; b < kFixBatch; ++b) {
            const int w = min(w0 + b, v_last);  // past the last segment: a valid slot, not added
            const int sid = gt == gtile_of(g, seg_lo(w, U, G)) ? 2 * w : 2 * w + 1;
            const float* p = g.slots + (size_t)sid * kSlot;
#pragma unroll
            for (int s = 0; s < kFixPer; ++s) t[b][s] = p[e0 + s * kThreads];
        }
#pragma unroll
        for (int b = 0; b < kFixBatch; ++b)
            if (w0 + b <= v_last) {
#pragma unroll
                for (int s = 0; s < kFixPer; ++s) acc[s] = w0 + b == v_first ? t[b][s] : acc[s] + t[b][s];
            }
    }
    rf_act::with_act(P.act, [&](auto F) {
#pragma unroll
        for (int s = 0; s < kFixPer; ++s) {
            if (row[s] >= P.M || col[s] >= P.N) continue;
            const float bv = P.bias ? P.bias[col[s]] : 0.f;
            P.C[(int64_t)row[s] * P.ldc + col[s]] = F(acc[s] + bv);
        }
    });
}

int cu_count() {
    static const int n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return cus > 0 ? cus : 256;
    }();
    return n;
}

int64_t tiles_of(int64_t M, int64_t N) { return ((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN); }
size_t slot_bytes() { return (size_t)2 * kWgPerCu * cu_count() * kSlot * sizeof(float); }  // 2 slots per workgroup
size_t cnt_bytes(int64_t tiles) { return (((size_t)std::max<int64_t>(tiles, 1) * 4) + 255) & ~(size_t)255; }

}  // namespace

extern "C" size_t rf_gemm_f32_ws_bytes(int64_t M, int64_t N, int64_t K) {
    (void)K;
    return cnt_bytes(tiles_of(M, N)) + slot_bytes();
}

extern "C" size_t rf_gemm_f32_grouped_ws_bytes(const rf_gemm_f32_problem* probs, int32_t n) {
    int64_t tiles = 0;
    for (int i = 0; probs && i < n; ++i) tiles += tiles_of(probs[i].M, probs[i].N);
    return cnt_bytes(tiles) + slot_bytes();
}

extern "C" int rf_gemm_f32_grouped(const rf_gemm_f32_problem* probs, int32_t n, int32_t a_kc, int32_t b_kc, void* ws,
                                   size_t ws_bytes, void* stream) {
    RF_REQUIRE(probs && n >= 1 && n <= kMaxProbs, "rf_gemm_f32_grouped: 1..%d problems", kMaxProbs);
    RF_REQUIRE(ws, "rf_gemm_f32_grouped: null workspace");
    GemmArgs g{};
    int64_t units = 0, tiles = 0;
    for (int i = 0; i < n; ++i) {
        const rf_gemm_f32_problem& q = probs[i];
        const int64_t M = q.M, N = q.N, K = q.K, lda = q.lda, ldb = q.ldb, ldc = q.ldc;
        RF_REQUIRE(M >= 0 && N >= 0 && K >= 0 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30),
                   "rf_gemm_f32: bad shape (problem %d)", i);
        RF_REQUIRE(q.act >= RF_ACT_NONE && q.act < RF_ACT_SOFTMAX, "rf_gemm_f32: activation must be elementwise");
        if (M == 0 || N == 0) continue;
        RF_REQUIRE((K == 0 || (q.A && q.B)) && q.C, "rf_gemm_f32: null pointer (problem %d)", i);
        RF_REQUIRE(K == 0 || (K % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)q.A & 15) == 0 &&
                              ((uintptr_t)q.B & 15) == 0),
                   "rf_gemm_f32: K, lda, ldb must be multiples of 4 and A, B 16-byte aligned");
        RF_REQUIRE(K == 0 || ((a_kc ? lda >= K : lda >= M) && (b_kc ? ldb >= K : ldb >= N)),
                   "rf_gemm_f32: leading dimension too small");
        RF_REQUIRE(ldc >= N, "rf_gemm_f32: leading dimension too small");
        // 32-bit buffer offsets: a k-contiguous operand's 128-row tile block, an m/n-contiguous operand's K + 192 rows
        RF_REQUIRE((a_kc ? 128 * (__int128)lda : (K + 192) * (__int128)lda) * 4 < ((__int128)1 << 31) &&
                       (b_kc ? 128 * (__int128)ldb : (K + 192) * (__int128)ldb) * 4 < ((__int128)1 << 31),
                   "rf_gemm_f32: operand block exceeds 2 GiB (32-bit buffer offsets)");
        Prob& P = g.p[g.np++];
        P.A = q.A;
        P.B = q.B;
        P.C = q.C;
        P.bias = q.bias;
        P.lda = lda;
        P.ldb = ldb;
        P.ldc = ldc;
        P.M = (int)M;
        P.N = (int)N;
        P.K = (int)K;
        P.act = q.act;
        P.tiles_n = (int)((N + kBN - 1) / kBN);
        P.nk = (int)std::max<int64_t>((K + kBK - 1) / kBK, 1);
        P.unit0 = units;
        P.tile0 = (int)tiles;
        tiles += tiles_of(M, N);
        units += tiles_of(M, N) * P.nk;
    }
    if (g.np == 0) return RF_OK;
    RF_REQUIRE(ws_bytes >= cnt_bytes(tiles) + slot_bytes(), "rf_gemm_f32: workspace too small");
    g.units = units;
    g.one = 1;
    // counters at the start, partial slots at the far end: one zeroed ws serves calls of any shape it is large
    // enough for (a smaller call's slots never land on a larger call's counters)
    g.cnt = static_cast<int*>(ws);
    g.slots = reinterpret_cast<float*>(static_cast<char*>(ws) + ((ws_bytes - slot_bytes()) & ~(size_t)255));
    const int64_t gmax = (int64_t)kWgPerCu * cu_count();
    int G = (int)std::max<int64_t>(1, std::min<int64_t>(gmax, g.units / kMinIters));
#ifdef RF_G32_LAB
    if (const char* e = getenv("RF_G32_GRID")) G = std::max(1, std::min(atoi(e), (int)gmax));
#endif
    hipStream_t st = rf_stream(stream);
    const int which = (a_kc ? 2 : 0) + (b_kc ? 1 : 0);
    static void (*const kerns[4])(GemmArgs) = {gemm32_kernel<false, false>, gemm32_kernel<false, true>,
                                               gemm32_kernel<true, false>, gemm32_kernel<true, true>};
    static bool attr_set[4] = {false, false, false, false};
    if (!attr_set[which]) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kerns[which]),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
        if (e != hipSuccess) return rf_set_error(RF_EHIP, "gemm32_kernel: %s", hipGetErrorString(e));
        attr_set[which] = true;
    }
    // many segments per cut tile (a WG's range under a quarter of some problem's k steps): defer the combine
    g.defer = 0;
    for (int i = 0; i < g.np; ++i)
        if ((int64_t)g.p[i].nk * G > 4 * g.units) g.defer = 1;
    hipLaunchKernelGGL(kerns[which], dim3(G), dim3(kThreads), kLdsBytes, st, g);
    if (g.defer) hipLaunchKernelGGL(gemm32_fixup_kernel, dim3((unsigned)(tiles * kFixParts)), dim3(kThreads), 0, st, g, G);
    return rf_check_launch("gemm32_kernel");
}

extern "C" int rf_gemm_f32(const float* A, int64_t lda, int32_t a_kc, const float* B, int64_t ldb, int32_t b_kc,
                           int64_t M, int64_t N, int64_t K, const float* bias, int32_t act, float* C, int64_t ldc,
                           void* ws, size_t ws_bytes, void* stream) {
    const rf_gemm_f32_problem p{A, lda, B, ldb, C, ldc, bias, M, N, K, act, 0};
    return rf_gemm_f32_grouped(&p, 1, a_kc, b_kc, ws, ws_bytes, stream);
}
