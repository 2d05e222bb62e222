// gemm_lab_f32.hip — standalone fp32 GEMM experiment (diagnostics only, not part of librf):
// y[M,N] = x[M,K] W[N,K]^T, fp32 in and out, on the LDS-DMA ring (128-byte rows = 32 floats per k-step) over a
// sweep of tile / wave / stage / MFMA-shape / split-K geometries (the DSSM tower shapes), checked against a naive
// fp32 kernel and timed with HIP events (interleaved rounds in one process).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_lab_f32 tools/gemm_lab_f32.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                              \
        }                                                                                         \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

// non-template wrapper: the builtin inside a template kernel's discarded branch breaks host-side instantiation
__device__ __forceinline__ void glds16(const float* src, float* dst) {
    __builtin_amdgcn_global_load_lds(src, (lds_void*)dst, 16, 0, 0);
}

__device__ unsigned long long g_stamp[4096][2][2];  // [workgroup][start/end][memtime, memrealtime]

template <int N>
__device__ __forceinline__ void vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Block tile BM x BN x 32 (fp32), WM x WN waves, STAGES-deep LDS ring, chunk c of row r at c ^ (r & 7).
// MF 0: v_mfma_f32_16x16x4f32 — lane (lr, lg) reads chunks lg and 4 + lg of its row (8 floats, 8 MFMAs);
// MF 1: v_mfma_f32_32x32x2f32 — lane (i = l & 31, h = l >> 5) reads chunks h, 2 + h, 4 + h, 6 + h (16 floats,
//       16 MFMAs); A and B in the same permuted k order. blockIdx.y = split (K range [y kspan, ...)).
template <int BM, int BN, int STAGES, int WM, int WN, int MF, int MODE = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_f32(const float* __restrict__ x, const float* __restrict__ w,
                                                         float* __restrict__ y, int M, int N, int K, int kspan) {
    constexpr int NW = WM * WN;
    constexpr int TM = BM / WM, TN = BN / WN;
    constexpr int A_EL = BM * 32, B_EL = BN * 32;
    constexpr int GA = BM / 8, GB = BN / 8;
    constexpr int L = (GA + GB) / NW;
    static_assert((GA + GB) % NW == 0, "loads must split evenly over waves");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    float* lds = reinterpret_cast<float*>(smem_raw);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int tiles_n = (N + BN - 1) / BN;
    const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
    const int kb = blockIdx.y * kspan;
    const int nk = min(kspan, K - kb) / 32;
    y += (int64_t)blockIdx.y * M * N;
    const int rr = lane >> 3, pos = lane & 7;

    auto stage = [&](int kt, int s) {
        float* As = lds + s * (A_EL + B_EL);
        float* Bs = As + A_EL;
        const int k0 = MODE == 1 ? 0 : kb + kt * 32;  // MODE 1: every step re-reads the first k-slab (L2-resident)
#pragma unroll
        for (int it = 0; it < L; ++it) {
            const int g = wave + NW * it;
            if (g < GA) {
                const int r = g * 8 + rr;
                const int row = m0 + r < M ? m0 + r : M - 1;
                __builtin_amdgcn_global_load_lds(x + (int64_t)row * K + k0 + ((pos ^ rr) << 2), (lds_void*)(As + g * 256), 16, 0, 0);
            } else {
                const int gb = g - GA, r = gb * 8 + rr;
                const int col = n0 + r < N ? n0 + r : N - 1;
                __builtin_amdgcn_global_load_lds(w + (int64_t)col * K + k0 + ((pos ^ rr) << 2), (lds_void*)(Bs + gb * 256), 16, 0, 0);
            }
        }
    };

    // MODE >= 3: the copy sources computed once (row clamps, swizzle, 64-bit products) and advanced by k only
    const float* srcp[L];
    uint32_t dsto[L];
#pragma unroll
    for (int it = 0; it < L; ++it) {
        const int g = wave + NW * it;
        if (g < GA) {
            const int r = g * 8 + rr;
            const int row = m0 + r < M ? m0 + r : M - 1;
            srcp[it] = x + (int64_t)row * K + kb + ((pos ^ rr) << 2);
            dsto[it] = g * 256;
        } else {
            const int gb = g - GA, r = gb * 8 + rr;
            const int col = n0 + r < N ? n0 + r : N - 1;
            srcp[it] = w + (int64_t)col * K + kb + ((pos ^ rr) << 2);
            dsto[it] = A_EL + gb * 256;
        }
    }
    auto stage2 = [&](int kt, int s) {
        float* base = lds + s * (A_EL + B_EL);
#pragma unroll
        for (int it = 0; it < L; ++it)
            glds16(srcp[it] + kt * 32, base + dsto[it]);
    };
    const bool stamp = MODE == 7 && tid == 0 && blockIdx.x < 4096 && blockIdx.y == 0;
    if (stamp) {
        g_stamp[blockIdx.x][0][0] = __builtin_amdgcn_s_memtime();
        g_stamp[blockIdx.x][0][1] = __builtin_amdgcn_s_memrealtime();
    }
    if constexpr (MF == 0 && (MODE == 12 || MODE == 13)) {
        // mode 5's mid-step barrier plus a hand-placed interleave (regions fenced by sched_barrier): phase A =
        // the first half's 64 MFMAs with this stage's 8 second-half fragment reads spread among them (one per 8
        // MFMAs); barrier; phase B = the second half's 64 MFMAs with stage kt + 2's 8 LDS-DMA copies and stage
        // kt + 1's 8 first-half reads spread among them (an LDS-DMA copy costs ~60 issue cycles: alone between
        // 32-cycle MFMAs it mostly hides; eight back to back stall the MFMA pipe). MODE 13: copies at one per
        // 8 MFMAs in phase A instead (reads of both kinds in phase B)
        static_assert(STAGES == 2, "two stages");
        constexpr int FM = TM / 16, FN = TN / 16;
        static_assert(FM == 4 && FN == 4 && L == 8, "64 MFMAs per half, 8 copies per wave");
        const int lr = lane & 15, lg = lane >> 4;
        f4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        f4 af[2][FM], bfr[2][FN];
        auto rd1 = [&](int st, int h, int f) {  // fragment f: 0..3 A rows, 4..7 B rows
            const float* A = lds + st * (A_EL + B_EL);
            const int ch = 4 * h + lg;
            if (f < 4) {
                const int r = wm * TM + f * 16 + lr;
                af[h][f] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
            } else {
                const int r = wn * TN + (f - 4) * 16 + lr;
                bfr[h][f - 4] = *reinterpret_cast<const f4*>(A + A_EL + r * 32 + ((ch ^ (r & 7)) << 2));
            }
        };
        auto mm8 = [&](int h, int g) {  // MFMAs 8g .. 8g + 7 of the half: e = g / 2, i = 2 (g & 1) + (0, 1)
            const int e = g >> 1;
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int i = 2 * (g & 1) + ii;
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
                }
        };
        auto copy1 = [&](int kt, int st, int it) {
            glds16(srcp[it] + kt * 32, lds + st * (A_EL + B_EL) + dsto[it]);
        };
        stage2(0, 0);
        if (nk > 1) stage2(1, 1);
        if (nk > 1) vmcnt<L>();
        else vmcnt<0>();
        __builtin_amdgcn_s_barrier();
#pragma unroll
        for (int f = 0; f < 8; ++f) rd1(0, 0, f);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = kt & 1;
            const int kc = min(kt + 2, nk - 1);  // past the end: re-copies the last stage into a dead buffer
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
            // phase A
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                mm8(0, g);
                __builtin_amdgcn_sched_barrier(0);
                rd1(s, 1, g);
                __builtin_amdgcn_sched_barrier(0);
            }
            const bool more = kt + 1 < nk;
            if (more) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_sched_barrier(0);
            // phase B (the next stage's reads only when it exists: a wave-uniform branch per read)
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                mm8(1, g);
                __builtin_amdgcn_sched_barrier(0);
                copy1(kc, s, g);  // last step: a dead buffer and stale reads, both unused
                rd1(s ^ 1, 0, g);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        vmcnt<0>();  // no LDS-DMA copy may land after the workgroup's LDS is released
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 1 && MODE == 11) {
        // 32x32x2, register-staged copies: step kt's global loads (16-byte chunks, 8 per thread at 128x128) are
        // issued at its top into registers, land under its MFMAs, and are written to the other LDS stage after
        // them (chunk c of row r at c ^ (r & 7)); one barrier per step. An LDS-DMA copy costs ~100 issue cycles
        // beside MFMAs; a global load + ds_write pair far less.
        static_assert(STAGES == 2, "two stages");
        constexpr int FM = TM / 32, FN = TN / 32;
        constexpr int CH = (BM + BN) * 8 / (64 * NW);  // 16-byte chunks per thread per stage
        const int li = lane & 31, hl = lane >> 5;
        f16v acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        const float* gsrc[CH];
        uint32_t ldo[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const int idx = tid + c * 64 * NW;  // chunk index over the stage: rows of A then B, 8 chunks per row
            const int r = idx >> 3, ch = idx & 7;
            if (r < BM) {
                const int row = m0 + r < M ? m0 + r : M - 1;
                gsrc[c] = x + (int64_t)row * K + kb + ch * 4;
                ldo[c] = r * 32 + ((ch ^ (r & 7)) << 2);
            } else {
                const int rb = r - BM;
                const int col = n0 + rb < N ? n0 + rb : N - 1;
                gsrc[c] = w + (int64_t)col * K + kb + ch * 4;
                ldo[c] = A_EL + rb * 32 + ((ch ^ (rb & 7)) << 2);
            }
        }
        f4 rg[CH];
        auto gload = [&](int kt) {
#pragma unroll
            for (int c = 0; c < CH; ++c) rg[c] = *reinterpret_cast<const f4*>(gsrc[c] + kt * 32);
        };
        auto lwrite = [&](int st) {
            float* base = lds + st * (A_EL + B_EL);
#pragma unroll
            for (int c = 0; c < CH; ++c) *reinterpret_cast<f4*>(base + ldo[c]) = rg[c];
        };
        gload(0);
        lwrite(0);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = kt & 1;
            __syncthreads();
            if (kt + 1 < nk) gload(kt + 1);
            const float* A = lds + s * (A_EL + B_EL);
            const float* B = A + A_EL;
            f4 af[4][FM], bfr[4][FN];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ch = 2 * q + hl;
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const int r = wm * TM + i * 32 + li;
                    af[q][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int r = wn * TN + j * 32 + li;
                    bfr[q][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][i][e], bfr[q][j][e], acc[i][j], 0, 0, 0);
            if (kt + 1 < nk) lwrite(s ^ 1);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 32 + li;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * TM + i * 32 + 8 * (r >> 2) + 4 * hl + (r & 3);
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 1 && (MODE == 5 || MODE == 4)) {
        // 32x32x2: MODE 5 = two-stage ring with the barrier mid-step (as MF 0 mode 5): stage kt's second-half
        // fragments read under its first-half MFMAs, stage kt + 1's first half under its second half;
        // MODE 4 = barrier at the step top, copies from precomputed pointers, halves' reads split as mode 5
        static_assert(STAGES == 2, "two stages");
        constexpr int FM = TM / 32, FN = TN / 32;
        const int li = lane & 31, hl = lane >> 5;
        f16v acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
        f4 af[2][2][FM], bfr[2][2][FN];  // [half][quarter within half]
        auto rd = [&](int st, int h) {
            const float* A = lds + st * (A_EL + B_EL);
            const float* B = A + A_EL;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const int ch = 2 * (2 * h + qq) + hl;
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const int r = wm * TM + i * 32 + li;
                    af[h][qq][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int r = wn * TN + j * 32 + li;
                    bfr[h][qq][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
                }
            }
        };
        auto mm = [&](int h) {
#pragma unroll
            for (int qq = 0; qq < 2; ++qq)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[h][qq][i][e], bfr[h][qq][j][e], acc[i][j], 0, 0, 0);
        };
        if constexpr (MODE == 5) {
            stage2(0, 0);
            if (nk > 1) stage2(1, 1);
            if (nk > 1) vmcnt<L>();
            else vmcnt<0>();
            __builtin_amdgcn_s_barrier();
            rd(0, 0);
            for (int kt = 0; kt < nk; ++kt) {
                const int s = kt & 1;
                rd(s, 1);
                __builtin_amdgcn_sched_barrier(0);
                mm(0);
                __builtin_amdgcn_sched_barrier(0);
                if (kt + 1 < nk) {
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_s_barrier();
                    __builtin_amdgcn_sched_barrier(0);
                    if (kt + 2 < nk) stage2(kt + 2, s);
                    rd(s ^ 1, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
                mm(1);
            }
        } else {
            stage2(0, 0);
            for (int kt = 0; kt < nk; ++kt) {
                const int s = kt & 1;
                vmcnt<0>();
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (kt + 1 < nk) stage2(kt + 1, s ^ 1);
                rd(s, 0);
                rd(s, 1);
                __builtin_amdgcn_sched_barrier(0);
                mm(0);
                mm(1);
            }
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 32 + li;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * TM + i * 32 + 8 * (r >> 2) + 4 * hl + (r & 3);
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 0 && MODE == 5) {
        // two-stage ring, barrier mid-step: step kt reads stage kt's second-half fragments under its first-half
        // MFMAs, then (stage kt + 1 landed, everyone done with stage kt's buffer) issues stage kt + 2's copies
        // into that buffer and reads stage kt + 1's first-half fragments under its second-half MFMAs
        static_assert(STAGES == 2, "mode 5: two stages");
        constexpr int FM = TM / 16, FN = TN / 16;
        const int lr = lane & 15, lg = lane >> 4;
        f4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        f4 af[2][FM], bfr[2][FN];
        auto rd = [&](int st, int h) {
            const float* A = lds + st * (A_EL + B_EL);
            const float* B = A + A_EL;
            const int ch = 4 * h + lg;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wm * TM + i * 16 + lr;
                af[h][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int r = wn * TN + j * 16 + lr;
                bfr[h][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
            }
        };
        auto mm = [&](int h) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
        };
        stage2(0, 0);
        if (nk > 1) stage2(1, 1);
        if (nk > 1) vmcnt<L>();
        else vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        rd(0, 0);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = kt & 1;
            rd(s, 1);
            __builtin_amdgcn_sched_barrier(0);
            mm(0);
            __builtin_amdgcn_sched_barrier(0);
            if (kt + 1 < nk) {
                asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                if (kt + 2 < nk) stage2(kt + 2, s);
                rd(s ^ 1, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
            mm(1);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 0 && (MODE == 3 || MODE == 4)) {
        constexpr int FM = TM / 16, FN = TN / 16;
        const int lr = lane & 15, lg = lane >> 4;
        f4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < STAGES - 1; ++p)
            if (p < nk) stage2(p, p);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = kt % STAGES;
            if (STAGES >= 3 && kt + 1 < nk) vmcnt<L>();
            else vmcnt<0>();
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (kt + STAGES - 1 < nk) stage2(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
            const float* A = lds + s * (A_EL + B_EL);
            const float* B = A + A_EL;
            f4 af[2][FM], bfr[2][FN];
            auto rd = [&](int h) {
                const int ch = 4 * h + lg;
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const int r = wm * TM + i * 16 + lr;
                    af[h][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int r = wn * TN + j * 16 + lr;
                    bfr[h][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
                }
            };
            auto mm = [&](int h, int e) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
            };
            rd(0);
            if constexpr (MODE == 4) {  // second half's reads issued under the first half's first MFMAs
                __builtin_amdgcn_sched_barrier(0);
                mm(0, 0);
                __builtin_amdgcn_sched_barrier(0);
                rd(1);
                __builtin_amdgcn_sched_barrier(0);
                mm(0, 1);
                mm(0, 2);
                mm(0, 3);
            } else {
                rd(1);
                __builtin_amdgcn_sched_barrier(0);
                mm(0, 0);
                mm(0, 1);
                mm(0, 2);
                mm(0, 3);
            }
            mm(1, 0);
            mm(1, 1);
            mm(1, 2);
            mm(1, 3);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 0 && (MODE < 3 || MODE >= 7)) {
        constexpr int FM = TM / 16, FN = TN / 16;
        const int lr = lane & 15, lg = lane >> 4;
        f4 acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < STAGES - 1; ++p)
            if (p < nk) stage(p, p);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = kt % STAGES;
            if constexpr (MODE != 2 && MODE != 10) {  // MODE 2 / 10: no waits, no barrier (timing only)
                if (STAGES >= 3 && kt + 1 < nk) vmcnt<L>();
                else vmcnt<0>();
                __builtin_amdgcn_s_barrier();
            }
            __builtin_amdgcn_sched_barrier(0);
            // MODE 9: no copies inside the loop (the prologue's stage is re-read: timing only)
            if (MODE != 9 && MODE != 10 && kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
            const float* A = lds + (MODE == 8 ? 0 : s) * (A_EL + B_EL);
            const float* B = A + A_EL;
            f4 af[2][FM], bfr[2][FN];
            // MODE 8: the fragment reads of one step only, fed to every step's MFMAs (timing only)
            if ((MODE != 8 && MODE != 10) || kt == 0)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ch = 4 * h + lg;
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const int r = wm * TM + i * 16 + lr;
                    af[h][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int r = wn * TN + j * 16 + lr;
                    bfr[h][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    } else if constexpr (MF == 1) {
        constexpr int FM = TM / 32, FN = TN / 32;
        const int li = lane & 31, h = lane >> 5;
        f16v acc[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
#pragma unroll
        for (int p = 0; p < STAGES - 1; ++p)
            if (p < nk) stage(p, p);
        for (int kt = 0; kt < nk; ++kt) {
            const int s = MODE == 10 ? 0 : kt % STAGES;
            if constexpr (MODE != 10 && MODE != 2) {
                if (STAGES >= 3 && kt + 1 < nk) vmcnt<L>();
                else vmcnt<0>();
                __builtin_amdgcn_s_barrier();
            }
            __builtin_amdgcn_sched_barrier(0);
            if (MODE != 10 && kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
            const float* A = lds + s * (A_EL + B_EL);
            const float* B = A + A_EL;
            f4 af[4][FM], bfr[4][FN];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ch = 2 * q + h;
#pragma unroll
                for (int i = 0; i < FM; ++i) {
                    const int r = wm * TM + i * 32 + li;
                    af[q][i] = *reinterpret_cast<const f4*>(A + r * 32 + ((ch ^ (r & 7)) << 2));
                }
#pragma unroll
                for (int j = 0; j < FN; ++j) {
                    const int r = wn * TN + j * 32 + li;
                    bfr[q][j] = *reinterpret_cast<const f4*>(B + r * 32 + ((ch ^ (r & 7)) << 2));
                }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int e = 0; e < 4; ++e)
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[q][i][e], bfr[q][j][e], acc[i][j], 0, 0, 0);
        }
        // C layout of 32x32: lane l, reg r: col = l & 31, row = 8 (r >> 2) + 4 (l >> 5) + (r & 3)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 32 + li;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * TM + i * 32 + 8 * (r >> 2) + 4 * h + (r & 3);
                    if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
    }
    if (stamp) {
        g_stamp[blockIdx.x][1][0] = __builtin_amdgcn_s_memtime();
        g_stamp[blockIdx.x][1][1] = __builtin_amdgcn_s_memrealtime();
    }
}

// k-width 64 floats per step (256-byte rows, 16 chunks; chunk c of row r at c ^ (r & 7)), 128x128 tile,
// 4 waves of 64x64, two-stage LDS-DMA ring (128 KiB: one workgroup per CU), fragment reads in two halves
// of 32 k (the second half's reads issued under the first half's first MFMAs)
template <int S_UNUSED>
__global__ __launch_bounds__(256) void gemm_f32_k64(const float* __restrict__ x, const float* __restrict__ w,
                                                    float* __restrict__ y, int M, int N, int K, int kspan) {
    constexpr int BM = 128, BN = 128, KW = 64, TM = 64, TN = 64, FM = 4, FN = 4;
    constexpr int A_EL = BM * KW, B_EL = BN * KW;
    constexpr int L = (BM / 4 + BN / 4) / 4;  // glds per thread per stage: 16
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    float* lds = reinterpret_cast<float*>(smem_raw);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int wm = wave >> 1, wn = wave & 1;
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int tiles_n = (N + BN - 1) / BN;
    const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
    const int kb = blockIdx.y * kspan;
    const int nk = min(kspan, K - kb) / KW;
    y += (int64_t)blockIdx.y * M * N;
    const int rr = lane >> 4, pos = lane & 15;  // one instruction: 4 rows x 16 chunks
    const float* srcp[L];
    uint32_t dsto[L];
#pragma unroll
    for (int it = 0; it < L; ++it) {
        const int g = wave + 4 * it;  // 0..63: 32 groups of A rows, 32 of B rows (4 rows each)
        if (g < BM / 4) {
            const int r = g * 4 + rr;
            const int row = m0 + r < M ? m0 + r : M - 1;
            srcp[it] = x + (int64_t)row * K + kb + ((pos ^ (r & 7)) << 2);
            dsto[it] = g * 4 * KW;
        } else {
            const int gb = g - BM / 4, r = gb * 4 + rr;
            const int col = n0 + r < N ? n0 + r : N - 1;
            srcp[it] = w + (int64_t)col * K + kb + ((pos ^ (r & 7)) << 2);
            dsto[it] = A_EL + gb * 4 * KW;
        }
    }
    auto stage = [&](int kt, int s) {
        float* base = lds + s * (A_EL + B_EL);
#pragma unroll
        for (int it = 0; it < L; ++it) glds16(srcp[it] + kt * KW, base + dsto[it]);
    };
    f4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    stage(0, 0);
    for (int kt = 0; kt < nk; ++kt) {
        const int s = kt & 1;
        vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) stage(kt + 1, s ^ 1);
        const float* A = lds + s * (A_EL + B_EL);
        const float* B = A + A_EL;
        f4 af[2][FM], bfr[2][FN];
        auto rd = [&](int q, int h) {  // quarter q (16 k: chunks 4q .. 4q + 3), into slot h
            const int ch = 4 * q + lg;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wm * TM + i * 16 + lr;
                af[h][i] = *reinterpret_cast<const f4*>(A + r * KW + ((ch ^ (r & 7)) << 2));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int r = wn * TN + j * 16 + lr;
                bfr[h][j] = *reinterpret_cast<const f4*>(B + r * KW + ((ch ^ (r & 7)) << 2));
            }
        };
        auto mm = [&](int h) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[h][i][e], bfr[h][j][e], acc[i][j], 0, 0, 0);
        };
        rd(0, 0);
        rd(1, 1);
        __builtin_amdgcn_sched_barrier(0);
        mm(0);
        __builtin_amdgcn_sched_barrier(0);
        rd(2, 0);
        __builtin_amdgcn_sched_barrier(0);
        mm(1);
        __builtin_amdgcn_sched_barrier(0);
        rd(3, 1);
        __builtin_amdgcn_sched_barrier(0);
        mm(0);
        mm(1);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
        const int col = n0 + wn * TN + j * 16 + lr;
        if (col >= N) continue;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                if (row < M) y[(int64_t)row * N + col] = acc[i][j][r];
            }
    }
}

__global__ void ref_gemm(const float* x, const float* w, float* y, int M, int N, int K) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)M * N) return;
    const int m = idx / N, n = idx % N;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(x[(int64_t)m * K + k], w[(int64_t)n * K + k], s);
    y[idx] = s;
}

__global__ void sum_splits(const float* p, float* y, int64_t n, int S) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float s = p[i];
    for (int k = 1; k < S; ++k) s += p[k * n + i];
    y[i] = s;
}

__global__ void fill_f32(float* p, int64_t n, uint32_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    p[i] = ((h & 0xffffff) / 16777216.0f) * 2.f - 1.f;
}

struct Variant {
    std::string name;
    void (*fn)(const float*, const float*, float*, int, int, int, int);
    int BM, BN, threads, S;
    size_t lds;
};

template <int BM, int BN, int STAGES, int WM, int WN, int MF, int MODE = 0>
Variant mk(const char* nm, int S) {
    Variant v;
    v.name = nm;
    v.fn = gemm_f32<BM, BN, STAGES, WM, WN, MF, MODE>;
    v.BM = BM;
    v.BN = BN;
    v.threads = 64 * WM * WN;
    v.S = S;
    v.lds = (size_t)STAGES * (BM + BN) * 128;
    CK(hipFuncSetAttribute((const void*)v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
    return v;
}

Variant mk64(const char* nm, int S) {
    Variant v;
    v.name = nm;
    v.fn = gemm_f32_k64<0>;
    v.BM = 128;
    v.BN = 128;
    v.threads = 256;
    v.S = S;
    v.lds = (size_t)2 * 256 * 256;
    CK(hipFuncSetAttribute((const void*)v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
    return v;
}

int main(int argc, char** argv) {
    std::vector<Variant> vs = {
        mk<128, 128, 2, 2, 2, 0>("128x128 s2 w4 16x16x4 S1 (rf)", 1),
        mk<128, 128, 2, 2, 2, 0>("128x128 s2 w4 16x16x4 S2 (rf)", 2),
        mk<128, 128, 2, 2, 2, 0, 5>("128x128 S1 m5", 1),
        mk<128, 128, 2, 2, 2, 0, 12>("128x128 S1 m12 interleaved", 1),
        mk<128, 128, 2, 2, 2, 0, 12>("128x128 S2 m12 interleaved", 2),
    };
    struct Shape { int M, K, N; };
    std::vector<Shape> shapes = {{4096, 8704, 1024}, {4096, 20480, 1024}};
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    for (auto sh : shapes) {
        const int M = sh.M, K = sh.K, N = sh.N;
        float *x, *w, *y, *yr, *part;
        CK(hipMalloc(&x, (size_t)M * K * 4));
        CK(hipMalloc(&w, (size_t)N * K * 4));
        CK(hipMalloc(&y, (size_t)M * N * 4));
        CK(hipMalloc(&yr, (size_t)M * N * 4));
        CK(hipMalloc(&part, (size_t)8 * M * N * 4));
        fill_f32<<<(M * (int64_t)K + 255) / 256, 256>>>(x, (int64_t)M * K, 1);
        fill_f32<<<(N * (int64_t)K + 255) / 256, 256>>>(w, (int64_t)N * K, 2);
        ref_gemm<<<(M * (int64_t)N + 255) / 256, 256>>>(x, w, yr, M, N, K);
        CK(hipDeviceSynchronize());
        std::vector<float> hr((size_t)M * N), hy((size_t)M * N);
        CK(hipMemcpy(hr.data(), yr, hr.size() * 4, hipMemcpyDeviceToHost));
        std::vector<std::vector<float>> ts(vs.size());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        auto launch = [&](const Variant& v) {
            const int tiles = ((M + v.BM - 1) / v.BM) * ((N + v.BN - 1) / v.BN);
            const int kspan = ((K + v.S - 1) / v.S + 63) / 64 * 64;
            hipLaunchKernelGGL(v.fn, dim3(tiles, v.S), dim3(v.threads), v.lds, 0, x, w, v.S > 1 ? part : y, M, N, K, kspan);
            if (v.S > 1) sum_splits<<<(M * (int64_t)N + 255) / 256, 256>>>(part, y, (int64_t)M * N, v.S);
        };
        for (size_t v = 0; v < vs.size(); ++v) {  // correctness
            CK(hipMemset(y, 0, (size_t)M * N * 4));
            launch(vs[v]);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hy.data(), y, hy.size() * 4, hipMemcpyDeviceToHost));
            double md = 0;
            for (size_t i = 0; i < hy.size(); ++i) md = std::max(md, (double)fabsf(hy[i] - hr[i]));
            if (md > 1e-2 && vs[v].name.find("mode") == std::string::npos && vs[v].name.find("clock") == std::string::npos) printf("MISMATCH %s M=%d K=%d: max|d| %g\n", vs[v].name.c_str(), M, K, md);
        }
        for (int r = 0; r < rounds; ++r)
            for (size_t v = 0; v < vs.size(); ++v) {
                for (int i = 0; i < 2; ++i) launch(vs[v]);
                const int it = 10;
                CK(hipEventRecord(a));
                for (int i = 0; i < it; ++i) launch(vs[v]);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts[v].push_back(ms / it * 1000.f);
            }
        printf("== M=%d K=%d N=%d (%.2f GFLOP)\n", M, K, N, 2.0 * M * N * K / 1e9);
        for (size_t v = 0; v < vs.size(); ++v) {
            if (vs[v].name.find("clock") == std::string::npos) continue;
            for (int i = 0; i < 20; ++i) launch(vs[v]);  // warm, then one stamped launch read back
            launch(vs[v]);
            CK(hipDeviceSynchronize());
            static unsigned long long hs[4096][2][2];
            CK(hipMemcpyFromSymbol(hs, HIP_SYMBOL(g_stamp), sizeof(hs)));
            const int tiles = ((M + vs[v].BM - 1) / vs[v].BM) * ((N + vs[v].BN - 1) / vs[v].BN);
            std::vector<double> ghz;
            for (int t = 0; t < tiles && t < 4096; ++t) {
                const double dc = (double)(hs[t][1][0] - hs[t][0][0]), dr = (double)(hs[t][1][1] - hs[t][0][1]);
                if (dr > 0) ghz.push_back(dc / dr * 0.1);
            }
            std::sort(ghz.begin(), ghz.end());
            if (!ghz.empty()) printf("  %-34s in-kernel clock median %.3f GHz (min %.3f, max %.3f)\n", vs[v].name.c_str(), ghz[ghz.size() / 2], ghz[0], ghz.back());
        }
        for (size_t v = 0; v < vs.size(); ++v) {
            auto t = ts[v];
            std::sort(t.begin(), t.end());
            const double med = t[t.size() / 2];
            printf("  %-34s lds %6zu  median %8.2f us  min %8.2f us  %7.1f TF\n", vs[v].name.c_str(), vs[v].lds, med, t[0],
                   2.0 * M * N * K / med / 1e6);
        }
        fflush(stdout);
        CK(hipFree(x));
        CK(hipFree(w));
        CK(hipFree(y));
        CK(hipFree(yr));
        CK(hipFree(part));
    }
    return 0;
}
