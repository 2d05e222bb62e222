// gemm_lab.hip — standalone bf16 GEMM experiment (diagnostics only, not part of librf):
// y[M,N] = x[M,K] W[N,K]^T, bf16 in, fp32 out, over a sweep of LDS-DMA ring geometries, checked against a
// naive fp32 reference kernel and timed with HIP events (interleaved rounds in one process).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gemm_lab tools/gemm_lab.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <algorithm>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ float gelu_erf(float x) {
    const float z = x * 0.70710678118654752440f, a = fabsf(z);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, a, 1.0f));
    float p = fmaf(t, 0.17087277f, -0.82215223f);
    p = fmaf(t, p, 1.48851587f);
    p = fmaf(t, p, -1.13520398f);
    p = fmaf(t, p, 0.27886807f);
    p = fmaf(t, p, -0.18628806f);
    p = fmaf(t, p, 0.09678418f);
    p = fmaf(t, p, 0.37409196f);
    p = fmaf(t, p, 1.00002368f);
    p = fmaf(t, p, -1.26551223f);
    const float e = t * __expf(fmaf(-a, a, p));
    return z >= 0.f ? x * fmaf(-0.5f, e, 1.0f) : 0.5f * x * e;
}

template <int N>
__device__ __forceinline__ void vmcnt() {
    if constexpr (N >= 63) asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most `pending` stages (of L loads each) issued after the one we need are outstanding
template <int L, int MAXP>
__device__ __forceinline__ void wait_stages(int pending) {
    if constexpr (MAXP >= 3) { if (pending >= 3) { vmcnt<3 * L>(); return; } }
    if constexpr (MAXP >= 2) { if (pending >= 2) { vmcnt<2 * L>(); return; } }
    if constexpr (MAXP >= 1) { if (pending >= 1) { vmcnt<L>(); return; } }
    vmcnt<0>();
}

// Block tile BM x BN x 64, WM x WN waves (wave tile BM/WM x BN/WN), 16x16x32 bf16 MFMA, STAGES-deep LDS ring
// filled by global_load_lds_dwordx4 (one instruction = 8 rows x 128 B, lane-linear; chunk c of row r lands at
// c ^ (r & 7) by swizzling the source). SCHED 0: all fragment reads, then all MFMAs; SCHED 1: reads of the
// second k-half issued among the first half's MFMAs (compiler-scheduled).
// EPI 0: raw fp32, lane-scattered stores; 1: bias + gelu fp32 scattered (rf_linear_fwd's epilogue); 2: the same
// through an LDS transpose (16-byte row stores); 3: bias + gelu -> bf16 scattered (the stats GEMM's output);
// 4: bf16 through the LDS transpose
template <int BM, int BN, int STAGES, int WM, int WN, int SCHED, int EPI = 0>
__global__ __launch_bounds__(64 * WM * WN) void gemm_v(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                       float* __restrict__ y, int M, int N, int K) {
    constexpr int NW = WM * WN, NT = 64 * NW;
    constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
    constexpr int A_EL = BM * 64, B_EL = BN * 64;
    constexpr int GA = BM / 8, GB = BN / 8;       // glds instructions per stage (block)
    constexpr int L = (GA + GB) / NW;              // per wave
    static_assert((GA + GB) % NW == 0, "loads must split evenly over waves");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    uint16_t* lds = reinterpret_cast<uint16_t*>(smem_raw);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
    const int wm = wave / WN, wn = wave % WN;
    const int nwg = gridDim.x, q8 = nwg / 8, r8 = nwg % 8, xcd = blockIdx.x % 8;
    const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + blockIdx.x / 8;
    const int tiles_n = (N + BN - 1) / BN;
    const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
    const int nk = K / 64;
    const int rr = lane >> 3, pos = lane & 7;

    auto stage = [&](int kt, int s) {
        uint16_t* As = lds + s * (A_EL + B_EL);
        uint16_t* Bs = As + A_EL;
        const int k0 = kt * 64;
#pragma unroll
        for (int it = 0; it < L; ++it) {
            const int g = wave + NW * it;
            if (g < GA) {
                const int r = g * 8 + rr;
                const int row = m0 + r < M ? m0 + r : M - 1;
                __builtin_amdgcn_global_load_lds(x + (int64_t)row * K + k0 + ((pos ^ rr) << 3), (lds_void*)(As + g * 512), 16, 0, 0);
            } else {
                const int gb = g - GA, r = gb * 8 + rr;
                const int col = n0 + r < N ? n0 + r : N - 1;
                __builtin_amdgcn_global_load_lds(w + (int64_t)col * K + k0 + ((pos ^ rr) << 3), (lds_void*)(Bs + gb * 512), 16, 0, 0);
            }
        }
    };

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
        const int pend = min(STAGES - 2, nk - 1 - kt);
        wait_stages<L, STAGES - 2>(pend);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + STAGES - 1 < nk) stage(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
        const uint16_t* A = lds + s * (A_EL + B_EL);
        const uint16_t* B = A + A_EL;
        bf16x8 af[2][FM], bfr[2][FN];
        auto rd = [&](int h) {
            const int ch = 4 * h + lg;
#pragma unroll
            for (int i = 0; i < FM; ++i) {
                const int r = wm * TM + i * 16 + lr;
                af[h][i] = *reinterpret_cast<const bf16x8*>(A + r * 64 + ((ch ^ (r & 7)) << 3));
            }
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                const int r = wn * TN + j * 16 + lr;
                bfr[h][j] = *reinterpret_cast<const bf16x8*>(B + r * 64 + ((ch ^ (r & 7)) << 3));
            }
        };
        auto mm = [&](int h) {
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[h][i], bfr[h][j], acc[i][j], 0, 0, 0);
        };
        if constexpr (SCHED == 0) {
            rd(0);
            rd(1);
            __builtin_amdgcn_sched_barrier(0);
            mm(0);
            mm(1);
        } else {
            rd(0);
            rd(1);
            mm(0);
            mm(1);
        }
    }
    if constexpr (EPI == 0 || EPI == 1 || EPI == 3) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int col = n0 + wn * TN + j * 16 + lr;
            if (col >= N) continue;
            const float bv = 0.001f * (col & 7);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wm * TM + i * 16 + lg * 4 + r;
                    if (row >= M) continue;
                    if constexpr (EPI == 0) y[(int64_t)row * N + col] = acc[i][j][r];
                    else if constexpr (EPI == 1) y[(int64_t)row * N + col] = gelu_erf(acc[i][j][r] + bv);
                    else reinterpret_cast<__bf16*>(y)[(int64_t)row * N + col] = (__bf16)gelu_erf(acc[i][j][r] + bv);
                }
        }
    } else {
        // LDS transpose: the wave's TM x TN tile row-major in LDS (row pitch TN + 4 floats), then each lane
        // stores 16-byte pieces of rows
        __syncthreads();  // every wave is done with the ring
        constexpr int PITCH = TN + 4;
        float* t = reinterpret_cast<float*>(smem_raw) + wave * TM * PITCH;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int cl = j * 16 + lr;
            const float bv = 0.001f * ((n0 + wn * TN + cl) & 7);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) t[(i * 16 + lg * 4 + r) * PITCH + cl] = gelu_erf(acc[i][j][r] + bv);
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes
        constexpr int EL = EPI == 2 ? 4 : 8;   // elements per 16-byte store
        constexpr int PER_ROW = TN / EL;
        for (int q = lane; q < TM * PER_ROW; q += 64) {
            const int rl = q / PER_ROW, c0 = (q % PER_ROW) * EL;
            const int row = m0 + wm * TM + rl, col = n0 + wn * TN + c0;
            if (row >= M || col >= N) continue;
            const float* src = t + rl * PITCH + c0;
            if constexpr (EPI == 2) {
                *reinterpret_cast<float4*>(y + (int64_t)row * N + col) = make_float4(src[0], src[1], src[2], src[3]);
            } else {
                typedef __bf16 b8 __attribute__((ext_vector_type(8)));
                b8 v;
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (__bf16)src[e];
                *reinterpret_cast<b8*>(reinterpret_cast<__bf16*>(y) + (int64_t)row * N + col) = v;
            }
        }
    }
}

__global__ void ref_gemm(const uint16_t* x, const uint16_t* w, float* y, int M, int N, int K) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (int64_t)M * N) return;
    const int m = idx / N, n = idx % N;
    float s = 0.f;
    for (int k = 0; k < K; ++k) {
        const float a = __uint_as_float((uint32_t)x[(int64_t)m * K + k] << 16);
        const float b = __uint_as_float((uint32_t)w[(int64_t)n * K + k] << 16);
        s = fmaf(a, b, s);
    }
    y[idx] = s;
}

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    const float v = ((h & 0xffffff) / 16777216.0f) * 2.f - 1.f;
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
}

struct Variant {
    std::string name;
    void (*fn)(const uint16_t*, const uint16_t*, float*, int, int, int);
    int BM, BN, threads, epi;
    size_t lds;
};

template <int BM, int BN, int STAGES, int WM, int WN, int SCHED, int EPI = 0>
Variant mk(const char* nm) {
    Variant v;
    v.name = nm;
    v.fn = gemm_v<BM, BN, STAGES, WM, WN, SCHED, EPI>;
    v.epi = EPI;
    v.BM = BM;
    v.BN = BN;
    v.threads = 64 * WM * WN;
    v.lds = (size_t)STAGES * (BM + BN) * 64 * 2;
    CK(hipFuncSetAttribute((const void*)v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)v.lds));
    return v;
}

int main(int argc, char** argv) {
    std::vector<Variant> vs = {
        mk<64, 128, 2, 1, 4, 0, 1>("64x128 s2 epi1 gelu f32 scat"),
        mk<64, 128, 3, 1, 4, 0, 1>("64x128 s3 epi1 gelu f32 scat"),
        mk<64, 64, 2, 2, 2, 0, 1>("64x64 s2 w2x2 epi1"),
        mk<64, 64, 3, 2, 2, 0, 1>("64x64 s3 w2x2 epi1"),
        mk<64, 64, 4, 2, 2, 0, 1>("64x64 s4 w2x2 epi1"),
        mk<64, 64, 2, 1, 4, 0, 1>("64x64 s2 w1x4 epi1"),
        mk<32, 128, 2, 1, 4, 0, 1>("32x128 s2 w1x4 epi1"),
        mk<32, 128, 3, 1, 4, 0, 1>("32x128 s3 w1x4 epi1"),
        mk<32, 64, 2, 1, 4, 0, 1>("32x64 s2 w1x4 epi1"),
        mk<32, 64, 3, 1, 2, 0, 1>("32x64 s3 w1x2 epi1"),
        mk<64, 64, 2, 2, 2, 0, 3>("64x64 s2 w2x2 epi3 bf16"),
        mk<64, 128, 2, 1, 4, 0, 3>("64x128 s2 epi3 gelu bf16 scat"),
    };
    struct Shape { int M, K, N; };
    std::vector<Shape> shapes = {{4096, 1280, 1024}, {4096, 1024, 512}};
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    for (auto sh : shapes) {
        const int M = sh.M, K = sh.K, N = sh.N;
        uint16_t *x, *w;
        float *y, *yr;
        CK(hipMalloc(&x, (size_t)M * K * 2));
        CK(hipMalloc(&w, (size_t)N * K * 2));
        CK(hipMalloc(&y, (size_t)M * N * 4));
        CK(hipMalloc(&yr, (size_t)M * N * 4));
        fill_bf16<<<(M * (int64_t)K + 255) / 256, 256>>>(x, (int64_t)M * K, 1);
        fill_bf16<<<(N * (int64_t)K + 255) / 256, 256>>>(w, (int64_t)N * K, 2);
        ref_gemm<<<(M * (int64_t)N + 255) / 256, 256>>>(x, w, yr, M, N, K);
        CK(hipDeviceSynchronize());
        std::vector<float> hr((size_t)M * N), hy((size_t)M * N);
        CK(hipMemcpy(hr.data(), yr, hr.size() * 4, hipMemcpyDeviceToHost));
        std::vector<std::vector<float>> ts(vs.size());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (size_t v = 0; v < vs.size(); ++v) {  // correctness
            CK(hipMemset(y, 0, (size_t)M * N * 4));
            const int tiles = ((M + vs[v].BM - 1) / vs[v].BM) * ((N + vs[v].BN - 1) / vs[v].BN);
            hipLaunchKernelGGL(vs[v].fn, dim3(tiles), dim3(vs[v].threads), vs[v].lds, 0, x, w, y, M, N, K);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(hy.data(), y, hy.size() * 4, hipMemcpyDeviceToHost));
            double md = 0;
            for (size_t i = 0; i < hy.size(); ++i) md = std::max(md, (double)fabsf(hy[i] - hr[i]));
            if (vs[v].epi == 0 && md > 1e-2) printf("MISMATCH %s M=%d: max|d| %g\n", vs[v].name.c_str(), M, md);
            if (vs[v].epi != 0) {  // epilogue variants: gelu(ref + bias) within bf16 / fp32 tolerance
                double me = 0;
                for (int64_t i = 0; i < (int64_t)M * N; i += 9973) {
                    const int col = i % N;
                    const double g = hr[i] + 0.001 * (col & 7);
                    const double want = 0.5 * g * (1.0 + erf(g / sqrt(2.0)));
                    double got = hy[i];
                    if (vs[v].epi >= 3) {
                        const uint32_t u = (uint32_t)reinterpret_cast<uint16_t*>(hy.data())[i] << 16;
                        float f;
                        memcpy(&f, &u, 4);
                        got = f;
                    }
                    me = std::max(me, fabs(got - want) / (1.0 + fabs(want)));
                }
                if (me > (vs[v].epi >= 3 ? 2e-2 : 1e-3)) printf("EPI MISMATCH %s M=%d: rel %g\n", vs[v].name.c_str(), M, me);
            }
        }
        for (int r = 0; r < rounds; ++r)
            for (size_t v = 0; v < vs.size(); ++v) {
                const int tiles = ((M + vs[v].BM - 1) / vs[v].BM) * ((N + vs[v].BN - 1) / vs[v].BN);
                for (int i = 0; i < 3; ++i)
                    hipLaunchKernelGGL(vs[v].fn, dim3(tiles), dim3(vs[v].threads), vs[v].lds, 0, x, w, y, M, N, K);
                const int it = 20;
                CK(hipEventRecord(a));
                for (int i = 0; i < it; ++i)
                    hipLaunchKernelGGL(vs[v].fn, dim3(tiles), dim3(vs[v].threads), vs[v].lds, 0, x, w, y, M, N, K);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts[v].push_back(ms / it * 1000.f);
            }
        printf("== M=%d K=%d N=%d (%.2f GFLOP)\n", M, K, N, 2.0 * M * N * K / 1e9);
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
    }
    return 0;
}
