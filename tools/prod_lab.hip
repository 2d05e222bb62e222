// prod_lab.hip — diagnostics only: librf's rf_linear_fwd / rf_linear_stats_fwd timed exactly like tools/gemm_lab
// (same fills, 20 back-to-back launches between HIP events, interleaved rounds), so the two can be compared on
// one box: a gap between them is the production kernel's code, not the measurement.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/prod_lab tools/prod_lab.hip \
//        -Lrecommendflow_amd/lib -lrf -Wl,-rpath,'$ORIGIN/../recommendflow_amd/lib'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../include/rf_api.h"

#define CK(x)                                                                                         \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);    \
            exit(1);                                                                                  \
        }                                                                                             \
    } while (0)

__global__ void fill_bf16(uint16_t* p, int64_t n, uint32_t seed, float scale) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    const float v = (((h & 0xffffff) / 16777216.0f) * 2.f - 1.f) * scale;
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    struct Shape { int M, K, N; };
    const std::vector<Shape> shapes = {{4096, 1280, 1024}, {4096, 1024, 512}, {51200, 1280, 1024}};
    const float scales[2] = {1.0f, 0.05f};
    for (auto sh : shapes) {
        const int M = sh.M, K = sh.K, N = sh.N;
        uint16_t *x, *w, *yb;
        float *y, *b, *st, *sv, *tv;
        CK(hipMalloc(&x, (size_t)M * K * 2));
        CK(hipMalloc(&w, (size_t)N * K * 2));
        CK(hipMalloc(&y, (size_t)M * N * 4));
        CK(hipMalloc(&yb, (size_t)M * N * 2));
        CK(hipMalloc(&b, (size_t)N * 4));
        CK(hipMalloc(&sv, (size_t)N * 4));
        CK(hipMalloc(&tv, (size_t)N * 4));
        CK(hipMalloc(&st, (size_t)M * 4 * ((std::max(N, K) + 127) / 128) * 8));
        CK(hipMemset(b, 0, (size_t)N * 4));
        CK(hipMemset(sv, 0, (size_t)N * 4));
        CK(hipMemset(tv, 0, (size_t)N * 4));
        for (float sc : scales) {
            fill_bf16<<<(M * (int64_t)K + 255) / 256, 256>>>(x, (int64_t)M * K, 1, sc);
            fill_bf16<<<(N * (int64_t)K + 255) / 256, 256>>>(w, (int64_t)N * K, 2, sc);
            // LN-fold statistics of x: (sum, M2) per 32-column slice = (0, 32) -> mu 0, var 1
            std::vector<float> hs((size_t)M * 4 * ((K + 127) / 128) * 2);
            for (size_t i = 0; i < hs.size(); i += 2) { hs[i] = 0.f; hs[i + 1] = 32.f; }
            CK(hipMemcpy(st, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
            float* st2;
            CK(hipMalloc(&st2, (size_t)M * 4 * ((N + 127) / 128) * 8));
            CK(hipDeviceSynchronize());
            struct V { std::string name; std::function<int()> f; };
            std::vector<V> vs = {
                {"rf_linear_fwd none", [&] { return rf_linear_fwd(x, RF_DTYPE_BF16, M, K, K, w, N, b, RF_ACT_NONE, y, N, nullptr); }},
                {"rf_linear_fwd gelu", [&] { return rf_linear_fwd(x, RF_DTYPE_BF16, M, K, K, w, N, b, RF_ACT_GELU, y, N, nullptr); }},
                {"rf_linear_stats_fwd gelu", [&] { return rf_linear_stats_fwd(x, M, K, K, w, N, b, RF_ACT_GELU, yb, N, st2, nullptr); }},
                {"rf_linear_lnfold_fwd gelu", [&] { return rf_linear_lnfold_fwd(x, M, K, K, w, N, sv, tv, st, 1e-6f, RF_ACT_GELU, y, N, nullptr); }},
            };
            std::vector<std::vector<float>> ts(vs.size());
            hipEvent_t a, e;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&e));
            for (int r = 0; r < rounds; ++r)
                for (size_t v = 0; v < vs.size(); ++v) {
                    for (int i = 0; i < 3; ++i)
                        if (vs[v].f() != 0) { fprintf(stderr, "%s failed\n", vs[v].name.c_str()); return 1; }
                    const int it = 20;
                    CK(hipEventRecord(a));
                    for (int i = 0; i < it; ++i) vs[v].f();
                    CK(hipEventRecord(e));
                    CK(hipEventSynchronize(e));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, e));
                    ts[v].push_back(ms / it * 1000.f);
                }
            printf("== M=%d K=%d N=%d scale %.2f\n", M, K, N, sc);
            for (size_t v = 0; v < vs.size(); ++v) {
                auto t = ts[v];
                std::sort(t.begin(), t.end());
                const double med = t[t.size() / 2];
                printf("  %-30s median %8.2f us  min %8.2f us  %7.1f TF\n", vs[v].name.c_str(), med, t[0],
                       2.0 * M * N * K / med / 1e6);
            }
            fflush(stdout);
            CK(hipFree(st2));
        }
        CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(yb)); CK(hipFree(b));
        CK(hipFree(sv)); CK(hipFree(tv)); CK(hipFree(st));
    }
    // chain: the cfg3 output MLP pair as the forward runs it (stats GEMM 1280 -> 1024 writes bf16 + row statistics,
    // the LN-fold GEMM 1024 -> 512 consumes them), 20 pairs back to back; under rocprofv3 --kernel-trace each
    // kernel's duration in the chain can be compared with its isolated, repeated timing above
    {
        const int M = 4096, K = 1280, N1 = 1024, N2 = 512;
        uint16_t *x, *w1, *w2, *yb;
        float *b1, *st, *sv, *tv, *y;
        CK(hipMalloc(&x, (size_t)M * K * 2));
        CK(hipMalloc(&w1, (size_t)N1 * K * 2));
        CK(hipMalloc(&w2, (size_t)N2 * N1 * 2));
        CK(hipMalloc(&yb, (size_t)M * N1 * 2));
        CK(hipMalloc(&y, (size_t)M * N2 * 4));
        CK(hipMalloc(&b1, (size_t)N1 * 4));
        CK(hipMalloc(&sv, (size_t)N2 * 4));
        CK(hipMalloc(&tv, (size_t)N2 * 4));
        CK(hipMalloc(&st, (size_t)M * 4 * (N1 / 128) * 8));
        CK(hipMemset(b1, 0, (size_t)N1 * 4));
        CK(hipMemset(sv, 0, (size_t)N2 * 4));
        CK(hipMemset(tv, 0, (size_t)N2 * 4));
        fill_bf16<<<(M * (int64_t)K + 255) / 256, 256>>>(x, (int64_t)M * K, 1, 1.f);
        fill_bf16<<<(N1 * (int64_t)K + 255) / 256, 256>>>(w1, (int64_t)N1 * K, 2, 0.05f);
        fill_bf16<<<(N2 * (int64_t)N1 + 255) / 256, 256>>>(w2, (int64_t)N2 * N1, 3, 0.05f);
        auto pair = [&] {
            rf_linear_stats_fwd(x, M, K, K, w1, N1, b1, RF_ACT_GELU, yb, N1, st, nullptr);
            rf_linear_lnfold_fwd(yb, M, N1, N1, w2, N2, sv, tv, st, 1e-6f, RF_ACT_GELU, y, N2, nullptr);
        };
        for (int i = 0; i < 3; ++i) pair();
        hipEvent_t a, e;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&e));
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i) pair();
            CK(hipEventRecord(e));
            CK(hipEventSynchronize(e));
            float ms;
            CK(hipEventElapsedTime(&ms, a, e));
            t.push_back(ms / 20 * 1000.f);
        }
        std::sort(t.begin(), t.end());
        printf("== chain stats(4096x1280->1024) + lnfold(->512): median %.2f us per pair\n", t[t.size() / 2]);
        // sustained: 2000 pairs back to back (~70 ms of continuous MFMA load), per-200-pair windows
        hipEvent_t ev[11];
        for (auto& x : ev) CK(hipEventCreate(&x));
        CK(hipEventRecord(ev[0]));
        for (int w = 0; w < 10; ++w) {
            for (int i = 0; i < 200; ++i) pair();
            CK(hipEventRecord(ev[w + 1]));
        }
        CK(hipEventSynchronize(ev[10]));
        printf("   sustained windows (us per pair):");
        for (int w = 0; w < 10; ++w) {
            float ms;
            CK(hipEventElapsedTime(&ms, ev[w], ev[w + 1]));
            printf(" %.2f", ms / 200 * 1000.f);
        }
        printf("\n");
        // the forward's order: LayerNorm (fp32 [M, 1280] -> bf16 x) writes the stats GEMM's input right before it
        float* xf;
        CK(hipMalloc(&xf, (size_t)M * K * 4));
        CK(hipMemset(xf, 0, (size_t)M * K * 4));
        fill_bf16<<<(M * (int64_t)K + 255) / 256, 256>>>(x, (int64_t)M * K, 1, 1.f);
        auto tri = [&] {
            rf_norm_fwd(xf, M, K, K, 0, 1e-6f, nullptr, nullptr, nullptr, nullptr, x, RF_DTYPE_BF16, K, nullptr);
            pair();
        };
        for (int i = 0; i < 3; ++i) tri();
        std::vector<float> t3;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(a));
            for (int i = 0; i < 20; ++i) tri();
            CK(hipEventRecord(e));
            CK(hipEventSynchronize(e));
            float ms;
            CK(hipEventElapsedTime(&ms, a, e));
            t3.push_back(ms / 20 * 1000.f);
        }
        std::sort(t3.begin(), t3.end());
        printf("== chain LayerNorm(1280, fp32 -> bf16) + stats + lnfold: median %.2f us per triple\n", t3[t3.size() / 2]);
    }
    return 0;
}
