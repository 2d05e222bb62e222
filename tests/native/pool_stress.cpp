// Stress test of rf_io.cpp's fork-join Pool (the feature pipe's host parse pool), built with
// -fsanitize=thread (and separately -fsanitize=address) by tests/test_pool_native.py.
//
// Thousands of back-to-back run() calls with a count that changes every call (the pattern of
// FeaturePipe's parse: pool_.run(T1, ...) then pool_.run(T2, ...), T varying with the batch), each
// index writing its own slot of a vector that lives on run()'s caller's stack. Checks that every index
// ran exactly once per call and that run() never returns while a worker is still inside the lambda.
#include "../../recommendflow_amd/csrc/rf_io.cpp"

#include <cstdio>

// rf_api.cpp's error slot (not linked into this test program)
int rf_set_error(int code, const char*, ...) { return code; }

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 5000;
    Pool pool(threads);
    std::atomic<int> inside{0};
    uint32_t x = 12345;
    for (int it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        const int n = 1 + static_cast<int>((x >> 8) % 67);  // 1 .. 67, varying every call
        std::vector<int> hits(n, 0);                        // on this frame: freed when the call returns
        pool.run(n, [&](int i) {
            inside.fetch_add(1);
            hits[i] += 1;  // a double execution is a data race TSan reports, and a count of 2 below
            if ((i & 7) == 0) std::this_thread::yield();
            inside.fetch_sub(1);
        });
        if (inside.load() != 0) {
            std::fprintf(stderr, "iteration %d: run() returned with a worker inside the lambda\n", it);
            return 2;
        }
        for (int i = 0; i < n; ++i)
            if (hits[i] != 1) {
                std::fprintf(stderr, "iteration %d: index %d of %d ran %d times\n", it, i, n, hits[i]);
                return 3;
            }
    }
    std::printf("pool ok: %d threads, %d runs\n", threads, iters);
    return 0;
}
