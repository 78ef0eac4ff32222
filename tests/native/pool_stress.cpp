// Stress test of ctws_host::WorkerPool (cluster_tools_amd/csrc/host_pool.h): many back-to-back
// parallel_for calls of varying sizes; every index must run exactly once per call and the call
// must not return before all of them finished.  Built with -fsanitize=thread by
// tests/test_host_pool.py (host code only).
#include <atomic>
#include <cstdio>
#include <vector>

#include "../../cluster_tools_amd/csrc/host_pool.h"

int main(int argc, char** argv) {
    const int calls = argc > 1 ? std::atoi(argv[1]) : 20000;
    ctws_host::WorkerPool pool(6);
    std::vector<std::atomic<int>> hits(257);
    for (int c = 0; c < calls; ++c) {
        const int n = 2 + (c * 37) % 255;
        for (int i = 0; i < n; ++i) hits[i].store(0, std::memory_order_relaxed);
        pool.parallel_for(n, [&](int64_t i) { hits[i].fetch_add(1, std::memory_order_relaxed); });
        for (int i = 0; i < n; ++i)
            if (hits[i].load() != 1) {
                std::fprintf(stderr, "call %d (n %d): index %d ran %d times\n", c, n, i, hits[i].load());
                return 1;
            }
    }
    std::printf("ok %d calls\n", calls);
    return 0;
}
