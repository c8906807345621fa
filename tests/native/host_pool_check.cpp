// Exercise aq::HostPool (ppls_amd/csrc/aq_host_pool.h) under ThreadSanitizer: every run executes each
// piece exactly once, runs follow each other with and without pauses (late-waking workers), and the
// pool is destroyed cleanly. Prints "ok <runs>" on success. Built and run by tests/test_host_pool.py.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "aq_host_pool.h"

int main(int argc, char** argv) {
    const int runs = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937 rng(12345);
    for (size_t workers : {0u, 1u, 7u}) {
        aq::HostPool pool(workers);
        for (int r = 0; r < runs; ++r) {
            const size_t parts = 1 + rng() % 64;
            std::vector<std::atomic<int>> hit(parts);
            for (auto& h : hit) h = 0;
            std::vector<long long> part_sum(parts, 0);   // plain writes, one piece each: tsan checks them
            const std::function<void(size_t)> f = [&](size_t p) {
                hit[p].fetch_add(1);
                long long s = 0;
                for (size_t i = 0; i < (p % 7) * 100; ++i) s += (long long)(i ^ p);
                part_sum[p] = s + 1;
            };
            pool.run(parts, f);
            for (size_t p = 0; p < parts; ++p)
                if (hit[p].load() != 1 || part_sum[p] == 0) {
                    fprintf(stderr, "run %d: piece %zu of %zu ran %d times\n", r, p, parts, hit[p].load());
                    return 1;
                }
            if (rng() % 16 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
        }
    }
    printf("ok %d\n", runs);
    return 0;
}
