// Host-side thread pool of the batch front end (aq_abi.inc host_parallel). Plain C++17, no HIP: the
// CPU suite builds it alone under ThreadSanitizer (tests/test_host_pool.py).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace aq {

// The batch front end's host threads, created once per context (r06: a fresh std::thread per piece on
// every call had made the first chunk's staging slower on 8 threads than on one -- 270-615 against 213
// us for 131072 integrals, profiles/r06p). run(n, f) runs f(0) .. f(n - 1) on the caller and the
// sleeping workers. Pieces are taken from one ticket word, (run << 32) | next piece, by compare-and-swap:
// a worker takes pieces only of the run it was woken for (a late one finds them taken, or a newer run's
// ticket, and goes back to sleep), and run returns only once no worker is inside it, so no worker ever
// calls a finished run's f.
struct HostPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable wake, done;
    std::atomic<unsigned long long> ticket{0};
    std::atomic<size_t> left{0};                 // pieces of the current run not yet finished
    const std::function<void(size_t)>* job = nullptr;   // under m: the current run
    size_t parts = 0;                            // under m
    unsigned long long gen = 0;                  // under m: the current run's number
    int busy = 0;                                // under m: workers inside a run
    bool stop = false;

    explicit HostPool(size_t workers) {
        try {
            for (size_t i = 0; i < workers; ++i) th.emplace_back([this] { loop(); });
        } catch (...) {   // no thread to be had (resource limits): fewer workers, the caller does the rest
        }
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
        }
        wake.notify_all();
        for (auto& t : th) t.join();
    }
    void pieces(unsigned long long g, const std::function<void(size_t)>* f, size_t n) {
        const unsigned long long run = (g & 0xffffffffull) << 32;
        unsigned long long t = ticket.load();
        for (;;) {
            if ((t & ~0xffffffffull) != run || (t & 0xffffffffull) >= n) return;
            if (!ticket.compare_exchange_weak(t, t + 1)) continue;   // t reloaded
            (*f)((size_t)(t & 0xffffffffull));
            if (left.fetch_sub(1) == 1) {
                std::lock_guard<std::mutex> lk(m);
                done.notify_all();
            }
            t = ticket.load();
        }
    }
    void loop() {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(size_t)>* f;
            size_t n;
            {
                std::unique_lock<std::mutex> lk(m);
                wake.wait(lk, [&] { return stop || gen != seen; });
                if (stop) return;
                seen = gen;
                f = job;
                n = parts;
                ++busy;
            }
            pieces(seen, f, n);   // (f of a finished run is never called: its ticket is used up)
            {
                std::lock_guard<std::mutex> lk(m);
                --busy;
            }
            done.notify_all();
        }
    }
    void run(size_t n, const std::function<void(size_t)>& f) {
        unsigned long long g;
        {
            std::lock_guard<std::mutex> lk(m);
            job = &f;
            parts = n;
            left = n;
            g = ++gen;
            ticket = (g & 0xffffffffull) << 32;
        }
        wake.notify_all();
        pieces(g, &f, n);
        std::unique_lock<std::mutex> lk(m);
        done.wait(lk, [&] { return left.load() == 0 && busy == 0; });
    }
};

}  // namespace aq
