// Host-side probe: is the pinned send / receive ring slow for the CPU?
// memcpy of 4 KiB payloads (1,000 of them, like one loopback connection) into
// kmws_host_alloc memory (hipHostMalloc) vs malloc, on 1 and 8 threads at once,
// after the GPU has masked the ring (zero-copy) or not; and the cost of
// steady_clock::now().  One JSON line per case.
//
// usage: host_mem_probe
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "kmws_gpu.h"

namespace {
using Clock = std::chrono::steady_clock;
double secs(Clock::duration d) { return std::chrono::duration<double>(d).count(); }

// one thread: 1,000 x 4 KiB copies into a 1 MiB ring (wrapping), `rounds` times; returns us per 4 KiB
double copy_us(uint8_t* ring, const uint8_t* src, bool gpu_touch)
{
    double best = 1e30;
    for (int r = 0; r < 5; ++r) {
        if (gpu_touch) {  // the GPU masks the whole ring in place (as the tx batch does), twice
            const uint8_t key[4] = {1, 2, 3, 4};
            uint8_t* seg[1] = {ring};
            size_t len[1] = {1u << 20};
            if (kmws_mask_host_chain(key, seg, len, 1, 0) != KMWS_OK) std::exit(3);
            if (kmws_mask_host_chain(key, seg, len, 1, 0) != KMWS_OK) std::exit(3);
        }
        const auto t0 = Clock::now();
        for (int i = 0; i < 1000; ++i) std::memcpy(ring + (size_t)(i % 256) * 4096, src + (size_t)i * 4096, 4096);
        best = std::min(best, secs(Clock::now() - t0));
    }
    return best / 1000 * 1e6;
}
}  // namespace

int main()
{
    {
        const auto t0 = Clock::now();
        uint64_t sink = 0;
        for (int i = 0; i < 1000000; ++i) sink += (uint64_t)Clock::now().time_since_epoch().count();
        std::printf("{\"case\": \"steady_clock_now\", \"ns_per_call\": %.1f, \"sink\": %llu}\n",
                    secs(Clock::now() - t0) * 1e3, (unsigned long long)(sink & 1));
    }
    if (kmws_device_count() < 1) return 1;
    for (int T : {1, 8}) {
        for (int kind = 0; kind < 3; ++kind) {  // 0 malloc, 1 pinned, 2 pinned after GPU masks
            std::vector<double> us(T);
            std::vector<std::thread> th;
            std::atomic<int> ready{0};
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    std::vector<uint8_t> src((size_t)1000 * 4096, (uint8_t)t);
                    uint8_t* ring = kind == 0 ? static_cast<uint8_t*>(std::malloc(1u << 20))
                                              : static_cast<uint8_t*>(kmws_host_alloc(1u << 20, 0));
                    std::memset(ring, 0, 1u << 20);
                    ready.fetch_add(1);
                    while (ready.load() < T) std::this_thread::yield();
                    us[t] = copy_us(ring, src.data(), kind == 2);
                    if (kind == 0) std::free(ring);
                    else kmws_host_free(ring);
                });
            for (auto& x : th) x.join();
            std::sort(us.begin(), us.end());
            std::printf("{\"case\": \"copy_4k\", \"memory\": \"%s\", \"threads\": %d, \"us_per_4k_min\": %.3f, "
                        "\"us_per_4k_max\": %.3f}\n",
                        kind == 0 ? "malloc" : kind == 1 ? "pinned" : "pinned_after_gpu", T, us.front(), us.back());
            std::fflush(stdout);
        }
    }
    return 0;
}
