// The resident grid's cost to a device batch.
//
// One process, as a deployment that mixes device batches (kmws_pipeline, the
// cfg2 unmask) with loop threads on the resident grid would run: BASELINE
// configs[1]'s batch (1 M x 64 KiB frames, 64 GiB, plain hipMalloc) is
// unmasked by kmws_unmask_plan + kmws_unmask_apply, `steps` launches per phase,
// each timed with HIP events on the launch stream; phases alternate between
// "quiet" (no other kmws work) and "busy" (`threads` host threads masking
// 4 KiB buffers with kmws_mask_host_chain back to back, i.e. every slot of the
// resident grid taken and polling, four workgroups of 1024 lanes per slot).
// Prints one JSON line: per phase the mean / min / max apply time, the HBM
// fraction (131,088 B per frame), and the masks completed meanwhile.  Every
// byte is verified at the end (kmws_check_unmasked).  Run it under
// `rocprofv3 --kernel-trace --stats` to see the same launches from the trace
// (tools/gpu_interference.sh).
//
// Attribution modes (5th argument): resident (the above), launch (the same
// masks with the grid switched off in every masking thread: a launch per
// call), one (thread 0 masks; the others claim a slot with one mask per phase
// and then idle, so the grid polls 16 claimed slots while one works).
//
// one_50us / one_1ms: as one, thread 0 sleeping that long between its masks.
// claim: every thread masks once per busy phase (claims its slot) and idles.
//
// usage: grid_interference [frames] [steps] [phases] [threads] [resident|launch|one|one_50us|one_1ms|claim]
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 10) : (1u << 20);
    const int steps = argc > 2 ? std::atoi(argv[2]) : 20;
    const int phases = argc > 3 ? std::atoi(argv[3]) : 6;
    const int threads = argc > 4 ? std::atoi(argv[4]) : 16;
    const std::string how = argc > 5 ? argv[5] : "resident";
    if (kmws_device_count() < 1) {
        std::printf("{\"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    const uint64_t L = 65536, span = (uint64_t)n * L;
    uint8_t* base = nullptr;
    kmws_desc* descs = nullptr;
    void* ws = nullptr;
    unsigned long long* mism = nullptr;
    const size_t wsb = kmws_unmask_workspace_size(span);
    if (hipMalloc(reinterpret_cast<void**>(&base), span) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&descs), (size_t)n * sizeof(kmws_desc)) != hipSuccess ||
        hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(reinterpret_cast<void**>(&mism), 8) != hipSuccess) {
        std::printf("{\"error\": \"hipMalloc\"}\n");
        return 2;
    }
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (std::getenv("GI_PRESTREAMS")) {  // harness variant: the streams tools/priority_probe.hip creates first
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        hipStream_t hp, np, cs, rs;
        (void)hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, greatest);
        (void)hipStreamCreateWithPriority(&np, hipStreamNonBlocking, least);
        (void)hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
        (void)hipStreamCreateWithPriority(&rs, hipStreamNonBlocking, greatest);
    }
    if (std::getenv("GI_HPONE")) {  // harness variant: one high-priority stream only
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        hipStream_t hp;
        (void)hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, greatest);
    }
    const uint64_t seed = 0x6B756D61;
    if (kmws_fill_synthetic(base, span, seed, s) != KMWS_OK ||
        kmws_fill_uniform_descs(descs, n, L, (uint32_t)L, seed ^ 0x5EED, s) != KMWS_OK ||
        kmws_unmask_plan(span, descs, n, ws, wsb, s) != KMWS_OK) {
        std::printf("{\"error\": \"setup\"}\n");
        return 3;
    }
    (void)hipStreamSynchronize(s);
    std::vector<hipEvent_t> ev(2 * (size_t)steps);
    for (auto& e : ev) (void)hipEventCreate(&e);

    std::atomic<int> mode{0};  // 0 idle, 1 masking, -1 quit
    std::atomic<long> masks{0}, bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            // GI_LEN: bytes per mask (default 4 KiB)
            const size_t mlen = std::getenv("GI_LEN") ? (size_t)std::strtoul(std::getenv("GI_LEN"), nullptr, 10) : 4096;
            std::vector<uint8_t> a(mlen, (uint8_t)t), b;
            uint8_t key[4] = {(uint8_t)(t + 1), 0x5A, 0xC3, 0x96};
            if (how == "launch") kmws_resident_enable(0, 0);
            int last_mode = 0;
            for (;;) {
                const int m = mode.load(std::memory_order_acquire);
                if (m < 0) break;
                const bool fresh = m != last_mode;
                last_mode = m;
                const bool one = how.rfind("one", 0) == 0;
                if (m == 0 || (one && t != 0 && !fresh) || (how == "claim" && !fresh)) {
                    std::this_thread::sleep_for(std::chrono::microseconds(200));
                    continue;
                }
                uint8_t* seg = a.data();
                size_t len = a.size();
                b = a;
                if (kmws_mask_host_chain(key, &seg, &len, 1, 0) != KMWS_OK) ++bad;
                for (size_t i = 0; i < b.size(); ++i) b[i] ^= key[i & 3];
                if (a != b) ++bad;
                masks.fetch_add(1, std::memory_order_relaxed);
                if (t == 0 && how == "one_50us") std::this_thread::sleep_for(std::chrono::microseconds(50));
                if (t == 0 && how == "one_1ms") std::this_thread::sleep_for(std::chrono::milliseconds(1));
            }
        });

    // warm: the schedule's first launches, and the grid once
    for (int i = 0; i < 3; ++i) (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
    (void)hipStreamSynchronize(s);
    std::string rows;
    double sum_q = 0, sum_b = 0;
    int nq = 0, nb = 0;
    for (int p = 0; p < phases; ++p) {
        const bool busy = p % 2 == 1;
        mode.store(busy ? 1 : 0, std::memory_order_release);
        if (busy) std::this_thread::sleep_for(std::chrono::milliseconds(20));  // every thread holds its slot
        else std::this_thread::sleep_for(std::chrono::milliseconds(5));        // the grid idles out (200 us)
        const long m0 = masks.load();
        const auto t0 = std::chrono::steady_clock::now();
        const bool one_by_one = std::getenv("GI_ONE") != nullptr;  // harness variant: wait for each apply
        for (int i = 0; i < steps; ++i) {
            (void)hipEventRecord(ev[2 * (size_t)i], s);
            (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
            (void)hipEventRecord(ev[2 * (size_t)i + 1], s);
            if (one_by_one)
                while (hipEventQuery(ev[2 * (size_t)i + 1]) == hipErrorNotReady)
                    std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        if (std::getenv("GI_POLL")) {  // harness variant: poll the last event instead of a blocking synchronize
            while (hipEventQuery(ev[2 * (size_t)steps - 1]) == hipErrorNotReady)
                std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        (void)hipStreamSynchronize(s);
        const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const long m1 = masks.load();
        double tot = 0, lo = 1e9, hi = 0;
        for (int i = 0; i < steps; ++i) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, ev[2 * (size_t)i], ev[2 * (size_t)i + 1]);
            tot += ms;
            lo = ms < lo ? ms : lo;
            hi = ms > hi ? ms : hi;
        }
        const double mean = tot / steps;
        const double frac = (double)n * (2 * L + 16) / (mean * 1e-3) / 8e12;
        (busy ? sum_b : sum_q) += mean;
        (busy ? nb : nq)++;
        char buf[512];
        std::snprintf(buf, sizeof buf,
                      "%s{\"phase\": %d, \"busy\": %s, \"mean_ms\": %.4f, \"min_ms\": %.4f, \"max_ms\": %.4f, "
                      "\"frac\": %.4f, \"masks\": %ld, \"mask_calls_per_s\": %.0f}",
                      rows.empty() ? "" : ", ", p, busy ? "true" : "false", mean, lo, hi, frac, m1 - m0,
                      (double)(m1 - m0) / wall);
        rows += buf;
    }
    mode.store(-1, std::memory_order_release);
    for (auto& t : th) t.join();
    // the batch went through 3 + phases * steps applies: bring it to the unmasked state and check every byte
    if ((3 + phases * steps) % 2 == 0) (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
    (void)hipMemsetAsync(mism, 0, 8, s);
    (void)kmws_check_unmasked(base, span, seed, descs, n, mism, s);
    unsigned long long mm = 0;
    (void)hipMemcpyAsync(&mm, mism, 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    uint64_t jobs = 0, launches = 0;
    kmws_resident_info(0, &jobs, &launches, nullptr);
    const double q = sum_q / (nq ? nq : 1), b = sum_b / (nb ? nb : 1);
    std::printf("{\"mode\": \"%s\", \"frames\": %u, \"frame_len\": %llu, \"steps_per_phase\": %d, \"threads\": %d, \"phases\": [%s], "
                "\"quiet_mean_ms\": %.4f, \"busy_mean_ms\": %.4f, \"busy_over_quiet\": %.4f, \"resident_jobs\": %llu, "
                "\"grid_launches\": %llu, \"mask_bad\": %ld, \"byte_mismatches\": %llu}\n",
                how.c_str(), n, (unsigned long long)L, steps, threads, rows.c_str(), q, b, b / q, (unsigned long long)jobs,
                (unsigned long long)launches, bad.load(), mm);
    return mm == 0 && bad.load() == 0 ? 0 : 1;
}
