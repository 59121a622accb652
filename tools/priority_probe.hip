// Does a resident kernel on another stream slow the cfg2 unmask, and does its
// stream priority matter?  (Diagnostic for tools/grid_interference: the
// resident grid cost a device batch 1.35x even with one thread's jobs and
// whatever the grid's block size, poll rate or acquire; on a normal-priority
// stream the grid could not get onto the GPU beside the batch at all.)
//
// A spinner kernel (`wgs` workgroups of `lanes` lanes that sleep-poll a
// pinned host flag, no other memory traffic) is launched first on a stream of
// the greatest or the least priority; then 20 applies of BASELINE configs[1]'s
// batch (1 M x 64 KiB, kmws_unmask_apply) are timed with HIP events; then the
// flag releases the spinner.  Prints one JSON line per configuration.
//
// usage: priority_probe [frames]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"

// every wave polls the flag itself (a system-scope load: pinned host memory),
// then sleeps: ~0.06 us (fast) or ~4 us (slow) between polls
__global__ void spin_kernel(uint64_t* flag, int fast)
{
    for (;;) {
        const uint64_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (__builtin_amdgcn_readfirstlane((int)v)) break;
        if (fast) __builtin_amdgcn_s_sleep(2);
        else __builtin_amdgcn_s_sleep(127);
    }
}

int main(int argc, char** argv)
{
    const uint32_t n = argc > 1 ? (uint32_t)std::strtoul(argv[1], nullptr, 10) : (1u << 20);
    const uint64_t L = 65536, span = (uint64_t)n * L;
    uint8_t* base = nullptr;
    kmws_desc* descs = nullptr;
    void* ws = nullptr;
    const size_t wsb = kmws_unmask_workspace_size(span);
    if (hipMalloc(reinterpret_cast<void**>(&base), span) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&descs), (size_t)n * sizeof(kmws_desc)) != hipSuccess ||
        hipMalloc(&ws, wsb) != hipSuccess)
        return 2;
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    hipStream_t s, hp, np;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    (void)hipStreamCreateWithPriority(&hp, hipStreamNonBlocking, greatest);
    (void)hipStreamCreateWithPriority(&np, hipStreamNonBlocking, least);
    uint64_t* flag = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void**>(&flag), 64, hipHostMallocCoherent | hipHostMallocMapped);
    uint64_t* dflag = nullptr;
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), flag, 0);
    if (kmws_fill_synthetic(base, span, 7, s) != KMWS_OK || kmws_fill_uniform_descs(descs, n, L, (uint32_t)L, 9, s) ||
        kmws_unmask_plan(span, descs, n, ws, wsb, s) != KMWS_OK)
        return 3;
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    struct Cfg {
        const char* name;
        int wgs, lanes, prio, poll_host;
    };
    const Cfg cfgs[] = {{"none", 0, 0, 0, 0},       {"hp_1x64", 1, 64, 1, 1},     {"np_1x64", 1, 64, 0, 1},
                        {"hp_64x1024", 64, 1024, 1, 1}, {"np_64x1024", 64, 1024, 0, 1}, {"hp_1x64_slowpoll", 1, 64, 1, 0},
                        {"none", 0, 0, 0, 0}};
    for (const Cfg& c : cfgs) {
        *flag = 0;
        if (c.wgs) {
            hipLaunchKernelGGL(spin_kernel, dim3(c.wgs), dim3(c.lanes), 0, c.prio ? hp : np, dflag, c.poll_host);
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        for (int i = 0; i < 3; ++i) (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
        double tot = 0;
        const int steps = 20;
        bool queued_behind = false;
        for (int i = 0; i < steps; ++i) {
            (void)hipEventRecord(e0, s);
            (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
            (void)hipEventRecord(e1, s);
            // bounded: should the batch's stream share a hardware queue with the
            // spinner, the batch waits for it -- release it after 3 s
            const auto t0 = std::chrono::steady_clock::now();
            while (hipEventQuery(e1) == hipErrorNotReady) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
                    __atomic_store_n(flag, 1ull, __ATOMIC_RELEASE);
                    queued_behind = true;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            (void)hipGetLastError();
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            tot += ms;
        }
        __atomic_store_n(flag, 1ull, __ATOMIC_RELEASE);
        (void)hipDeviceSynchronize();
        const double mean = tot / steps;
        std::printf("{\"config\": \"%s\", \"spinner_workgroups\": %d, \"lanes\": %d, \"priority\": \"%s\", "
                    "\"queued_behind_spinner\": %s, \"mean_ms\": %.4f, \"frac\": %.4f}\n",
                    c.name, c.wgs, c.lanes, c.prio ? "greatest" : "least", queued_behind ? "true" : "false", mean,
                    (double)n * (2 * L + 16) / (mean * 1e-3) / 8e12);
        std::fflush(stdout);
    }
    return 0;
}
