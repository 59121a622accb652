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

#include <atomic>
#include <chrono>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <cstring>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"

// The spinner's poll, by `how`:
//  0  every wave polls the pinned host flag (system-scope load), ~0.06 us sleeps
//  1  the same, ~4 us sleeps
//  2  every wave polls a flag in uncached device memory (agent-scope load)
//  3  every wave polls a flag in ordinary device memory (agent-scope load:
//     L2-served, so a copy engine's write may never be seen -- not run)
//  4  only wave 0 of each workgroup polls the host flag; the others wait at a
//     barrier (the resident grid's shape)
//  5  as 4, each workgroup polling its own host word (256 B apart)
//  6  as 5, reading the constant-rate clock (s_memrealtime) at every poll, as
//     the resident grid does for its idle and lease bounds
//  7  as 5, reading the shader clock (s_memtime) at every poll
//  8  one wave: between polls it reads and rewrites a 4 KiB block of pinned
//     host memory (write-through), then sleeps ~4 us: a trickle of PCIe
//     traffic, like a few resident jobs a second
// Configuration "sdma": no spinner; a host thread keeps 4 MiB pinned H2D and
// D2H copies running on another stream during the timed applies.
// Device flags are released by a copy of the host flag.
__global__ void spin_kernel(uint64_t* hflag, uint64_t* dflag_uc, uint64_t* dflag, int how)
{
    uint64_t* f = how == 2 ? dflag_uc : how == 3 ? dflag : how >= 5 ? hflag + 32 * (blockIdx.x % 64) : hflag;
    uint64_t clk = 0;
    const bool poller = how < 4 || threadIdx.x < 64;
    if (poller) {
        for (;;) {
            const uint64_t v = how == 2 || how == 3 ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                    : __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (__builtin_amdgcn_readfirstlane((int)v)) break;
            if (how == 6) clk += __builtin_amdgcn_s_memrealtime();
            if (how == 8 && threadIdx.x < 64) {
                uint64_t* blk = hflag + 4096;  // 4 KiB at +32 KiB of the flag area
                for (int i = 0; i < 8; ++i) {
                    uint64_t x = __hip_atomic_load(blk + threadIdx.x + 64 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(blk + threadIdx.x + 64 * i, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                __builtin_amdgcn_s_sleep(127);
            }
            if (how == 7) clk += __builtin_amdgcn_s_memtime();
            if (how == 1) __builtin_amdgcn_s_sleep(127);
            else __builtin_amdgcn_s_sleep(2);
        }
    }
    if (how >= 4) __syncthreads();
    if (clk == 0x123456789ull) hflag[1] = clk;  // keeps the clock reads
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
    (void)hipHostMalloc(reinterpret_cast<void**>(&flag), 64 * 1024, hipHostMallocCoherent | hipHostMallocMapped);
    uint64_t *duc = nullptr, *dl2 = nullptr;
    (void)hipExtMallocWithFlags(reinterpret_cast<void**>(&duc), 256, hipDeviceMallocUncached);
    (void)hipMalloc(reinterpret_cast<void**>(&dl2), 256);
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
        int wgs, lanes, prio, how;
    };
    const Cfg cfgs[] = {{"none", 0, 0, 0, 0}, {"pcie_trickle_1x64", 1, 64, 1, 8}, {"sdma", 0, 0, 0, 0},
                        {"none", 0, 0, 0, 0}};
    std::vector<uint8_t> dummy;
    uint8_t *hbuf = nullptr, *dbuf = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void**>(&hbuf), 8u << 20, hipHostMallocDefault);
    (void)hipMalloc(reinterpret_cast<void**>(&dbuf), 8u << 20);
    hipStream_t cs;
    (void)hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    hipStream_t rs;
    (void)hipStreamCreateWithPriority(&rs, hipStreamNonBlocking, greatest);
    const uint64_t one = 1;
    auto release = [&] {
        for (int i = 0; i < 64; ++i) __atomic_store_n(flag + 32 * i, 1ull, __ATOMIC_RELEASE);
        (void)hipMemcpyAsync(duc, &one, 8, hipMemcpyHostToDevice, rs);
        (void)hipMemcpyAsync(dl2, &one, 8, hipMemcpyHostToDevice, rs);
        (void)hipStreamSynchronize(rs);
    };
    for (const Cfg& c : cfgs) {
        std::memset(flag, 0, 64 * 1024);
        (void)hipMemset(duc, 0, 256);
        (void)hipMemset(dl2, 0, 256);
        (void)hipDeviceSynchronize();
        if (c.wgs) {
            hipLaunchKernelGGL(spin_kernel, dim3(c.wgs), dim3(c.lanes), 0, c.prio ? hp : np, dflag, duc, dl2, c.how);
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        std::atomic<bool> copying{std::string(c.name) == "sdma"};
        std::thread copier([&] {
            while (copying.load()) {
                (void)hipMemcpyAsync(dbuf, hbuf, 4u << 20, hipMemcpyHostToDevice, cs);
                (void)hipMemcpyAsync(hbuf + (4u << 20), dbuf + (4u << 20), 4u << 20, hipMemcpyDeviceToHost, cs);
                (void)hipStreamSynchronize(cs);
            }
        });
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
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3) && !queued_behind) {
                    release();
                    queued_behind = true;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            (void)hipGetLastError();
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            tot += ms;
        }
        release();
        copying.store(false);
        copier.join();
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
