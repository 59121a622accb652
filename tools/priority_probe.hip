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
// Configurations "relaunch_*": a host thread relaunches the spinner every
// millisecond (releases it, waits for it, launches it again), as the resident
// grid's lease does.
// Configurations "*_hostread" / "*_hostwrite": beside the spinner (5: 64
// workgroups, wave 0 polling its own host word), a host thread spins reading a
// pinned word on a line of its own / writes the second word of each polled
// line in turn (the polled words keep their value), as a loop thread posting
// jobs and waiting for them does.
// Configurations "*_stages": first 16 host threads each run one kmws mask
// with the resident grid off for them (each borrows a pinned stage with its
// own stream, as loop threads do), so the process holds as many streams as a
// loop-thread process.
// Configuration "grid_claim16": 16 host threads each run one kmws mask on the
// resident grid (claiming their slots) and stay alive until the
// configuration ends; run with a keep-alive build of the library
// (tools/patches/meas_keepalive.patch) the grid then stays on the GPU.
// Configuration "sdma": no spinner; a host thread keeps 4 MiB pinned H2D and
// D2H copies running on another stream during the timed applies.
// Device flags are released by a copy of the host flag.
//  9  as 8 on ordinary (non-coherent, hipHostMallocDefault) pinned memory
//     with plain 16-byte loads and stores, as the staging of the resident jobs
// 10  as 9 with write-through (sc0 sc1) stores, as the resident grid's
__global__ void spin_kernel(uint64_t* hflag, uint64_t* dflag_uc, uint64_t* dflag, int how, uint8_t* nc)
{
    uint64_t* f = how == 2 ? dflag_uc : how == 3 ? dflag : (how >= 5 && how <= 7) ? hflag + 32 * (blockIdx.x % 64) : hflag;
    uint64_t clk = 0;
    const bool poller = how < 4 || how >= 8 || threadIdx.x < 64;
    if (poller) {
        for (;;) {
            const uint64_t v = how == 2 || how == 3 ? __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                    : __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (__builtin_amdgcn_readfirstlane((int)v)) break;
            if (how == 6) clk += __builtin_amdgcn_s_memrealtime();
            if ((how == 9 || how == 10) && threadIdx.x < 64) {
                typedef uint32_t v4 __attribute__((ext_vector_type(4)));
                for (int i = 0; i < 4; ++i) {
                    v4* q = reinterpret_cast<v4*>(nc) + threadIdx.x + 64 * i;
                    v4 x = *q;
                    x.x += 1;
                    if (how == 9) *q = x;
                    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(q), "v"(x) : "memory");
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_sleep(127);
            }
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
    if (how >= 4 && how <= 7) __syncthreads();
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
    uint8_t *nch = nullptr, *ncbuf = nullptr;
    (void)hipHostMalloc(reinterpret_cast<void**>(&nch), 1 << 16, hipHostMallocDefault);
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&ncbuf), nch, 0);
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
    const Cfg cfgs[] = {{"none", 0, 0, 0, 0}, {"own16", 16, 1024, 1, 5}, {"grid_claim16", 0, 0, 0, 0},
                        {"none_after_grid", 0, 0, 0, 0}};
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
    bool staged = false;
    for (const Cfg& c : cfgs) {
        const std::string nm = c.name;
        if (nm.find("stages") != std::string::npos && !staged) {
            std::vector<std::thread> ts;
            for (int t = 0; t < 16; ++t)
                ts.emplace_back([] {
                    kmws_resident_enable(0, 0);
                    std::vector<uint8_t> a(4096, 1);
                    uint8_t key[4] = {1, 2, 3, 4};
                    uint8_t* seg = a.data();
                    size_t len = a.size();
                    (void)kmws_mask_host_chain(key, &seg, &len, 1, 0);
                });
            for (auto& t : ts) t.join();
            staged = true;
        }
        std::memset(flag, 0, 64 * 1024);
        (void)hipMemset(duc, 0, 256);
        (void)hipMemset(dl2, 0, 256);
        (void)hipDeviceSynchronize();
        const bool relaunch = std::string(c.name).rfind("relaunch", 0) == 0;
        std::atomic<bool> relaunching{relaunch};
        std::thread relauncher;
        if (c.wgs && !relaunch) {
            hipLaunchKernelGGL(spin_kernel, dim3(c.wgs), dim3(c.lanes), 0, c.prio ? hp : np, dflag, duc, dl2, c.how, ncbuf);
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        if (relaunch)
            relauncher = std::thread([&] {
                hipStream_t q = c.prio ? hp : np;
                while (relaunching.load()) {
                    for (int i = 0; i < 64; ++i) __atomic_store_n(flag + 32 * i, 0ull, __ATOMIC_RELEASE);
                    hipLaunchKernelGGL(spin_kernel, dim3(c.wgs), dim3(c.lanes), 0, q, dflag, duc, dl2, c.how, ncbuf);
                    std::this_thread::sleep_for(std::chrono::milliseconds(1));
                    for (int i = 0; i < 64; ++i) __atomic_store_n(flag + 32 * i, 1ull, __ATOMIC_RELEASE);
                    (void)hipStreamSynchronize(q);
                }
            });
        std::atomic<bool> copying{std::string(c.name) == "sdma"};
        std::atomic<bool> claiming{nm == "grid_claim16"};
        std::vector<std::thread> claimers;
        if (claiming.load()) {
            for (int t = 0; t < 16; ++t)
                claimers.emplace_back([&claiming, t] {
                    std::vector<uint8_t> a(4096, (uint8_t)t);
                    uint8_t key[4] = {(uint8_t)t, 2, 3, 4};
                    uint8_t* seg = a.data();
                    size_t len = a.size();
                    (void)kmws_mask_host_chain(key, &seg, &len, 1, 0);
                    while (claiming.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
                });
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
        }
        std::atomic<bool> hosting{nm.find("_host") != std::string::npos};
        std::thread hoster([&] {
            uint64_t sink = 0, i = 0;
            const bool wr = nm.find("hostwrite") != std::string::npos;
            while (hosting.load(std::memory_order_relaxed)) {
                if (wr) {
                    __atomic_store_n(flag + 32 * (i % 64) + 1, i, __ATOMIC_RELEASE);
                    for (int k = 0; k < 200; ++k) __builtin_ia32_pause();
                } else {
                    sink += __atomic_load_n(flag + 32 * 64 + 8, __ATOMIC_ACQUIRE);
                }
                ++i;
            }
            if (sink == 42) std::printf("#");
        });
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
        const bool batched = nm.find("_q20") != std::string::npos;
        std::vector<hipEvent_t> evs(2 * steps);
        if (batched) {
            for (auto& e : evs) (void)hipEventCreate(&e);
            for (int i = 0; i < steps; ++i) {
                (void)hipEventRecord(evs[2 * i], s);
                (void)kmws_unmask_apply(base, span, descs, n, ws, wsb, s);
                (void)hipEventRecord(evs[2 * i + 1], s);
            }
            const auto t0 = std::chrono::steady_clock::now();
            while (hipEventQuery(evs[2 * steps - 1]) == hipErrorNotReady) {
                if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10) && !queued_behind) {
                    release();
                    queued_behind = true;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(100));
            }
            for (int i = 0; i < steps; ++i) {
                float ms = 0;
                (void)hipEventElapsedTime(&ms, evs[2 * i], evs[2 * i + 1]);
                tot += ms;
            }
            for (auto& e : evs) (void)hipEventDestroy(e);
        }
        for (int i = 0; i < (batched ? 0 : steps); ++i) {
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
        relaunching.store(false);
        if (relauncher.joinable()) relauncher.join();
        hosting.store(false);
        hoster.join();
        claiming.store(false);
        for (auto& t : claimers) t.join();
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
