// Zero-copy probe: what bounds a resident job's bytes over PCIe?
//
// One launch per case; every workgroup timestamps (s_memrealtime, 100 MHz)
// its own start and end, so launch overhead is excluded.  A case XORs S bytes
// of pinned host memory in place (the resident worker's job, kmws_resident.hip)
// split evenly over G workgroups of L lanes, W 16-byte words per lane per
// round, every load of a round issued before its stores, then a fence:
//   fence 0: none; 1: release at agent scope; 2: release at system scope (the
//   resident worker's, before it signals done).
// Also the system-scope acquire alone (acq = 1), as the worker does before it
// reads a job's payload.  Reports the slowest workgroup's microseconds and the
// payload GB/s (each byte read and written).  Memory: hipHostMalloc default
// (the decoder's staging) or coherent (the mailbox).
//
// usage: zc_probe  -> one JSON line per case
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int W, int FENCE, int ACQ>
__global__ void zc_kernel(u32x4* buf, uint32_t words_per_block, uint64_t* times)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (ACQ == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (ACQ == 2) {  // one wave acquires, the others wait at the barrier
        if (threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __syncthreads();
    }
    u32x4* p = buf + (uint64_t)blockIdx.x * words_per_block;
    for (uint32_t w0 = 0; w0 < words_per_block; w0 += blockDim.x * W) {
        u32x4 v[W];
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t w = w0 + threadIdx.x + blockDim.x * i;
            v[i] = w < words_per_block ? p[w] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < W; ++i) {
            const uint32_t w = w0 + threadIdx.x + blockDim.x * i;
            if (w < words_per_block) p[w] = v[i] ^ 0x5a5a5a5au;
        }
    }
    if (FENCE == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (FENCE == 2) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (FENCE == 3) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // each wave: its own stores done
    __syncthreads();
    if (FENCE == 3 && threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // then one wave
    if (FENCE == 3) __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        times[2 * blockIdx.x] = t0;
        times[2 * blockIdx.x + 1] = t1;
    }
}

// The job of zc_kernel (W = 4, system-scope release) on the first G
// workgroups while P more poll one host word each (a system-scope load, then
// s_sleep SLEEP), as the resident grid's other workgroups do; the pollers stop
// once every job workgroup has counted itself done.
template <int SLEEP>
__global__ void zc_polled_kernel(u32x4* buf, uint32_t words_per_block, uint64_t* times, const uint64_t* host_word,
                                 uint32_t* done_count, uint32_t G)
{
    if (blockIdx.x >= G) {  // a poller
        uint64_t sink = 0;
        while (__hip_atomic_load(done_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < G) {
            if (threadIdx.x < 64) sink += __hip_atomic_load(host_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __builtin_amdgcn_s_sleep(SLEEP);
        }
        if (sink == 0x123456789ull) times[0] = sink;  // keeps the loads
        return;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    u32x4* p = buf + (uint64_t)blockIdx.x * words_per_block;
    for (uint32_t w0 = 0; w0 < words_per_block; w0 += blockDim.x * 4) {
        u32x4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t w = w0 + threadIdx.x + blockDim.x * i;
            v[i] = w < words_per_block ? p[w] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t w = w0 + threadIdx.x + blockDim.x * i;
            if (w < words_per_block) p[w] = v[i] ^ 0x5a5a5a5au;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        times[2 * blockIdx.x] = t0;
        times[2 * blockIdx.x + 1] = t1;
        __hip_atomic_fetch_add(done_count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// G workgroups, each its own job of `words` 16-byte words of pinned host
// memory, K times in a row, as the resident worker runs them: (ACQ) one wave
// acquires at system scope, every lane XORs its words, each wave waits for its
// stores, then (REL) one lane stores the job number to a host word with a
// system-scope release.  Does a job take longer when other workgroups run
// theirs at the same time?
template <int ACQ, int REL>
__global__ void zc_multi_kernel(u32x4* buf, uint32_t words, uint64_t* done_words, uint32_t K, uint64_t* times)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    u32x4* p = buf + (uint64_t)blockIdx.x * words;
    for (uint32_t k = 1; k <= K; ++k) {
        if (ACQ && threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __syncthreads();
        for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) p[w] = p[w] ^ 0x5a5a5a5au;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (REL) __hip_atomic_store(&done_words[16 * blockIdx.x], (uint64_t)k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            else __hip_atomic_store(&done_words[16 * blockIdx.x], (uint64_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        times[2 * blockIdx.x] = t0;
        times[2 * blockIdx.x + 1] = t1;
    }
}

template <int ACQ, int REL>
double run_multi(u32x4* d, uint32_t words, int G, uint32_t K, uint64_t* dw, uint64_t* dtimes, uint64_t* htimes)
{
    double best = 1e30;
    for (int rep = 0; rep < 8; ++rep) {
        hipLaunchKernelGGL((zc_multi_kernel<ACQ, REL>), dim3(G), dim3(1024), 0, 0, d, words, dw, K, dtimes);
        if (hipDeviceSynchronize() != hipSuccess) std::exit(3);
        if (hipMemcpy(htimes, dtimes, 16 * G, hipMemcpyDeviceToHost) != hipSuccess) std::exit(4);
        double worst = 0;  // the slowest workgroup's microseconds per job
        for (int g = 0; g < G; ++g) {
            const double us = (double)(htimes[2 * g + 1] - htimes[2 * g]) / 100.0 / K;
            worst = us > worst ? us : worst;
        }
        if (rep >= 2 && worst < best) best = worst;
    }
    return best;
}

template <int SLEEP>
double run_polled(u32x4* dbuf, uint64_t bytes, int G, int L, int P, uint64_t* dtimes, uint64_t* htimes,
                  const uint64_t* dword, uint32_t* dcount)
{
    const uint32_t wpb = (uint32_t)(bytes / 16 / G);
    double best = 1e30;
    for (int rep = 0; rep < 20; ++rep) {
        if (hipMemset(dcount, 0, 4) != hipSuccess) std::exit(3);
        hipLaunchKernelGGL((zc_polled_kernel<SLEEP>), dim3(G + P), dim3(L), 0, 0, dbuf, wpb, dtimes, dword, dcount,
                           (uint32_t)G);
        if (hipDeviceSynchronize() != hipSuccess) std::exit(3);
        if (hipMemcpy(htimes, dtimes, 16 * G, hipMemcpyDeviceToHost) != hipSuccess) std::exit(4);
        uint64_t lo = ~0ull, hi = 0;
        for (int g = 0; g < G; ++g) {
            lo = htimes[2 * g] < lo ? htimes[2 * g] : lo;
            hi = htimes[2 * g + 1] > hi ? htimes[2 * g + 1] : hi;
        }
        const double us = (double)(hi - lo) / 100.0;
        if (rep >= 3 && us < best) best = us;
    }
    return best;
}

template <int W, int FENCE, int ACQ>
double run(u32x4* dbuf, uint64_t bytes, int G, int L, uint64_t* dtimes, uint64_t* htimes)
{
    const uint32_t wpb = (uint32_t)(bytes / 16 / G);
    double best = 1e30;
    for (int rep = 0; rep < 20; ++rep) {
        hipLaunchKernelGGL((zc_kernel<W, FENCE, ACQ>), dim3(G), dim3(L), 0, 0, dbuf, wpb, dtimes);
        if (hipDeviceSynchronize() != hipSuccess) std::exit(3);
        if (hipMemcpy(htimes, dtimes, 16 * G, hipMemcpyDeviceToHost) != hipSuccess) std::exit(4);
        uint64_t lo = ~0ull, hi = 0;
        for (int g = 0; g < G; ++g) {
            lo = htimes[2 * g] < lo ? htimes[2 * g] : lo;
            hi = htimes[2 * g + 1] > hi ? htimes[2 * g + 1] : hi;
        }
        const double us = (double)(hi - lo) / 100.0;  // 100 MHz
        if (rep >= 3 && us < best) best = us;
    }
    return best;
}

int main(int argc, char** argv)
{
    if (argc > 1 && std::string(argv[1]) == "multi") {  // concurrent jobs only
        uint64_t *dtimes = nullptr, *htimes = static_cast<uint64_t*>(std::malloc(16 * 256));
        if (hipMalloc(&dtimes, 16 * 256) != hipSuccess) return 2;
        for (int mem = 0; mem < 2; ++mem) {
            void *h = nullptr, *hw = nullptr;
            if (hipHostMalloc(&h, 64u << 20, mem ? hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess) return 2;
            if (hipHostMalloc(&hw, 64 * 128, hipHostMallocCoherent) != hipSuccess) return 2;
            u32x4* d = nullptr;
            uint64_t* dw = nullptr;
            if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 2;
            if (hipHostGetDevicePointer(reinterpret_cast<void**>(&dw), hw, 0) != hipSuccess) return 2;
            for (uint32_t bytes : {4096u, 65536u}) {
                const uint32_t K = bytes == 4096 ? 400 : 100;
                for (int G : {1, 2, 4, 8, 16, 32, 64}) {
                    const double none = run_multi<0, 0>(d, bytes / 16, G, K, dw, dtimes, htimes);
                    const double rel = run_multi<0, 1>(d, bytes / 16, G, K, dw, dtimes, htimes);
                    const double both = run_multi<1, 1>(d, bytes / 16, G, K, dw, dtimes, htimes);
                    std::printf("{\"multi\": true, \"mem\": \"%s\", \"bytes\": %u, \"workgroups\": %d, \"jobs_each\": %u, "
                                "\"us_per_job_no_fence\": %.3f, \"us_per_job_release\": %.3f, "
                                "\"us_per_job_acquire_release\": %.3f, \"jobs_per_s_acquire_release\": %.0f}\n",
                                mem ? "coherent" : "default", bytes, G, K, none, rel, both, G / both * 1e6);
                    std::fflush(stdout);
                }
            }
            (void)hipHostFree(h);
            (void)hipHostFree(hw);
        }
        return 0;
    }
    uint64_t *dtimes = nullptr, *htimes = nullptr;
    if (hipMalloc(&dtimes, 16 * 256) != hipSuccess) return 2;
    htimes = static_cast<uint64_t*>(std::malloc(16 * 256));
    for (int mem = 0; mem < 2; ++mem) {
        void* h = nullptr;
        const uint64_t cap = 1 << 20;
        if (hipHostMalloc(&h, cap, mem ? hipHostMallocCoherent : hipHostMallocDefault) != hipSuccess) return 2;
        u32x4* d = nullptr;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 2;
        const char* mname = mem ? "coherent" : "default";
        for (uint64_t bytes : {4096ull, 16384ull, 65536ull, 262144ull}) {
            for (int G : {1, 2, 4, 8, 16}) {
                if (bytes / G < 1024) continue;
                for (int L : {256, 1024}) {
                    const double none = run<4, 0, 0>(d, bytes, G, L, dtimes, htimes);
                    const double agent = run<4, 1, 0>(d, bytes, G, L, dtimes, htimes);
                    const double sys = run<4, 2, 0>(d, bytes, G, L, dtimes, htimes);
                    const double acq_sys = run<4, 2, 1>(d, bytes, G, L, dtimes, htimes);
                    const double w1 = run<1, 2, 0>(d, bytes, G, L, dtimes, htimes);
                    const double one = run<4, 3, 0>(d, bytes, G, L, dtimes, htimes);
                    const double one_acq = run<4, 3, 2>(d, bytes, G, L, dtimes, htimes);
                    std::printf("{\"mem\": \"%s\", \"bytes\": %llu, \"workgroups\": %d, \"lanes\": %d, "
                                "\"us_no_fence\": %.2f, \"us_agent_release\": %.2f, \"us_system_release\": %.2f, "
                                "\"us_acquire_and_system_release\": %.2f, \"us_1word_system_release\": %.2f, "
                                "\"us_waitcnt_then_one_wave_release\": %.2f, \"us_one_wave_acquire_and_release\": %.2f, "
                                "\"GB_s_system_release\": %.2f}\n",
                                mname, (unsigned long long)bytes, G, L, none, agent, sys, acq_sys, w1, one, one_acq,
                                2.0 * bytes / sys / 1e3);
                    std::fflush(stdout);
                }
            }
        }
        (void)hipHostFree(h);
    }
    // a job beside polling workgroups
    {
        void *h = nullptr, *hw = nullptr;
        if (hipHostMalloc(&h, 1 << 20, hipHostMallocDefault) != hipSuccess) return 2;
        if (hipHostMalloc(&hw, 4096, hipHostMallocCoherent) != hipSuccess) return 2;
        u32x4* d = nullptr;
        uint64_t* dw = nullptr;
        uint32_t* dcount = nullptr;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 2;
        if (hipHostGetDevicePointer(reinterpret_cast<void**>(&dw), hw, 0) != hipSuccess) return 2;
        if (hipMalloc(&dcount, 4) != hipSuccess) return 2;
        for (uint64_t bytes : {4096ull, 65536ull}) {
            for (int G : {1, 4}) {
                for (int P : {0, 15, 31, 63}) {
                    const double s2 = run_polled<2>(d, bytes, G, 1024, P, dtimes, htimes, dw, dcount);
                    const double s127 = run_polled<127>(d, bytes, G, 1024, P, dtimes, htimes, dw, dcount);
                    std::printf("{\"polled\": true, \"bytes\": %llu, \"workgroups\": %d, \"lanes\": 1024, "
                                "\"pollers\": %d, \"us_pollers_sleep2\": %.2f, \"us_pollers_sleep127\": %.2f}\n",
                                (unsigned long long)bytes, G, P, s2, s127);
                    std::fflush(stdout);
                }
            }
        }
    }
    return 0;
}
