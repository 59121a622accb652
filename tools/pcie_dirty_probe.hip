// Does writing host memory from the GPU cost more when the CPU has just
// written the same lines (still in its caches), and does it depend on how the
// GPU stores: through the L2 with one release at the end (the resident grid's
// large jobs), or write-through (sc0 sc1, its small jobs)?  The loopback writes
// its receive ring on the CPU and has the grid unmask it in place at once;
// write-through stores halved its decode at 4-8 connections.
//
// For a pinned buffer of `bytes` (default 4 MiB, LLC-sized): per mode and state,
// the best of 20 passes of a kernel XOR-ing the buffer in place (each 16-byte
// word read, XORed, written back).  State "dirty": the CPU memsets the buffer
// right before each pass; "clean": it does not.  One JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool WT>
__global__ void __launch_bounds__(1024) xor_in_place(u32x4* p, size_t n)
{
    for (size_t i = blockIdx.x * 1024ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 1024ull) {
        u32x4 v = p[i];
        v.x ^= 0x5A5A5A5Au;
        if (WT) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(p + i), "v"(v) : "memory");
        else p[i] = v;
    }
    __syncthreads();
    if (!WT && threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: L2 written back
}

int main(int argc, char** argv)
{
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (4u << 20), n = bytes / 16;
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) return 1;
    u32x4* d = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 1;
    std::memset(h, 1, bytes);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const unsigned grid = 64;  // the resident grid's size: 16 slots x 4 parts
    std::printf("{\"bytes\": %zu, \"grid\": %u", bytes, grid);
    for (int wt = 0; wt < 2; ++wt)
        for (int dirty = 0; dirty < 2; ++dirty) {
            float best = 1e30f;
            for (int r = 0; r < 20; ++r) {
                if (dirty) std::memset(h, r, bytes);
                (void)hipEventRecord(e0, s);
                if (wt) hipLaunchKernelGGL(xor_in_place<true>, dim3(grid), dim3(1024), 0, s, d, n);
                else hipLaunchKernelGGL(xor_in_place<false>, dim3(grid), dim3(1024), 0, s, d, n);
                (void)hipEventRecord(e1, s);
                (void)hipStreamSynchronize(s);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            std::printf(", \"%s_%s_GB_s\": %.2f", wt ? "write_through" : "l2_release", dirty ? "dirty" : "clean",
                        bytes / (best * 1e6));
        }
    std::printf("}\n");
    return 0;
}
