// Host<->device transfer probe for the end-to-end (host-memory) unmask path.
// Compares SDMA copies (alone and H2D || D2H on two streams), a zero-copy
// kernel that XORs pinned host memory in place over PCIe, and the product
// kmws_pipeline at several chunk sizes / depths.
//
// build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -Iinclude tools/pcie_probe.hip \
//        -Lkuma_amd/lib -lkmws_gpu -Wl,-rpath,'$ORIGIN/../kuma_amd/lib' -o tools/pcie_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>

#include "kmws_gpu.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

template <bool NT>
__global__ void __launch_bounds__(256) xor_host(u32x4* p, uint64_t nw, uint32_t c)
{
    for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256) {
        u32x4 v = NT ? __builtin_nontemporal_load(p + w) : p[w];
        if (NT) __builtin_nontemporal_store(v ^ c, p + w); else p[w] = v ^ c;
    }
}

int main(int argc, char** argv)
{
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : 4ull) << 30;
    uint8_t *h1, *h2, *hnc, *d1, *d2;
    CK(hipHostMalloc((void**)&h1, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h2, bytes, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&hnc, bytes, hipHostMallocNonCoherent));
    CK(hipMalloc(&d1, bytes));
    CK(hipMalloc(&d2, bytes));
    memset(h1, 1, bytes); memset(h2, 2, bytes); memset(hnc, 3, bytes);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const double gib = bytes / 1073741824.0;
    auto rep = [&](const char* name, double moved_gib, auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        double best = 1e9;
        for (int r = 0; r < 3; ++r) {
            double t0 = now();
            fn();
            CK(hipDeviceSynchronize());
            best = std::min(best, now() - t0);
        }
        printf("%-52s %8.2f GiB/s (%.3f s)\n", name, moved_gib / best, best);
    };
    rep("H2D hipMemcpyAsync", gib, [&] { CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1)); });
    rep("D2H hipMemcpyAsync", gib, [&] { CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s1)); });
    rep("H2D || D2H (two streams), total", 2 * gib, [&] {
        CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
    });
    rep("H2D || D2H chunked 64 MiB interleaved, total", 2 * gib, [&] {
        const uint64_t c = 64ull << 20;
        for (uint64_t o = 0; o < bytes; o += c) {
            CK(hipMemcpyAsync(d1 + o, h1 + o, c, hipMemcpyHostToDevice, s1));
            CK(hipMemcpyAsync(h2 + o, d2 + o, c, hipMemcpyDeviceToHost, s2));
        }
    });
    const uint64_t nw = bytes / 16;
    for (int grid : {1024, 4096, 16384}) {
        char name[96];
        snprintf(name, sizeof name, "zero-copy XOR coherent pinned, grid %d (payload)", grid);
        rep(name, gib, [&] { hipLaunchKernelGGL(xor_host<false>, dim3(grid), dim3(256), 0, s1, (u32x4*)h1, nw, 0x5au); });
        snprintf(name, sizeof name, "zero-copy XOR non-coherent pinned, grid %d", grid);
        rep(name, gib, [&] { hipLaunchKernelGGL(xor_host<false>, dim3(grid), dim3(256), 0, s1, (u32x4*)hnc, nw, 0x5au); });
        snprintf(name, sizeof name, "zero-copy XOR nt non-coherent, grid %d", grid);
        rep(name, gib, [&] { hipLaunchKernelGGL(xor_host<true>, dim3(grid), dim3(256), 0, s1, (u32x4*)hnc, nw, 0x5au); });
    }
    // product pipeline on a 64 KiB-frame wire image in h1
    const uint64_t L = 65536, fsz = L + 14;
    const uint32_t nf = (uint32_t)(bytes / fsz);
    std::vector<kmws_desc> d(nf);
    for (uint32_t i = 0; i < nf; ++i) d[i] = kmws_desc{(uint64_t)i * fsz + 14, (uint32_t)L, 0x12345678u + i};
    for (uint64_t chunk : {16ull << 20, 64ull << 20, 256ull << 20}) {
        for (int depth : {2, 3, 4}) {
            kmws_pipeline* p = kmws_pipeline_create(0, chunk, 1 << 16, depth);
            if (!p) { printf("pipeline create failed\n"); continue; }
            char name[96];
            snprintf(name, sizeof name, "kmws_pipeline chunk %llu MiB depth %d (payload)",
                     (unsigned long long)(chunk >> 20), depth);
            rep(name, (double)nf * L / 1073741824.0, [&] {
                if (kmws_pipeline_unmask(p, h1, bytes, d.data(), nf) != KMWS_OK) { printf("pipeline error\n"); exit(1); }
            });
            kmws_pipeline_destroy(p);
        }
    }
    return 0;
}
