// Can the unmask kernel write its output to pinned host memory itself while the
// copy engines bring the next chunk in?  (The host-resident pipeline,
// kmws_pipeline_unmask, moves payload H2D and back D2H by SDMA on two streams:
// 45 GiB/s of payload, 0.84 of one direction's copy rate; two directions of
// copy-engine traffic at once ran 40 GiB/s each: tools/pcie_duplex.py.)
//
// Measures, for 1 GiB: (a) a kernel copying HBM -> pinned host memory (16-byte
// stores, plain / non-temporal / write-through), alone; (b) SDMA H2D alone;
// (c) both at once on two streams.  One JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) copy_to_host(const u32x4* __restrict__ src, u32x4* dst, size_t n)
{
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256ull) {
        u32x4 v = src[i];
        v.x ^= 0x5A5A5A5Au;
        if (MODE == 0) dst[i] = v;
        else if (MODE == 1) __builtin_nontemporal_store(v, dst + i);
        else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1\n\ts_nop 1" ::"v"(dst + i), "v"(v) : "memory");
    }
}

int main()
{
    const size_t bytes = 1ull << 30, n = bytes / 16;
    u32x4 *d_src = nullptr, *d_in = nullptr, *h_out = nullptr, *dv_out = nullptr;
    void* h_in = nullptr;
    (void)hipMalloc(reinterpret_cast<void**>(&d_src), bytes);
    (void)hipMalloc(reinterpret_cast<void**>(&d_in), bytes);
    (void)hipHostMalloc(reinterpret_cast<void**>(&h_out), bytes, hipHostMallocDefault);
    (void)hipHostMalloc(&h_in, bytes, hipHostMallocDefault);
    (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&dv_out), h_out, 0);
    (void)hipMemset(d_src, 1, bytes);
    (void)hipDeviceSynchronize();
    hipStream_t sk, sc;
    (void)hipStreamCreateWithFlags(&sk, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&sc, hipStreamNonBlocking);
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    const int grids[] = {256, 1024, 4096};
    std::printf("{");
    bool first = true;
    for (int mode = 0; mode < 3; ++mode)
        for (int g : grids) {
            auto launch = [&] {
                if (mode == 0) hipLaunchKernelGGL(copy_to_host<0>, dim3(g), dim3(256), 0, sk, d_src, dv_out, n);
                else if (mode == 1) hipLaunchKernelGGL(copy_to_host<1>, dim3(g), dim3(256), 0, sk, d_src, dv_out, n);
                else hipLaunchKernelGGL(copy_to_host<2>, dim3(g), dim3(256), 0, sk, d_src, dv_out, n);
            };
            double ka = 1e9, both_k = 1e9, both = 1e9;
            for (int r = 0; r < 3; ++r) {
                (void)hipDeviceSynchronize();
                auto t0 = now();
                launch();
                (void)hipStreamSynchronize(sk);
                ka = std::min(ka, secs(t0, now()));
                (void)hipDeviceSynchronize();
                t0 = now();
                (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, sc);
                launch();
                (void)hipStreamSynchronize(sk);
                const double tk = secs(t0, now());
                (void)hipStreamSynchronize(sc);
                both_k = std::min(both_k, tk);
                both = std::min(both, secs(t0, now()));
            }
            std::printf("%s\"%s_grid%d\": {\"kernel_alone_GiB_s\": %.2f, \"with_h2d_kernel_GiB_s\": %.2f, "
                        "\"with_h2d_both_done_GiB_s_each\": %.2f}",
                        first ? "" : ", ", mode == 0 ? "plain" : mode == 1 ? "nt" : "sc0sc1", g, 1.0 / ka, 1.0 / both_k,
                        1.0 / both);
            first = false;
        }
    double h = 1e9;
    for (int r = 0; r < 3; ++r) {
        (void)hipDeviceSynchronize();
        auto t0 = now();
        (void)hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, sc);
        (void)hipStreamSynchronize(sc);
        h = std::min(h, secs(t0, now()));
    }
    std::printf(", \"sdma_h2d_alone_GiB_s\": %.2f}\n", 1.0 / h);
    return 0;
}
