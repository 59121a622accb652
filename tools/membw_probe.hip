// Streaming-bandwidth probe for the unmask kernel's access pattern on MI355X.
// Interleaves variants in one process (guide sec.5.4 rule 24) over a 64 GiB
// buffer and prints achieved GB/s (algorithmic bytes: read + write).
//
// build: hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -Iinclude tools/membw_probe.hip \
//        -Lkuma_amd/lib -lkmws_gpu -Wl,-rpath,'$ORIGIN/../kuma_amd/lib' -o tools/membw_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kmws_gpu.h"

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int V, int B>
__global__ void __launch_bounds__(B) xor_tiles(u32x4* p, uint32_t c)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[base + (uint64_t)B * i];
#pragma unroll
    for (int i = 0; i < V; ++i) p[base + (uint64_t)B * i] = v[i] ^ c;
}

template <int V, int B>
__global__ void __launch_bounds__(B) xor_tiles_nt(u32x4* p, uint32_t c)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = __builtin_nontemporal_load(p + base + (uint64_t)B * i);
#pragma unroll
    for (int i = 0; i < V; ++i) __builtin_nontemporal_store(v[i] ^ c, p + base + (uint64_t)B * i);
}

template <int V, int B>
__global__ void __launch_bounds__(B) xor_tiles_ntst(u32x4* p, uint32_t c)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[base + (uint64_t)B * i];
#pragma unroll
    for (int i = 0; i < V; ++i) __builtin_nontemporal_store(v[i] ^ c, p + base + (uint64_t)B * i);
}

// persistent: each block walks tiles b, b+G, ...; next tile's loads issued before this tile's stores
template <int V, int B>
__global__ void __launch_bounds__(B) xor_persist(u32x4* p, uint32_t c, uint64_t ntiles)
{
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = p[t * B * V + threadIdx.x + (uint64_t)B * i];
    for (;;) {
        const uint64_t tn = t + gridDim.x;
        u32x4 w[V];
        if (tn < ntiles) {
#pragma unroll
            for (int i = 0; i < V; ++i) w[i] = p[tn * B * V + threadIdx.x + (uint64_t)B * i];
        }
#pragma unroll
        for (int i = 0; i < V; ++i) p[t * B * V + threadIdx.x + (uint64_t)B * i] = v[i] ^ c;
        if (tn >= ntiles) break;
#pragma unroll
        for (int i = 0; i < V; ++i) v[i] = w[i];
        t = tn;
    }
}

template <int V, int B, bool NT>
__global__ void __launch_bounds__(B) xor_persist2(u32x4* p, uint32_t c, uint64_t ntiles)
{
    auto ld = [&](uint64_t i) { return NT ? __builtin_nontemporal_load(p + i) : p[i]; };
    auto st = [&](u32x4 x, uint64_t i) { if (NT) __builtin_nontemporal_store(x, p + i); else p[i] = x; };
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = ld(t * B * V + threadIdx.x + (uint64_t)B * i);
    for (;;) {
        const uint64_t tn = t + gridDim.x;
        u32x4 w[V];
        if (tn < ntiles) {
#pragma unroll
            for (int i = 0; i < V; ++i) w[i] = ld(tn * B * V + threadIdx.x + (uint64_t)B * i);
        }
#pragma unroll
        for (int i = 0; i < V; ++i) st(v[i] ^ c, t * B * V + threadIdx.x + (uint64_t)B * i);
        if (tn >= ntiles) break;
#pragma unroll
        for (int i = 0; i < V; ++i) v[i] = w[i];
        t = tn;
    }
}

template <int V, int B, bool NT>
__global__ void __launch_bounds__(B) xor_loop(u32x4* p, uint32_t c, uint64_t ntiles)
{
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        u32x4 v[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint64_t j = t * B * V + threadIdx.x + (uint64_t)B * i;
            v[i] = NT ? __builtin_nontemporal_load(p + j) : p[j];
        }
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint64_t j = t * B * V + threadIdx.x + (uint64_t)B * i;
            if (NT) __builtin_nontemporal_store(v[i] ^ c, p + j); else p[j] = v[i] ^ c;
        }
    }
}

template <int V, int B>
__global__ void __launch_bounds__(B) copy_tiles(const u32x4* a, u32x4* b)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = a[base + (uint64_t)B * i];
#pragma unroll
    for (int i = 0; i < V; ++i) b[base + (uint64_t)B * i] = v[i];
}

// one block per tile, tiles dealt over K parts of the buffer (the product's split schedule)
template <int V, int B, int K>
__global__ void __launch_bounds__(B) xor_split_nt(u32x4* p, uint32_t c)
{
    const uint64_t q = gridDim.x / K;
    const uint64_t t = K > 1 ? (blockIdx.x % K) * q + blockIdx.x / K : blockIdx.x;
    const uint64_t base = t * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = __builtin_nontemporal_load(p + base + (uint64_t)B * i);
#pragma unroll
    for (int i = 0; i < V; ++i) __builtin_nontemporal_store(v[i] ^ c, p + base + (uint64_t)B * i);
}

// xor_split_nt with plain (temporal) loads and/or stores
template <int V, int B, int K, bool NTL, bool NTS>
__global__ void __launch_bounds__(B) xor_split_pol(u32x4* p, uint32_t c)
{
    const uint64_t q = gridDim.x / K;
    const uint64_t t = K > 1 ? (blockIdx.x % K) * q + blockIdx.x / K : blockIdx.x;
    const uint64_t base = t * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = NTL ? __builtin_nontemporal_load(p + base + (uint64_t)B * i) : p[base + (uint64_t)B * i];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        if (NTS) __builtin_nontemporal_store(v[i] ^ c, p + base + (uint64_t)B * i);
        else p[base + (uint64_t)B * i] = v[i] ^ c;
    }
}

// read-only ceiling: XOR-reduce a tile, one word per block out (negligible writes)
template <int V, int B, int K>
__global__ void __launch_bounds__(B) read_split_nt(const u32x4* p, u32x4* out)
{
    const uint64_t q = gridDim.x / K;
    const uint64_t t = K > 1 ? (blockIdx.x % K) * q + blockIdx.x / K : blockIdx.x;
    const uint64_t base = t * B * V + threadIdx.x;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < V; ++i) acc ^= __builtin_nontemporal_load(p + base + (uint64_t)B * i);
    if ((acc.x | acc.y | acc.z | acc.w) == 0x9e3779b9u) out[blockIdx.x] = acc;  // practically never
}

// write-only ceiling
template <int V, int B, int K>
__global__ void __launch_bounds__(B) write_split_nt(u32x4* p, uint32_t c)
{
    const uint64_t q = gridDim.x / K;
    const uint64_t t = K > 1 ? (blockIdx.x % K) * q + blockIdx.x / K : blockIdx.x;
    const uint64_t base = t * B * V + threadIdx.x;
#pragma unroll
    for (int i = 0; i < V; ++i) __builtin_nontemporal_store(u32x4{c, c, c, (uint32_t)i}, p + base + (uint64_t)B * i);
}

// copy half -> half with the split mapping
template <int V, int B, int K>
__global__ void __launch_bounds__(B) copy_split_nt(const u32x4* a, u32x4* b)
{
    const uint64_t q = gridDim.x / K;
    const uint64_t t = K > 1 ? (blockIdx.x % K) * q + blockIdx.x / K : blockIdx.x;
    const uint64_t base = t * B * V + threadIdx.x;
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = __builtin_nontemporal_load(a + base + (uint64_t)B * i);
#pragma unroll
    for (int i = 0; i < V; ++i) __builtin_nontemporal_store(v[i], b + base + (uint64_t)B * i);
}

__global__ void __launch_bounds__(256) fill_kernel(u32x4* p, uint64_t nw)
{
    for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256)
        p[w] = u32x4{(uint32_t)w, 1u, 2u, 3u};
}

int main(int argc, char** argv)
{
    const uint64_t bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : 64ull) << 30;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    uint8_t* buf = nullptr;
    CK(hipMalloc(&buf, bytes));
    const uint64_t nw = bytes / 16;
    // argv[4] == "rand": splitmix64 payload (as bench.py) instead of the low-entropy counter pattern
    const bool rand_fill = argc > 4 && std::string(argv[4]) == "rand";
    if (rand_fill) kmws_fill_synthetic(buf, bytes, 12345, 0);
    else hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (u32x4*)buf, nw);
    // product path inputs: 64 KiB frames over the same buffer
    const uint32_t nf = (uint32_t)(bytes / 65536);
    kmws_desc* d = nullptr;
    CK(hipMalloc(&d, (size_t)nf * sizeof(kmws_desc)));
    kmws_fill_uniform_descs(d, nf, 65536, 65536, 7, 0);
    size_t wsb = kmws_unmask_workspace_size(bytes);
    void* ws = nullptr;
    CK(hipMalloc(&ws, wsb));
    kmws_unmask_plan(bytes, d, nf, ws, wsb, 0);
    CK(hipDeviceSynchronize());

    struct Var { const char* name; int kind; };
    std::vector<Var> vars = {
        {"copy V4 B256 (half buffer -> half)", 0}, {"xor V4 B256", 1}, {"xor V8 B256", 2},
        {"xor V4 B512", 3}, {"xor V2 B256", 4}, {"xor nt V4 B256", 5}, {"xor nt-store V4 B256", 6},
        {"xor persistent V4 B256 x2048", 7}, {"xor persistent V4 B256 x4096", 8},
        {"product kmws_unmask_apply", 9}, {"xor V16 B256", 10}, {"product kmws_unmask_batch (plan+apply)", 11},
        {"persist2 nt V4 x4096", 12}, {"persist2 nt V4 x8192", 13}, {"persist2 nt V4 x2048", 14},
        {"persist2 V4 x8192", 15}, {"persist2 nt V2 x8192", 16}, {"persist2 nt V8 x4096", 17},
        {"loop nt V4 x4096 (no prefetch)", 18}, {"loop nt V4 x8192 (no prefetch)", 19}, {"persist2 nt V4 x6144", 20},
        {"product variant 3 (persistent x8192)", 23}, {"product variant 4 (persistent x16384)", 24},
        {"product variant 5 (persistent x24576)", 25}, {"product variant 0 (default, again)", 26},
        {"product variant 6 (persistent x32768)", 27}, {"product variant 7 (persistent x65536)", 28},
        {"product variant 8 (>=6 waves/SIMD)", 29}, {"product variant 9 (>=8 waves/SIMD)", 30},
    };
    const bool ceil_mode = argc > 3 && std::string(argv[3]) == "ceil";
    if (ceil_mode) {  // read-only / write-only / copy / in-place ceilings, in order vs split
        vars = {{"read-only nt V4, in order", 40}, {"read-only nt V4, split 8", 41},
                {"write-only nt V4, in order", 42}, {"write-only nt V4, split 8", 43},
                {"copy nt V4 (half -> half), in order", 44}, {"copy nt V4 (half -> half), split 8", 45},
                {"xor nt V4, in order", 46}, {"xor nt V4, split 2", 47}, {"xor nt V4, split 8", 48},
                {"product kmws_unmask_apply (default schedule)", 9}};
    } else if (argc > 3 && std::string(argv[3]) == "split") {  // in-place XOR shapes under the split-8 mapping
        vars = {{"xor nt V4 B256, split 8", 48}, {"xor nt V2 B256, split 8", 50}, {"xor nt V8 B256, split 8", 51},
                {"xor nt V4 B512, split 8", 52}, {"xor nt V2 B512, split 8", 53}, {"xor nt V4 B128, split 8", 54},
                {"xor plain-load nt-store V4, split 8", 55}, {"xor nt-load plain-store V4, split 8", 56},
                {"xor plain V4, split 8", 57}, {"xor nt V4 B256, split 4", 58}, {"xor nt V8 B256, split 2", 59},
                {"product kmws_unmask_apply (default schedule)", 9}};
    } else if (argc > 3) {  // "product": only the product variants, interleaved
        std::vector<Var> keep;
        for (auto& v : vars)
            if (v.kind == 9 || v.kind == 11 || v.kind >= 23) keep.push_back(v);
        vars = keep;
    }
    u32x4* sink = nullptr;
    CK(hipMalloc(&sink, (nw / 1024) * sizeof(u32x4)));
    std::vector<std::vector<float>> ms(vars.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps + 1; ++r) {
        for (size_t k = 0; k < vars.size(); ++k) {
            CK(hipEventRecord(e0, 0));
            switch (vars[k].kind) {
            case 0: hipLaunchKernelGGL((copy_tiles<4, 256>), dim3(nw / 2 / 1024), dim3(256), 0, 0,
                                       (const u32x4*)buf, (u32x4*)(buf + bytes / 2)); break;
            case 1: hipLaunchKernelGGL((xor_tiles<4, 256>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 2: hipLaunchKernelGGL((xor_tiles<8, 256>), dim3(nw / 2048), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 3: hipLaunchKernelGGL((xor_tiles<4, 512>), dim3(nw / 2048), dim3(512), 0, 0, (u32x4*)buf, 0x5au); break;
            case 4: hipLaunchKernelGGL((xor_tiles<2, 256>), dim3(nw / 512), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 5: hipLaunchKernelGGL((xor_tiles_nt<4, 256>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 6: hipLaunchKernelGGL((xor_tiles_ntst<4, 256>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 7: hipLaunchKernelGGL((xor_persist<4, 256>), dim3(2048), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 8: hipLaunchKernelGGL((xor_persist<4, 256>), dim3(4096), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 9: kmws_unmask_apply(buf, bytes, d, nf, ws, wsb, 0); break;
            case 10: hipLaunchKernelGGL((xor_tiles<16, 256>), dim3(nw / 4096), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 11: kmws_unmask_batch(buf, bytes, d, nf, ws, wsb, 0); break;
            case 12: hipLaunchKernelGGL((xor_persist2<4, 256, true>), dim3(4096), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 13: hipLaunchKernelGGL((xor_persist2<4, 256, true>), dim3(8192), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 14: hipLaunchKernelGGL((xor_persist2<4, 256, true>), dim3(2048), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 15: hipLaunchKernelGGL((xor_persist2<4, 256, false>), dim3(8192), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 16: hipLaunchKernelGGL((xor_persist2<2, 256, true>), dim3(8192), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 512); break;
            case 17: hipLaunchKernelGGL((xor_persist2<8, 256, true>), dim3(4096), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 2048); break;
            case 18: hipLaunchKernelGGL((xor_loop<4, 256, true>), dim3(4096), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 19: hipLaunchKernelGGL((xor_loop<4, 256, true>), dim3(8192), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 20: hipLaunchKernelGGL((xor_persist2<4, 256, true>), dim3(6144), dim3(256), 0, 0, (u32x4*)buf, 0x5au, nw / 1024); break;
            case 23: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 3); break;
            case 24: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 4); break;
            case 25: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 5); break;
            case 26: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 0); break;
            case 27: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 6); break;
            case 28: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 7); break;
            case 29: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 8); break;
            case 30: kmws_unmask_batch_variant(buf, bytes, d, nf, ws, wsb, 0, 9); break;
            case 40: hipLaunchKernelGGL((read_split_nt<4, 256, 1>), dim3(nw / 1024), dim3(256), 0, 0, (const u32x4*)buf, sink); break;
            case 41: hipLaunchKernelGGL((read_split_nt<4, 256, 8>), dim3(nw / 1024), dim3(256), 0, 0, (const u32x4*)buf, sink); break;
            case 42: hipLaunchKernelGGL((write_split_nt<4, 256, 1>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 43: hipLaunchKernelGGL((write_split_nt<4, 256, 8>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 44: hipLaunchKernelGGL((copy_split_nt<4, 256, 1>), dim3(nw / 2 / 1024), dim3(256), 0, 0,
                                        (const u32x4*)buf, (u32x4*)(buf + bytes / 2)); break;
            case 45: hipLaunchKernelGGL((copy_split_nt<4, 256, 8>), dim3(nw / 2 / 1024), dim3(256), 0, 0,
                                        (const u32x4*)buf, (u32x4*)(buf + bytes / 2)); break;
            case 46: hipLaunchKernelGGL((xor_split_nt<4, 256, 1>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 47: hipLaunchKernelGGL((xor_split_nt<4, 256, 2>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 48: hipLaunchKernelGGL((xor_split_nt<4, 256, 8>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 50: hipLaunchKernelGGL((xor_split_nt<2, 256, 8>), dim3(nw / 512), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 51: hipLaunchKernelGGL((xor_split_nt<8, 256, 8>), dim3(nw / 2048), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 52: hipLaunchKernelGGL((xor_split_nt<4, 512, 8>), dim3(nw / 2048), dim3(512), 0, 0, (u32x4*)buf, 0x5au); break;
            case 53: hipLaunchKernelGGL((xor_split_nt<2, 512, 8>), dim3(nw / 1024), dim3(512), 0, 0, (u32x4*)buf, 0x5au); break;
            case 54: hipLaunchKernelGGL((xor_split_nt<4, 128, 8>), dim3(nw / 512), dim3(128), 0, 0, (u32x4*)buf, 0x5au); break;
            case 55: hipLaunchKernelGGL((xor_split_pol<4, 256, 8, false, true>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 56: hipLaunchKernelGGL((xor_split_pol<4, 256, 8, true, false>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 57: hipLaunchKernelGGL((xor_split_pol<4, 256, 8, false, false>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 58: hipLaunchKernelGGL((xor_split_nt<4, 256, 4>), dim3(nw / 1024), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            case 59: hipLaunchKernelGGL((xor_split_nt<8, 256, 2>), dim3(nw / 2048), dim3(256), 0, 0, (u32x4*)buf, 0x5au); break;
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r > 0) ms[k].push_back(t);
        }
    }
    printf("fill: %s\n", rand_fill ? "splitmix64 random" : "counter pattern {w, 1, 2, 3}");
    printf("buffer %.1f GiB, %d reps (GB/s = bytes moved / time: 2 x buffer for in-place, 1 x for read-only,\n"
           "write-only and copy (half -> half))\n",
           bytes / 1073741824.0, reps);
    for (size_t k = 0; k < vars.size(); ++k) {
        std::vector<float> v = ms[k];
        std::sort(v.begin(), v.end());
        const int kd = vars[k].kind;
        const double moved = (kd == 0 || kd == 44 || kd == 45 || (kd >= 40 && kd <= 43)) ? (double)bytes : 2.0 * bytes;
        printf("%-42s median %8.3f ms  best %8.3f ms  -> %7.0f GB/s (%.1f%% of 8 TB/s)\n", vars[k].name,
               v[v.size() / 2], v[0], moved / (v[v.size() / 2] * 1e-3) / 1e9,
               100.0 * moved / (v[v.size() / 2] * 1e-3) / 8e12);
    }
    return 0;
}
