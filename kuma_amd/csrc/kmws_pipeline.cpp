// Host-resident batches for kmws: the receive path starts and ends in host
// memory (TcpConnection.cpp:229 reads sockets into a 64 KiB host buffer).
//   - pinned host buffers under two chunks: ONE zero-copy unmask launch that
//     reads and writes the host bytes over PCIe (41.8 GiB/s on MI355X);
//   - pageable buffers, pinned batches of two chunks or more, or
//     KMWS_XFER_COPY: a ring of SDMA copies H2D -> unmask -> D2H on three
//     streams, chunks cut on frame boundaries (43-45 GiB/s on pinned memory).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "kmws_gpu.h"
#include "kmws_host_util.hpp"

using namespace kmws;

struct kmws_pipeline {
    // Copy ring: a slot's chunk goes H2D on s_in, is unmasked on s_kern and
    // goes D2H on s_out, ordered by events.  One stream per direction keeps
    // the copies of a direction back to back and lets H2D of chunk k+1 run
    // beside D2H of chunk k (two DMA directions at once: 90 GiB/s on MI355X vs
    // 53 for one); three streams stay within the 4 hardware queues a process
    // gets, where a stream per slot would share queues and serialize.
    hipStream_t s_in = nullptr, s_kern = nullptr, s_out = nullptr;
    struct Slot {
        hipEvent_t in_done = nullptr, kern_done = nullptr, done = nullptr;
        uint8_t* d_buf = nullptr;
        kmws_desc* d_desc = nullptr;
        kmws_desc* h_desc = nullptr;  // pinned staging for rebased descriptors
        void* d_ws = nullptr;
        size_t ws_bytes = 0;
        bool busy = false;
    };
    int device = 0;
    uint64_t chunk = 0;
    uint32_t max_frames = 0;
    std::vector<Slot> slots;
    int xfer = KMWS_XFER_AUTO;
    // zero-copy path (pinned host buffers): whole-batch descriptors + workspace
    kmws_desc* zc_desc = nullptr;
    size_t zc_desc_cap = 0;
    void* zc_ws = nullptr;
    size_t zc_ws_cap = 0;
    ~kmws_pipeline()
    {
        if (zc_desc) (void)hipFree(zc_desc);
        if (zc_ws) (void)hipFree(zc_ws);
        for (hipStream_t st : {s_in, s_kern, s_out})
            if (st) (void)hipStreamSynchronize(st);
        for (Slot& s : slots) {
            if (s.d_buf) (void)hipFree(s.d_buf);
            if (s.d_desc) (void)hipFree(s.d_desc);
            if (s.h_desc) (void)hipHostFree(s.h_desc);
            if (s.d_ws) (void)hipFree(s.d_ws);
            for (hipEvent_t e : {s.in_done, s.kern_done, s.done})
                if (e) (void)hipEventDestroy(e);
        }
        for (hipStream_t st : {s_in, s_kern, s_out})
            if (st) (void)hipStreamDestroy(st);
    }
};

extern "C" {

kmws_pipeline* kmws_pipeline_create(int device, uint64_t chunk_bytes, uint32_t max_frames_per_chunk, int depth)
{
    device = resolve_device(device);
    if (device < 0 || device >= kmws_device_count() || chunk_bytes < 4096 || depth < 1 || depth > 8 ||
        max_frames_per_chunk == 0)
        return nullptr;
    DevGuard g(device);
    kmws_pipeline* p = new (std::nothrow) kmws_pipeline();
    if (!p) return nullptr;
    p->device = device;
    p->chunk = (chunk_bytes + 15) & ~(uint64_t)15;
    p->max_frames = max_frames_per_chunk;
    p->slots.resize(depth);
    const uint64_t dev_bytes = p->chunk + 32;  // + alignment slack at both ends
    for (hipStream_t* st : {&p->s_in, &p->s_kern, &p->s_out})
        if (hipStreamCreateWithFlags(st, hipStreamNonBlocking) != hipSuccess) {
            delete p;
            return nullptr;
        }
    for (auto& s : p->slots) {
        s.ws_bytes = kmws_unmask_workspace_size(dev_bytes);
        if (hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.kern_done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&s.d_buf), dev_bytes) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&s.d_desc), (size_t)p->max_frames * sizeof(kmws_desc)) != hipSuccess ||
            hipHostMalloc(reinterpret_cast<void**>(&s.h_desc), (size_t)p->max_frames * sizeof(kmws_desc),
                          hipHostMallocDefault) != hipSuccess ||
            hipMalloc(&s.d_ws, s.ws_bytes) != hipSuccess) {
            delete p;
            return nullptr;
        }
    }
    return p;
}

kmws_status kmws_pipeline_set_transfer(kmws_pipeline* p, int mode)
{
    if (!p || mode < KMWS_XFER_AUTO || mode > KMWS_XFER_ZEROCOPY) return KMWS_ERR_INVALID_PARAM;
    p->xfer = mode;
    return KMWS_OK;
}

void kmws_pipeline_destroy(kmws_pipeline* p)
{
    if (p) {
        DevGuard g(p->device);
        delete p;
    }
}

kmws_status kmws_pipeline_unmask(kmws_pipeline* p, uint8_t* host_base, uint64_t span, const kmws_desc* descs,
                                 uint32_t n)
{
    if (!p || (n && (!host_base || !descs))) return KMWS_ERR_INVALID_PARAM;
    DevGuard g(p->device);
    if (n == 0) return KMWS_OK;
    uint8_t* dv = p->xfer == KMWS_XFER_COPY ? nullptr : static_cast<uint8_t*>(device_view(host_base));
    if (p->xfer == KMWS_XFER_ZEROCOPY && !dv) return KMWS_ERR_INVALID_PARAM;  // needs pinned memory
    // AUTO on pinned memory: the copy ring once the batch spans two chunks (its
    // two DMA directions overlap: 43-45 GiB/s vs 41.8 for the zero-copy kernel,
    // profiles/r01e_e2e_ring.txt), the single zero-copy launch below that.
    if (p->xfer == KMWS_XFER_AUTO && dv && span >= 2 * p->chunk) dv = nullptr;
    if (dv) {
        // Pinned host memory: one zero-copy unmask over PCIe, in place.
        hipStream_t zs = p->s_kern;
        if (n > p->zc_desc_cap) {
            if (p->zc_desc) (void)hipFree(p->zc_desc);
            p->zc_desc = nullptr;
            p->zc_desc_cap = 0;
            if (hipMalloc(reinterpret_cast<void**>(&p->zc_desc), (size_t)n * sizeof(kmws_desc)) != hipSuccess)
                return KMWS_ERR_FAILED;
            p->zc_desc_cap = n;
        }
        const size_t ws = kmws_unmask_workspace_size(span);
        if (ws > p->zc_ws_cap) {
            if (p->zc_ws) (void)hipFree(p->zc_ws);
            p->zc_ws = nullptr;
            p->zc_ws_cap = 0;
            if (hipMalloc(&p->zc_ws, ws) != hipSuccess) return KMWS_ERR_FAILED;
            p->zc_ws_cap = ws;
        }
        if (hipMemcpyAsync(p->zc_desc, descs, (size_t)n * sizeof(kmws_desc), hipMemcpyHostToDevice, zs) !=
            hipSuccess)
            return KMWS_ERR_FAILED;
        kmws_status st = kmws_unmask_batch(dv, span, p->zc_desc, n, p->zc_ws, p->zc_ws_cap, zs);
        if (st != KMWS_OK) return st;
        uint32_t status = 0;
        if (hipMemcpyAsync(&status, p->zc_ws, sizeof(status), hipMemcpyDeviceToHost, zs) != hipSuccess ||
            hipStreamSynchronize(zs) != hipSuccess)
            return KMWS_ERR_FAILED;
        return status == 0 ? KMWS_OK : KMWS_ERR_INVALID_PARAM;
    }
    // Every descriptor is checked before the first chunk is queued (sorted, in
    // the span, each frame's 16-B aligned hull within one chunk), so a bad batch
    // is rejected with nothing in flight and the host buffer untouched.
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = descs[i].off, end = off + descs[i].len;
        if (end < off || end > span || (i && off < descs[i - 1].off + descs[i - 1].len))
            return KMWS_ERR_INVALID_PARAM;
        if (end - (off & ~(uint64_t)15) > p->chunk) return KMWS_ERR_BUFFER_TOO_SMALL;  // one frame larger than a chunk
    }
    uint32_t f = 0;
    size_t k = 0;
    kmws_status st = KMWS_OK;
    // From here on every failure leaves the loop and goes through the drain
    // below: no slot is still copying into host_base when the call returns.
    while (f < n && st == KMWS_OK) {
        // frames [f, e) whose 16-B aligned hull fits the chunk (e > f: checked above)
        const uint64_t lo = descs[f].off & ~(uint64_t)15;
        uint32_t e = f;
        uint64_t hi = descs[f].off;
        while (e < n && e - f < p->max_frames) {
            const uint64_t end = descs[e].off + descs[e].len;
            if (end - lo > p->chunk) break;
            hi = end;
            ++e;
        }
        // at most 3 slots in flight: with 4, H2D runs far enough ahead to hold
        // the DMA engines the D2H needs (26 GiB/s instead of 45)
        kmws_pipeline::Slot& s = p->slots[k % std::min<size_t>(p->slots.size(), 3)];
        if (s.busy && hipEventSynchronize(s.done) != hipSuccess) {
            st = KMWS_ERR_FAILED;
            break;
        }
        s.busy = false;
        const uint64_t first = descs[f].off;
        for (uint32_t i = f; i < e; ++i) {
            s.h_desc[i - f] = descs[i];
            s.h_desc[i - f].off -= lo;
        }
        const uint64_t bytes = (hi + 15 - lo) & ~(uint64_t)15;
        const uint64_t h2d = hi - lo;  // never read past the caller's span
        if (hipMemcpyAsync(s.d_buf, host_base + lo, h2d, hipMemcpyHostToDevice, p->s_in) != hipSuccess ||
            hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)(e - f) * sizeof(kmws_desc), hipMemcpyHostToDevice,
                           p->s_in) != hipSuccess ||
            hipEventRecord(s.in_done, p->s_in) != hipSuccess ||
            hipStreamWaitEvent(p->s_kern, s.in_done, 0) != hipSuccess) {
            st = KMWS_ERR_FAILED;
            break;
        }
        // the H2D copies may be in flight: the slot counts as busy until its
        // last recorded event (s_in's work is drained below in any case)
        s.busy = true;
        if (hipEventRecord(s.done, p->s_in) != hipSuccess) {
            st = KMWS_ERR_FAILED;
            break;
        }
        st = kmws_unmask_batch(s.d_buf, bytes, s.d_desc, e - f, s.d_ws, s.ws_bytes, p->s_kern);
        if (st != KMWS_OK) break;
        // write back exactly the frames' extent: neighbours' bytes stay untouched
        if (hipEventRecord(s.kern_done, p->s_kern) != hipSuccess ||
            hipStreamWaitEvent(p->s_out, s.kern_done, 0) != hipSuccess ||
            hipMemcpyAsync(host_base + first, s.d_buf + (first - lo), hi - first, hipMemcpyDeviceToHost,
                           p->s_out) != hipSuccess ||
            hipEventRecord(s.done, p->s_out) != hipSuccess) {
            st = KMWS_ERR_FAILED;
            break;
        }
        f = e;
        ++k;
    }
    if (st != KMWS_OK) {  // whatever was queued finishes before the caller gets its buffer back
        for (hipStream_t q : {p->s_in, p->s_kern, p->s_out}) (void)hipStreamSynchronize(q);
    }
    for (auto& s : p->slots) {
        if (s.busy && hipEventSynchronize(s.done) != hipSuccess) st = KMWS_ERR_FAILED;
        s.busy = false;
    }
    return st;
}

}  // extern "C"
