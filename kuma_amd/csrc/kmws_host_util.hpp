// Host-side helpers shared by the decoder, the rx batch and the pipeline:
// device guard, pinned-memory detection and the pinned staging area whose
// payloads the unmask kernel processes in place over PCIe (zero-copy).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "kmws_gpu.h"

namespace kmws {

// Switch to `dev` for the scope; restore the caller's current device on exit.
struct DevGuard {
    int prev = -1;
    explicit DevGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DevGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Device-visible address of pinned host memory (hipHostMalloc / hipHostRegister),
// or nullptr for pageable memory.
inline void* device_view(void* host)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, host) != hipSuccess) {
        (void)hipGetLastError();  // clear the error left for pageable pointers
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost) return nullptr;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

inline size_t grow(size_t need, size_t have)
{
    size_t c = have ? have : (size_t)1 << 20;
    while (c < need) c *= 2;
    return c;
}

// A batch of payloads unmasked in place by the GPU.  Payloads are appended to
// a pinned host area (16-B aligned starts, so whole-frame tiles take the
// kernel's fast path); run() copies the descriptors to the device, launches
// kmws_unmask_batch on the pinned area itself (zero-copy over PCIe) and waits.
// An optional second batch of descriptors can target another pinned buffer
// (a caller's registered receive buffer).
class PinnedStage {
public:
    ~PinnedStage() { release(); }

    kmws_status init(int device)
    {
        if (dev_ok_ < 0) {
            device_ = device;
            dev_ok_ = (device >= 0 && kmws_device_count() > device) ? 1 : 0;
        }
        if (!dev_ok_) return KMWS_ERR_NOT_SUPPORTED;
        if (!stream_) {
            DevGuard g(device_);
            if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return KMWS_ERR_FAILED;
        }
        return KMWS_OK;
    }
    int device() const { return device_; }
    hipStream_t stream() const { return stream_; }

    // Room for `bytes` more payload bytes (plus alignment) without moving offsets.
    kmws_status reserve(size_t bytes)
    {
        const size_t need = len_ + 16 + bytes;
        if (need <= cap_) return KMWS_OK;
        DevGuard g(device_);
        const size_t c = grow(need, cap_);
        uint8_t* p = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), c, hipHostMallocDefault) != hipSuccess) return KMWS_ERR_FAILED;
        if (h_) {
            std::memcpy(p, h_, len_);
            (void)hipHostFree(h_);
        }
        h_ = p;
        cap_ = c;
        return KMWS_OK;
    }
    size_t append(const uint8_t* p, size_t n)  // after reserve(n)
    {
        const size_t off = (len_ + 15) & ~(size_t)15;
        if (n) std::memcpy(h_ + off, p, n);
        len_ = off + n;
        return off;
    }
    // Room for n bytes at a 16-B aligned offset (after reserve(n)); the caller fills it.
    uint8_t* alloc(size_t n, size_t* off)
    {
        *off = (len_ + 15) & ~(size_t)15;
        len_ = *off + n;
        return h_ + *off;
    }
    uint8_t* data() { return h_; }
    void add_desc(uint64_t off, uint32_t len, uint32_t key) { descs_.push_back(kmws_desc{off, len, key}); }
    size_t n_desc() const { return descs_.size(); }
    void clear()
    {
        len_ = 0;
        descs_.clear();
    }

    // Unmask every staged descriptor (and `extra` over `extra_base`, a pinned
    // buffer of extra_span bytes, if given), then wait for the GPU.
    kmws_status run(uint8_t* extra_base = nullptr, uint64_t extra_span = 0,
                    const std::vector<kmws_desc>* extra = nullptr)
    {
        const size_t n1 = descs_.size(), n2 = extra ? extra->size() : 0;
        if (n1 + n2 == 0) return KMWS_OK;
        DevGuard g(device_);
        kmws_status st = ensure_dev(n1 + n2, std::max<uint64_t>((len_ + 15) & ~(size_t)15, extra_span));
        if (st != KMWS_OK) return st;
        std::memcpy(h_desc_, descs_.data(), n1 * sizeof(kmws_desc));
        if (n2) std::memcpy(h_desc_ + n1, extra->data(), n2 * sizeof(kmws_desc));
        if (n1 && hipMemcpyAsync(d_desc_, h_desc_, n1 * sizeof(kmws_desc), hipMemcpyHostToDevice, stream_) !=
                      hipSuccess)
            return KMWS_ERR_FAILED;
        uint32_t status[2] = {0, 0};
        if (n1) {
            uint8_t* dv = static_cast<uint8_t*>(device_view(h_));
            if (!dv) return KMWS_ERR_FAILED;
            st = kmws_unmask_batch(dv, (len_ + 15) & ~(size_t)15, d_desc_, (uint32_t)n1, d_ws_[0], ws_cap_, stream_);
            if (st != KMWS_OK) return st;
            if (hipMemcpyAsync(&status[0], d_ws_[0], 4, hipMemcpyDeviceToHost, stream_) != hipSuccess)
                return KMWS_ERR_FAILED;
        }
        if (n2) {
            // Only the extent the descriptors cover is processed: rebase them
            // onto its 16-B aligned start (a large pinned ring may hold few frames).
            uint64_t lo = ~0ull, hi = 0;
            for (const kmws_desc& x : *extra) {
                lo = std::min<uint64_t>(lo, x.off);
                hi = std::max<uint64_t>(hi, x.off + x.len);
            }
            lo &= ~(uint64_t)15;
            if (hi > extra_span) return KMWS_ERR_INVALID_PARAM;
            for (size_t i = 0; i < n2; ++i) h_desc_[n1 + i].off -= lo;
            if (hipMemcpyAsync(d_desc_ + n1, h_desc_ + n1, n2 * sizeof(kmws_desc), hipMemcpyHostToDevice, stream_) !=
                hipSuccess)
                return KMWS_ERR_FAILED;
            uint8_t* dv = static_cast<uint8_t*>(device_view(extra_base));
            if (!dv) return KMWS_ERR_INVALID_PARAM;
            st = kmws_unmask_batch(dv + lo, hi - lo, d_desc_ + n1, (uint32_t)n2, d_ws_[1], ws_cap_, stream_);
            if (st != KMWS_OK) return st;
            if (hipMemcpyAsync(&status[1], d_ws_[1], 4, hipMemcpyDeviceToHost, stream_) != hipSuccess)
                return KMWS_ERR_FAILED;
        }
        if (hipStreamSynchronize(stream_) != hipSuccess) return KMWS_ERR_FAILED;
        return (status[0] | status[1]) == 0 ? KMWS_OK : KMWS_ERR_INVALID_STATE;
    }

private:
    kmws_status ensure_dev(size_t nd, uint64_t span)
    {
        if (nd > desc_cap_) {
            const size_t c = std::max<size_t>(nd * 2, 1024);
            if (h_desc_) (void)hipHostFree(h_desc_);
            if (d_desc_) (void)hipFree(d_desc_);
            h_desc_ = nullptr;
            d_desc_ = nullptr;
            desc_cap_ = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&h_desc_), c * sizeof(kmws_desc), hipHostMallocDefault) !=
                    hipSuccess ||
                hipMalloc(reinterpret_cast<void**>(&d_desc_), c * sizeof(kmws_desc)) != hipSuccess)
                return KMWS_ERR_FAILED;
            desc_cap_ = c;
        }
        const size_t ws = kmws_unmask_workspace_size(span);
        if (ws > ws_cap_) {
            for (void*& w : d_ws_) {
                if (w) (void)hipFree(w);
                w = nullptr;
            }
            ws_cap_ = grow(ws, ws_cap_);
            for (void*& w : d_ws_)
                if (hipMalloc(&w, ws_cap_) != hipSuccess) {
                    ws_cap_ = 0;
                    return KMWS_ERR_FAILED;
                }
        }
        return KMWS_OK;
    }
    void release()
    {
        if (stream_) (void)hipStreamSynchronize(stream_);
        if (h_) (void)hipHostFree(h_);
        if (h_desc_) (void)hipHostFree(h_desc_);
        if (d_desc_) (void)hipFree(d_desc_);
        for (void* w : d_ws_)
            if (w) (void)hipFree(w);
        if (stream_) (void)hipStreamDestroy(stream_);
    }

    int device_ = 0;
    int dev_ok_ = -1;
    hipStream_t stream_ = nullptr;
    uint8_t* h_ = nullptr;
    size_t cap_ = 0, len_ = 0;
    std::vector<kmws_desc> descs_;
    kmws_desc* h_desc_ = nullptr;
    kmws_desc* d_desc_ = nullptr;
    size_t desc_cap_ = 0;
    void* d_ws_[2] = {nullptr, nullptr};
    size_t ws_cap_ = 0;
};

}  // namespace kmws
