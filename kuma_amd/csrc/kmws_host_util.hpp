// Host-side helpers shared by the decoder, the rx batch and the pipeline:
// device guard, pinned-memory detection and the pinned staging area whose
// payloads the unmask kernel processes in place over PCIe (zero-copy).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "kmws_common.hpp"
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
// a pinned host area (16-B aligned starts); launch() posts them as one job on
// the calling thread's slot of the resident worker when they fit one, else
// enqueues the pieces kernel on the pinned area itself (zero-copy over PCIe)
// on the stage's own stream and records its completion event; done() / wait()
// follow whichever ran; run() = launch() + wait.  An optional second
// batch of descriptors can target another pinned buffer (a caller's registered
// receive or send ring).  The asynchronous rx / tx batches keep one stage per
// generation in flight (kmws_decoder.cpp).
// A stream a batch owns and its stages share; declared first in the batch so
// it is destroyed after every stage.
struct BatchStream {
    hipStream_t s = nullptr;
    int device = -1;
    kmws_status create(int dev)
    {
        device = dev;
        if (dev < 0 || kmws_device_count() <= dev) return KMWS_ERR_NOT_SUPPORTED;
        DevGuard g(dev);
        return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? KMWS_OK : KMWS_ERR_FAILED;
    }
    ~BatchStream()
    {
        if (!s) return;
        DevGuard g(device);
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
};

class PinnedStage {
public:
    ~PinnedStage() { release(); }

    // shared: a stream the owner keeps for all its stages (a batch's
    // generations), else the stage creates its own.  Creating a stream can
    // take milliseconds -- a loop iteration that needed a new stage stalled
    // for 2-3.5 ms (r05i/r05j loopback, rx_task_max) -- so the batches create
    // theirs once.
    kmws_status init(int device, hipStream_t shared = nullptr)
    {
        if (dev_ok_ < 0) {
            device_ = device;
            dev_ok_ = (device >= 0 && kmws_device_count() > device) ? 1 : 0;
        }
        if (!dev_ok_) return KMWS_ERR_NOT_SUPPORTED;
        if (!stream_) {
            DevGuard g(device_);
            if (shared) {
                stream_ = shared;
                own_stream_ = false;
            } else if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
                return KMWS_ERR_FAILED;
            }
            if (hipEventCreateWithFlags(&done_, hipEventDisableTiming) != hipSuccess) return KMWS_ERR_FAILED;
        }
        return KMWS_OK;
    }
    int device() const { return device_; }
    hipStream_t stream() const { return stream_; }

    // Allocates the pinned staging area and descriptor / piece arrays ahead
    // of use (hipHostMalloc can take milliseconds inside a loop iteration).
    kmws_status warm()
    {
        kmws_status st = reserve(64u << 10);
        if (st == KMWS_OK) st = ensure_host(kResMaxDescs, 4 * kResMaxDescs);
        return st;
    }

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
        dv_h_ = static_cast<uint8_t*>(device_view(h_));
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
    // buffer of extra_span bytes, if given), then wait for the GPU: launch() +
    // wait().  extra_dv: the device view of extra_base if the caller has it (a
    // ring attached once); else it is looked up here (hipPointerGetAttributes).
    kmws_status run(uint8_t* extra_base = nullptr, uint64_t extra_span = 0,
                    const std::vector<kmws_desc>* extra = nullptr, uint8_t* extra_dv = nullptr)
    {
        kmws_status st = launch(extra_base, extra_span, extra, extra_dv, kResMaxBytes);
        if (st != KMWS_OK) return st;
        return wait();
    }

    // Has the last launch() finished?  (true when nothing was launched)
    bool done()
    {
        if (!launched_) return true;
        if (res_pending_) {
            const int r = resident_test(res_);
            if (r == 1) return true;
            if (r == 0) return false;
            res_pending_ = false;
            if (r != KMWS_ERR_NOT_SUPPORTED || launch_saved() != KMWS_OK) return true;  // wait() reports it
        }
        const hipError_t e = hipEventQuery(done_);
        if (e == hipErrorNotReady) return false;
        (void)hipGetLastError();
        return true;  // finished, or failed: wait() reports which
    }
    // A launched job: spins on the event for a time that grows with its bytes
    // (a loop thread waiting for a small job should not be parked and woken by
    // the runtime; a large one should not burn a core), then parks.
    kmws_status wait()
    {
        if (!launched_) return KMWS_OK;
        if (res_pending_) {
            res_pending_ = false;
            const kmws_status st = resident_wait(res_);
            if (st == KMWS_ERR_TIMEOUT) abandon();
            if (st != KMWS_ERR_NOT_SUPPORTED) {
                launched_ = false;
                return st;
            }
            const kmws_status ls = launch_saved();  // withdrawn, never run: launch it now
            if (ls != KMWS_OK) {
                launched_ = false;
                return ls;
            }
        }
        launched_ = false;
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            const hipError_t e = hipEventQuery(done_);
            if (e == hipSuccess) return KMWS_OK;
            if (e != hipErrorNotReady) {
                (void)hipGetLastError();
                return KMWS_ERR_FAILED;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) break;
        }
        return hipEventSynchronize(done_) == hipSuccess ? KMWS_OK : KMWS_ERR_FAILED;
    }

    // Enqueue the unmask of every staged descriptor (and `extra`) without
    // waiting: a job of at most kResMaxDescs payloads and max_res_bytes bytes is
    // posted on the calling thread's slot of the device's resident worker (no
    // launch; kmws_resident.hip), anything else is launched on the stage's
    // stream (launch_unmask_pieces: no plan kernels, no copies, no status
    // read-back) with its completion event recorded.
    // max_res_bytes: the largest job posted on the worker (a synchronous run()
    // keeps kResMaxBytes: one workgroup is slower than a launch's many above it).
    kmws_status launch(uint8_t* extra_base = nullptr, uint64_t extra_span = 0,
                       const std::vector<kmws_desc>* extra = nullptr, uint8_t* extra_dv = nullptr,
                       uint64_t max_res_bytes = kResMaxBytesAsync)
    {
        const size_t n1 = descs_.size(), n2 = extra ? extra->size() : 0;
        if (n1 + n2 == 0) return KMWS_OK;
        if (launched_) return KMWS_ERR_INVALID_STATE;
        for (size_t i = 0; i < n2; ++i)
            if ((*extra)[i].off + (*extra)[i].len > extra_span) return KMWS_ERR_INVALID_PARAM;
        if (n2 && !extra_dv) extra_dv = static_cast<uint8_t*>(device_view(extra_base));
        if (n2 && !extra_dv) return KMWS_ERR_INVALID_PARAM;  // must be pinned
        if (n1 && !dv_h_) return KMWS_ERR_FAILED;
        if (n1 + n2 <= (size_t)kResMaxDescs) {
            const kmws_status st = resident_post(device_, descs_.data(), dv_h_, n1, n2 ? extra->data() : nullptr,
                                                 extra_dv, n2, &res_, max_res_bytes);
            if (st == KMWS_OK) {  // kept for a launch if the worker withdraws the job
                saved_base_ = extra_base;
                saved_span_ = extra_span;
                saved_dv_ = extra_dv;
                saved_extra_.assign(extra ? extra->begin() : saved_extra_.end(), extra ? extra->end() : saved_extra_.end());
                res_pending_ = true;
                launched_ = true;
                return KMWS_OK;
            }
            if (st != KMWS_ERR_NOT_SUPPORTED) return st;
        }
        return launch_kernels(extra_base, extra_span, extra, extra_dv);
    }

private:
    kmws_status launch_saved()
    {
        return launch_kernels(saved_base_, saved_span_, saved_extra_.empty() ? nullptr : &saved_extra_, saved_dv_);
    }

    // The device may still write the staging area (a resident job that timed
    // out): it is left to the device -- never freed, never reused.
    void abandon()
    {
        h_ = nullptr;
        dv_h_ = nullptr;
        cap_ = 0;
        len_ = 0;
        descs_.clear();
    }

    kmws_status launch_kernels(uint8_t* extra_base, uint64_t extra_span, const std::vector<kmws_desc>* extra,
                               uint8_t* extra_dv)
    {
        const size_t n1 = descs_.size(), n2 = extra ? extra->size() : 0;
        if (n1 + n2 == 0) return KMWS_OK;
        DevGuard g(device_);
        // the extra buffer's 16-B aligned base, descriptors rebased onto it
        uint8_t* eb = reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(extra_base) & ~(uintptr_t)15);
        const uint64_t delta = (uint64_t)(extra_base - eb);
        uint64_t p1 = 0, p2 = 0, bytes = 0;
        for (const kmws_desc& x : descs_) {
            p1 += piece_count(x.off, x.len);
            bytes += x.len;
        }
        for (size_t i = 0; i < n2; ++i) {
            const kmws_desc& x = (*extra)[i];
            if (x.off + x.len > extra_span) return KMWS_ERR_INVALID_PARAM;
            p2 += piece_count(x.off + delta, x.len);
            bytes += x.len;
        }
        if (p1 + p2 > 0x7FFFFFFFull) return KMWS_ERR_INVALID_PARAM;
        kmws_status st = ensure_host(n1 + n2, p1 + p2);
        if (st != KMWS_OK) return st;
        std::memcpy(h_desc_, descs_.data(), n1 * sizeof(kmws_desc));
        size_t k = 0;
        for (size_t i = 0; i < n1; ++i)
            for (uint64_t j = 0, c = piece_count(descs_[i].off, descs_[i].len); j < c; ++j)
                h_piece_[k++] = PieceRec{(uint32_t)i, (uint32_t)j};
        for (size_t i = 0; i < n2; ++i) {
            kmws_desc x = (*extra)[i];
            x.off += delta;
            h_desc_[n1 + i] = x;
            for (uint64_t j = 0, c = piece_count(x.off, x.len); j < c; ++j)
                h_piece_[k++] = PieceRec{(uint32_t)i, (uint32_t)j};
        }
        if (p1) {
            uint8_t* dv = dv_h_;  // device view of the staging area, taken when it was allocated
            if (!dv) return KMWS_ERR_FAILED;
            st = launch_unmask_pieces(dv, dv_desc_, dv_piece_, (uint32_t)p1, stream_);
            if (st != KMWS_OK) return st;
        }
        if (p2) {
            if (!extra_dv) extra_dv = static_cast<uint8_t*>(device_view(extra_base));
            if (!extra_dv) return KMWS_ERR_INVALID_PARAM;
            uint8_t* dv = extra_dv - delta;  // the aligned base's view (one mapping per allocation)
            st = launch_unmask_pieces(dv, dv_desc_ + n1, dv_piece_ + p1, (uint32_t)p2, stream_);
            if (st != KMWS_OK) return st;
        }
        if (hipEventRecord(done_, stream_) != hipSuccess) return KMWS_ERR_FAILED;
        // spin for about twice what the job should take (a launch's ~20 us, then
        // the payload over PCIe at ~8 GB/s each way), at least 1 ms -- a kernel
        // queued behind the resident grid on a shared hardware queue waits up
        // to its 1 ms lease, and a parked thread is woken milliseconds late
        // (loopback rx flushes of 2.6-5.1 ms with a 104 us spin, r05g) -- at
        // most 2 ms
        spin_us_ = std::min<uint64_t>(2000, std::max<uint64_t>(1000, 2 * (20 + (bytes >> 13))));
        launched_ = true;
        return KMWS_OK;
    }

    // Pinned descriptor and piece arrays (and their device views) for nd / np entries.
    kmws_status ensure_host(size_t nd, size_t np)
    {
        if (nd > desc_cap_) {
            const size_t c = std::max<size_t>(nd * 2, 1024);
            if (h_desc_) (void)hipHostFree(h_desc_);
            h_desc_ = nullptr;
            dv_desc_ = nullptr;
            desc_cap_ = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&h_desc_), c * sizeof(kmws_desc), hipHostMallocDefault) !=
                hipSuccess)
                return KMWS_ERR_FAILED;
            dv_desc_ = static_cast<kmws_desc*>(device_view(h_desc_));
            if (!dv_desc_) return KMWS_ERR_FAILED;
            desc_cap_ = c;
        }
        if (np > piece_cap_) {
            const size_t c = std::max<size_t>(np * 2, 1024);
            if (h_piece_) (void)hipHostFree(h_piece_);
            h_piece_ = nullptr;
            dv_piece_ = nullptr;
            piece_cap_ = 0;
            if (hipHostMalloc(reinterpret_cast<void**>(&h_piece_), c * sizeof(PieceRec), hipHostMallocDefault) !=
                hipSuccess)
                return KMWS_ERR_FAILED;
            dv_piece_ = static_cast<PieceRec*>(device_view(h_piece_));
            if (!dv_piece_) return KMWS_ERR_FAILED;
            piece_cap_ = c;
        }
        return KMWS_OK;
    }
    void release()
    {
        if (launched_) (void)wait();  // nothing may outlive its pinned memory (a timed-out job's is abandoned)
        if (stream_ && own_stream_) (void)hipStreamSynchronize(stream_);
        if (done_) (void)hipEventDestroy(done_);
        if (h_) (void)hipHostFree(h_);
        if (h_desc_) (void)hipHostFree(h_desc_);
        if (h_piece_) (void)hipHostFree(h_piece_);
        if (stream_ && own_stream_) (void)hipStreamDestroy(stream_);
    }

    int device_ = 0;
    int dev_ok_ = -1;
    hipStream_t stream_ = nullptr;
    bool own_stream_ = true;
    hipEvent_t done_ = nullptr;
    bool launched_ = false;
    bool res_pending_ = false;  // launched_ on the resident worker: res_ says which job
    ResidentJob res_;
    uint8_t* saved_base_ = nullptr;  // extra of a resident job, for launch_saved()
    uint64_t saved_span_ = 0;
    uint8_t* saved_dv_ = nullptr;
    std::vector<kmws_desc> saved_extra_;
    uint64_t spin_us_ = 1000;
    uint8_t* h_ = nullptr;
    uint8_t* dv_h_ = nullptr;
    size_t cap_ = 0, len_ = 0;
    std::vector<kmws_desc> descs_;
    kmws_desc* h_desc_ = nullptr;   // pinned, read by the kernel over PCIe
    kmws_desc* dv_desc_ = nullptr;  // its device view
    size_t desc_cap_ = 0;
    PieceRec* h_piece_ = nullptr;
    PieceRec* dv_piece_ = nullptr;
    size_t piece_cap_ = 0;
};

}  // namespace kmws
