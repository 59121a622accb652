// Host side of the kmws C ABI: header pack and the WSHandler-compatible
// streaming decoder (src/ws/WSHandler.{h,cpp} in the reference).
//
// The decoder keeps kuma's per-byte header state machine on the event-loop
// thread (headers arrive byte-serially on one connection, WSHandler.cpp:
// 108-280) and moves the payload work -- the reference's scalar unmask loop
// (WSHandler.cpp:303-310) -- to the GPU: every masked frame completed by one
// feed call is staged into pinned memory, unmasked by ONE kmws_unmask_batch
// launch, and then delivered in order.  There is no CPU unmask path: without a
// usable gfx950 device a masked frame fails the call with
// KMWS_ERR_NOT_SUPPORTED.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "kmws_gpu.h"

namespace {

enum class St : uint8_t { HDR1, HDR2, HDREX, MASKEY, DATA, CLOSED, IN_ERROR };  // WSHandler.h:57-65

bool is_control(uint8_t op) { return op >= 8; }  // WSHandler.h:52-54

// Where a completed frame's payload lives until delivery.
enum Origin : int {
    kInChunk = 0,        // unmasked (or empty): view into the caller's chunk
    kInChunkMasked = 1,  // masked, wholly in the chunk: staged, written back in place
    kStagedMasked = 2,   // masked, reassembled across chunks: view into staging
    kHeld = 3,           // unmasked, reassembled: view into a held reassembly buffer
};

struct Pending {
    kmws_frame_hdr hdr;
    uint8_t* data_ptr;   // kInChunk / kInChunkMasked: payload position in the chunk
    size_t stage_off;    // masked: payload offset in the pinned staging area
    size_t hold_idx;     // kHeld: index into kmws_decoder::held
    Origin where;
};

}  // namespace

struct kmws_decoder {
    int mode = KMWS_MODE_CLIENT;
    int device = 0;
    // DecodeContext (WSHandler.h:66-78)
    kmws_frame_hdr hdr{};
    St state = St::HDR1;
    std::vector<uint8_t> buf;
    uint8_t pos = 0;

    // per-call delivery lists
    std::vector<Pending> pending;
    std::vector<std::vector<uint8_t>> held;

    // GPU staging (lazily created on the first masked frame)
    hipStream_t stream = nullptr;
    uint8_t* h_stage = nullptr;  // pinned
    size_t h_stage_cap = 0;
    kmws_desc* h_desc = nullptr;  // pinned
    kmws_desc* d_desc = nullptr;
    size_t desc_cap = 0;
    void* d_ws = nullptr;
    size_t ws_cap = 0;
    size_t stage_len = 0;
    int dev_ok = -1;  // cached: is `device` a usable gfx950?

    void reset_ctx()
    {
        std::memset(&hdr, 0, sizeof(hdr));
        state = St::HDR1;
        buf.clear();
        pos = 0;
    }
    ~kmws_decoder() { release_gpu(); }
    void release_gpu()
    {
        if (h_stage) (void)hipHostFree(h_stage);
        if (h_desc) (void)hipHostFree(h_desc);
        if (d_desc) (void)hipFree(d_desc);
        if (d_ws) (void)hipFree(d_ws);
        if (stream) (void)hipStreamDestroy(stream);
        h_stage = nullptr;
        h_desc = d_desc = nullptr;
        d_ws = nullptr;
        stream = nullptr;
        h_stage_cap = desc_cap = ws_cap = 0;
    }
    kmws_status stage_reserve(size_t bytes, size_t nframes);
    size_t stage_append(const uint8_t* p, size_t n);
    kmws_status unmask_staged();
};

namespace {

struct DevGuard {  // switch to the decoder's device, restore the caller's on exit
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
void* device_view(void* host)
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

size_t grow(size_t need, size_t have)
{
    size_t c = have ? have : (size_t)1 << 20;
    while (c < need) c *= 2;
    return c;
}

}  // namespace

kmws_status kmws_decoder::stage_reserve(size_t bytes, size_t nframes)
{
    if (dev_ok < 0) dev_ok = (device >= 0 && kmws_device_count() > device) ? 1 : 0;
    if (!dev_ok) return KMWS_ERR_NOT_SUPPORTED;
    DevGuard g(device);
    if (!stream && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return KMWS_ERR_FAILED;
    if (bytes > h_stage_cap) {
        size_t c = grow(bytes, h_stage_cap);
        uint8_t* p = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), c, hipHostMallocDefault) != hipSuccess) return KMWS_ERR_FAILED;
        if (h_stage) {
            std::memcpy(p, h_stage, stage_len);
            (void)hipHostFree(h_stage);
        }
        h_stage = p;
        h_stage_cap = c;
    }
    if (nframes > desc_cap) {
        size_t c = std::max<size_t>(nframes * 2, 1024);
        kmws_desc* hp = nullptr;
        if (hipHostMalloc(reinterpret_cast<void**>(&hp), c * sizeof(kmws_desc), hipHostMallocDefault) != hipSuccess)
            return KMWS_ERR_FAILED;
        if (h_desc) (void)hipHostFree(h_desc);
        if (d_desc) (void)hipFree(d_desc);
        d_desc = nullptr;
        h_desc = hp;
        desc_cap = c;
        if (hipMalloc(reinterpret_cast<void**>(&d_desc), c * sizeof(kmws_desc)) != hipSuccess) return KMWS_ERR_FAILED;
    }
    return KMWS_OK;
}

size_t kmws_decoder::stage_append(const uint8_t* p, size_t n)
{
    size_t off = (stage_len + 15) & ~(size_t)15;  // 16-B aligned payloads take the kernel's fast path
    std::memcpy(h_stage + off, p, n);
    stage_len = off + n;
    return off;
}

kmws_status kmws_decoder::unmask_staged()
{
    size_t nd = 0;
    for (const Pending& q : pending) {
        if (q.where == kInChunkMasked || q.where == kStagedMasked) {
            kmws_desc d;
            d.off = q.stage_off;
            d.len = q.hdr.length;
            std::memcpy(&d.key, q.hdr.maskey, 4);
            h_desc[nd++] = d;
        }
    }
    if (nd == 0) return KMWS_OK;
    DevGuard g(device);
    // Zero-copy: the kernel unmasks the pinned staging area in place over
    // PCIe (measured 43.7 GiB/s on MI355X, at the ~45 GiB/s per-direction
    // ceiling of concurrent H2D + D2H, tools/pcie_probe.hip), so no H2D/D2H
    // copies of the payload; only the descriptors are copied.
    const size_t span = (stage_len + 15) & ~(size_t)15;
    uint8_t* dview = static_cast<uint8_t*>(device_view(h_stage));
    if (!dview) return KMWS_ERR_FAILED;
    const size_t ws = kmws_unmask_workspace_size(span);
    if (ws > ws_cap) {
        if (d_ws) (void)hipFree(d_ws);
        d_ws = nullptr;
        ws_cap = grow(ws, ws_cap);
        if (hipMalloc(&d_ws, ws_cap) != hipSuccess) {
            ws_cap = 0;
            return KMWS_ERR_FAILED;
        }
    }
    if (hipMemcpyAsync(d_desc, h_desc, nd * sizeof(kmws_desc), hipMemcpyHostToDevice, stream) != hipSuccess)
        return KMWS_ERR_FAILED;
    kmws_status st = kmws_unmask_batch(dview, span, d_desc, (uint32_t)nd, d_ws, ws_cap, stream);
    if (st != KMWS_OK) return st;
    uint32_t status = 0;
    if (hipMemcpyAsync(&status, d_ws, sizeof(status), hipMemcpyDeviceToHost, stream) != hipSuccess)
        return KMWS_ERR_FAILED;
    if (hipStreamSynchronize(stream) != hipSuccess) return KMWS_ERR_FAILED;
    return status == 0 ? KMWS_OK : KMWS_ERR_INVALID_STATE;
}

// ---------------------------------------------------------------------------
// Host-resident batches: chunked, multi-slot H2D -> unmask -> D2H pipeline
// (the receive path starts and ends in host memory, TcpConnection.cpp:229).
// Chunks are cut on frame boundaries; slot k's H2D overlaps slot k-1's
// kernel and slot k-2's D2H (separate streams; PCIe is full duplex).
struct kmws_pipeline {
    struct Slot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
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
        for (Slot& s : slots) {
            if (s.stream) (void)hipStreamSynchronize(s.stream);
            if (s.d_buf) (void)hipFree(s.d_buf);
            if (s.d_desc) (void)hipFree(s.d_desc);
            if (s.h_desc) (void)hipHostFree(s.h_desc);
            if (s.d_ws) (void)hipFree(s.d_ws);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.stream) (void)hipStreamDestroy(s.stream);
        }
    }
};

extern "C" {

kmws_pipeline* kmws_pipeline_create(int device, uint64_t chunk_bytes, uint32_t max_frames_per_chunk, int depth)
{
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
    for (auto& s : p->slots) {
        s.ws_bytes = kmws_unmask_workspace_size(dev_bytes);
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess ||
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
    if (dv) {
        // Pinned host memory: one zero-copy unmask over PCIe, in place.
        kmws_pipeline::Slot& s = p->slots[0];
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
        if (hipMemcpyAsync(p->zc_desc, descs, (size_t)n * sizeof(kmws_desc), hipMemcpyHostToDevice, s.stream) !=
            hipSuccess)
            return KMWS_ERR_FAILED;
        kmws_status st = kmws_unmask_batch(dv, span, p->zc_desc, n, p->zc_ws, p->zc_ws_cap, s.stream);
        if (st != KMWS_OK) return st;
        uint32_t status = 0;
        if (hipMemcpyAsync(&status, p->zc_ws, sizeof(status), hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
            hipStreamSynchronize(s.stream) != hipSuccess)
            return KMWS_ERR_FAILED;
        return status == 0 ? KMWS_OK : KMWS_ERR_INVALID_PARAM;
    }
    uint32_t f = 0;
    size_t k = 0;
    kmws_status st = KMWS_OK;
    while (f < n && st == KMWS_OK) {
        // frames [f, e) whose 16-B aligned hull fits the chunk
        const uint64_t lo = descs[f].off & ~(uint64_t)15;
        if (descs[f].off + descs[f].len > span) return KMWS_ERR_INVALID_PARAM;
        uint32_t e = f;
        uint64_t hi = descs[f].off;
        while (e < n && e - f < p->max_frames) {
            const uint64_t end = descs[e].off + descs[e].len;
            if (descs[e].off < hi || end > span) return KMWS_ERR_INVALID_PARAM;  // sorted, in range
            if (end - lo > p->chunk) break;
            hi = end;
            ++e;
        }
        if (e == f) return KMWS_ERR_BUFFER_TOO_SMALL;  // one frame larger than a chunk
        kmws_pipeline::Slot& s = p->slots[k % p->slots.size()];
        if (s.busy && hipEventSynchronize(s.done) != hipSuccess) return KMWS_ERR_FAILED;
        s.busy = false;
        const uint64_t first = descs[f].off;
        for (uint32_t i = f; i < e; ++i) {
            s.h_desc[i - f] = descs[i];
            s.h_desc[i - f].off -= lo;
        }
        const uint64_t bytes = (hi + 15 - lo) & ~(uint64_t)15;
        const uint64_t h2d = hi - lo;  // never read past the caller's span
        if (hipMemcpyAsync(s.d_buf, host_base + lo, h2d, hipMemcpyHostToDevice, s.stream) != hipSuccess ||
            hipMemcpyAsync(s.d_desc, s.h_desc, (size_t)(e - f) * sizeof(kmws_desc), hipMemcpyHostToDevice,
                           s.stream) != hipSuccess)
            return KMWS_ERR_FAILED;
        st = kmws_unmask_batch(s.d_buf, bytes, s.d_desc, e - f, s.d_ws, s.ws_bytes, s.stream);
        if (st != KMWS_OK) break;
        // write back exactly the frames' extent: neighbours' bytes stay untouched
        if (hipMemcpyAsync(host_base + first, s.d_buf + (first - lo), hi - first, hipMemcpyDeviceToHost,
                           s.stream) != hipSuccess ||
            hipEventRecord(s.done, s.stream) != hipSuccess)
            return KMWS_ERR_FAILED;
        s.busy = true;
        f = e;
        ++k;
    }
    for (auto& s : p->slots) {
        if (s.busy && hipEventSynchronize(s.done) != hipSuccess) st = KMWS_ERR_FAILED;
        s.busy = false;
    }
    return st;
}

int kmws_header_size(uint32_t length, int mask)
{
    const int n = length <= 125 ? 2 : (length <= 0xFFFF ? 4 : 10);
    return n + (mask ? KMWS_MASK_KEY_SIZE : 0);
}

// WSHandler::encodeFrameHeader, WSHandler.cpp:46-106.
int kmws_encode_header(const kmws_frame_hdr* h, uint8_t out[KMWS_MAX_HEADER_SIZE])
{
    if (!h || !out) return KMWS_ERR_INVALID_PARAM;
    const uint32_t L = h->length;
    out[0] = (uint8_t)((h->fin ? 0x80 : 0) | (h->rsv1 ? 0x40 : 0) | (h->rsv2 ? 0x20 : 0) | (h->rsv3 ? 0x10 : 0) |
                       (h->opcode & 0x0F));
    const uint8_t m = h->mask ? 0x80 : 0;
    int n;
    if (L <= 125) {
        out[1] = (uint8_t)(m | L);
        n = 2;
    } else if (L <= 0xFFFF) {
        out[1] = m | 126;
        out[2] = (uint8_t)(L >> 8);
        out[3] = (uint8_t)L;
        n = 4;
    } else {
        // 8-byte length: the reference writes 4 zero bytes then the 32-bit
        // length (hdr.length is a uint32), big-endian.
        out[1] = m | 127;
        const uint64_t L64 = L;
        for (int i = 0; i < 8; ++i) out[2 + i] = (uint8_t)(L64 >> (56 - 8 * i));
        n = 10;
    }
    if (h->mask) {
        std::memcpy(out + n, h->maskey, KMWS_MASK_KEY_SIZE);
        n += KMWS_MASK_KEY_SIZE;
    }
    return n;
}

// Header chain walk (boundary discovery) over complete frames.  Lengths use
// the reference's semantics (127-class quirk, 10 MiB cap) so the chain is the
// one WSHandler would follow.
kmws_status kmws_find_headers(const uint8_t* wire, uint64_t len, uint64_t* hdr_off, uint32_t cap,
                              uint32_t* n_out, uint64_t* consumed)
{
    if (!n_out || (len && !wire) || (cap && !hdr_off)) return KMWS_ERR_INVALID_PARAM;
    uint64_t p = 0, done = 0;
    uint32_t n = 0;
    while (p < len && n < cap) {
        hdr_off[n++] = p;
        if (p + 2 > len) break;
        const uint8_t b0 = wire[p], b1 = wire[p + 1];
        const uint32_t plen = b1 & 0x7F, mask = b1 >> 7;
        const uint64_t ext = plen == 126 ? 2 : (plen == 127 ? 8 : 0);
        if (p + 2 + ext > len) break;
        uint64_t L;
        if (plen == 126) {
            L = ((uint32_t)wire[p + 2] << 8) | wire[p + 3];
        } else if (plen == 127) {
            uint64_t x = 0;
            for (uint32_t k = 0; k < 8; ++k)
                x |= (uint64_t)(int64_t)(int32_t)((uint32_t)wire[p + 2 + k] << (((7u - k) * 8u) & 31u));
            if ((x >> 63) != 0 || (uint32_t)x > KMWS_MAX_FRAME_DATA_LENGTH) break;
            L = (uint32_t)x;
        } else {
            L = plen;
        }
        const uint64_t end = p + 2 + ext + (mask ? 4 : 0) + L;
        if (end > len) break;
        p = done = end;
        if ((b0 & 0x0F) == KMWS_OP_CLOSE) break;
    }
    *n_out = n;
    if (consumed) *consumed = done;
    return KMWS_OK;
}

kmws_decoder* kmws_decoder_create(int mode, int device)
{
    kmws_decoder* d = new (std::nothrow) kmws_decoder();
    if (d) {
        d->mode = mode;
        d->device = device;
    }
    return d;
}

void kmws_decoder_destroy(kmws_decoder* dec) { delete dec; }
void kmws_decoder_set_mode(kmws_decoder* dec, int mode)
{
    if (dec) dec->mode = mode;
}
void kmws_decoder_reset(kmws_decoder* dec)
{
    if (dec) dec->reset_ctx();
}

// WSHandler::handleData -> decodeFrame (WSHandler.cpp:41-44, 108-280), in three
// phases: (1) parse the chunk with the reference's state machine, staging the
// payload of every completed masked frame; (2) one GPU unmask batch over the
// staged payloads; (3) deliver the frames in order (masked frames that lay in
// the caller's chunk are first written back there, unmasked in place, as the
// reference does), stopping at a callback that destroyed the decoder.
int kmws_decoder_feed(kmws_decoder* dec, uint8_t* data, size_t len, kmws_frame_cb cb, void* user)
{
    if (!dec) return KMWS_ERR_INVALID_PARAM;
    dec->pending.clear();
    dec->held.clear();
    dec->stage_len = 0;
    int result = -100;  // set by the parse loop
    size_t p = 0;
    auto& h = dec->hdr;

    // ---- phase 1: parse ----
    while (result == -100 && p < len) {
        switch (dec->state) {
        case St::HDR1: {  // :118-135
            const uint8_t b = data[p++];
            h.fin = b >> 7;
            h.opcode = b & 0x0F;
            h.rsv1 = (b >> 6) & 1;
            h.rsv2 = (b >> 5) & 1;
            h.rsv3 = (b >> 4) & 1;
            if (!h.fin && is_control(h.opcode)) {
                dec->state = St::IN_ERROR;
                result = KMWS_WS_PROTOCOL_ERROR;
                break;
            }
            dec->state = St::HDR2;
        }
            [[fallthrough]];
        case St::HDR2: {  // :136-156
            if (p >= len) {
                result = KMWS_WS_NEED_MORE_DATA;
                break;
            }
            const uint8_t b = data[p++];
            h.mask = b >> 7;
            h.plen = b & 0x7F;
            h.xpl64 = 0;
            dec->pos = 0;
            dec->buf.clear();
            if (is_control(h.opcode) && h.plen > 125) {
                dec->state = St::IN_ERROR;
                result = KMWS_WS_PROTOCOL_ERROR;
                break;
            }
            dec->state = St::HDREX;
        }
            [[fallthrough]];
        case St::HDREX: {  // :157-204
            if (h.plen == 126) {
                for (; p < len && dec->pos < 2; ++p, ++dec->pos)
                    h.xpl64 = (h.xpl64 & ~0xFFFFull) |
                              (uint16_t)((uint16_t)h.xpl64 | (uint16_t)(data[p] << ((1 - dec->pos) * 8)));
                if (dec->pos < 2) {
                    result = KMWS_WS_NEED_MORE_DATA;
                    break;
                }
                dec->pos = 0;
                if ((uint16_t)h.xpl64 < 126) {
                    dec->state = St::IN_ERROR;
                    result = KMWS_WS_INVALID_LENGTH;
                    break;
                }
                h.length = (uint16_t)h.xpl64;
            } else if (h.plen == 127) {
                // Reference quirk (WSHandler.cpp:179): a promoted 32-bit int
                // shifted by (7-k)*8; x86-64 takes the count mod 32 and the
                // int result is sign-extended into the u64.
                for (; p < len && dec->pos < 8; ++p, ++dec->pos) {
                    const uint32_t sh = ((7u - dec->pos) * 8u) & 31u;
                    h.xpl64 |= (uint64_t)(int64_t)(int32_t)((uint32_t)data[p] << sh);
                }
                if (dec->pos < 8) {
                    result = KMWS_WS_NEED_MORE_DATA;
                    break;
                }
                dec->pos = 0;
                if ((h.xpl64 >> 63) != 0) {
                    dec->state = St::IN_ERROR;
                    result = KMWS_WS_INVALID_LENGTH;
                    break;
                }
                h.length = (uint32_t)h.xpl64;
                if (h.length > KMWS_MAX_FRAME_DATA_LENGTH) {
                    dec->state = St::IN_ERROR;
                    result = KMWS_WS_INVALID_LENGTH;
                    break;
                }
            } else {
                h.length = h.plen;
            }
            dec->state = St::MASKEY;
        }
            [[fallthrough]];
        case St::MASKEY: {  // :205-234
            if (h.mask) {
                if (dec->mode == KMWS_MODE_CLIENT) {
                    dec->state = St::IN_ERROR;
                    result = KMWS_WS_PROTOCOL_ERROR;
                    break;
                }
                size_t c = 4u - dec->pos;
                if (c > len - p) c = len - p;
                std::memcpy(h.maskey + dec->pos, data + p, c);
                p += c;
                dec->pos = (uint8_t)(dec->pos + c);
                if (dec->pos < 4) {
                    result = KMWS_WS_NEED_MORE_DATA;
                    break;
                }
                dec->pos = 0;
            } else if (dec->mode == KMWS_MODE_SERVER && h.length > 0) {
                dec->state = St::IN_ERROR;
                result = KMWS_WS_PROTOCOL_ERROR;
                break;
            }
            dec->buf.clear();
            dec->state = St::DATA;
        }
            [[fallthrough]];
        case St::DATA: {  // :235-272
            if (len - p + dec->buf.size() < h.length) {
                dec->buf.insert(dec->buf.end(), data + p, data + len);
                p = len;
                result = KMWS_WS_NEED_MORE_DATA;
                break;
            }
            Pending q{};
            q.hdr = h;
            const bool masked = h.mask && h.length;  // handleDataMask no-op otherwise (:293, :305)
            if (masked) {
                kmws_status st = dec->stage_reserve(dec->stage_len + 16 + h.length, dec->pending.size() + 1);
                if (st != KMWS_OK) return st;
            }
            if (dec->buf.empty()) {  // whole payload in this chunk (:247-250)
                q.data_ptr = data + p;
                if (masked) {
                    q.stage_off = dec->stage_append(data + p, h.length);
                    q.where = kInChunkMasked;
                } else {
                    q.where = kInChunk;
                }
                p += h.length;
            } else {  // reassembled in ctx_.buf (:251-258)
                const size_t read_len = h.length - dec->buf.size();
                dec->buf.insert(dec->buf.end(), data + p, data + p + read_len);
                p += read_len;
                if (masked) {
                    q.stage_off = dec->stage_append(dec->buf.data(), h.length);
                    q.where = kStagedMasked;
                } else {
                    dec->held.emplace_back();
                    dec->held.back().swap(dec->buf);
                    q.hold_idx = dec->held.size() - 1;
                    q.where = kHeld;
                }
            }
            dec->pending.push_back(q);
            if (h.opcode == KMWS_OP_CLOSE) {  // :265-268
                dec->state = St::CLOSED;
                result = KMWS_WS_CLOSED;
                break;
            }
            dec->reset_ctx();  // :270
            break;
        }
        default:
            result = KMWS_WS_INVALID_FRAME;  // :273-276
            break;
        }
    }
    if (result == -100) result = dec->state == St::HDR1 ? KMWS_WS_NOERR : KMWS_WS_NEED_MORE_DATA;  // :279

    // ---- phase 2: GPU unmask of every staged masked payload ----
    kmws_status st = dec->unmask_staged();
    if (st != KMWS_OK) return st;

    // ---- phase 3: in-order delivery ----
    std::vector<Pending> todo;
    todo.swap(dec->pending);
    std::vector<std::vector<uint8_t>> held;
    held.swap(dec->held);
    uint8_t* stage = dec->h_stage;
    for (Pending& q : todo) {
        uint8_t* payload;
        switch (q.where) {
        case kInChunkMasked:  // unmasked in place in the caller's buffer, as kuma does (:260)
            std::memcpy(q.data_ptr, stage + q.stage_off, q.hdr.length);
            payload = q.data_ptr;
            break;
        case kStagedMasked: payload = stage + q.stage_off; break;
        case kHeld: payload = held[q.hold_idx].data(); break;
        default: payload = q.data_ptr; break;
        }
        // WSHandler::handleFrame (:282-289): a callback that destroyed its
        // owner ends the call; the decoder must not be touched afterwards.
        if (cb && cb(&q.hdr, payload, q.hdr.length, user)) return KMWS_WS_DESTROYED;
    }
    return result;
}

}  // extern "C"
