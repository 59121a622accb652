// WSHandler-compatible streaming decoder of the kmws C ABI
// (src/ws/WSHandler.{h,cpp} in the reference).
//
// The per-byte header state machine stays on the event-loop thread, as in kuma
// (headers arrive byte-serially per connection, WSHandler.cpp:108-280).  The
// payload work -- the reference's scalar unmask loop (WSHandler.cpp:303-310) --
// runs on the GPU, batched:
//   kmws_decoder_feed           one GPU batch per call, callbacks before return
//                               (the drop-in for WSHandler::handleData);
//   kmws_decoder_feed_deferred  frames of many calls / connections staged into
//   + kmws_rx_batch_flush       a kmws_rx_batch; one GPU batch per flush (once
//                               per event-loop iteration), callbacks at flush.
// There is no CPU unmask path: without a usable gfx950 device a masked frame
// fails the call with KMWS_ERR_NOT_SUPPORTED.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "kmws_gpu.h"
#include "kmws_host_util.hpp"

using namespace kmws;

namespace {

enum class St : uint8_t { HDR1, HDR2, HDREX, MASKEY, DATA, CLOSED, IN_ERROR };  // WSHandler.h:57-65

bool is_control(uint8_t op) { return op >= 8; }  // WSHandler.h:52-54

constexpr int kParsing = -100;

// Where a completed frame's payload lives until delivery (synchronous feed).
enum Origin : int {
    kInChunk = 0,        // unmasked (or empty): view into the caller's chunk
    kInChunkPinned = 1,  // masked, caller's chunk is pinned: unmasked there in place by the kernel
    kInChunkStaged = 2,  // masked, pageable chunk: staged, written back in place before delivery
    kStagedMasked = 3,   // masked, reassembled across chunks: view into staging
    kHeld = 4,           // unmasked, reassembled: view into a held reassembly buffer
};

struct Pending {
    kmws_frame_hdr hdr;
    uint8_t* data_ptr;  // in-chunk kinds: payload position in the chunk
    size_t stage_off;   // staged kinds: payload offset in the staging area
    size_t hold_idx;    // kHeld: index into the held buffers
    Origin where;
};

}  // namespace

struct kmws_decoder {
    int mode = KMWS_MODE_CLIENT;
    int device = 0;
    bool in_place = true;  // kmws_decoder_set_in_place
    // The last chunk base found pageable: kuma reads into the same buffer every
    // time (TcpConnection.cpp:229), and hipPointerGetAttributes per feed costs
    // more than a small read's unmask.  Only that verdict is remembered: memory
    // pinned since then is still staged (correct, slower), never the reverse.
    const uint8_t* last_pageable = nullptr;
    // DecodeContext (WSHandler.h:66-78)
    kmws_frame_hdr hdr{};
    St state = St::HDR1;
    std::vector<uint8_t> buf;
    uint8_t pos = 0;
    // synchronous-feed delivery lists (the staging is borrowed per call: StagePool)
    std::vector<Pending> pending;
    std::vector<std::vector<uint8_t>> held;
    std::vector<kmws_desc> chunk_descs;

    void reset_ctx()  // DecodeContext::reset, WSHandler.h:66-72 (capacity kept)
    {
        std::memset(&hdr, 0, sizeof(hdr));
        state = St::HDR1;
        buf.clear();
        pos = 0;
    }
};

// Stages a batch makes before its first loop iteration (a generation in
// flight each; more are made if needed).
constexpr int kWarmStages = 4;

struct kmws_rx_batch {
    BatchStream bstream;  // first: destroyed after every stage that uses it
    struct Item {
        kmws_decoder* dec;  // identity only; never dereferenced at delivery
        kmws_frame_cb cb;
        void* user;
        kmws_frame_hdr hdr;
        size_t off;       // payload offset in the generation's staging area (direct == nullptr)
        uint8_t* direct;  // payload in the attached ring (no copy)
        bool live;        // false once discarded
    };
    // One submitted generation: its frames, and the pinned stage that holds
    // their staged payloads and the unmask launch in flight.
    struct Gen {
        std::unique_ptr<PinnedStage> stage;
        std::vector<Item> items;
    };
    std::unique_ptr<PinnedStage> stage;  // the generation being fed
    std::vector<Item> items;
    uint64_t pending_bytes = 0;  // masked payload bytes of `items`
    std::vector<kmws_desc> ring_descs;
    std::deque<Gen> inflight;            // submitted, not yet delivered (submit order)
    std::vector<std::unique_ptr<PinnedStage>> spare;
    std::vector<Item>* delivering = nullptr;  // the generation whose callbacks are running
    uint8_t* ring = nullptr;  // caller's pinned receive ring (optional)
    uint8_t* ring_dv = nullptr;  // its device view, looked up once at attach
    size_t ring_bytes = 0;
    int device = 0;
    bool flushing = false;  // feeding / submitting / polling from inside a delivery is refused

    std::unique_ptr<PinnedStage> take_stage()
    {
        if (!spare.empty()) {
            std::unique_ptr<PinnedStage> s = std::move(spare.back());
            spare.pop_back();
            return s;
        }
        std::unique_ptr<PinnedStage> s(new (std::nothrow) PinnedStage());
        if (s && s->init(device, bstream.s) != KMWS_OK) s.reset();
        return s;
    }
    // the stream and a few warm stages, made before the first loop iteration
    kmws_status prepare(int dev)
    {
        device = dev;
        kmws_status st = bstream.create(dev);
        for (int i = 0; st == KMWS_OK && i < kWarmStages; ++i) {
            std::unique_ptr<PinnedStage> s = take_stage();
            if (!s) return KMWS_ERR_FAILED;
            st = s->warm();
            spare.push_back(std::move(s));
        }
        return st;
    }
};

namespace {

// Pinned stages for the synchronous entries (kmws_decoder_feed,
// kmws_mask_host_chain), shared by every connection and thread of the process.
// A stage is used only within one call -- its payloads are unmasked and
// delivered before the call returns -- so a call borrows one and gives it back;
// a callback that feeds another decoder borrows another.  The pool holds as
// many stages as calls ever ran at once, each with its stream, event and
// pinned area made once: a decoder per connection (kuma's WSHandler) would
// otherwise create a stream (milliseconds) and 1 MiB of pinned memory per
// connection, and a new loop thread its own.  Never freed (pinned memory must
// not be released after the HIP runtime's teardown at process exit).  Each
// thread keeps the stage it gave back last in front of the pool, so its calls
// take no lock (16 threads masking at once contended on the pool's mutex); a
// nested call, or a call for another device, goes to the pool, and a thread's
// kept stage returns to it when the thread exits.
class StagePool;
StagePool& stage_pool();

// The calling thread's kept stage.  Plain data (zero-initialised, trivially
// destructible), so a call from another thread_local object's destructor after
// the thread's exit hook ran still finds it valid: such a call gives its stage
// to the pool instead of keeping it (which would leak it with the thread).
struct HotStage {
    PinnedStage* s;
    bool gone;  // the thread's exit hook ran
};
thread_local HotStage t_hot;
struct HotStageExit {  // returns the kept stage to the pool at thread exit
    bool armed = false;
    ~HotStageExit();
};
thread_local HotStageExit t_hot_exit;

class StagePool {
public:
    PinnedStage* take(int device, kmws_status* st)
    {
        *st = KMWS_OK;
        if (t_hot.s && t_hot.s->device() == device) {
            PinnedStage* s = t_hot.s;
            t_hot.s = nullptr;
            return s;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (size_t i = free_.size(); i-- > 0;)  // the most recently used first (warm in cache)
                if (free_[i]->device() == device) {
                    PinnedStage* s = free_[i];
                    free_.erase(free_.begin() + (ptrdiff_t)i);
                    return s;
                }
        }
        PinnedStage* s = new (std::nothrow) PinnedStage();
        if (!s) {
            *st = KMWS_ERR_FAILED;
            return nullptr;
        }
        *st = s->init(device);  // KMWS_ERR_NOT_SUPPORTED: no such gfx950 device
        if (*st == KMWS_OK) *st = s->warm();
        if (*st != KMWS_OK) {
            delete s;
            s = nullptr;
        }
        return s;
    }
    void give(PinnedStage* s, bool keep = true)
    {
        s->clear();
        if (keep && !t_hot.s && !t_hot.gone) {
            t_hot_exit.armed = true;  // constructed before the stage is kept: it gives it back
            t_hot.s = s;
            return;
        }
        std::lock_guard<std::mutex> lk(mu_);
        free_.push_back(s);
    }

private:
    std::mutex mu_;
    std::vector<PinnedStage*> free_;
};

StagePool& stage_pool()
{
    static StagePool* p = new StagePool();
    return *p;
}

HotStageExit::~HotStageExit()
{
    t_hot.gone = true;
    if (PinnedStage* s = t_hot.s) {
        t_hot.s = nullptr;
        stage_pool().give(s, false);
    }
}

// A stage borrowed for the scope of one call (taken at first use).
struct BorrowedStage {
    int device;
    PinnedStage* s = nullptr;
    kmws_status st = KMWS_OK;  // why get() failed
    explicit BorrowedStage(int dev) : device(dev) {}
    ~BorrowedStage()
    {
        if (s) stage_pool().give(s);
    }
    PinnedStage* get()
    {
        if (!s) s = stage_pool().take(device, &st);
        return s;
    }
};

// The reference's decodeFrame loop (WSHandler.cpp:108-280).  At every
// completed frame, sink(hdr, payload, reassembly) is called with the payload
// contiguous in memory: in the caller's chunk (reassembly == nullptr) or in
// the decoder's reassembly buffer (the sink may steal it).  Returns the
// WSError of the call, or a negative status the sink returned.
template <class Sink>
int parse_chunk(kmws_decoder* dec, uint8_t* data, size_t len, Sink&& sink)
{
    int result = kParsing;
    size_t p = 0;
    auto& h = dec->hdr;
    while (result == kParsing && p < len) {
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
            int st;
            if (dec->buf.empty()) {  // whole payload in this chunk (:247-250)
                st = sink(h, data + p, (std::vector<uint8_t>*)nullptr);
                p += h.length;
            } else {  // reassembled in ctx_.buf (:251-258)
                const size_t read_len = h.length - dec->buf.size();
                dec->buf.insert(dec->buf.end(), data + p, data + p + read_len);
                p += read_len;
                st = sink(h, dec->buf.data(), &dec->buf);
            }
            if (st != KMWS_OK) return st;
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
    if (result == kParsing) result = dec->state == St::HDR1 ? KMWS_WS_NOERR : KMWS_WS_NEED_MORE_DATA;  // :279
    return result;
}

}  // namespace

extern "C" {

kmws_decoder* kmws_decoder_create(int mode, int device)
{
    kmws_decoder* d = new (std::nothrow) kmws_decoder();
    if (d) {
        d->mode = mode;
        d->device = resolve_device(device);  // KMWS_DEVICE_AUTO: the creating (loop) thread's GPU
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

void kmws_decoder_set_in_place(kmws_decoder* dec, int on)
{
    if (dec) dec->in_place = on != 0;
}

// WSHandler::handleData (WSHandler.cpp:41-44, decodeFrame :108-280) in three
// phases: (1) parse the chunk, collecting completed frames; (2) one GPU unmask
// batch over their masked payloads -- in place in the caller's chunk when it
// is pinned memory, else on a pinned staging copy; (3) deliver in order
// (staged frames that lay in the chunk are first written back there, as the
// reference unmasks them in place), stopping at a callback that destroyed
// the decoder.
int kmws_decoder_feed(kmws_decoder* dec, uint8_t* data, size_t len, kmws_frame_cb cb, void* user)
{
    if (!dec || (len && !data)) return KMWS_ERR_INVALID_PARAM;
    dec->pending.clear();
    dec->held.clear();
    dec->chunk_descs.clear();
    BorrowedStage bs(dec->device);  // given back when the call returns (the decoder may be gone by then)
    int chunk_pinned = -1;  // resolved at the first masked in-chunk frame
    uint8_t* chunk_dv = nullptr;
    uint8_t* chunk_base = reinterpret_cast<uint8_t*>(reinterpret_cast<uintptr_t>(data) & ~(uintptr_t)15);

    auto sink = [&](const kmws_frame_hdr& h, uint8_t* payload, std::vector<uint8_t>* reasm) -> int {
        Pending q{};
        q.hdr = h;
        const bool masked = h.mask && h.length;  // handleDataMask is a no-op otherwise (:293, :305)
        uint32_t key;
        std::memcpy(&key, h.maskey, 4);
        if (masked && !bs.get()) return bs.st;
        if (!reasm) {
            q.data_ptr = payload;
            if (!masked) {
                q.where = kInChunk;
            } else {
                if (chunk_pinned < 0) {
                    chunk_dv = chunk_base == dec->last_pageable ? nullptr
                                                                : static_cast<uint8_t*>(device_view(chunk_base));
                    chunk_pinned = chunk_dv != nullptr;
                    if (!chunk_pinned) dec->last_pageable = chunk_base;
                }
                if (chunk_pinned) {
                    dec->chunk_descs.push_back(kmws_desc{(uint64_t)(payload - chunk_base), h.length, key});
                    q.where = kInChunkPinned;
                } else {
                    kmws_status st = bs.s->reserve(h.length);
                    if (st != KMWS_OK) return st;
                    q.stage_off = bs.s->append(payload, h.length);
                    bs.s->add_desc(q.stage_off, h.length, key);
                    q.where = kInChunkStaged;
                }
            }
        } else if (masked) {
            kmws_status st = bs.s->reserve(h.length);
            if (st != KMWS_OK) return st;
            q.stage_off = bs.s->append(payload, h.length);
            bs.s->add_desc(q.stage_off, h.length, key);
            q.where = kStagedMasked;
        } else {
            dec->held.emplace_back();
            dec->held.back().swap(*reasm);
            q.hold_idx = dec->held.size() - 1;
            q.where = kHeld;
        }
        dec->pending.push_back(q);
        return KMWS_OK;
    };

    const int result = parse_chunk(dec, data, len, sink);
    if (result < 0) return result;

    // ---- GPU unmask of every masked payload of this call ----
    if (bs.s && (bs.s->n_desc() || !dec->chunk_descs.empty())) {
        const uint64_t chunk_span = (uint64_t)((data + len) - chunk_base);
        kmws_status st = bs.s->run(chunk_base, chunk_span, &dec->chunk_descs, chunk_dv);
        if (st != KMWS_OK) return st;
    }

    // ---- in-order delivery ----
    const bool in_place = dec->in_place;  // the callbacks may destroy the decoder
    std::vector<Pending> todo;
    todo.swap(dec->pending);
    std::vector<std::vector<uint8_t>> held;
    held.swap(dec->held);
    uint8_t* stage = bs.s ? bs.s->data() : nullptr;
    for (Pending& q : todo) {
        uint8_t* payload;
        switch (q.where) {
        case kInChunkStaged:  // unmasked in place in the caller's buffer, as kuma does (:260)
            if (!in_place) {     // or the view points at the unmasked staging copy
                payload = stage + q.stage_off;
                break;
            }
            std::memcpy(q.data_ptr, stage + q.stage_off, q.hdr.length);
            payload = q.data_ptr;
            break;
        case kStagedMasked: payload = stage + q.stage_off; break;
        case kHeld: payload = held[q.hold_idx].data(); break;
        default: payload = q.data_ptr; break;  // kInChunk, kInChunkPinned
        }
        // WSHandler::handleFrame (:282-289): a callback that destroyed its
        // owner ends the call; the decoder must not be touched afterwards.
        if (cb && cb(&q.hdr, payload, q.hdr.length, user)) return KMWS_WS_DESTROYED;
    }
    return result;
}

// ---- host-buffer masking: WSHandler::handleDataMask statics (a-1, a-2) ----

// Masks a chain of host segments in place with the key phase continuing across
// segments (WSHandler.cpp:312-322; one segment = :303-310).  The segments are
// gathered back to back into pinned staging -- so the chain is one payload and
// one descriptor -- unmasked by the GPU in place there, and scattered back.
kmws_status kmws_mask_host_chain(const uint8_t key[KMWS_MASK_KEY_SIZE], uint8_t* const* segs, const size_t* lens,
                                 size_t nseg, int device)
{
    if (!key || (nseg && (!segs || !lens))) return KMWS_ERR_INVALID_PARAM;
    size_t total = 0;
    for (size_t i = 0; i < nseg; ++i) {
        if (lens[i] && !segs[i]) return KMWS_ERR_INVALID_PARAM;
        total += lens[i];
    }
    if (total == 0) return KMWS_OK;  // nothing to do (:305)
    if (total > 0xFFFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    if (device == KMWS_DEVICE_AUTO) {
        device = kmws_thread_device();
        if (device < 0) return device;
    }
    if (device < 0) return KMWS_ERR_INVALID_PARAM;
    BorrowedStage bs(device);  // a stage of the process's pool for this call (StagePool)
    PinnedStage* s = bs.get();
    if (!s) return bs.st;
    kmws_status st = s->reserve(total);
    if (st != KMWS_OK) return st;
    size_t off = 0;
    uint8_t* dst = s->alloc(total, &off);
    size_t pos = 0;
    for (size_t i = 0; i < nseg; ++i) {
        if (lens[i]) std::memcpy(dst + pos, segs[i], lens[i]);
        pos += lens[i];
    }
    uint32_t k;
    std::memcpy(&k, key, 4);
    s->add_desc(off, (uint32_t)total, k);
    st = s->run();
    if (st != KMWS_OK) return st;
    pos = 0;
    for (size_t i = 0; i < nseg; ++i) {
        if (lens[i]) std::memcpy(segs[i], dst + pos, lens[i]);
        pos += lens[i];
    }
    return KMWS_OK;
}

// ---- pinned host rings ----

void* kmws_host_alloc(size_t bytes, int device)
{
    device = resolve_device(device);
    if (bytes == 0 || device < 0 || kmws_device_count() <= device) return nullptr;
    DevGuard g(device);
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void kmws_host_free(void* p)
{
    if (p) (void)hipHostFree(p);
}

// ---- batched send path (SURVEY f-2) ----
//
// Sends queued with kmws_tx_batch_add form the current generation;
// kmws_tx_batch_submit enqueues ONE mask launch for it and returns a ticket;
// kmws_tx_batch_poll(ticket) completes generations up to the ticket (staged
// segments are copied back into the caller's buffers) -- the loop writes a
// generation's iovecs once its ticket completed, and can fill and submit the
// next generation meanwhile.  kmws_tx_batch_flush = submit + poll(wait).

struct kmws_tx_batch {
    BatchStream bstream;  // first: destroyed after every stage that uses it
    struct Seg {
        uint8_t* p;
        size_t len;
    };
    struct Frame {
        size_t seg0, nseg;  // range in segs
        size_t bytes;
        uint32_t key;
    };
    struct Gen {  // submitted: the stage with the launch in flight, segments to copy back
        std::unique_ptr<PinnedStage> stage;
        std::vector<Seg> segs;
        std::vector<size_t> offs;  // staging offset per segment (SIZE_MAX: masked in the ring)
        int64_t ticket;
    };
    std::unique_ptr<PinnedStage> stage;
    std::vector<Seg> segs;
    std::vector<Frame> frames;
    size_t bytes = 0;
    int device = 0;
    uint8_t* ring = nullptr;  // caller's pinned send ring (optional)
    uint8_t* ring_dv = nullptr;  // its device view, looked up once at attach
    size_t ring_bytes = 0;
    std::vector<kmws_desc> ring_descs;
    std::deque<Gen> inflight;
    std::vector<std::unique_ptr<PinnedStage>> spare;
    int64_t next_ticket = 1, done_ticket = 0;
    bool in_ring(const uint8_t* p, size_t n) const
    {
        return ring && p >= ring && n <= ring_bytes && (size_t)(p - ring) <= ring_bytes - n;
    }
    std::unique_ptr<PinnedStage> take_stage()
    {
        if (!spare.empty()) {
            std::unique_ptr<PinnedStage> s = std::move(spare.back());
            spare.pop_back();
            return s;
        }
        std::unique_ptr<PinnedStage> s(new (std::nothrow) PinnedStage());
        if (s && s->init(device, bstream.s) != KMWS_OK) s.reset();
        return s;
    }
    // the stream and a few warm stages, made before the first loop iteration
    kmws_status prepare(int dev)
    {
        device = dev;
        kmws_status st = bstream.create(dev);
        for (int i = 0; st == KMWS_OK && i < kWarmStages; ++i) {
            std::unique_ptr<PinnedStage> s = take_stage();
            if (!s) return KMWS_ERR_FAILED;
            st = s->warm();
            spare.push_back(std::move(s));
        }
        return st;
    }
};

kmws_tx_batch* kmws_tx_batch_create(int device)
{
    device = resolve_device(device);
    kmws_tx_batch* b = new (std::nothrow) kmws_tx_batch();
    if (!b) return nullptr;
    if (b->prepare(device) != KMWS_OK) {
        delete b;
        return nullptr;
    }
    b->stage = b->take_stage();
    if (!b->stage) {
        delete b;
        return nullptr;
    }
    return b;
}

void kmws_tx_batch_destroy(kmws_tx_batch* b)
{
    if (!b) return;
    for (auto& g : b->inflight) (void)g.stage->wait();  // no launch may outlive its pinned memory
    delete b;
}

int kmws_tx_batch_pending(const kmws_tx_batch* b) { return b ? (int)b->frames.size() : 0; }

// sendWsFrame (WebSocketImpl.cpp:405-436) up to the socket write: length =
// u32(chain length) (:415), header packed (:416), payload queued for masking
// when the header says so and it is not empty (:410-414); more than 128
// non-empty segments -> BUFFER_TOO_LONG after the mask, as kuma (:419-431).
int kmws_tx_batch_add(kmws_tx_batch* b, const kmws_frame_hdr* hdr, uint8_t* const* segs, const size_t* lens,
                      size_t nseg, uint8_t hdr_out[KMWS_MAX_HEADER_SIZE])
{
    if (!b || !hdr || !hdr_out || (nseg && (!segs || !lens))) return KMWS_ERR_INVALID_PARAM;
    size_t plen = 0, nonempty = 0;
    for (size_t i = 0; i < nseg; ++i) {
        if (lens[i] && !segs[i]) return KMWS_ERR_INVALID_PARAM;
        plen += lens[i];
        nonempty += lens[i] != 0;
    }
    if (plen > 0xFFFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    kmws_frame_hdr h = *hdr;
    h.length = (uint32_t)plen;
    const int hl = kmws_encode_header(&h, hdr_out);
    if (h.mask && plen > 0) {
        uint32_t key;
        std::memcpy(&key, h.maskey, 4);
        b->frames.push_back(kmws_tx_batch::Frame{b->segs.size(), 0, plen, key});
        for (size_t i = 0; i < nseg; ++i)
            if (lens[i]) b->segs.push_back(kmws_tx_batch::Seg{segs[i], lens[i]});
        b->frames.back().nseg = b->segs.size() - b->frames.back().seg0;
        b->bytes += plen;
    }
    return 1 + nonempty > 129 ? KMWS_ERR_BUFFER_TOO_LONG : hl;
}

// kmws_tx_batch_attach_ring: segments inside it are masked there (zero-copy).
kmws_status kmws_tx_batch_attach_ring(kmws_tx_batch* b, uint8_t* ring, size_t ring_bytes)
{
    if (!b || (ring && !ring_bytes)) return KMWS_ERR_INVALID_PARAM;
    // queued segments were classified already; a mask in flight may still be writing into the old ring
    if (!b->frames.empty() || !b->inflight.empty()) return KMWS_ERR_INVALID_STATE;
    uint8_t* dv = ring ? static_cast<uint8_t*>(device_view(ring)) : nullptr;
    if (ring && !dv) return KMWS_ERR_INVALID_PARAM;  // must be pinned
    b->ring = ring;
    b->ring_dv = dv;
    b->ring_bytes = ring ? ring_bytes : 0;
    return KMWS_OK;
}

// One descriptor per segment, its key rotated by the frame bytes before it
// (the phase continues across segments, WSHandler.cpp:312-322): segments in
// the attached pinned ring are masked in place there, the others gathered
// into pinned staging and copied back when the generation completes; one
// launch per buffer -- or, for a flush (sync), one synchronous job on the
// device's resident worker (kmws_resident.hip) when it fits one.
static int64_t tx_submit(kmws_tx_batch* b, bool sync)
{
    if (!b) return KMWS_ERR_INVALID_PARAM;
    if (b->frames.empty()) return 0;
    std::unique_ptr<PinnedStage> next = b->take_stage();
    if (!next) return KMWS_ERR_FAILED;
    PinnedStage& s = *b->stage;
    s.clear();
    b->ring_descs.clear();
    size_t staged = 0;
    for (const kmws_tx_batch::Seg& g : b->segs)
        if (!b->in_ring(g.p, g.len)) staged += g.len + 16;
    kmws_status st = s.reserve(staged);
    std::vector<size_t> offs(b->segs.size(), SIZE_MAX);
    if (st == KMWS_OK) {
        for (const kmws_tx_batch::Frame& fr : b->frames) {
            size_t phase = 0;
            for (size_t i = fr.seg0; i < fr.seg0 + fr.nseg; ++i) {
                const kmws_tx_batch::Seg& g = b->segs[i];
                const uint32_t key = __builtin_rotateright32(fr.key, 8u * (uint32_t)(phase & 3u));
                if (b->in_ring(g.p, g.len)) {
                    b->ring_descs.push_back(kmws_desc{(uint64_t)(g.p - b->ring), (uint32_t)g.len, key});
                } else {
                    uint8_t* dst = s.alloc(g.len, &offs[i]);
                    std::memcpy(dst, g.p, g.len);
                    s.add_desc(offs[i], (uint32_t)g.len, key);
                }
                phase += g.len;
            }
        }
        if (sync)
            st = b->ring_descs.empty() ? s.run() : s.run(b->ring, b->ring_bytes, &b->ring_descs, b->ring_dv);
        else
            st = b->ring_descs.empty() ? s.launch() : s.launch(b->ring, b->ring_bytes, &b->ring_descs, b->ring_dv);
    }
    b->frames.clear();
    b->ring_descs.clear();
    b->bytes = 0;
    if (st != KMWS_OK) {
        b->segs.clear();
        s.clear();
        b->spare.push_back(std::move(next));
        return st;
    }
    kmws_tx_batch::Gen g;
    g.stage = std::move(b->stage);
    g.segs.swap(b->segs);
    g.offs.swap(offs);
    g.ticket = b->next_ticket++;
    b->inflight.push_back(std::move(g));
    b->stage = std::move(next);
    return b->inflight.back().ticket;
}

int64_t kmws_tx_batch_submit(kmws_tx_batch* b) { return tx_submit(b, false); }

int kmws_tx_batch_poll(kmws_tx_batch* b, int64_t ticket, int wait)
{
    if (!b || ticket < 0) return KMWS_ERR_INVALID_PARAM;
    kmws_status err = KMWS_OK;
    while (!b->inflight.empty() && b->inflight.front().ticket <= ticket) {
        kmws_tx_batch::Gen& g = b->inflight.front();
        if (!wait && !g.stage->done()) break;
        const kmws_status st = g.stage->wait();
        if (st == KMWS_OK) {
            for (size_t i = 0; i < g.segs.size(); ++i)
                if (g.offs[i] != SIZE_MAX) std::memcpy(g.segs[i].p, g.stage->data() + g.offs[i], g.segs[i].len);
        } else {
            err = st;
        }
        b->done_ticket = g.ticket;
        g.stage->clear();
        b->spare.push_back(std::move(g.stage));
        b->inflight.pop_front();
    }
    if (err != KMWS_OK) return err;
    return ticket <= b->done_ticket || b->inflight.empty() || b->inflight.front().ticket > ticket ? 1 : 0;
}

int64_t kmws_tx_batch_flush(kmws_tx_batch* b)
{
    if (!b) return KMWS_ERR_INVALID_PARAM;
    const int64_t nf = (int64_t)b->frames.size();
    // what is in flight first: the thread's resident slot holds one job, and a
    // job posted while the previous one runs launches instead
    if (!b->inflight.empty()) {
        const int r0 = kmws_tx_batch_poll(b, b->next_ticket - 1, 1);
        if (r0 < 0) return r0;
    }
    const int64_t t = tx_submit(b, true);  // masked when it returns: the poll only copies back
    if (t < 0) return t;
    const int r = kmws_tx_batch_poll(b, b->next_ticket - 1, 1);
    if (r < 0) return r;
    return nf;
}

// ---- deferred delivery across calls and connections ----
//
// Frames fed with kmws_decoder_feed_deferred collect in the batch's current
// generation (payloads copied into its pinned stage, or left where they lie in
// the attached ring).  kmws_rx_batch_submit enqueues ONE unmask launch for the
// generation and returns at once; kmws_rx_batch_poll delivers the callbacks of
// every generation whose launch has finished, in submit order (wait != 0: all
// of them).  kmws_rx_batch_flush = submit + poll(wait).  So an event loop can
// submit at the end of an iteration and deliver at the next one: the GPU round
// trip overlaps the loop's socket reads instead of stalling them.

kmws_rx_batch* kmws_rx_batch_create(int device)
{
    device = resolve_device(device);
    kmws_rx_batch* b = new (std::nothrow) kmws_rx_batch();
    if (!b) return nullptr;
    if (b->prepare(device) != KMWS_OK) {
        delete b;
        return nullptr;
    }
    b->stage = b->take_stage();
    if (!b->stage) {
        delete b;
        return nullptr;
    }
    return b;
}

void kmws_rx_batch_destroy(kmws_rx_batch* b)
{
    if (!b) return;
    for (auto& g : b->inflight) (void)g.stage->wait();  // no launch may outlive its pinned memory
    delete b;
}

int kmws_decoder_feed_deferred(kmws_decoder* dec, kmws_rx_batch* b, const uint8_t* data, size_t len,
                               kmws_frame_cb cb, void* user)
{
    if (!dec || !b || (len && !data)) return KMWS_ERR_INVALID_PARAM;
    if (b->flushing) return KMWS_ERR_INVALID_STATE;
    // The chunk does not outlive this call (kuma reads into a stack buffer,
    // TcpConnection.cpp:229), so every payload is copied into the batch unless
    // it lies in the attached ring.  The parse does not write into the chunk.
    auto sink = [&](const kmws_frame_hdr& h, uint8_t* payload, std::vector<uint8_t>* reasm) -> int {
        uint32_t key;
        std::memcpy(&key, h.maskey, 4);
        const bool masked = h.mask && h.length;
        if (masked) b->pending_bytes += h.length;
        if (!reasm && b->ring && payload >= b->ring && payload + h.length <= b->ring + b->ring_bytes) {
            // payload lies in the caller's pinned ring: unmasked there, no copy
            if (masked) b->ring_descs.push_back(kmws_desc{(uint64_t)(payload - b->ring), h.length, key});
            b->items.push_back(kmws_rx_batch::Item{dec, cb, user, h, 0, payload, true});
            return KMWS_OK;
        }
        kmws_status st = b->stage->reserve(h.length);
        if (st != KMWS_OK) return st;
        const size_t off = b->stage->append(payload, h.length);
        if (masked) b->stage->add_desc(off, h.length, key);
        b->items.push_back(kmws_rx_batch::Item{dec, cb, user, h, off, nullptr, true});
        return KMWS_OK;
    };
    return parse_chunk(dec, const_cast<uint8_t*>(data), len, sink);
}

kmws_status kmws_rx_batch_attach_ring(kmws_rx_batch* b, uint8_t* ring, size_t bytes)
{
    if (!b || b->flushing || !b->items.empty() || !b->inflight.empty()) return KMWS_ERR_INVALID_STATE;
    uint8_t* dv = ring && bytes ? static_cast<uint8_t*>(device_view(ring)) : nullptr;
    if (ring && !dv) return KMWS_ERR_INVALID_PARAM;  // must be pinned
    b->ring = ring;
    b->ring_dv = dv;
    b->ring_bytes = ring ? bytes : 0;
    return KMWS_OK;
}

int kmws_rx_batch_pending(const kmws_rx_batch* b) { return b ? (int)b->items.size() : 0; }

uint64_t kmws_rx_batch_pending_bytes(const kmws_rx_batch* b) { return b ? b->pending_bytes : 0; }

int kmws_rx_batch_inflight(const kmws_rx_batch* b) { return b ? (int)b->inflight.size() : 0; }

void kmws_rx_batch_discard(kmws_rx_batch* b, const kmws_decoder* dec)
{
    if (!b) return;
    for (auto& it : b->items)
        if (it.dec == dec) it.live = false;
    for (auto& g : b->inflight)
        for (auto& it : g.items)
            if (it.dec == dec) it.live = false;
    if (b->delivering)
        for (auto& it : *b->delivering)
            if (it.dec == dec) it.live = false;
}

// sync (a flush): one synchronous job on the device's resident worker when it
// fits one (else a launch and a wait), instead of an enqueued launch.
static int rx_submit(kmws_rx_batch* b, bool sync)
{
    if (!b) return KMWS_ERR_INVALID_PARAM;
    if (b->flushing) return KMWS_ERR_INVALID_STATE;
    if (b->items.empty()) return 0;
    std::unique_ptr<PinnedStage> next = b->take_stage();
    if (!next) return KMWS_ERR_FAILED;
    kmws_status st = sync ? b->stage->run(b->ring, b->ring_bytes, &b->ring_descs, b->ring_dv)
                          : b->stage->launch(b->ring, b->ring_bytes, &b->ring_descs, b->ring_dv);
    b->ring_descs.clear();
    b->pending_bytes = 0;
    if (st != KMWS_OK) {
        // nothing of this generation can be delivered masked: drop it
        b->items.clear();
        b->stage->clear();
        b->spare.push_back(std::move(next));
        return st;
    }
    const int n = (int)b->items.size();
    kmws_rx_batch::Gen g;
    g.stage = std::move(b->stage);
    g.items.swap(b->items);
    b->inflight.push_back(std::move(g));
    b->stage = std::move(next);
    return n;
}

int kmws_rx_batch_submit(kmws_rx_batch* b) { return rx_submit(b, false); }

int kmws_rx_batch_poll(kmws_rx_batch* b, int wait)
{
    if (!b) return KMWS_ERR_INVALID_PARAM;
    if (b->flushing) return KMWS_ERR_INVALID_STATE;
    int delivered = 0;
    kmws_status err = KMWS_OK;
    while (!b->inflight.empty()) {
        kmws_rx_batch::Gen& g = b->inflight.front();
        if (!wait && !g.stage->done()) break;
        const kmws_status st = g.stage->wait();
        std::vector<kmws_rx_batch::Item> items;
        items.swap(g.items);
        std::unique_ptr<PinnedStage> stage = std::move(g.stage);
        b->inflight.pop_front();
        if (st != KMWS_OK) {  // the launch failed: these payloads are still masked, never delivered
            err = st;
            stage->clear();
            b->spare.push_back(std::move(stage));
            continue;
        }
        b->flushing = true;
        b->delivering = &items;
        for (auto& it : items) {
            if (!it.live) continue;
            ++delivered;  // a NULL callback consumes the frame, like WSHandler without frame_cb_ (:286)
            uint8_t* payload = it.direct ? it.direct : stage->data() + it.off;
            // "destroyed" (WSHandler.cpp:284-287): none of that decoder's frames
            // may reach its callback again -- the rest of this generation, every
            // later generation in flight and the one still being fed
            if (it.cb && it.cb(&it.hdr, payload, it.hdr.length, it.user)) kmws_rx_batch_discard(b, it.dec);
        }
        b->delivering = nullptr;
        b->flushing = false;
        stage->clear();
        b->spare.push_back(std::move(stage));
    }
    return err != KMWS_OK ? err : delivered;
}

int kmws_rx_batch_flush(kmws_rx_batch* b)
{
    // the generations in flight first (delivered in order, before this one):
    // the thread's resident slot holds one job, and a job posted while the
    // previous one runs launches instead (the loopback's ring-wrap flushes did)
    int d0 = 0;
    if (b && !b->flushing && !b->inflight.empty()) {
        d0 = kmws_rx_batch_poll(b, 1);
        if (d0 < 0) return d0;
    }
    const int s = rx_submit(b, true);
    const int d = kmws_rx_batch_poll(b, 1);
    return s < 0 ? s : d < 0 ? d : d0 + d;
}

}  // extern "C"
