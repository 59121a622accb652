// kmws_wshandler.hpp -- C++ drop-in for kuma's WSHandler over the kmws C ABI.
//
// Reference interface: kuma::ws::WSHandler (src/ws/WSHandler.h:32-91), the
// codec member of WebSocket::Impl (src/ws/WebSocketImpl.h:140).  This header
// gives the same class shape -- setMode/getMode, handleData, setFrameCallback,
// reset, the static encodeFrameHeader / handleDataMask (x2) / isControlFrame --
// on top of include/kmws_gpu.h, so WebSocket::Impl can hold either type.
//
// The class is a template over the caller's own types, so kuma instantiates it
// with ITS FrameHeader, KMBuffer, WSError, WSMode and KMError
// (INTEGRATION.md sec.3):
//
//   using KmwsHandler = kmws::BasicWSHandler<FrameHeader, KMBuffer, WSError, WSMode, KMError>;
//
// Requirements on the types (all met by kuma's):
//   FrameHeader  fields fin rsv1 rsv2 rsv3 opcode mask plen (bitfields or
//                integers), xpl.xpl64, maskey[4], length  (wsdefs.h:74-88)
//   Buffer       Buffer(void* data, size_t capacity, size_t size) makes a
//                non-owning view (kmbuffer.h:229-233, WSHandler.cpp:285);
//                begin()/end() iterate the chain, it->readPtr(), it->length()
//                (kmbuffer.h:706-772)
//   WSError      enum with the values of wsdefs.h:56-67 (NOERR = 0 ...)
//   WSMode       enum with CLIENT and SERVER (wsdefs.h:69-72)
//   CbResult     whatever the frame callback returns (kuma: KMError); ignored,
//                as WSHandler::handleFrame ignores it (WSHandler.cpp:286)
//
// kmws::ws below provides standalone types with those shapes, used by the
// tests and by programs without kuma.
//
// Behaviour differences from the reference, all observable-byte-neutral:
//  * payload unmasking runs on the GPU.  There is no CPU fallback: without a
//    gfx950 device a masked frame makes handleData return INVALID_STATE and
//    lastStatus() the kmws_status (KMWS_ERR_NOT_SUPPORTED); handleDataMask
//    returns that status instead of void (callers that ignore the result, as
//    kuma's do, compile unchanged).
//  * self-destruction from inside the frame callback (the reference's
//    DestroyDetector, WSHandler.cpp:284-287) is supported: the decoder state
//    is reference-counted and outlives the feed that is delivering.
//
// Batched mode (RxLoop below): kuma calls handleData once per 64 KiB socket
// read; a GPU round trip per read costs about what the CPU's whole unmask of
// the read does.  With an RxLoop attached (one per event-loop thread), handleData
// parses and validates at once -- same return values -- and queues the frames
// on the loop's receive batch; the loop's posted task (kuma: EventLoop::post,
// kmapi.h:204-210) submits ONE GPU unmask for everything queued in the
// iteration and delivers the callbacks of finished generations at the next
// iterations, so the GPU round trip overlaps the loop's socket reads.  A CLOSE
// frame or a decode error makes handleData deliver everything queued before it
// returns, so kuma's onWsData (WebSocketImpl.cpp:225-246) sees the same state
// and return value as with the reference.
#ifndef KMWS_WSHANDLER_HPP
#define KMWS_WSHANDLER_HPP

#include <sys/uio.h>

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <new>
#include <utility>
#include <vector>

#include "kmws_gpu.h"

namespace kmws {

// kuma's FrameHeader (wsdefs.h:74-88: bitfields fin..plen, xpl, maskey,
// length) -- or any type with those fields -- as the C ABI's kmws_frame_hdr.
template <class FrameHeader>
inline kmws_frame_hdr to_c_header(const FrameHeader& hdr)
{
    kmws_frame_hdr k;
    std::memset(&k, 0, sizeof(k));
    k.fin = hdr.fin;
    k.rsv1 = hdr.rsv1;
    k.rsv2 = hdr.rsv2;
    k.rsv3 = hdr.rsv3;
    k.opcode = hdr.opcode;
    k.mask = hdr.mask;
    k.plen = hdr.plen;
    k.length = hdr.length;
    std::memcpy(k.maskey, hdr.maskey, KMWS_MASK_KEY_SIZE);
    return k;
}
inline kmws_frame_hdr to_c_header(const kmws_frame_hdr& hdr) { return hdr; }

// The deferred receive batch of one event-loop thread, shared by every handler
// on that loop, and the once-per-iteration hook that runs it.
class RxLoop {
public:
    using Task = std::function<void()>;
    using Poster = std::function<void(Task)>;  // kuma: [loop](Task t) { loop->post(std::move(t)); }

    // async: submit at the end of an iteration, deliver at the next ones (the
    // default); false: one synchronous flush per iteration.
    // device: KMWS_DEVICE_AUTO (the default) = the constructing thread's GPU
    // (kmws_thread_device: pinned, or its NUMA node's), so construct the loop
    // on its event-loop thread.  attach: claim that thread's resident slot now
    // (kmws_thread_attach) -- for a loop that is a thread_local of its own loop
    // thread (forThisThread): the thread then gives the slot back only after
    // this loop's destructor has flushed on it.
    explicit RxLoop(Poster post, int device = KMWS_DEVICE_AUTO, bool async = true, bool attach = false)
        : post_(std::move(post)), device_(device == KMWS_DEVICE_AUTO ? kmws_thread_device() : device),
          batch_(kmws_rx_batch_create(device_)), async_(async), alive_(std::make_shared<bool>(true))
    {
        if (batch_ && attach) (void)kmws_thread_attach(device_);
    }
    ~RxLoop()
    {
        *alive_ = false;  // a posted task still queued on the loop becomes a no-op
        if (batch_) {
            (void)kmws_rx_batch_flush(batch_);
            kmws_rx_batch_destroy(batch_);
        }
    }
    RxLoop(const RxLoop&) = delete;
    RxLoop& operator=(const RxLoop&) = delete;

    // The RxLoop of the calling (event-loop) thread, created on first use.
    static RxLoop& forThisThread(Poster post, int device = KMWS_DEVICE_AUTO)
    {
        thread_local RxLoop loop(std::move(post), device, true, true);
        return loop;
    }

    bool valid() const { return batch_ != nullptr; }
    int device() const { return device_; }
    kmws_rx_batch* batch() const { return batch_; }
    // (Re)binds the loop's post function (e.g. when the loop object is created
    // before its event loop runs).
    // A new poster holds none of this loop's tasks: the next arm() posts again
    // (a task left with the old one never ran, or runs as a harmless extra pass).
    void setPoster(Poster post)
    {
        post_ = std::move(post);
        armed_ = false;
        if (pending() > 0 || inflight() > 0) arm();
    }

    // Pinned receive ring the loop reads sockets into (kmws_host_alloc): payloads
    // lying in it are unmasked there, without copies.  Ring bytes of a frame
    // must stay unmodified until it was delivered (inflight() == 0 frees all).
    int attachRing(uint8_t* ring, size_t bytes) { return kmws_rx_batch_attach_ring(batch_, ring, bytes); }

    // Called after every deferred feed: posts the iteration's task once, and
    // keeps generations within the resident worker's job limits -- frames fed
    // while a generation is in flight wait for it, and once they reach half the
    // limits (a 64 KiB read adds at most 64 KiB) the one in flight is waited
    // for (its frames delivered now) and they are submitted at once: a
    // generation that outgrew the limits would launch, and a loop that had
    // fallen behind would stay behind (r05ao).
    void fed()
    {
        if (async_ && batch_ &&
            (kmws_rx_batch_pending(batch_) >= KMWS_RESIDENT_MAX_PAYLOADS / 2 ||
             kmws_rx_batch_pending_bytes(batch_) >= KMWS_RESIDENT_MAX_BYTES / 2)) {
            int r = kmws_rx_batch_inflight(batch_) > 0 ? kmws_rx_batch_poll(batch_, 1) : 0;
            if (r >= 0) r = kmws_rx_batch_submit(batch_);
            if (r < 0) last_ = r;
        }
        arm();
    }

    // Posts the iteration's task once.
    void arm()
    {
        if (armed_ || !post_) return;
        armed_ = true;
        std::weak_ptr<bool> alive = alive_;
        post_([this, alive] {
            std::shared_ptr<bool> a = alive.lock();
            if (a && *a) runIteration();
        });
    }

    // The posted task: deliver what finished, then submit what was fed since
    // -- once the loop's previous generation has finished: one generation in
    // flight per loop thread, so it always runs on the thread's slot of the
    // resident grid (a second one posted while the first runs finds the slot
    // busy and launches; with several in flight the loopback's connections
    // launched most of their jobs, r05an).  Frames fed meanwhile wait and go
    // with the next.  Never waits; re-arms itself while anything is queued.
    void runIteration()
    {
        armed_ = false;
        if (!async_) {
            last_ = kmws_rx_batch_flush(batch_);
            return;
        }
        int r = kmws_rx_batch_poll(batch_, 0);
        if (r >= 0 && kmws_rx_batch_inflight(batch_) == 0 && kmws_rx_batch_pending(batch_) > 0) {
            const int s = kmws_rx_batch_submit(batch_);
            if (s < 0) r = s;
        }
        last_ = r;
        if (kmws_rx_batch_inflight(batch_) > 0 || kmws_rx_batch_pending(batch_) > 0) arm();
    }

    // Deliver everything queued and in flight now (synchronous).
    int flush() { return last_ = kmws_rx_batch_flush(batch_); }
    int inflight() const { return kmws_rx_batch_inflight(batch_); }
    int pending() const { return kmws_rx_batch_pending(batch_); }
    int lastResult() const { return last_; }  // frames delivered by the last run, or a kmws_status

private:
    Poster post_;
    int device_;
    kmws_rx_batch* batch_;
    bool async_;
    bool armed_ = false;
    int last_ = 0;
    std::shared_ptr<bool> alive_;
};

// The batched send path of one event-loop thread: WebSocket::Impl::sendWsFrame
// (WebSocketImpl.cpp:381-436) masks the caller's payload with one
// handleDataMask per send, packs the header and writes both as one iovec.
// With a TxLoop, send() packs the header at once and copies the payload into
// the loop's pinned send ring (the bytes kuma would hand the socket); the
// loop's posted task (kuma: EventLoop::post, kmapi.h:204-210) masks every
// payload queued in the iteration with ONE GPU job and writes each
// connection's frames, in send order, as soon as their generation's mask has
// completed -- the GPU round trip overlaps the next iterations instead of
// stalling every send.  The task never waits: it writes the generations whose
// masks completed and posts what was sent since as the next generation once
// fewer than `max_inflight` are in flight (1, the default: one job per loop
// thread, always on its slot of the resident grid -- a second posted while the
// first runs finds the slot busy and launches; frames sent meanwhile go with
// the next generation).
//
// Differences from sendWsFrame, observable only to the sender:
//  * the frame reaches the socket at the iteration's task, not before send()
//    returns; a writer error is reported by Conn::lastResult() / lastResult(),
//    not by send();
//  * the caller's payload buffer is not modified (kuma masks it in place,
//    :388/:414) and may be reused as soon as send() returns;
//  * an unmasked frame (server mode) whose connection has nothing queued is
//    written at once, without a copy -- exactly sendWsFrame's path.
class TxLoop {
public:
    using Task = std::function<void()>;
    using Poster = std::function<void(Task)>;
    // kuma: [conn](const iovec* v, int n) { return conn->send(v, n); } (negative: error, :432)
    using Writer = std::function<int(const iovec* iov, int cnt)>;

    // One connection's queue: its frames are written in send order.
    class Conn {
    public:
        int lastResult() const { return last_; }  // the writer's last result (negative: an error)
        int queued() const { return queued_; }    // frames sent but not yet written

    private:
        friend class TxLoop;
        explicit Conn(Writer w) : write_(std::move(w)) {}
        Writer write_;
        int queued_ = 0;
        int last_ = 0;
    };

    // ring_bytes: the pinned send ring (a small one stays in the CPU's caches:
    // the payload copies and the socket writes hit it); a payload that does
    // not fit goes through a buffer of its own
    // device, attach: as RxLoop's (KMWS_DEVICE_AUTO: the constructing thread's
    // GPU; attach: its resident slot claimed now, given back after this loop's
    // destructor -- forThisThread does)
    explicit TxLoop(Poster post, int device = KMWS_DEVICE_AUTO, size_t ring_bytes = (size_t)1 << 20,
                    int max_inflight = 1, bool attach = false)
        : post_(std::move(post)), device_(device == KMWS_DEVICE_AUTO ? kmws_thread_device() : device),
          batch_(kmws_tx_batch_create(device_)), max_inflight_(max_inflight < 1 ? 1 : max_inflight),
          alive_(std::make_shared<bool>(true))
    {
        if (!batch_) return;
        if (attach) (void)kmws_thread_attach(device_);
        ring_ = static_cast<uint8_t*>(kmws_host_alloc(ring_bytes, device_));
        if (ring_ && kmws_tx_batch_attach_ring(batch_, ring_, ring_bytes) == KMWS_OK) {
            ring_bytes_ = ring_bytes;
        } else {
            kmws_host_free(ring_);
            ring_ = nullptr;
        }
    }
    ~TxLoop()
    {
        *alive_ = false;  // a posted task still queued on the loop becomes a no-op
        if (batch_) {
            (void)flush();  // every queued frame is written: close connections first
            kmws_tx_batch_destroy(batch_);
        }
        // after a mask that timed out the device may still write the ring: it
        // is never freed (nor reused)
        if (broken_ != KMWS_ERR_TIMEOUT) kmws_host_free(ring_);
    }
    TxLoop(const TxLoop&) = delete;
    TxLoop& operator=(const TxLoop&) = delete;

    // The TxLoop of the calling (event-loop) thread, created on first use.
    static TxLoop& forThisThread(Poster post, int device = KMWS_DEVICE_AUTO)
    {
        thread_local TxLoop loop(std::move(post), device, (size_t)1 << 20, 1, true);
        return loop;
    }

    bool valid() const { return batch_ != nullptr && ring_ != nullptr && broken_ == 0; }
    int device() const { return device_; }
    // Frames dropped because their generation's mask failed (never written;
    // their connections' lastResult() says why).  A mask that timed out
    // (KMWS_ERR_TIMEOUT) also retires the loop: later sends return it.
    uint64_t dropped() const { return dropped_; }
    int broken() const { return broken_; }
    // A new poster holds none of this loop's tasks: the next arm() posts again
    // (a task left with the old one never ran, or runs as a harmless extra pass).
    void setPoster(Poster post)
    {
        post_ = std::move(post);
        armed_ = false;
        if (pending() > 0 || inflight() > 0) arm();
    }

    // A connection's queue (kuma: per WebSocket::Impl, around ws_conn_->send).
    Conn* open(Writer w)
    {
        conns_.emplace_back(new Conn(std::move(w)));
        return conns_.back().get();
    }
    // Writes everything queued (every connection's frames), then forgets c.
    int close(Conn* c)
    {
        const int r = flush();
        for (size_t i = 0; i < conns_.size(); ++i)
            if (conns_[i].get() == c) {
                conns_.erase(conns_.begin() + (std::ptrdiff_t)i);
                break;
            }
        return r;
    }

    // sendWsFrame(hdr, payload, plen) (WebSocketImpl.cpp:381-403): length =
    // plen, header packed now; masked with hdr.maskey when hdr.mask is set and
    // plen > 0 (kuma's client mode, :384-388).  Returns the header length
    // (2..14) or a negative kmws_status.
    // (hdr: kuma's FrameHeader or a kmws_frame_hdr)
    template <class FrameHeader>
    int send(Conn* c, const FrameHeader& hdr, const uint8_t* payload, size_t plen)
    {
        const uint8_t* segs[1] = {payload};
        const size_t lens[1] = {plen};
        return sendChain(c, to_c_header(hdr), segs, lens, plen ? 1 : 0);
    }

    // sendWsFrame(hdr, const KMBuffer&) (:405-436) over kuma's chain
    // (KMBuffer::begin/end, readPtr, length: kmbuffer.h:706-772).
    template <class FrameHeader, class Buffer>
    int sendBuffer(Conn* c, const FrameHeader& hdr, const Buffer& buf)
    {
        std::vector<const uint8_t*> segs;
        std::vector<size_t> lens;
        for (auto it = buf.begin(); it != buf.end(); ++it) {
            segs.push_back(static_cast<const uint8_t*>(it->readPtr()));
            lens.push_back(it->length());
        }
        return sendChain(c, to_c_header(hdr), segs.data(), lens.data(), segs.size());
    }

    // sendWsFrame(hdr, KMBuffer) (:405-436): the chain's segments, the key
    // phase continuing across them; more than 128 non-empty segments return
    // KMWS_ERR_BUFFER_TOO_LONG and send nothing (as kuma, :427).
    int sendChain(Conn* c, const kmws_frame_hdr& hdr, const uint8_t* const* segs, const size_t* lens, size_t nseg)
    {
        if (broken_) return broken_;
        if (!valid() || !c) return KMWS_ERR_INVALID_STATE;
        size_t plen = 0, nonempty = 0;
        for (size_t i = 0; i < nseg; ++i) {
            plen += lens[i];
            nonempty += lens[i] != 0;
        }
        if (nonempty > 128) return KMWS_ERR_BUFFER_TOO_LONG;
        if (plen > 0xFFFFFFFFull) return KMWS_ERR_INVALID_PARAM;
        Frame f;
        f.conn = c;
        f.plen = plen;
        kmws_frame_hdr h = hdr;
        h.length = (uint32_t)plen;
        const bool masked = h.mask && plen > 0;
        if (!masked && c->queued_ == 0) {  // nothing of this connection is waiting: sendWsFrame's own path
            uint8_t hb[KMWS_MAX_HEADER_SIZE];
            const int hl = kmws_encode_header(&h, hb);
            std::vector<iovec> iov(1, iovec{hb, (size_t)hl});
            for (size_t i = 0; i < nseg; ++i)
                if (lens[i]) iov.push_back(iovec{const_cast<uint8_t*>(segs[i]), lens[i]});
            c->last_ = c->write_(iov.data(), (int)iov.size());
            return hl;
        }
        // the generation stays within the resident worker's job limits: one
        // that would outgrow them is posted first, after the one in flight
        // (a larger generation would launch, and a loop that fell behind
        // would stay behind, r05ao)
        if (masked && !cur_.frames.empty() &&
            (cur_.nmasked + 1 > KMWS_RESIDENT_MAX_PAYLOADS || cur_.bytes + plen > KMWS_RESIDENT_MAX_BYTES)) {
            int r = 0;
            while (r >= 0 && !inflight_.empty()) r = completeOldest();
            if (r >= 0) r = submit();
            if (r < 0) return r;
        }
        uint8_t* p = place(plen, &f);
        if (!p) return broken_ ? broken_ : KMWS_ERR_FAILED;
        for (size_t i = 0, pos = 0; i < nseg; pos += lens[i], ++i)
            if (lens[i]) std::memcpy(p + pos, segs[i], lens[i]);
        f.payload = p;
        if (masked) {
            size_t one = plen;
            f.hlen = kmws_tx_batch_add(batch_, &h, &p, &one, 1, f.hdr);
            cur_.masked = true;
            ++cur_.nmasked;
            cur_.bytes += plen;
        } else {
            f.hlen = kmws_encode_header(&h, f.hdr);
        }
        if (f.hlen < 0) return f.hlen;
        cur_.frames.push_back(std::move(f));
        ++c->queued_;
        arm();
        return cur_.frames.back().hlen;
    }

    // Posts the iteration's task once (after a send).
    void arm()
    {
        if (armed_ || !post_) return;
        armed_ = true;
        std::weak_ptr<bool> alive = alive_;
        post_([this, alive] {
            std::shared_ptr<bool> a = alive.lock();
            if (a && *a) runIteration();
        });
    }

    // The posted task: write every generation whose masks completed, then
    // post what was sent since if fewer than max_inflight generations are in
    // flight; re-arms itself while anything is queued or in flight.
    void runIteration()
    {
        armed_ = false;
        int r = complete(false);
        if (r >= 0 && (int)inflight_.size() < max_inflight_) {
            const int s = submit();
            if (s < 0) r = s;
        }
        last_ = r;
        if (!inflight_.empty() || !cur_.frames.empty()) arm();
    }

    // Everything sent so far masked and written, synchronously (what is in
    // flight first, so the last generation's job finds the slot free).
    int flush()
    {
        int r = complete(true);
        if (r >= 0) {
            const int s = submit();
            const int w = s < 0 ? s : complete(true);
            r = w < 0 ? w : r + w;
        }
        return last_ = r;
    }

    int inflight() const { return (int)inflight_.size(); }
    int pending() const { return (int)cur_.frames.size(); }
    int lastResult() const { return last_; }  // frames written by the last run, or a kmws_status

private:
    struct Frame {
        Conn* conn = nullptr;
        uint8_t hdr[KMWS_MAX_HEADER_SIZE];
        int hlen = 0;
        uint8_t* payload = nullptr;
        size_t plen = 0;
        std::unique_ptr<uint8_t[]> own;  // a payload larger than the ring
    };
    struct Gen {
        std::vector<Frame> frames;
        bool masked = false;
        uint32_t nmasked = 0;  // masked payloads (one job descriptor each)
        uint64_t bytes = 0;    // their bytes
        int64_t ticket = 0;
        size_t ring_used = 0;  // ring bytes (with alignment and wrap waste) freed when written
        bool dropped = false;  // its mask failed: never written
    };

    // Room for n payload bytes: 16-byte aligned in the ring, after the bytes
    // in use (written generations free theirs in order); a full ring writes
    // the oldest generation first; a payload larger than the ring gets a heap
    // buffer (staged by the tx batch).
    uint8_t* place(size_t n, Frame* f)
    {
        if (n == 0) return ring_;
        if (n + 16 > ring_bytes_) {
            f->own.reset(new (std::nothrow) uint8_t[n]);
            return f->own.get();
        }
        for (;;) {
            const size_t head = (tail_ + used_) % ring_bytes_;
            const size_t pad = (16 - (head & 15)) & 15;
            size_t waste = pad, at = head + pad;
            if (at + n > ring_bytes_) {  // wrap: the end of the ring stays unused
                waste = ring_bytes_ - head;
                at = 0;
            }
            if (used_ + waste + n <= ring_bytes_) {
                used_ += waste + n;
                cur_.ring_used += waste + n;
                return ring_ + at;
            }
            // full: free the oldest generation, or everything if only the current one holds the ring
            const int r = inflight_.empty() ? flush() : completeOldest();
            if (r < 0) return nullptr;
        }
    }

    int submit()
    {
        if (cur_.frames.empty()) return 0;
        if (cur_.masked) {
            const int64_t t = kmws_tx_batch_submit(batch_);
            if (t <= 0) {
                // the batch dropped the generation's masks (nothing runs on
                // them): its frames are never written -- their payloads are not
                // masked although their headers say so
                const int st = t < 0 ? (int)t : KMWS_ERR_FAILED;
                drop(cur_, st);
                used_ -= cur_.ring_used;  // the newest ring bytes: nothing writes them
                cur_ = Gen();
                return st;
            }
            cur_.ticket = t;
        }
        inflight_.push_back(std::move(cur_));
        cur_ = Gen();
        return 0;
    }

    // Writes finished generations in order (wait: all of them); returns the
    // frames written or a negative status.
    int complete(bool wait)
    {
        int n = 0;
        while (!inflight_.empty()) {
            Gen& g = inflight_.front();
            if (g.ticket > 0) {
                const int p = kmws_tx_batch_poll(batch_, g.ticket, wait ? 1 : 0);
                if (p < 0) return failOldest(p);
                if (p == 0) break;
            }
            n += write(g);
            retireOldest();
        }
        if (inflight_.empty() && cur_.frames.empty() && cur_.ring_used == 0) tail_ = used_ = 0;
        return n;
    }
    int completeOldest()
    {
        Gen& g = inflight_.front();
        if (g.ticket > 0) {
            const int p = kmws_tx_batch_poll(batch_, g.ticket, 1);
            if (p < 0) return failOldest(p);
        }
        const int n = write(g);
        retireOldest();
        return n;
    }
    void retireOldest()
    {
        Gen& g = inflight_.front();
        used_ -= g.ring_used;
        tail_ = (tail_ + g.ring_used) % ring_bytes_;
        inflight_.pop_front();
    }
    // The oldest generation's mask failed (the batch has retired it): its
    // frames are dropped, not written.  KMWS_ERR_TIMEOUT: the device may still
    // write its ring bytes -- the loop is retired (later generations written
    // if their masks finish, frames not yet submitted dropped, the ring never
    // reused or freed); any other failure frees them.
    int failOldest(int st)
    {
        drop(inflight_.front(), st);
        if (st != KMWS_ERR_TIMEOUT) {
            retireOldest();
            return st;
        }
        broken_ = st;
        inflight_.pop_front();  // its ring bytes stay allocated: the ring is never reused
        while (!inflight_.empty()) {  // later generations: written if their masks finish
            Gen& g = inflight_.front();
            const int p = g.ticket > 0 ? kmws_tx_batch_poll(batch_, g.ticket, 1) : 1;
            if (p == 1) (void)write(g);
            else drop(g, p < 0 ? p : st);
            inflight_.pop_front();
        }
        drop(cur_, st);
        cur_ = Gen();
        return st;
    }
    void drop(Gen& g, int st)
    {
        if (g.dropped) return;
        g.dropped = true;
        for (Frame& f : g.frames) {
            --f.conn->queued_;
            f.conn->last_ = st;
        }
        dropped_ += g.frames.size();
    }

    // Each connection's consecutive frames of the generation as one writev
    // (kuma's send takes an iovec array, :432), at most 1024 entries at a time.
    int write(Gen& g)
    {
        std::vector<iovec> iov;
        Conn* c = nullptr;
        auto out = [&] {
            if (c && !iov.empty()) c->last_ = c->write_(iov.data(), (int)iov.size());
            iov.clear();
        };
        for (Frame& f : g.frames) {
            if (f.conn != c || iov.size() + 2 > 1024) {
                out();
                c = f.conn;
            }
            iov.push_back(iovec{f.hdr, (size_t)f.hlen});
            if (f.plen) iov.push_back(iovec{f.payload, f.plen});
            --f.conn->queued_;
        }
        out();
        return (int)g.frames.size();
    }

    Poster post_;
    int device_;
    kmws_tx_batch* batch_;
    int max_inflight_;
    std::shared_ptr<bool> alive_;
    uint8_t* ring_ = nullptr;
    size_t ring_bytes_ = 0;
    size_t tail_ = 0, used_ = 0;  // ring bytes in use: [tail_, tail_ + used_) mod ring_bytes_
    Gen cur_;
    std::deque<Gen> inflight_;
    std::vector<std::unique_ptr<Conn>> conns_;
    bool armed_ = false;
    int last_ = 0;
    int broken_ = 0;         // KMWS_ERR_TIMEOUT once a mask timed out
    uint64_t dropped_ = 0;
};

template <class FrameHeader, class Buffer, class WSError, class WSMode, class CbResult>
class BasicWSHandler {
public:
    using FrameCallback = std::function<CbResult(FrameHeader, Buffer&)>;  // WSHandler.h:35

    // device: KMWS_DEVICE_AUTO (the default) = the constructing thread's GPU;
    // kuma creates a connection's handler on its loop thread
    explicit BasicWSHandler(int device = KMWS_DEVICE_AUTO) : st_(std::make_shared<State>(device)) {}
    ~BasicWSHandler()
    {
        if (st_) {
            st_->alive = false;  // a feed in progress keeps the state until it returns
            if (st_->rx && st_->dec) kmws_rx_batch_discard(st_->rx->batch(), st_->dec);  // queued frames: dropped
        }
    }
    BasicWSHandler(const BasicWSHandler&) = delete;
    BasicWSHandler& operator=(const BasicWSHandler&) = delete;

    // false if the decoder could not be created (bad device index)
    bool valid() const { return st_->dec != nullptr; }

    void setMode(WSMode mode)  // WSHandler.h:40
    {
        st_->mode = mode;
        if (st_->dec) kmws_decoder_set_mode(st_->dec, mode == WSMode::SERVER ? KMWS_MODE_SERVER : KMWS_MODE_CLIENT);
    }
    WSMode getMode() const { return st_->mode; }  // WSHandler.h:41

    // WSHandler::handleData (WSHandler.cpp:41-44): same return values and
    // callback sequence; masked payloads lying wholly in `data` are unmasked
    // there, in place.
    WSError handleData(uint8_t* data, size_t len)
    {
        std::shared_ptr<State> keep = st_;
        if (!keep->dec) return WSError::INVALID_STATE;
        if (keep->rx) return handleDeferred(keep, data, len);
        const int r = kmws_decoder_feed(keep->dec, data, len, &State::on_frame, keep.get());
        if (!keep->alive) return WSError::DESTROYED;
        keep->last_status = r < 0 ? r : KMWS_OK;
        if (r < 0) return WSError::INVALID_STATE;  // device step failed: lastStatus() says why
        return static_cast<WSError>(r);
    }

    // Batched mode: queue decoded frames on the loop's receive batch (see the
    // file comment).  nullptr returns to one GPU batch per handleData.  Switch
    // only while none of this handler's frames are queued.
    void setRxLoop(RxLoop* loop) { st_->rx = loop && loop->valid() ? loop : nullptr; }
    RxLoop* rxLoop() const { return st_->rx; }

    // kmws_status of the last handleData: KMWS_OK, or why the GPU step failed
    int lastStatus() const { return st_->last_status; }

    // kmws_decoder_set_in_place: false delivers masked payloads of a pageable
    // read buffer as views of their unmasked staging copy (one host copy fewer;
    // kuma does not read its buffer after handleData returns).
    void setInPlace(bool on)
    {
        if (st_->dec) kmws_decoder_set_in_place(st_->dec, on ? 1 : 0);
    }

    void setFrameCallback(FrameCallback cb) { st_->cb = std::move(cb); }  // WSHandler.h:46

    void reset()  // WSHandler.cpp:324-327
    {
        if (st_->dec) kmws_decoder_reset(st_->dec);
    }

    // WSHandler::encodeFrameHeader (WSHandler.cpp:46-106): 2/4/10 (+4) bytes
    static int encodeFrameHeader(FrameHeader hdr, uint8_t hdr_buf[KMWS_MAX_HEADER_SIZE])
    {
        const kmws_frame_hdr k = to_c_header(hdr);
        return kmws_encode_header(&k, hdr_buf);
    }

    // WSHandler::handleDataMask(key, data, len) (WSHandler.cpp:303-310), on the GPU
    static kmws_status handleDataMask(const uint8_t mask_key[KMWS_MASK_KEY_SIZE], uint8_t* data, size_t len,
                                      int device = KMWS_DEVICE_AUTO)
    {
        if (data == nullptr || len == 0) return KMWS_OK;  // :305
        uint8_t* segs[1] = {data};
        const size_t lens[1] = {len};
        return kmws_mask_host_chain(mask_key, segs, lens, 1, device);
    }

    // WSHandler::handleDataMask(key, KMBuffer&) (WSHandler.cpp:312-322): the key
    // phase continues across the chain's segments; on the GPU, one launch
    static kmws_status handleDataMask(const uint8_t mask_key[KMWS_MASK_KEY_SIZE], Buffer& buf,
                                      int device = KMWS_DEVICE_AUTO)
    {
        std::vector<uint8_t*> segs;
        std::vector<size_t> lens;
        collectSegments(buf, segs, lens);
        if (segs.empty()) return KMWS_OK;
        return kmws_mask_host_chain(mask_key, segs.data(), lens.data(), segs.size(), device);
    }

    // The chain's segments in order (KMBuffer::begin/end, kmbuffer.h:706-772), as
    // handleDataMask hands them to kmws_mask_host_chain.
    static void collectSegments(const Buffer& buf, std::vector<uint8_t*>& segs, std::vector<size_t>& lens)
    {
        for (auto it = buf.begin(); it != buf.end(); ++it) {
            segs.push_back(static_cast<uint8_t*>(it->readPtr()));
            lens.push_back(it->length());
        }
    }

    static bool isControlFrame(uint8_t opcode) { return opcode >= 8; }  // WSHandler.h:52-54

private:
    struct State;

    static WSError handleDeferred(const std::shared_ptr<State>& keep, uint8_t* data, size_t len)
    {
        RxLoop* rx = keep->rx;
        const int r = kmws_decoder_feed_deferred(keep->dec, rx->batch(), data, len, &State::on_frame, keep.get());
        if (r == KMWS_WS_NOERR || r == KMWS_WS_NEED_MORE_DATA) {
            rx->fed();  // may deliver earlier frames (this handler's callback may destroy it)
            if (!keep->alive) return WSError::DESTROYED;
            keep->last_status = KMWS_OK;
            return static_cast<WSError>(r);
        }
        // CLOSE or an error: deliver everything queued first, so the caller sees
        // the connection state the reference's synchronous delivery leaves
        // (kuma's onWsData checks it before the return value)
        const int f = rx->flush();
        if (!keep->alive) return WSError::DESTROYED;
        keep->last_status = r < 0 ? r : (f < 0 ? f : KMWS_OK);
        if (r < 0) return WSError::INVALID_STATE;
        return static_cast<WSError>(r);
    }

    struct State : std::enable_shared_from_this<State> {
        explicit State(int device) : dec(kmws_decoder_create(KMWS_MODE_CLIENT, device)) {}
        ~State()
        {
            if (dec) kmws_decoder_destroy(dec);
        }
        State(const State&) = delete;
        State& operator=(const State&) = delete;

        // WSHandler::handleFrame (WSHandler.cpp:282-289): FrameHeader by value, a
        // non-owning view of the payload, "destroyed" if the callback deleted
        // the handler
        static int on_frame(const kmws_frame_hdr* k, uint8_t* payload, size_t len, void* user)
        {
            // held for the call: the callback may destroy the handler (deferred
            // delivery runs outside handleData, with no caller holding the state)
            std::shared_ptr<State> s = static_cast<State*>(user)->shared_from_this();
            FrameHeader h;
            std::memset(static_cast<void*>(&h), 0, sizeof(h));
            h.fin = k->fin;
            h.rsv1 = k->rsv1;
            h.rsv2 = k->rsv2;
            h.rsv3 = k->rsv3;
            h.opcode = k->opcode;
            h.mask = k->mask;
            h.plen = k->plen;
            h.xpl.xpl64 = k->xpl64;
            std::memcpy(h.maskey, k->maskey, KMWS_MASK_KEY_SIZE);
            h.length = k->length;
            Buffer view(static_cast<void*>(payload), len, len);
            if (s->cb) {
                FrameCallback cb = s->cb;  // the callback may replace or drop itself
                (void)cb(h, view);
            }
            return s->alive ? 0 : 1;
        }

        kmws_decoder* dec;
        FrameCallback cb;
        WSMode mode = WSMode::CLIENT;
        bool alive = true;
        int last_status = KMWS_OK;
        RxLoop* rx = nullptr;
    };
    std::shared_ptr<State> st_;
};

// Standalone types with the reference's shapes, for programs without kuma.
namespace ws {

enum class WSError : int {  // wsdefs.h:56-67
    NOERR = 0, NEED_MORE_DATA = 1, HANDSHAKE = 2, INVALID_PARAM = 3, INVALID_STATE = 4,
    INVALID_FRAME = 5, INVALID_LENGTH = 6, PROTOCOL_ERROR = 7, CLOSED = 8, DESTROYED = 9
};

enum class WSMode { CLIENT, SERVER };  // wsdefs.h:69-72

struct FrameHeader {  // wsdefs.h:74-88
    uint8_t fin : 1;
    uint8_t rsv1 : 1;
    uint8_t rsv2 : 1;
    uint8_t rsv3 : 1;
    uint8_t opcode : 4;
    uint8_t mask : 1;
    uint8_t plen : 7;
    union {
        uint16_t xpl16;
        uint64_t xpl64;
    } xpl;
    uint8_t maskey[KMWS_MASK_KEY_SIZE];
    uint32_t length = 0;
};

// A non-owning segment chain with KMBuffer's view constructor and iteration
// surface (kmbuffer.h:229-233, 706-772).
class BufferChain {
public:
    struct Segment {
        void* ptr;
        size_t len;
        void* readPtr() const { return ptr; }
        size_t length() const { return len; }
    };
    BufferChain() = default;
    BufferChain(void* data, size_t capacity, size_t size = 0) : segs_{Segment{data, size}}
    {
        (void)capacity;
    }
    void append(void* data, size_t size) { segs_.push_back(Segment{data, size}); }
    std::vector<Segment>::const_iterator begin() const { return segs_.begin(); }
    std::vector<Segment>::const_iterator end() const { return segs_.end(); }
    void* readPtr() const { return segs_.empty() ? nullptr : segs_[0].ptr; }
    size_t length() const { return segs_.empty() ? 0 : segs_[0].len; }
    size_t chainLength() const  // kmbuffer.h:388-398
    {
        size_t n = 0;
        for (const Segment& s : segs_) n += s.len;
        return n;
    }

private:
    std::vector<Segment> segs_;
};

using WSHandler = BasicWSHandler<FrameHeader, BufferChain, WSError, WSMode, int>;

}  // namespace ws
}  // namespace kmws

#endif  // KMWS_WSHANDLER_HPP
