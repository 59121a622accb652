// BASELINE configs[0] over a real loopback TCP connection: a client thread
// sends 1,000 x 4 KiB masked TEXT frames to a server thread, which reads the
// socket in <= 64 KiB reads (kuma's TcpConnection::onReceive,
// TcpConnection.cpp:220-249) and decodes them (WebSocket::Impl::onWsData ->
// WSHandler::handleData, WebSocketImpl.cpp:225-246).  Both ends run one codec:
//   cpu  kuma's codec as restated in oracle/ (byte-loop mask, state machine),
//        one encode + mask per send, one feed per read -- the reference's shape;
//   gpu  kmws: sends queued in a kmws_tx_batch over a pinned send ring, one
//        flush per loop iteration (16 frames), then writev; reads land in a
//        pinned receive ring fed with kmws_decoder_feed_deferred, one
//        kmws_rx_batch_flush per loop iteration (socket drained to EAGAIN).
//        The batches and rings belong to the loop threads (created once); the
//        decoder is per connection, as kuma's WSHandler.
//   sync  the plain member swap: the server holds a
//        kmws::BasicWSHandler WITHOUT an RxLoop and calls handleData once per
//        read into a pageable buffer, synchronously, like kuma's WSHandler (the
//        thread's resident worker unmasks each read, no launch); the client masks
//        each payload with the static handleDataMask (sendWsFrame,
//        WebSocketImpl.cpp:388) and packs the header with encodeFrameHeader.
//   adapter  the drop-in as kuma would run it: the server
//        holds a kmws::BasicWSHandler (include/kmws_wshandler.hpp) in batched
//        mode -- handleData per read, as WebSocket::Impl::onWsData calls it,
//        frames queued on the loop thread's kmws::RxLoop, whose posted task
//        submits the iteration's unmask and delivers finished generations at the
//        next iterations (asynchronous, the GPU round trip overlaps the reads);
//        the client sends through its loop thread's kmws::TxLoop (sendWsFrame's
//        replacement: header packed and payload copied into the pinned send
//        ring at send, one mask job per iteration, frames written by the posted
//        task once their generation completed, one generation in flight after
//        each task).
// Every delivered payload is compared with what the client sent.  Prints one
// JSON line per mode.  Test infrastructure (links the oracle): tests/test_abi_build.py.
//
//   replay_cpu / replay_adapter  the server alone: each client replays the
//        connection's masked wire image, built once before the run (remote
//        peers' bytes: no codec work on this box's client side), and the server
//        decodes with kuma's codec or with the drop-in's RxLoop adapter -- what
//        a kuma server with the drop-in would meet; only the receive side
//        crosses PCIe.
//   sink_cpu / sink_adapter  the client alone: it sends with kuma's codec or with
//        the drop-in's TxLoop, and the server only reads and compares the bytes
//        with the expected masked wire image (no decode) -- a kuma client's
//        send side; only it crosses PCIe.
// usage: loopback_cfg1 cpu|gpu|sync|adapter|replay_cpu|replay_adapter|sink_cpu|sink_adapter [reps] [frames per send iteration] [rx flush bytes] [variant] [connections]
// (variant noresident: both loop threads switch their resident worker off --
// every GPU job a launch and a wait, the A/B of kmws_resident.hip; submitpoll:
// the gpu mode's flushes replaced by submit + poll(wait); inflight2: the
// adapter's TxLoop keeps two generations in flight instead of one; ring16m: its
// send ring is 16 MiB instead of 1 MiB; "0" or "-": none).  connections (1-8): that many
// client / server loop-thread pairs at once, each with its own connection and loop
// objects, 1,000 frames each; GiB_s is the aggregate from the first send of any
// connection to the last frame delivered on any (kuma runs several loop threads)
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"
#include "kmws_wshandler.hpp"

extern "C" {  // oracle/kmws_oracle.c (test infrastructure)
typedef struct orc_hdr {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, plen, _pad;
    uint64_t xpl64;
    uint8_t maskey[4];
    uint32_t length;
} orc_hdr;
typedef struct orc_decoder orc_decoder;
typedef int (*orc_frame_cb)(const orc_hdr* hdr, const uint8_t* payload, size_t len, void* user);
void orc_mask(const uint8_t key[4], uint8_t* data, size_t len, size_t phase);
int orc_encode_header(const orc_hdr* h, uint8_t out[14]);
orc_decoder* orc_decoder_create(int mode);
void orc_decoder_destroy(orc_decoder* d);
int orc_decoder_feed(orc_decoder* d, uint8_t* data, size_t len, orc_frame_cb cb, void* user);
}

namespace {

constexpr int kFrames = 1000;
constexpr size_t kLen = 4096;
int kGroup = 16;                      // frames per client loop iteration (64 KiB; argv[3])
size_t kFlushBytes = 0;               // server: hold a drained batch until this many bytes (argv[4]; 0 = every iteration)
constexpr size_t kRead = 64 * 1024;   // kuma's receive buffer (TcpConnection.cpp:229)
constexpr size_t kRing = 8u << 20;    // pinned receive ring

uint64_t splitmix(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double cpu_s()  // CPU time of every thread of the process so far (user + system)
{
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return (double)u.ru_utime.tv_sec + u.ru_utime.tv_usec * 1e-6 + (double)u.ru_stime.tv_sec + u.ru_stime.tv_usec * 1e-6;
}

double thread_cpu_s()
{
    rusage u{};
    getrusage(RUSAGE_THREAD, &u);
    return (double)u.ru_utime.tv_sec + u.ru_utime.tv_usec * 1e-6 + (double)u.ru_stime.tv_sec + u.ru_stime.tv_usec * 1e-6;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// Seconds spent per step of one connection (breakdown).  The client's and the
// server's fields are on cache lines of their own, and so is each connection's
// record: a server spinning on recv updates its fields at every pass, and
// fields shared with a client or another connection's record made those
// threads ping-pong the line (it cost the other threads milliseconds per
// connection at 8 connections).
struct alignas(64) Times {
    // client thread
    double tx_flush = 0, writev = 0, client = 0, t0 = 0;  // t0: this connection's first send (steady clock)
    double sends = 0;          // adapter client: inside TxLoop::send
    double client_cpu = 0;     // the client thread's own CPU time
    long client_nivcsw = 0;    // its involuntary context switches
    int client_slot = -1;      // its slot of the resident grid (-1: none)
    // server thread
    alignas(64) double rx_feed = 0, rx_flush = 0, recv = 0;
    double rx_task_max = 0, rx_wrap = 0;  // adapter: the longest posted rx task; flushes at ring wraps
    int rx_wraps = 0, rx_inflight_max = 0;
    double t_end = 0;        // the last delivered frame (steady clock)
    double server_cpu = 0;   // the server thread's own CPU time
    int server_slot = -1;
};

struct alignas(64) Expect {  // one connection's (a line of its own: the server thread updates it per frame)
    std::vector<uint8_t> plain;  // kFrames * kLen
    std::vector<uint8_t> wire;   // replay modes: every frame, header + masked payload
    std::vector<size_t> frame_off;  // where frame k starts in `wire` (kFrames + 1 entries)
    std::atomic<int> got{0};
    std::atomic<int> bad{0};
};

void check_frame(Expect* e, const uint8_t* p, size_t len, int opcode)
{
    const int k = e->got.load(std::memory_order_relaxed);
    if (k >= kFrames || len != kLen || opcode != 1 || std::memcmp(p, e->plain.data() + (size_t)k * kLen, kLen) != 0)
        e->bad.fetch_add(1);
    e->got.store(k + 1, std::memory_order_release);
}

int kmws_cb(const kmws_frame_hdr* h, uint8_t* p, size_t len, void* user)
{
    check_frame(static_cast<Expect*>(user), p, len, h->opcode);
    return 0;
}

int orc_cb(const orc_hdr* h, const uint8_t* p, size_t len, void* user)
{
    check_frame(static_cast<Expect*>(user), p, len, h->opcode);
    return 0;
}

void send_all(int fd, std::vector<iovec>& iov)
{
    size_t i = 0;
    while (i < iov.size()) {
        const int cnt = (int)std::min<size_t>(iov.size() - i, 1024);
        ssize_t w = writev(fd, iov.data() + i, cnt);
        if (w < 0) {
            std::perror("writev");
            std::exit(2);
        }
        while (w > 0 && i < iov.size()) {  // advance over what was written
            if ((size_t)w >= iov[i].iov_len) {
                w -= (ssize_t)iov[i].iov_len;
                ++i;
            } else {
                iov[i].iov_base = static_cast<uint8_t*>(iov[i].iov_base) + w;
                iov[i].iov_len -= (size_t)w;
                w = 0;
            }
        }
    }
}

// Per loop thread, long-lived (created once, as a loop's batches and rings would be).
struct LoopObjs {
    kmws_rx_batch* rx = nullptr;
    uint8_t* rring = nullptr;
    kmws_tx_batch* tx = nullptr;
    uint8_t* sring = nullptr;
    kmws::RxLoop* rxloop = nullptr;  // adapter mode: the server loop's RxLoop (owns its own batch)
    kmws::TxLoop* txloop = nullptr;  // adapter mode: the client loop's TxLoop (owns its batch and ring)
};

// One connection: returns seconds from the first send to the last delivered frame.
bool g_sync = false;  // mode "sync": the synchronous member swap on both ends
bool g_noresident = false;
bool g_submitpoll = false;  // gpu mode: submit + poll(wait) instead of the flushes
bool g_replay = false;      // replay_* modes: clients replay a pre-built masked wire image
bool g_sink = false;        // sink_* modes: the server compares the bytes with that image, no decode
int g_inflight = 1;         // adapter mode: the TxLoop's generations in flight after a run (inflight2: 2)
size_t g_tx_ring = (size_t)1 << 20;  // adapter mode: the TxLoop's pinned send ring (ring16m: 16 MiB)

double run_once(bool gpu, bool adapter, Expect& e, const std::vector<uint32_t>& keys, const LoopObjs& lo, Times& T,
                std::atomic<int>* gate = nullptr, int conns = 1)
{
    int ls = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    a.sin_port = 0;
    socklen_t al = sizeof a;
    if (bind(ls, (sockaddr*)&a, sizeof a) != 0 || listen(ls, 1) != 0 || getsockname(ls, (sockaddr*)&a, &al) != 0) {
        std::perror("listen");
        std::exit(2);
    }
    e.got = 0;
    e.bad = 0;
    T = Times();
    std::atomic<bool> ready{false};
    std::chrono::steady_clock::time_point t_end;

    std::thread server([&] {
        if (g_noresident) kmws_resident_enable(0, 0);
        int fd = accept(ls, nullptr, nullptr);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        ready = true;
        const double sc0 = thread_cpu_s();
        if (g_sink) {  // reads compared with the expected wire image; a frame counted per frame's bytes
            std::vector<uint8_t> buf(kRead);
            size_t pos = 0;
            const size_t total = e.wire.size();
            while (pos < total) {
                double t = now_s();
                const ssize_t r = recv(fd, buf.data(), kRead, 0);
                T.recv += now_s() - t;
                if (r <= 0) break;
                if ((size_t)r > total - pos || std::memcmp(buf.data(), e.wire.data() + pos, (size_t)r) != 0)
                    e.bad.fetch_add(1);
                pos += (size_t)r;
            }
            e.got.store(pos == total ? kFrames : 0, std::memory_order_release);
        } else if (g_sync) {
            kmws::ws::WSHandler h;  // per connection; no RxLoop: one synchronous GPU job per read
            h.setMode(kmws::ws::WSMode::SERVER);
            h.setInPlace(false);
            h.setFrameCallback([&e](kmws::ws::FrameHeader hdr, kmws::ws::BufferChain& buf) {
                check_frame(&e, static_cast<const uint8_t*>(buf.readPtr()), buf.length(), hdr.opcode);
                return 0;
            });
            std::vector<uint8_t> buf(kRead);  // kuma's read buffer (pageable)
            while (e.got.load(std::memory_order_acquire) < kFrames) {
                double t = now_s();
                const ssize_t r = recv(fd, buf.data(), kRead, 0);
                T.recv += now_s() - t;
                if (r <= 0) break;
                t = now_s();
                const kmws::ws::WSError err = h.handleData(buf.data(), (size_t)r);
                T.rx_feed += now_s() - t;
                if (err != kmws::ws::WSError::NOERR && err != kmws::ws::WSError::NEED_MORE_DATA) std::exit(4);
            }
        } else if (gpu && !adapter) {
            kmws_decoder* d = kmws_decoder_create(KMWS_MODE_SERVER, 0);  // per connection, as in kuma
            kmws_rx_batch* b = lo.rx;
            uint8_t* ring = lo.rring;
            if (!d) std::exit(3);
            size_t pos = 0;
            bool closed = false;
            while (!closed && e.got.load(std::memory_order_acquire) < kFrames) {
                // one loop iteration: read until the socket is drained, then one GPU batch
                int flags = 0;
                for (;;) {
                    if (pos + kRead > kRing) break;  // ring full: flush first
                    double t = now_s();
                    const ssize_t r = recv(fd, ring + pos, kRead, flags);
                    T.recv += now_s() - t;
                    if (r == 0) closed = true;
                    if (r <= 0) break;
                    t = now_s();
                    if (kmws_decoder_feed_deferred(d, b, ring + pos, (size_t)r, kmws_cb, &e) < 0) std::exit(4);
                    T.rx_feed += now_s() - t;
                    pos += (size_t)r;
                    flags = MSG_DONTWAIT;
                }
                // throughput policy (argv[4]): keep collecting across iterations until enough
                // bytes are pending, the ring is full, or every frame has been parsed
                if (!closed && pos < kFlushBytes && pos + kRead <= kRing &&
                    e.got.load() + kmws_rx_batch_pending(b) < kFrames)
                    continue;
                const double tf = now_s();
                if (g_submitpoll) {  // the asynchronous pair, waited at once
                    if (kmws_rx_batch_submit(b) < 0 || kmws_rx_batch_poll(b, 1) < 0) std::exit(5);
                } else if (kmws_rx_batch_flush(b) < 0) {
                    std::exit(5);
                }
                T.rx_flush += now_s() - tf;
                pos = 0;  // ring bytes are free again after the flush
            }
            kmws_decoder_destroy(d);
        } else if (adapter) {
            // the loop thread: its RxLoop (posted tasks run once per iteration) and ring
            std::vector<kmws::RxLoop::Task> tasks;
            kmws::RxLoop& rx = *lo.rxloop;
            rx.setPoster([&tasks](kmws::RxLoop::Task t) { tasks.push_back(std::move(t)); });
            kmws::ws::WSHandler h;  // per connection: WebSocket::Impl's ws_handler_
            h.setMode(kmws::ws::WSMode::SERVER);
            h.setRxLoop(&rx);
            h.setFrameCallback([&e](kmws::ws::FrameHeader hdr, kmws::ws::BufferChain& buf) {
                check_frame(&e, static_cast<const uint8_t*>(buf.readPtr()), buf.length(), hdr.opcode);
                return 0;
            });
            uint8_t* ring = lo.rring;
            size_t pos = 0;
            bool closed = false;
            while (e.got.load(std::memory_order_acquire) < kFrames) {
                // one loop iteration: reads until the socket is drained (blocking only
                // when nothing is queued or in flight), then the posted tasks
                const bool busy = !tasks.empty() || rx.inflight() > 0 || rx.pending() > 0;
                int flags = busy || closed ? MSG_DONTWAIT : 0;
                for (;;) {
                    if (pos + kRead > kRing) {  // wrap: ring bytes are free once every frame was delivered
                        const double tf = now_s();
                        if (rx.flush() < 0) std::exit(5);
                        T.rx_flush += now_s() - tf;
                        T.rx_wrap += now_s() - tf;
                        ++T.rx_wraps;
                        pos = 0;
                    }
                    double t = now_s();
                    const ssize_t r = closed ? -1 : recv(fd, ring + pos, kRead, flags);
                    T.recv += now_s() - t;
                    if (r == 0) closed = true;
                    if (r <= 0) break;
                    t = now_s();
                    const kmws::ws::WSError err = h.handleData(ring + pos, (size_t)r);  // onWsData
                    T.rx_feed += now_s() - t;
                    if (err != kmws::ws::WSError::NOERR && err != kmws::ws::WSError::NEED_MORE_DATA) std::exit(4);
                    pos += (size_t)r;
                    flags = MSG_DONTWAIT;
                }
                const double tf = now_s();
                std::vector<kmws::RxLoop::Task> now;
                now.swap(tasks);
                for (auto& t : now) t();
                if (rx.lastResult() < 0) std::exit(5);
                T.rx_flush += now_s() - tf;
                T.rx_task_max = std::max(T.rx_task_max, now_s() - tf);
                T.rx_inflight_max = std::max(T.rx_inflight_max, rx.inflight());
                if (closed && tasks.empty() && rx.inflight() == 0 && rx.pending() == 0) break;
            }
        } else {
            orc_decoder* d = orc_decoder_create(1);
            std::vector<uint8_t> buf(kRead);
            while (e.got.load(std::memory_order_acquire) < kFrames) {
                const ssize_t r = recv(fd, buf.data(), kRead, 0);
                if (r <= 0) break;
                orc_decoder_feed(d, buf.data(), (size_t)r, orc_cb, &e);
            }
            orc_decoder_destroy(d);
        }
        t_end = std::chrono::steady_clock::now();
        T.server_cpu = thread_cpu_s() - sc0;
        if (gpu) kmws_resident_counters(0, &T.server_slot, nullptr, nullptr, nullptr);
        close(fd);
    });

    int fd = socket(AF_INET, SOCK_STREAM, 0);
    if (connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        std::perror("connect");
        std::exit(2);
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    while (!ready) std::this_thread::yield();
    if (gate) {  // several connections at once: every one connected before any sends
        gate->fetch_add(1);
        while (gate->load() < conns) std::this_thread::yield();
    }

    kmws_tx_batch* tx = lo.tx;
    uint8_t* sring = lo.sring;
    std::vector<uint8_t> sbuf;
    // the client's codec (replay modes: none, the wire image is pre-built)
    const bool cgpu = gpu && !g_replay, cadapter = adapter && !g_replay;
    if (!cgpu || g_sync) sbuf.resize(kGroup * kLen);
    std::vector<std::array<uint8_t, KMWS_MAX_HEADER_SIZE>> hdrs(kGroup);
    std::vector<int> hlen(kGroup);
    std::vector<iovec> iov;
    const auto t0 = std::chrono::steady_clock::now();
    const double cc0 = thread_cpu_s();
    rusage ru0{};
    getrusage(RUSAGE_THREAD, &ru0);
    if (g_replay) {
        for (int g0 = 0; g0 < kFrames; g0 += kGroup) {  // one loop iteration: the next kGroup frames' bytes
            const int ng = std::min(kGroup, kFrames - g0);
            std::vector<iovec> one(1, iovec{e.wire.data() + e.frame_off[g0], e.frame_off[g0 + ng] - e.frame_off[g0]});
            const double tt = now_s();
            send_all(fd, one);
            T.writev += now_s() - tt;
        }
    }
    if (cadapter) {
        // the client loop thread: its TxLoop (the posted task masks the
        // iteration's sends with one GPU job and writes finished generations)
        std::vector<kmws::TxLoop::Task> ctasks;
        kmws::TxLoop& txl = *lo.txloop;
        txl.setPoster([&ctasks](kmws::TxLoop::Task t) { ctasks.push_back(std::move(t)); });
        kmws::TxLoop::Conn* conn = txl.open([&](const iovec* v, int cnt) {  // ws_conn_->send(iovs, cnt)
            const double tt = now_s();
            iov.assign(v, v + cnt);
            send_all(fd, iov);
            T.writev += now_s() - tt;
            return 0;
        });
        for (int g0 = 0; g0 < kFrames; g0 += kGroup) {
            // one loop iteration: the application's sends (sendWsFrame), then the posted tasks
            const int ng = std::min(kGroup, kFrames - g0);
            for (int j = 0; j < ng; ++j) {
                const uint32_t key = keys[g0 + j];
                kmws_frame_hdr h;
                std::memset(&h, 0, sizeof h);
                h.fin = 1;
                h.opcode = KMWS_OP_TEXT;
                h.mask = 1;
                std::memcpy(h.maskey, &key, 4);
                const double ts = now_s();
                if (txl.send(conn, h, e.plain.data() + (size_t)(g0 + j) * kLen, kLen) < 0) std::exit(7);
                T.sends += now_s() - ts;
            }
            const double tt = now_s(), w0 = T.writev;
            std::vector<kmws::TxLoop::Task> now;
            now.swap(ctasks);
            for (auto& t : now) t();
            if (txl.lastResult() < 0 || conn->lastResult() < 0) std::exit(7);
            T.tx_flush += now_s() - tt - (T.writev - w0);
        }
        const double tt = now_s(), w0 = T.writev;
        if (txl.close(conn) < 0) std::exit(7);  // the last generations: masked and written
        T.tx_flush += now_s() - tt - (T.writev - w0);
    }
    for (int g0 = 0; g0 < kFrames && !cadapter && !g_replay; g0 += kGroup) {
        const int ng = std::min(kGroup, kFrames - g0);
        uint8_t* base = cgpu && !g_sync ? sring : sbuf.data();
        // the application writes its payloads (the send buffer is reused per iteration)
        std::memcpy(base, e.plain.data() + (size_t)g0 * kLen, (size_t)ng * kLen);
        for (int j = 0; j < ng; ++j) {
            uint8_t* p = base + (size_t)j * kLen;
            const uint32_t key = keys[g0 + j];
            if (g_sync) {  // sendWsFrame with the drop-in's statics (WebSocketImpl.cpp:381-392)
                kmws::ws::FrameHeader h;
                std::memset(static_cast<void*>(&h), 0, sizeof h);
                h.fin = 1;
                h.opcode = KMWS_OP_TEXT;
                h.mask = 1;
                std::memcpy(h.maskey, &key, 4);
                if (kmws::ws::WSHandler::handleDataMask(h.maskey, p, kLen) != KMWS_OK) std::exit(7);
                h.length = (uint32_t)kLen;
                hlen[j] = kmws::ws::WSHandler::encodeFrameHeader(h, hdrs[j].data());
            } else if (cgpu) {
                kmws_frame_hdr h;
                std::memset(&h, 0, sizeof h);
                h.fin = 1;
                h.opcode = KMWS_OP_TEXT;
                h.mask = 1;
                std::memcpy(h.maskey, &key, 4);
                size_t len = kLen;
                hlen[j] = kmws_tx_batch_add(tx, &h, &p, &len, 1, hdrs[j].data());
            } else {  // sendWsFrame: mask in place, then encodeFrameHeader (WebSocketImpl.cpp:405-417)
                orc_hdr h;
                std::memset(&h, 0, sizeof h);
                h.fin = 1;
                h.opcode = 1;
                h.mask = 1;
                std::memcpy(h.maskey, &key, 4);
                orc_mask(h.maskey, p, kLen, 0);
                h.length = (uint32_t)kLen;
                hlen[j] = orc_encode_header(&h, hdrs[j].data());
            }
        }
        double tt = now_s();
        if (cgpu && !g_sync && g_submitpoll) {
            const int64_t tk = kmws_tx_batch_submit(tx);
            if (tk <= 0 || kmws_tx_batch_poll(tx, tk, 1) != 1) std::exit(7);
        } else if (cgpu && !g_sync && kmws_tx_batch_flush(tx) != ng) {
            std::exit(7);
        }
        T.tx_flush += now_s() - tt;
        iov.clear();
        for (int j = 0; j < ng; ++j) {
            iov.push_back(iovec{hdrs[j].data(), (size_t)hlen[j]});
            iov.push_back(iovec{base + (size_t)j * kLen, kLen});
        }
        tt = now_s();
        send_all(fd, iov);
        T.writev += now_s() - tt;
    }
    T.client = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    T.client_cpu = thread_cpu_s() - cc0;
#ifdef KMWS_PROF
    std::fprintf(stderr, "{\"place_ms\": %.3f, \"copy_ms\": %.3f, \"add_ms\": %.3f, \"push_ms\": %.3f, \"arm_ms\": %.3f, \"waits\": %ld}\n",
                 kmws::t_txprof.place * 1e3, kmws::t_txprof.copy * 1e3, kmws::t_txprof.add * 1e3, kmws::t_txprof.push * 1e3,
                 kmws::t_txprof.arm * 1e3, kmws::t_txprof.waits);
    kmws::t_txprof = kmws::TxProf();
#endif
    rusage ru1{};
    getrusage(RUSAGE_THREAD, &ru1);
    T.client_nivcsw = ru1.ru_nivcsw - ru0.ru_nivcsw;
    if (cgpu) kmws_resident_counters(0, &T.client_slot, nullptr, nullptr, nullptr);
    server.join();
    close(fd);
    close(ls);
    T.t0 = std::chrono::duration<double>(t0.time_since_epoch()).count();
    T.t_end = std::chrono::duration<double>(t_end.time_since_epoch()).count();
    return std::chrono::duration<double>(t_end - t0).count();
}

}  // namespace

int main(int argc, char** argv)
{
    const std::string mode = argc > 1 ? argv[1] : "cpu";
    const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
    if (argc > 3) kGroup = std::max(1, std::atoi(argv[3]));
    if (argc > 4) kFlushBytes = (size_t)std::atoll(argv[4]);
    g_noresident = argc > 5 && std::string(argv[5]) == "noresident";
    g_submitpoll = argc > 5 && std::string(argv[5]) == "submitpoll";
    if (argc > 5 && std::string(argv[5]) == "inflight2") g_inflight = 2;
    if (argc > 5 && std::string(argv[5]) == "ring16m") g_tx_ring = (size_t)16 << 20;
    const int conns = argc > 6 ? std::max(1, std::min(8, std::atoi(argv[6]))) : 1;
    if (g_noresident) kmws_resident_enable(0, 0);  // the client (main) thread
    g_replay = mode == "replay_cpu" || mode == "replay_adapter";
    g_sink = mode == "sink_cpu" || mode == "sink_adapter";
    const bool adapter = mode == "adapter" || mode == "replay_adapter" || mode == "sink_adapter";
    g_sync = mode == "sync";
    const bool gpu = mode == "gpu" || adapter || g_sync;
    if (gpu && kmws_device_count() < 1) {
        std::printf("{\"mode\": \"gpu\", \"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    std::vector<uint8_t> plain((size_t)kFrames * kLen);
    for (size_t i = 0; i < plain.size(); ++i) plain[i] = (uint8_t)(0x20 + splitmix(i) % 95);
    std::vector<uint32_t> keys(kFrames);
    for (int i = 0; i < kFrames; ++i) keys[i] = (uint32_t)splitmix(0x6b756d61ull + i);
    // one client and one server loop thread per connection, each pair with its own
    // long-lived loop objects (kuma runs several loop threads, each with its connections)
    std::vector<Expect> es(conns);
    std::vector<LoopObjs> los(conns);
    std::vector<Times> ts(conns);
    std::vector<uint8_t> wire;  // the masked wire image the replay clients send
    std::vector<size_t> frame_off;
    if (g_replay || g_sink) {
        for (int f = 0; f < kFrames; ++f) {
            frame_off.push_back(wire.size());
            orc_hdr h;
            std::memset(&h, 0, sizeof h);
            h.fin = 1;
            h.opcode = 1;
            h.mask = 1;
            std::memcpy(h.maskey, &keys[f], 4);
            h.length = (uint32_t)kLen;
            uint8_t hb[14];
            const int hl = orc_encode_header(&h, hb);
            wire.insert(wire.end(), hb, hb + hl);
            const size_t p0 = wire.size();
            wire.insert(wire.end(), plain.begin() + (size_t)f * kLen, plain.begin() + (size_t)(f + 1) * kLen);
            orc_mask(h.maskey, wire.data() + p0, kLen, 0);
        }
        frame_off.push_back(wire.size());
    }
    for (int c = 0; c < conns; ++c) {
        es[c].plain = plain;
        es[c].wire = wire;
        es[c].frame_off = frame_off;
        if (!gpu) continue;
        LoopObjs& lo = los[c];
        lo.rx = kmws_rx_batch_create(0);
        lo.rring = static_cast<uint8_t*>(kmws_host_alloc(kRing, 0));
        lo.tx = kmws_tx_batch_create(0);
        lo.sring = static_cast<uint8_t*>(kmws_host_alloc((size_t)2 * kGroup * kLen, 0));  // 2 slots (adapter)
        if (!lo.rx || !lo.rring || !lo.tx || !lo.sring || kmws_tx_batch_attach_ring(lo.tx, lo.sring, (size_t)2 * kGroup * kLen) != KMWS_OK)
            return 3;
        if (adapter) {
            lo.rxloop = new kmws::RxLoop(nullptr, 0);
            if (!lo.rxloop->valid() || lo.rxloop->attachRing(lo.rring, kRing) != KMWS_OK) return 3;
            lo.txloop = new kmws::TxLoop(nullptr, 0, g_tx_ring, g_inflight);
            if (!lo.txloop->valid()) return 3;
        } else if (kmws_rx_batch_attach_ring(lo.rx, lo.rring, kRing) != KMWS_OK) {
            return 3;
        }
    }
    double best = 1e9, best_cpu = 0, best_wall = 0;
    // the best rep's connections, ms: [start offset, span, client, tx_flush, writev, server recv, rx_flush,
    // sends (adapter), client thread CPU, server thread CPU, client involuntary switches, client slot, server slot]
    std::string spans = "[]";
    bool ok = true;
    for (int r = 0; r < reps + 1; ++r) {  // first round of connections warms up (staging growth, GPU context)
        double t = 0;
        const double c0 = cpu_s(), w0 = now_s();
        if (conns == 1) {
            t = run_once(gpu, adapter, es[0], keys, los[0], ts[0]);
        } else {
            std::atomic<int> gate{0};
            std::vector<std::thread> th;
            for (int c = 0; c < conns; ++c)
                th.emplace_back([&, c] {
                    if (g_noresident) kmws_resident_enable(0, 0);  // this client thread
                    run_once(gpu, adapter, es[c], keys, los[c], ts[c], &gate, conns);
                });
            for (auto& x : th) x.join();
            double t0 = 1e30, t1 = 0;  // the first send of any connection to the last frame of any
            for (const Times& x : ts) {
                t0 = std::min(t0, x.t0);
                t1 = std::max(t1, x.t_end);
            }
            t = t1 - t0;
        }
        for (const Expect& x : es) ok = ok && x.got.load() == kFrames && x.bad.load() == 0;
        if (r && t < best) {
            best = t;
            best_cpu = cpu_s() - c0;  // the whole rep: connection set-up and thread start included
            best_wall = now_s() - w0;
            double t0 = 1e30;
            for (const Times& x : ts) t0 = std::min(t0, x.t0);
            spans = "[";
            for (size_t c = 0; c < ts.size(); ++c) {
                char b[240];
                std::snprintf(b, sizeof b, "%s[%.3f, %.3f, %.3f, %.3f, %.3f, %.3f, %.3f, %.3f, %.3f, %.3f, %ld, %d, %d]",
                              c ? ", " : "", (ts[c].t0 - t0) * 1e3, (ts[c].t_end - ts[c].t0) * 1e3, ts[c].client * 1e3,
                              ts[c].tx_flush * 1e3, ts[c].writev * 1e3, ts[c].recv * 1e3, ts[c].rx_flush * 1e3,
                              ts[c].sends * 1e3, ts[c].client_cpu * 1e3, ts[c].server_cpu * 1e3, ts[c].client_nivcsw,
                              ts[c].client_slot, ts[c].server_slot);
                spans += b;
            }
            spans += "]";
        }
    }
    if (gpu) {
        for (LoopObjs& lo : los) {
            delete lo.rxloop;
            delete lo.txloop;
            kmws_rx_batch_destroy(lo.rx);
            kmws_tx_batch_destroy(lo.tx);
            kmws_host_free(lo.rring);
            kmws_host_free(lo.sring);
        }
    }
    const Times& g = ts[0];
    const double bytes = (double)kFrames * kLen * conns;
    std::printf("{\"mode\": \"%s\", \"connections\": %d, \"frames\": %d, \"frame_len\": %zu, \"frames_per_send_iteration\": %d, "
                "\"rx_flush_bytes\": %zu, \"best_of\": %d, \"GiB_s\": %.3f, \"us_per_frame\": %.3f, "
                "\"cpu_cores_busy\": %.2f, \"cpu_ms_per_MiB\": %.4f, \"connection_start_span_ms\": %s, "
                "\"verified\": %s, \"breakdown_ms_last_connection\": {\"client_total\": %.3f, "
                "\"tx_flush\": %.3f, \"writev\": %.3f, \"server_recv\": %.3f, \"rx_feed\": %.3f, "
                "\"rx_flush\": %.3f, \"rx_task_max\": %.3f, \"rx_wrap_flush\": %.3f, \"rx_wraps\": %d, \"rx_inflight_max\": %d}}\n",
                mode.c_str(), conns, kFrames, kLen, kGroup, kFlushBytes, reps, bytes / best / (1u << 30),
                best / (kFrames * conns) * 1e6, best_wall > 0 ? best_cpu / best_wall : 0.0,
                best_cpu * 1e3 / (bytes / (1 << 20)), spans.c_str(), ok ? "true" : "false", g.client * 1e3, g.tx_flush * 1e3, g.writev * 1e3,
                g.recv * 1e3, g.rx_feed * 1e3, g.rx_flush * 1e3, g.rx_task_max * 1e3, g.rx_wrap * 1e3,
                g.rx_wraps, g.rx_inflight_max);
    return ok ? 0 : 1;
}
