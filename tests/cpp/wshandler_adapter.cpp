// Drives include/kmws_wshandler.hpp the way kuma's WebSocket::Impl drives
// WSHandler (src/ws/WebSocketImpl.cpp:152-246, 381-436), with the standalone
// kmws::ws types.  Expected bytes are RFC 6455 sec.5.7 frames and the
// reference outputs recorded in SURVEY.md sec.8 (tests/golden/reference_vectors.json).
//
// usage: wshandler_adapter          host-only checks (no GPU needed)
//        wshandler_adapter gpu      + masked paths on the GPU
//        wshandler_adapter nogpu    + masked paths must fail loudly (no device)
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <string>
#include <vector>

#include "kmws_wshandler.hpp"

using kmws::ws::BufferChain;
using kmws::ws::FrameHeader;
using kmws::ws::WSError;
using kmws::ws::WSHandler;
using kmws::ws::WSMode;

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);   \
            ++g_fail;                                                   \
        }                                                               \
    } while (0)

static std::vector<uint8_t> hex(const char* s)
{
    std::vector<uint8_t> v;
    for (; s[0] && s[1]; s += 2) {
        while (*s == ' ') ++s;
        unsigned b = 0;
        std::sscanf(s, "%2x", &b);
        v.push_back((uint8_t)b);
    }
    return v;
}

struct Rec {
    int fin, rsv1, opcode, mask;
    uint32_t length;
    std::string payload;
};

static void collect(WSHandler& h, std::vector<Rec>& out)
{
    h.setFrameCallback([&out](FrameHeader hdr, BufferChain& buf) {
        out.push_back(Rec{hdr.fin, hdr.rsv1, hdr.opcode, hdr.mask, hdr.length,
                          std::string(static_cast<const char*>(buf.readPtr()), buf.length())});
        return 0;
    });
}

static FrameHeader make_hdr(int fin, int rsv1, int opcode, int mask, uint32_t len, const uint8_t key[4])
{
    FrameHeader h;
    std::memset(static_cast<void*>(&h), 0, sizeof(h));
    h.fin = fin;
    h.rsv1 = rsv1;
    h.opcode = opcode;
    h.mask = mask;
    h.length = len;
    if (key) std::memcpy(h.maskey, key, 4);
    return h;
}

static void host_checks()
{
    // encodeFrameHeader: SURVEY.md sec.8 a-4 vectors
    const uint8_t k[4] = {0xde, 0xad, 0xbe, 0xef};
    uint8_t out[14];
    int n = WSHandler::encodeFrameHeader(make_hdr(1, 1, 2, 1, 65536, k), out);
    CHECK(n == 14 && std::vector<uint8_t>(out, out + n) == hex("c2ff0000000000010000deadbeef"));
    n = WSHandler::encodeFrameHeader(make_hdr(1, 1, 2, 1, 126, k), out);
    CHECK(n == 8 && std::vector<uint8_t>(out, out + n) == hex("c2fe007edeadbeef"));
    n = WSHandler::encodeFrameHeader(make_hdr(1, 0, 1, 0, 5, nullptr), out);
    CHECK(n == 2 && out[0] == 0x81 && out[1] == 0x05);
    CHECK(WSHandler::isControlFrame(8) && WSHandler::isControlFrame(11) && !WSHandler::isControlFrame(2));

    // CLIENT mode, unmasked server frames (RFC 6455 sec.5.7): no GPU involved
    {
        WSHandler h;
        CHECK(h.valid());
        std::vector<Rec> got;
        collect(h, got);
        CHECK(h.getMode() == WSMode::CLIENT);
        std::vector<uint8_t> w = hex("810548656c6c6f");
        std::vector<int> rets;
        for (size_t i = 0; i < w.size(); ++i) rets.push_back((int)h.handleData(&w[i], 1));  // byte at a time
        CHECK(rets == std::vector<int>({1, 1, 1, 1, 1, 1, 0}));
        CHECK(got.size() == 1 && got[0].payload == "Hello" && got[0].opcode == 1 && got[0].fin == 1);
        std::vector<uint8_t> f = hex("010348656c80026c6f");  // fragmented "Hel" + "lo"
        CHECK(h.handleData(f.data(), f.size()) == WSError::NOERR);
        CHECK(got.size() == 3 && got[1].payload == "Hel" && got[1].fin == 0 && got[1].opcode == 1 &&
              got[2].payload == "lo" && got[2].fin == 1 && got[2].opcode == 0);
        // masked frame in CLIENT mode: PROTOCOL_ERROR (WSHandler.cpp:207-229), then INVALID_FRAME
        std::vector<uint8_t> m = hex("818537fa213d7f9f4d5158");
        CHECK(h.handleData(m.data(), m.size()) == WSError::PROTOCOL_ERROR);
        CHECK(h.handleData(w.data(), w.size()) == WSError::INVALID_FRAME);
        h.reset();
        CHECK(h.handleData(w.data(), w.size()) == WSError::NOERR);
        CHECK(got.size() == 4 && got[3].payload == "Hello");
    }
    // the callback destroys its handler (DestroyDetector, WSHandler.cpp:284-287)
    {
        WSHandler* h = new WSHandler();
        int calls = 0;
        h->setFrameCallback([&](FrameHeader, BufferChain&) {
            ++calls;
            delete h;
            h = nullptr;
            return 0;
        });
        std::vector<uint8_t> w = hex("810548656c6c6f810548656c6c6f");  // two frames in one read
        WSHandler* self = h;
        CHECK(self->handleData(w.data(), w.size()) == WSError::DESTROYED);
        CHECK(calls == 1 && h == nullptr);
    }
    // CLOSE: delivered, then CLOSED; trailing bytes not parsed (WSHandler.cpp:262-268)
    {
        WSHandler h;
        std::vector<Rec> got;
        collect(h, got);
        std::vector<uint8_t> w = hex("880203e8810548656c6c6f");
        CHECK(h.handleData(w.data(), w.size()) == WSError::CLOSED);
        CHECK(got.size() == 1 && got[0].opcode == 8);
    }
    // an empty chain / empty buffer is a no-op (WSHandler.cpp:305)
    {
        BufferChain empty;
        CHECK(WSHandler::handleDataMask(k, empty) == KMWS_OK);
        CHECK(WSHandler::handleDataMask(k, nullptr, 0) == KMWS_OK);
    }
}

// WebSocket::Impl::send (WebSocketImpl.cpp:152-212) + sendWsFrame (:381-404) in
// CLIENT mode: opcode rule, mask the caller's buffer in place, header, iovec
// order -> one wire image.
struct Sender {
    bool fragmented = false;
    std::vector<uint8_t> wire;
    int send(uint8_t* data, size_t len, bool is_text, bool is_fin, const uint8_t key[4])
    {
        const int op = fragmented ? 0 : (is_text ? 1 : 2);
        fragmented = !is_fin;
        FrameHeader h = make_hdr(is_fin, 0, op, len > 0, (uint32_t)len, len > 0 ? key : nullptr);
        if (len > 0 && WSHandler::handleDataMask(h.maskey, data, len) != KMWS_OK) return -1;
        uint8_t hb[14];
        const int n = WSHandler::encodeFrameHeader(h, hb);
        wire.insert(wire.end(), hb, hb + n);
        wire.insert(wire.end(), data, data + len);
        return (int)len;
    }
};

static void gpu_checks()
{
    // SERVER mode, masked "Hello" (RFC 6455 sec.5.7), unmasked in place
    {
        WSHandler h;
        h.setMode(WSMode::SERVER);
        std::vector<Rec> got;
        collect(h, got);
        std::vector<uint8_t> m = hex("818537fa213d7f9f4d5158");
        CHECK(h.handleData(m.data(), m.size()) == WSError::NOERR);
        CHECK(got.size() == 1 && got[0].payload == "Hello" && got[0].mask == 1);
        CHECK(std::memcmp(m.data() + 6, "Hello", 5) == 0);  // in place, as kuma
    }
    // handleDataMask over a chain: SURVEY.md sec.8 a-2 vector
    {
        uint8_t a[3] = {0, 0, 0}, b[5] = {0, 0, 0, 0, 0};
        const uint8_t key[4] = {1, 2, 3, 4};
        BufferChain c(a, 3, 3);
        c.append(b, 5);
        CHECK(WSHandler::handleDataMask(key, c) == KMWS_OK);
        uint8_t both[8];
        std::memcpy(both, a, 3);
        std::memcpy(both + 3, b, 5);
        // the phase continues across segments: bytes 0..7 = key[i % 4]
        const uint8_t want[8] = {1, 2, 3, 4, 1, 2, 3, 4};
        CHECK(std::memcmp(both, want, 8) == 0);
    }
    // a client sends a 16-fragment message (cfg4 shape, a-12), a server decodes it
    {
        Sender tx;
        std::vector<std::string> sent;
        for (int i = 0; i < 16; ++i) {
            std::string frag(4096 + i, 'a' + i);
            sent.push_back(frag);
            std::vector<uint8_t> buf(frag.begin(), frag.end());
            const uint8_t key[4] = {(uint8_t)(0x10 + i), 0x77, (uint8_t)(0x30 ^ i), 0xC5};
            CHECK(tx.send(buf.data(), buf.size(), true, i == 15, key) == (int)buf.size());
            CHECK(buf[0] != (uint8_t)('a' + i) || key[0] == 0);  // the caller's buffer is left masked
        }
        WSHandler rx;
        rx.setMode(WSMode::SERVER);
        std::vector<Rec> got;
        collect(rx, got);
        for (size_t p = 0; p < tx.wire.size(); p += 65536) {  // 64 KiB socket reads
            const size_t len = tx.wire.size() - p < 65536 ? tx.wire.size() - p : 65536;
            const WSError r = rx.handleData(tx.wire.data() + p, len);
            CHECK(r == WSError::NOERR || r == WSError::NEED_MORE_DATA);
        }
        CHECK(got.size() == 16);
        for (size_t i = 0; i < got.size() && i < 16; ++i) {
            CHECK(got[i].payload == sent[i]);
            CHECK(got[i].opcode == (i == 0 ? 1 : 0) && got[i].fin == (i == 15 ? 1 : 0) && got[i].mask == 1);
        }
    }
}

// A minimal event loop: EventLoop::post appends a task, every iteration runs
// the tasks queued before it (kmapi.h:204-210 "run the task at next time").
struct FakeLoop {
    std::deque<std::function<void()>> tasks;
    kmws::RxLoop::Poster poster()
    {
        return [this](kmws::RxLoop::Task t) { tasks.push_back(std::move(t)); };
    }
    int iterate()
    {
        std::deque<std::function<void()>> now;
        now.swap(tasks);
        for (auto& t : now) t();
        return (int)now.size();
    }
};

static std::vector<uint8_t> masked_frame(int opcode, const std::string& payload, const uint8_t key[4], int fin = 1)
{
    std::vector<uint8_t> data(payload.begin(), payload.end());
    FrameHeader h = make_hdr(fin, 0, opcode, 1, (uint32_t)data.size(), key);
    uint8_t hb[14];
    const int n = WSHandler::encodeFrameHeader(h, hb);
    for (size_t i = 0; i < data.size(); ++i) data[i] ^= key[i % 4];
    std::vector<uint8_t> w(hb, hb + n);
    w.insert(w.end(), data.begin(), data.end());
    return w;
}

// Batched mode: two connections on one loop, frames queued by handleData,
// delivered by the loop's posted task (asynchronously: submit, then poll at
// the next iterations), in order per connection; CLOSE and errors deliver
// everything queued before handleData returns; a handler deleted by its own
// callback during deferred delivery stops its delivery.
static void batched_checks(bool async)
{
    FakeLoop loop;
    kmws::RxLoop rx(loop.poster(), 0, async);
    CHECK(rx.valid());
    WSHandler a, b;
    a.setMode(WSMode::SERVER);
    b.setMode(WSMode::SERVER);
    a.setRxLoop(&rx);
    b.setRxLoop(&rx);
    std::vector<Rec> ga, gb;
    collect(a, ga);
    collect(b, gb);
    std::vector<std::string> sa, sb;
    for (int it = 0; it < 6; ++it) {  // 6 loop iterations of reads on both connections
        std::vector<uint8_t> wa, wb;
        for (int j = 0; j < 3; ++j) {
            const uint8_t key[4] = {(uint8_t)(it * 7 + j), 0x5a, (uint8_t)(j + 1), 0x0f};
            std::string pa(100 + 517 * j + it, (char)('A' + (it + j) % 26));
            std::string pb(3000 + j, (char)('a' + (it * 3 + j) % 26));
            sa.push_back(pa);
            sb.push_back(pb);
            std::vector<uint8_t> fa = masked_frame(2, pa, key), fb = masked_frame(1, pb, key);
            wa.insert(wa.end(), fa.begin(), fa.end());
            wb.insert(wb.end(), fb.begin(), fb.end());
        }
        // reads cut mid-frame: the decoder reassembles across reads
        const size_t cut = wa.size() / 2 + 3;
        CHECK(a.handleData(wa.data(), cut) == WSError::NEED_MORE_DATA);
        CHECK(b.handleData(wb.data(), wb.size()) == WSError::NOERR);
        CHECK(a.handleData(wa.data() + cut, wa.size() - cut) == WSError::NOERR);
        loop.iterate();
    }
    for (int spin = 0; spin < 100000 && (rx.inflight() || rx.pending() || !loop.tasks.empty()); ++spin) loop.iterate();
    CHECK(ga.size() == sa.size() && gb.size() == sb.size());
    for (size_t i = 0; i < ga.size() && i < sa.size(); ++i) CHECK(ga[i].payload == sa[i] && ga[i].opcode == 2);
    for (size_t i = 0; i < gb.size() && i < sb.size(); ++i) CHECK(gb[i].payload == sb[i] && gb[i].opcode == 1);

    // CLOSE on a: everything queued (b's frame too) is delivered before handleData returns CLOSED
    {
        const uint8_t key[4] = {9, 8, 7, 6};
        std::vector<uint8_t> fb = masked_frame(2, std::string(777, 'q'), key);
        CHECK(b.handleData(fb.data(), fb.size()) == WSError::NOERR);
        std::vector<uint8_t> fa = masked_frame(1, "bye?", key);
        std::vector<uint8_t> cl = masked_frame(8, std::string("\x03\xe8", 2), key);
        fa.insert(fa.end(), cl.begin(), cl.end());
        const size_t na = ga.size(), nb = gb.size();
        CHECK(a.handleData(fa.data(), fa.size()) == WSError::CLOSED);
        CHECK(ga.size() == na + 2 && ga[na].payload == "bye?" && ga[na + 1].opcode == 8);
        CHECK(gb.size() == nb + 1 && gb[nb].payload == std::string(777, 'q'));
    }
    // a decode error: the frames before it are delivered first, then the error returns
    {
        const uint8_t key[4] = {1, 1, 2, 3};
        std::vector<uint8_t> w = masked_frame(2, "first", key);
        w.push_back(0x09);  // PING without FIN: PROTOCOL_ERROR (WSHandler.cpp:120-130)
        w.push_back(0x80);
        const size_t nb = gb.size();
        CHECK(b.handleData(w.data(), w.size()) == WSError::PROTOCOL_ERROR);
        CHECK(gb.size() == nb + 1 && gb[nb].payload == "first");
    }
    // a handler deleted by its own callback during deferred delivery
    {
        WSHandler* h = new WSHandler();
        h->setMode(WSMode::SERVER);
        h->setRxLoop(&rx);
        int calls = 0;
        h->setFrameCallback([&](FrameHeader, BufferChain&) {
            ++calls;
            delete h;
            h = nullptr;
            return 0;
        });
        const uint8_t key[4] = {4, 3, 2, 1};
        std::vector<uint8_t> w = masked_frame(2, "one", key), w2 = masked_frame(2, "two", key);
        w.insert(w.end(), w2.begin(), w2.end());
        CHECK(h->handleData(w.data(), w.size()) == WSError::NOERR);
        for (int spin = 0; spin < 100000 && (rx.inflight() || rx.pending() || !loop.tasks.empty()); ++spin)
            loop.iterate();
        CHECK(calls == 1 && h == nullptr);
    }
    // a handler destroyed while its frames are queued: they are dropped, nothing touches it
    {
        WSHandler* h = new WSHandler();
        h->setMode(WSMode::SERVER);
        h->setRxLoop(&rx);
        int calls = 0;
        h->setFrameCallback([&](FrameHeader, BufferChain&) {
            ++calls;
            return 0;
        });
        const uint8_t key[4] = {4, 3, 2, 1};
        std::vector<uint8_t> w = masked_frame(2, "dropped", key);
        CHECK(h->handleData(w.data(), w.size()) == WSError::NOERR);
        delete h;
        for (int spin = 0; spin < 100000 && (rx.inflight() || rx.pending() || !loop.tasks.empty()); ++spin)
            loop.iterate();
        CHECK(calls == 0);
    }
}

static void nogpu_checks()
{
    {  // batched mode needs a device: the loop object is invalid and handlers stay synchronous
        FakeLoop loop;
        kmws::RxLoop rx(loop.poster(), 0);
        CHECK(!rx.valid());
        WSHandler h;
        h.setRxLoop(&rx);
        CHECK(h.rxLoop() == nullptr);
    }
    WSHandler h;
    h.setMode(WSMode::SERVER);
    std::vector<Rec> got;
    collect(h, got);
    std::vector<uint8_t> m = hex("818537fa213d7f9f4d5158");
    CHECK(h.handleData(m.data(), m.size()) == WSError::INVALID_STATE);
    CHECK(h.lastStatus() == KMWS_ERR_NOT_SUPPORTED && got.empty());
    uint8_t b[4] = {0, 0, 0, 0};
    const uint8_t key[4] = {1, 2, 3, 4};
    CHECK(WSHandler::handleDataMask(key, b, 4) == KMWS_ERR_NOT_SUPPORTED);
}

int main(int argc, char** argv)
{
    host_checks();
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "gpu") {
        gpu_checks();
        batched_checks(true);
        batched_checks(false);
    }
    if (mode == "nogpu") nogpu_checks();
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK\n");
    return 0;
}
