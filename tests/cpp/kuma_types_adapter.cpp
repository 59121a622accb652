// The C++ drop-in (include/kmws_wshandler.hpp) instantiated with kuma's OWN
// types -- kuma::ws::FrameHeader / WSError / WSMode (src/ws/wsdefs.h:56-88),
// kuma::KMBuffer (include/kmbuffer.h:183-784) and kuma::KMError
// (include/kmdefs.h:61-86) -- exactly as INTEGRATION.md sec.3 aliases it, and
// driven the way WebSocket::Impl drives ws::WSHandler (WebSocketImpl.cpp:56-60,
// 225-246, 381-436).  Built only in the container that holds the reference
// checkout (tests/test_kuma_types.py); nothing of it travels to the GPU box.
//
// Needs no GPU: CLIENT-mode decoding of unmasked frames touches no kernel; the
// masked paths must fail loudly without a device (no CPU fallback).
#include "kmbuffer.h"  // a build-directory copy with the one-token createSharedData fix
#include "kmdefs.h"
#include "wsdefs.h"

#include "kmws_wshandler.hpp"

#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

using namespace kuma;
using namespace kuma::ws;

// the one type WebSocket::Impl swaps (WebSocketImpl.h:140)
using KmwsHandler = kmws::BasicWSHandler<ws::FrameHeader, KMBuffer, ws::WSError, ws::WSMode, KMError>;

static_assert(std::is_same<KmwsHandler::FrameCallback, std::function<KMError(FrameHeader, KMBuffer&)>>::value,
              "FrameCallback is WSHandler::FrameCallback (WSHandler.h:35)");
static_assert(std::is_same<decltype(std::declval<KmwsHandler&>().handleData(nullptr, 0)), WSError>::value,
              "handleData returns kuma's WSError");
static_assert(std::is_same<decltype(std::declval<KmwsHandler&>().getMode()), WSMode>::value, "getMode");

static int g_fail = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                 \
        }                                                             \
    } while (0)

static std::vector<uint8_t> hex(const char* s)
{
    std::vector<uint8_t> v;
    for (; s[0] && s[1]; s += 2) {
        unsigned b = 0;
        std::sscanf(s, "%2x", &b);
        v.push_back((uint8_t)b);
    }
    return v;
}

struct Got {
    FrameHeader hdr;
    std::string payload;
    size_t chain_len;
};

int main()
{
    // encodeFrameHeader with kuma's bitfield FrameHeader (SURVEY 8 a-4 vectors)
    {
        FrameHeader h;
        std::memset(static_cast<void*>(&h), 0, sizeof(h));
        h.fin = 1;
        h.rsv1 = 1;
        h.opcode = (uint8_t)WSOpcode::BINARY;
        h.mask = 1;
        h.length = 65536;
        const uint8_t key[4] = {0xde, 0xad, 0xbe, 0xef};
        std::memcpy(h.maskey, key, 4);
        uint8_t out[WS_MAX_HEADER_SIZE];
        KmwsHandler handler;
        int n = handler.encodeFrameHeader(h, out);  // called on the member, as WebSocketImpl.cpp:391
        CHECK(n == 14 && std::vector<uint8_t>(out, out + n) == hex("c2ff0000000000010000deadbeef"));
        h.length = 126;
        n = KmwsHandler::encodeFrameHeader(h, out);
        CHECK(n == 8 && std::vector<uint8_t>(out, out + n) == hex("c2fe007edeadbeef"));
        CHECK(KmwsHandler::isControlFrame((uint8_t)WSOpcode::PING) && !KmwsHandler::isControlFrame(2));
    }
    // CLIENT mode (WebSocketImpl.cpp:101): unmasked server frames, RFC 6455 sec.5.7,
    // with WebSocket::Impl's callback shape (WebSocketImpl.cpp:58-60)
    {
        KmwsHandler h;
        h.setMode(WSMode::CLIENT);
        std::vector<Got> got;
        h.setFrameCallback([&got](ws::FrameHeader hdr, KMBuffer& buf) {
            got.push_back(Got{hdr, std::string(static_cast<const char*>(buf.readPtr()), buf.length()),
                              buf.chainLength()});
            return KMError::NOERR;
        });
        CHECK(h.getMode() == WSMode::CLIENT);
        std::vector<uint8_t> w = hex("810548656c6c6f");
        std::vector<int> rets;
        for (size_t i = 0; i < w.size(); ++i) rets.push_back((int)h.handleData(&w[i], 1));
        CHECK(rets == std::vector<int>({1, 1, 1, 1, 1, 1, 0}));
        CHECK(got.size() == 1 && got[0].payload == "Hello" && got[0].chain_len == 5);
        CHECK(got.size() == 1 && got[0].hdr.fin == 1 && got[0].hdr.opcode == 1 && got[0].hdr.length == 5 &&
              got[0].hdr.plen == 5 && got[0].hdr.mask == 0);
        // fragmented "Hel" + "lo", and a 256-byte binary frame (16-bit length, xpl16)
        std::vector<uint8_t> f = hex("010348656c80026c6f");
        std::vector<uint8_t> big = hex("827e0100");
        for (int i = 0; i < 256; ++i) big.push_back((uint8_t)i);
        f.insert(f.end(), big.begin(), big.end());
        CHECK(h.handleData(f.data(), f.size()) == WSError::NOERR);
        CHECK(got.size() == 4 && got[1].payload == "Hel" && got[1].hdr.fin == 0 && got[2].payload == "lo" &&
              got[2].hdr.opcode == 0 && got[3].hdr.plen == 126 && got[3].hdr.xpl.xpl16 == 256 &&
              got[3].hdr.length == 256 && got[3].payload.size() == 256 && (uint8_t)got[3].payload[255] == 255);
        // a masked frame in CLIENT mode is a protocol error (WSHandler.cpp:207-229)
        std::vector<uint8_t> m = hex("818537fa213d7f9f4d5158");
        CHECK(h.handleData(m.data(), m.size()) == WSError::PROTOCOL_ERROR);
        CHECK(h.handleData(w.data(), w.size()) == WSError::INVALID_FRAME);
        h.reset();
        CHECK(h.handleData(w.data(), w.size()) == WSError::NOERR && got.size() == 5);
    }
    // CLOSE delivered, then CLOSED (WSHandler.cpp:262-268)
    {
        KmwsHandler h;
        int closes = 0;
        h.setFrameCallback([&closes](FrameHeader hdr, KMBuffer&) {
            closes += hdr.opcode == (uint8_t)WSOpcode::CLOSE;
            return KMError::NOERR;
        });
        std::vector<uint8_t> w = hex("880203e8810548656c6c6f");
        CHECK(h.handleData(w.data(), w.size()) == WSError::CLOSED && closes == 1);
    }
    // the callback destroys its owner (DestroyDetector, WSHandler.cpp:284-287)
    {
        KmwsHandler* h = new KmwsHandler();
        int calls = 0;
        h->setFrameCallback([&](FrameHeader, KMBuffer&) {
            ++calls;
            delete h;
            h = nullptr;
            return KMError::NOERR;
        });
        std::vector<uint8_t> w = hex("810548656c6c6f810548656c6c6f");
        KmwsHandler* self = h;
        CHECK(self->handleData(w.data(), w.size()) == WSError::DESTROYED && calls == 1 && h == nullptr);
    }
    // handleDataMask(key, KMBuffer&) over a real 2-segment chain (a-2, WebSocketImpl.cpp:414):
    // the adapter walks kuma's circular chain with its const Iterator (kmbuffer.h:706-772)
    {
        uint8_t s1[3] = {0, 0, 0}, s2[5] = {0, 0, 0, 0, 0};
        KMBuffer tail(s2, sizeof s2, sizeof s2);
        KMBuffer head(s1, sizeof s1, sizeof s1);
        head.append(&tail);
        CHECK(head.chainLength() == 8);
        std::vector<uint8_t*> segs;
        std::vector<size_t> lens;
        KmwsHandler::collectSegments(head, segs, lens);
        CHECK(segs.size() == 2 && segs[0] == s1 && segs[1] == s2 && lens[0] == 3 && lens[1] == 5);
        const uint8_t key[4] = {1, 2, 3, 4};
        const int r = KmwsHandler::handleDataMask(key, const_cast<KMBuffer&>(static_cast<const KMBuffer&>(head)));
        if (kmws_device_count() == 0) {
            CHECK(r == KMWS_ERR_NOT_SUPPORTED);  // no CPU fallback
            CHECK(s1[0] == 0 && s2[4] == 0);       // untouched
        } else {
            const uint8_t want[8] = {1, 2, 3, 4, 1, 2, 3, 4};  // phase continues across segments
            CHECK(r == KMWS_OK && std::memcmp(s1, want, 3) == 0 && std::memcmp(s2, want + 3, 5) == 0);
        }
        // the (data, len) form the send path uses (WebSocketImpl.cpp:388)
        uint8_t one[4] = {0, 0, 0, 0};
        const int r1 = KmwsHandler::handleDataMask(key, one, sizeof one);
        CHECK(kmws_device_count() == 0 ? r1 == KMWS_ERR_NOT_SUPPORTED : (r1 == KMWS_OK && one[3] == 4));
    }
    // SERVER mode masked frame: the GPU unmask, or a loud failure without a device
    {
        KmwsHandler h;
        h.setMode(WSMode::SERVER);
        std::string payload;
        h.setFrameCallback([&payload](FrameHeader, KMBuffer& buf) {
            payload.assign(static_cast<const char*>(buf.readPtr()), buf.length());
            return KMError::NOERR;
        });
        std::vector<uint8_t> m = hex("818537fa213d7f9f4d5158");
        const WSError r = h.handleData(m.data(), m.size());
        if (kmws_device_count() == 0)
            CHECK(r == WSError::INVALID_STATE && h.lastStatus() == (int)KMError::NOT_SUPPORTED && payload.empty());
        else
            CHECK(r == WSError::NOERR && payload == "Hello");
    }
    // batched mode with kuma's loop shape: without a device the RxLoop is invalid
    // and the handler stays synchronous
    {
        std::vector<kmws::RxLoop::Task> tasks;
        kmws::RxLoop loop([&tasks](kmws::RxLoop::Task t) { tasks.push_back(std::move(t)); });
        KmwsHandler h;
        h.setRxLoop(&loop);
        CHECK(loop.valid() == (kmws_device_count() > 0) && (h.rxLoop() != nullptr) == loop.valid());
    }
    // the send side, as WebSocket::Impl::sendWsFrame would call it (INTEGRATION.md
    // sec.3.3) with kuma's FrameHeader and a two-segment KMBuffer chain; without
    // a device the TxLoop is invalid and refuses the send
    {
        std::vector<kmws::TxLoop::Task> tasks;
        kmws::TxLoop tx([&tasks](kmws::TxLoop::Task t) { tasks.push_back(std::move(t)); });
        std::string wrote;
        kmws::TxLoop::Conn* conn = tx.open([&wrote](const iovec* v, int n) {
            for (int i = 0; i < n; ++i) wrote.append(static_cast<const char*>(v[i].iov_base), v[i].iov_len);
            return 0;
        });
        FrameHeader hdr;
        std::memset(static_cast<void*>(&hdr), 0, sizeof(hdr));
        hdr.fin = 1;
        hdr.opcode = (uint8_t)WSOpcode::TEXT;
        char a[] = "Hel", b[] = "lo";
        KMBuffer b1(a, 3, 3), b2(b, 2, 2);
        b1.append(&b2);
        const int r = tx.sendBuffer(conn, hdr, b1);  // unmasked (server mode): written at once
        if (kmws_device_count() == 0) {
            CHECK(!tx.valid() && r == KMWS_ERR_INVALID_STATE && wrote.empty());
        } else {
            CHECK(r == 2 && wrote == std::string("\x81\x05Hello", 7));
            (void)tx.close(conn);
        }
    }
    if (g_fail) {
        std::printf("%d checks failed\n", g_fail);
        return 1;
    }
    std::printf("OK kuma types\n");
    return 0;
}
