// kmws::TxLoop (include/kmws_wshandler.hpp), the batched replacement of
// WebSocket::Impl::sendWsFrame (WebSocketImpl.cpp:381-436), against kuma's
// send path restated in oracle/ (encodeFrameHeader + the byte-loop mask,
// WSHandler.cpp:46-106, 303-322): random sends on three connections of one
// loop -- masked (client) and unmasked (server) frames, empty payloads,
// KMBuffer-style chains of 1-5 segments, payloads larger than the pinned send
// ring (the heap path) -- with the loop's posted tasks run every few sends,
// a ring small enough to wrap many times, then every connection closed.
// Each connection's written bytes must equal the oracle's frames in send order,
// and the callers' payload buffers must be unchanged.  Test infrastructure
// (links the oracle): tests/test_abi_build.py.
//
// usage: txloop_check [seed] [sends]
//        txloop_check timeout      (linked against the test build: the error path)
#include <sys/uio.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kmws_gpu.h"
#include "kmws_wshandler.hpp"

extern "C" {  // oracle/kmws_oracle.c (test infrastructure)
typedef struct orc_hdr {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, plen, _pad;
    uint64_t xpl64;
    uint8_t maskey[4];
    uint32_t length;
} orc_hdr;
void orc_mask(const uint8_t key[4], uint8_t* data, size_t len, size_t phase);
int orc_encode_header(const orc_hdr* h, uint8_t out[14]);
}

namespace {

uint64_t g_rng = 1;
uint64_t rnd()
{
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// a generation whose mask fails is never written.  Needs the test
// build (kuma_amd/build.py TEST_DEFINES: a resident job whose first key is
// 0xDEAD5Exx stalls its workgroup xx * 10 ms; timeout 50 ms, drain 150 ms).
// An 80 ms stall is withdrawn and launched: exact.  A 400 ms stall outlives
// timeout + drain: the flush returns KMWS_ERR_TIMEOUT, the generation's frames
// are dropped (not one masked header goes out with a plain payload), their
// connections report the status, and the loop refuses later sends.
int timeout_case()
{
    std::vector<kmws::TxLoop::Task> tasks;
    kmws::TxLoop tx([&tasks](kmws::TxLoop::Task t) { tasks.push_back(std::move(t)); }, 0, 64 << 10);
    if (!tx.valid()) return 3;
    std::string wrote[2], want[2];
    kmws::TxLoop::Conn* conn[2];
    for (int c = 0; c < 2; ++c)
        conn[c] = tx.open([&wrote, c](const iovec* v, int n) {
            for (int i = 0; i < n; ++i) wrote[c].append(static_cast<const char*>(v[i].iov_base), v[i].iov_len);
            return 0;
        });
    auto send = [&](int c, uint32_t key, size_t plen, bool expect) {
        std::vector<uint8_t> payload(plen);
        for (auto& b : payload) b = (uint8_t)rnd();
        kmws_frame_hdr h;
        std::memset(&h, 0, sizeof h);
        h.fin = 1;
        h.opcode = KMWS_OP_BINARY;
        h.mask = 1;
        std::memcpy(h.maskey, &key, 4);
        const int r = tx.send(conn[c], h, payload.data(), plen);
        if (!expect) return r;
        orc_hdr o;
        std::memset(&o, 0, sizeof o);
        o.fin = 1;
        o.opcode = KMWS_OP_BINARY;
        o.mask = 1;
        std::memcpy(o.maskey, &key, 4);
        o.length = (uint32_t)plen;
        uint8_t hb[14];
        const int hl = orc_encode_header(&o, hb);
        orc_mask(o.maskey, payload.data(), plen, 0);
        want[c].append(reinterpret_cast<const char*>(hb), (size_t)hl);
        want[c].append(reinterpret_cast<const char*>(payload.data()), plen);
        return r;
    };
    const uint32_t stall80 = 0xDEAD5E00u | 8, stall400 = 0xDEAD5E00u | 40;
    int r0 = send(0, 0x11223344u, 3000, true);
    const int f0 = tx.flush();                  // a normal generation
    int r1 = send(1, stall80, 5000, true);      // first key of its generation: stalls 80 ms
    int r2 = send(0, 0x55667788u, 700, true);
    const int f1 = tx.flush();                  // withdrawn after 50 ms, launched: exact
    const std::string before0 = wrote[0], before1 = wrote[1];
    int r3 = send(1, stall400, 4000, false);    // stalls past timeout + drain
    int r4 = send(0, 0x99AABBCCu, 900, false);
    const int f2 = tx.flush();
    const int after = send(0, 0x01010101u, 100, false);
    const bool dropped_ok = wrote[0] == before0 && wrote[1] == before1 && tx.dropped() == 2 &&
                            conn[0]->lastResult() == KMWS_ERR_TIMEOUT && conn[1]->lastResult() == KMWS_ERR_TIMEOUT &&
                            conn[0]->queued() == 0 && conn[1]->queued() == 0;
    const bool ok = r0 > 0 && r1 > 0 && r2 > 0 && r3 > 0 && r4 > 0 && f0 == 1 && f1 == 2 && f2 == KMWS_ERR_TIMEOUT &&
                    after == KMWS_ERR_TIMEOUT && tx.broken() == KMWS_ERR_TIMEOUT && !tx.valid() && dropped_ok &&
                    wrote[0] == want[0] && wrote[1] == want[1];
    std::printf("{\"case\": \"timeout\", \"flush\": [%d, %d, %d], \"send_after\": %d, \"dropped\": %llu, "
                "\"conn_results\": [%d, %d], \"bytes\": [%zu, %zu], \"exact\": %s}\n",
                f0, f1, f2, after, (unsigned long long)tx.dropped(), conn[0]->lastResult(), conn[1]->lastResult(),
                wrote[0].size(), wrote[1].size(), ok ? "true" : "false");
    return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv)
{
    if (kmws_device_count() < 1) {
        std::printf("{\"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    if (argc > 1 && std::strcmp(argv[1], "timeout") == 0) return timeout_case();
    g_rng = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
    const int sends = argc > 2 ? std::atoi(argv[2]) : 3000;
    std::vector<kmws::TxLoop::Task> tasks;
    constexpr size_t kRing = 64 << 10;  // small: the ring wraps every few iterations
    kmws::TxLoop tx([&tasks](kmws::TxLoop::Task t) { tasks.push_back(std::move(t)); }, 0, kRing);
    if (!tx.valid()) return 3;
    constexpr int kConns = 3;
    std::string wrote[kConns], want[kConns];
    kmws::TxLoop::Conn* conn[kConns];
    for (int c = 0; c < kConns; ++c)
        conn[c] = tx.open([&wrote, c](const iovec* v, int n) {
            for (int i = 0; i < n; ++i) wrote[c].append(static_cast<const char*>(v[i].iov_base), v[i].iov_len);
            return 0;
        });
    int bad_src = 0, heap = 0, masked_n = 0, runs = 0;
    for (int i = 0; i < sends; ++i) {
        const int c = (int)(rnd() % kConns);
        const bool masked = rnd() % 4 != 0;
        size_t plen;
        const uint64_t k = rnd() % 100;
        if (k < 5) plen = 0;
        else if (k < 8) plen = kRing + rnd() % 50000;  // larger than the ring
        else if (k < 40) plen = rnd() % 126;
        else plen = rnd() % 20000;
        heap += plen + 16 > kRing;
        std::vector<uint8_t> payload(plen);
        for (auto& b : payload) b = (uint8_t)rnd();
        const std::vector<uint8_t> orig = payload;
        // the frame header as sendWsFrame fills it (:384-390)
        kmws_frame_hdr h;
        std::memset(&h, 0, sizeof h);
        h.fin = 1;
        h.opcode = (uint8_t)(rnd() % 2 ? KMWS_OP_BINARY : KMWS_OP_TEXT);
        h.mask = masked && plen > 0;
        const uint32_t key = (uint32_t)rnd();
        std::memcpy(h.maskey, &key, 4);
        masked_n += h.mask;
        // 1-5 segments (a KMBuffer chain), some empty
        const int nseg = 1 + (int)(rnd() % 5);
        std::vector<const uint8_t*> segs;
        std::vector<size_t> lens;
        size_t pos = 0;
        for (int s = 0; s < nseg; ++s) {
            const size_t l = s == nseg - 1 ? plen - pos : (plen - pos ? rnd() % (plen - pos + 1) : 0);
            segs.push_back(payload.data() + pos);
            lens.push_back(l);
            pos += l;
        }
        const int r = nseg == 1 ? tx.send(conn[c], h, payload.data(), plen)
                                : tx.sendChain(conn[c], h, segs.data(), lens.data(), segs.size());
        // the oracle's frame
        orc_hdr o;
        std::memset(&o, 0, sizeof o);
        o.fin = 1;
        o.opcode = h.opcode;
        o.mask = h.mask;
        std::memcpy(o.maskey, h.maskey, 4);
        o.length = (uint32_t)plen;
        uint8_t hb[14];
        const int hl = orc_encode_header(&o, hb);
        if (r != hl) {
            std::printf("{\"error\": \"send %d returned %d, header length %d\"}\n", i, r, hl);
            return 4;
        }
        std::vector<uint8_t> m = payload;
        if (o.mask) orc_mask(o.maskey, m.data(), m.size(), 0);
        want[c].append(reinterpret_cast<const char*>(hb), (size_t)hl);
        want[c].append(reinterpret_cast<const char*>(m.data()), m.size());
        bad_src += payload != orig;
        if (rnd() % 6 == 0) {  // the end of a loop iteration: its posted tasks
            std::vector<kmws::TxLoop::Task> now;
            now.swap(tasks);
            for (auto& t : now) t();
            ++runs;
            if (tx.lastResult() < 0) return 5;
        }
    }
    // A loop that drops a posted task (it was torn down, or the caller's task
    // list was discarded), then a new poster: sends are posted again (a stale
    // armed flag once kept every later send queued until the ring filled).
    int reposted = 0;
    {
        if (tx.flush() < 0) return 8;  // everything written; then the loop's queued tasks run out
        while (!tasks.empty()) {
            std::vector<kmws::TxLoop::Task> now;
            now.swap(tasks);
            for (auto& t : now) t();
        }
        auto frame = [&](uint32_t key, size_t plen, int c) {
            std::vector<uint8_t> payload(plen);
            for (auto& b : payload) b = (uint8_t)rnd();
            kmws_frame_hdr h;
            std::memset(&h, 0, sizeof h);
            h.fin = 1;
            h.opcode = KMWS_OP_BINARY;
            h.mask = 1;
            std::memcpy(h.maskey, &key, 4);
            if (tx.send(conn[c], h, payload.data(), plen) < 0) std::exit(7);
            orc_hdr o;
            std::memset(&o, 0, sizeof o);
            o.fin = 1;
            o.opcode = KMWS_OP_BINARY;
            o.mask = 1;
            std::memcpy(o.maskey, &key, 4);
            o.length = (uint32_t)plen;
            uint8_t hb[14];
            const int hl = orc_encode_header(&o, hb);
            orc_mask(o.maskey, payload.data(), plen, 0);
            want[c].append(reinterpret_cast<const char*>(hb), (size_t)hl);
            want[c].append(reinterpret_cast<const char*>(payload.data()), plen);
        };
        frame(0x01020304u, 3000, 0);
        reposted += tasks.size() == 1;
        tasks.clear();  // dropped unrun
        std::vector<kmws::TxLoop::Task> tasks2;
        tx.setPoster([&tasks2](kmws::TxLoop::Task t) { tasks2.push_back(std::move(t)); });
        reposted += tasks2.size() == 1;  // something is queued: the new poster gets a task at once
        frame(0x0a0b0c0du, 5000, 1);
        reposted += tasks2.size() == 1;  // armed: no second task
        while (!tasks2.empty()) {
            std::vector<kmws::TxLoop::Task> now;
            now.swap(tasks2);
            for (auto& t : now) t();
        }
        reposted += tx.pending() == 0 && tx.inflight() == 0;
        tx.setPoster([&tasks](kmws::TxLoop::Task t) { tasks.push_back(std::move(t)); });
    }
    for (int c = 0; c < kConns; ++c)
        if (tx.close(conn[c]) < 0) return 6;
    bool ok = bad_src == 0 && reposted == 4;
    for (int c = 0; c < kConns; ++c) ok &= wrote[c] == want[c];
    std::printf("{\"sends\": %d, \"masked\": %d, \"larger_than_ring\": %d, \"iterations\": %d, \"bytes\": [%zu, %zu, %zu], "
                "\"callers_buffers_changed\": %d, \"reposted_checks\": %d, \"exact\": %s}\n",
                sends, masked_n, heap, runs, wrote[0].size(), wrote[1].size(), wrote[2].size(), bad_src, reposted,
                ok ? "true" : "false");
    return ok ? 0 : 1;
}
