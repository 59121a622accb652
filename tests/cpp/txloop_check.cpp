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

}  // namespace

int main(int argc, char** argv)
{
    g_rng = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
    const int sends = argc > 2 ? std::atoi(argv[2]) : 3000;
    if (kmws_device_count() < 1) {
        std::printf("{\"error\": \"no gfx950 device\"}\n");
        return 1;
    }
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
