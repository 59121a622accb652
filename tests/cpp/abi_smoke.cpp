// C++ consumer of the kmws C ABI (what kuma's WebSocket::Impl would link):
// host codec entries checked against RFC 6455 / SURVEY a-4 known answers;
// on a GPU box also a masked frame and a device-less failure mode otherwise.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kmws_gpu.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } } while (0)

static std::string hex(const uint8_t* p, size_t n)
{
    static const char* d = "0123456789abcdef";
    std::string s;
    for (size_t i = 0; i < n; ++i) { s += d[p[i] >> 4]; s += d[p[i] & 15]; }
    return s;
}

struct Got { std::vector<std::string> payloads; std::vector<int> ops; };

static int on_frame(const kmws_frame_hdr* h, uint8_t* p, size_t n, void* user)
{
    auto* g = static_cast<Got*>(user);
    g->payloads.emplace_back(reinterpret_cast<const char*>(p), n);
    g->ops.push_back(h->opcode);
    return 0;
}

int main()
{
    // SURVEY a-4: len 65536, masked, key de ad be ef, fin=1 rsv1=1 op=2
    kmws_frame_hdr h{};
    h.fin = 1; h.rsv1 = 1; h.opcode = KMWS_OP_BINARY; h.mask = 1; h.length = 65536;
    const uint8_t key[4] = {0xde, 0xad, 0xbe, 0xef};
    std::memcpy(h.maskey, key, 4);
    uint8_t out[KMWS_MAX_HEADER_SIZE];
    int n = kmws_encode_header(&h, out);
    CHECK(n == 14 && hex(out, n) == "c2ff0000000000010000deadbeef");
    h.length = 126;
    n = kmws_encode_header(&h, out);
    CHECK(n == 8 && hex(out, n) == "c2fe007edeadbeef");
    CHECK(kmws_header_size(125, 0) == 2 && kmws_header_size(65535, 1) == 8 && kmws_header_size(65536, 0) == 10);

    // RFC 6455 5.7 fragmented unmasked "Hel" + "lo" (CLIENT mode needs no device)
    uint8_t frag[] = {0x01, 0x03, 0x48, 0x65, 0x6c, 0x80, 0x02, 0x6c, 0x6f};
    kmws_decoder* dec = kmws_decoder_create(KMWS_MODE_CLIENT, 0);
    Got g;
    CHECK(kmws_decoder_feed(dec, frag, sizeof frag, on_frame, &g) == KMWS_WS_NOERR);
    CHECK(g.payloads.size() == 2 && g.payloads[0] == "Hel" && g.payloads[1] == "lo");
    CHECK(g.ops[0] == KMWS_OP_TEXT && g.ops[1] == KMWS_OP_CONTINUE);
    // byte at a time: 1, 1, ..., 0
    Got g2;
    kmws_decoder_reset(dec);
    int last = -1;
    for (size_t i = 0; i < sizeof frag; ++i) last = kmws_decoder_feed(dec, frag + i, 1, on_frame, &g2);
    CHECK(last == KMWS_WS_NOERR && g2.payloads.size() == 2);
    kmws_decoder_destroy(dec);

    // header walk
    uint64_t offs[4];
    uint32_t nf = 0;
    uint64_t used = 0;
    CHECK(kmws_find_headers(frag, sizeof frag, offs, 4, &nf, &used) == KMWS_OK);
    CHECK(nf == 2 && offs[0] == 0 && offs[1] == 5 && used == sizeof frag);

    // RFC 6455 5.7 masked "Hello" in SERVER mode: GPU unmask, or a loud failure without a device
    uint8_t masked[] = {0x81, 0x85, 0x37, 0xfa, 0x21, 0x3d, 0x7f, 0x9f, 0x4d, 0x51, 0x58};
    kmws_decoder* srv = kmws_decoder_create(KMWS_MODE_SERVER, 0);
    Got g3;
    const int r = kmws_decoder_feed(srv, masked, sizeof masked, on_frame, &g3);
    if (kmws_device_count() > 0) {
        CHECK(r == KMWS_WS_NOERR && g3.payloads.size() == 1 && g3.payloads[0] == "Hello");
        CHECK(std::memcmp(masked + 6, "Hello", 5) == 0);  // unmasked in place in the caller's buffer
        uint8_t seg1[3] = {0, 0, 0}, seg2[5] = {0, 0, 0, 0, 0};
        uint8_t* segs[2] = {seg1, seg2};
        size_t lens[2] = {3, 5};
        const uint8_t k[4] = {1, 2, 3, 4};
        CHECK(kmws_mask_host_chain(k, segs, lens, 2, 0) == KMWS_OK);  // SURVEY a-2 vector
        CHECK(hex(seg1, 3) == "010203" && hex(seg2, 5) == "0401020304");
        // batched send path: RFC 6455 5.7 masked "Hello" built from two segments, one flush
        kmws_tx_batch* tx = kmws_tx_batch_create(0);
        CHECK(tx != nullptr);
        uint8_t he[2] = {'H', 'e'}, llo[3] = {'l', 'l', 'o'};
        uint8_t* tsegs[2] = {he, llo};
        size_t tlens[2] = {2, 3};
        kmws_frame_hdr th;
        std::memset(&th, 0, sizeof th);
        th.fin = 1;
        th.opcode = KMWS_OP_TEXT;
        th.mask = 1;
        const uint8_t tk[4] = {0x37, 0xfa, 0x21, 0x3d};
        std::memcpy(th.maskey, tk, 4);
        uint8_t hb[KMWS_MAX_HEADER_SIZE];
        CHECK(kmws_tx_batch_add(tx, &th, tsegs, tlens, 2, hb) == 6 && hex(hb, 6) == "818537fa213d");
        CHECK(kmws_tx_batch_pending(tx) == 1 && kmws_tx_batch_flush(tx) == 1);
        CHECK(hex(he, 2) == "7f9f" && hex(llo, 3) == "4d5158");
        kmws_tx_batch_destroy(tx);
    } else {
        CHECK(r == KMWS_ERR_NOT_SUPPORTED && g3.payloads.empty());
        CHECK(kmws_tx_batch_create(0) == nullptr);
    }
    kmws_decoder_destroy(srv);
    std::printf("%s (%d failures)\n", fails ? "FAILED" : "OK", fails);
    return fails ? 1 : 0;
}
