// Host codec entries of the kmws C ABI that need no device: header pack
// (WSHandler::encodeFrameHeader) and the serial header-chain walk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "kmws_gpu.h"
#include "kmws_host_util.hpp"

using namespace kmws;

extern "C" {

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

}  // extern "C"
