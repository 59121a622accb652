// Frame-header parsing shared by the device kernels (kmws_pack.hip,
// kmws_unmask.hip): the reference's HDR1..MASKEY rules of
// WSHandler::decodeFrame (WSHandler.cpp:118-234), including the x86-64 shift
// quirk of the 127 length class, for one frame whose header offset is known
// (descriptor-indexed decode), plus the 16-byte window helpers they use.
#pragma once
#include "kmws_common.hpp"

namespace kmws {

__host__ __device__ __forceinline__ uint32_t hdr_len(uint32_t len, uint32_t mask)
{
    return (len <= 125 ? 2u : (len <= 0xFFFFu ? 4u : 10u)) + (mask ? 4u : 0u);
}

// Dword I of the 8-dword window lo||hi (I fixed at compile time).
template <int I>
__device__ __forceinline__ uint32_t dw(const u32x4& lo, const u32x4& hi)
{
    if constexpr (I == 0) return lo.x;
    else if constexpr (I == 1) return lo.y;
    else if constexpr (I == 2) return lo.z;
    else if constexpr (I == 3) return lo.w;
    else if constexpr (I == 4) return hi.x;
    else if constexpr (I == 5) return hi.y;
    else if constexpr (I == 6) return hi.z;
    else return hi.w;
}

// Dword q + K of the window for q in 0..3 (per lane): a select chain over
// distinct registers (an indexed register array would be placed in scratch).
template <int K>
__device__ __forceinline__ uint32_t pick(const u32x4& lo, const u32x4& hi, uint32_t q)
{
    const uint32_t a = (q & 1u) ? dw<K + 1>(lo, hi) : dw<K>(lo, hi);
    const uint32_t b = (q & 1u) ? dw<K + 3>(lo, hi) : dw<K + 2>(lo, hi);
    return (q & 2u) ? b : a;
}

// 16 bytes starting at byte delta (0..15) of the 32-byte window lo||hi.
__device__ __forceinline__ u32x4 funnel16(const u32x4& lo, const u32x4& hi, uint32_t delta)
{
    const uint32_t q = delta >> 2;
    const uint32_t r = (delta & 3u) * 8u;
    const uint32_t c0 = pick<0>(lo, hi, q), c1 = pick<1>(lo, hi, q), c2 = pick<2>(lo, hi, q),
                   c3 = pick<3>(lo, hi, q), c4 = pick<4>(lo, hi, q);
    // v_alignbit_b32(hi, lo, 0) == lo, so r == 0 needs no special case
    return u32x4{__builtin_amdgcn_alignbit(c1, c0, r), __builtin_amdgcn_alignbit(c2, c1, r),
                 __builtin_amdgcn_alignbit(c3, c2, r), __builtin_amdgcn_alignbit(c4, c3, r)};
}

// Byte k (0..15) of a 16-byte register word.
__device__ __forceinline__ uint32_t byte_of(const u32x4& v, uint32_t k)
{
    const uint32_t q = k >> 2;
    const uint32_t w = (q & 2u) ? ((q & 1u) ? v.w : v.z) : ((q & 1u) ? v.y : v.x);
    return (w >> (8u * (k & 3u))) & 0xFFu;
}

// The 127-class extended length as the reference computes it on x86-64
// (WSHandler.cpp:176-197): xpl64 |= data[pos] << ((8-k-1) << 3) with a 32-bit
// int operand, so byte k (0..7) contributes (u64)(i64)(i32)(b << ((7-k)*8 & 31))
// -- bytes 0..3 alias onto bits 24/16/8/0, bytes 0 and 4 sign-extend.
// hw holds the header from byte 0; the length bytes are 2..9.
__device__ __forceinline__ uint64_t ext_len127(const u32x4& hw)
{
    uint64_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) x |= (uint64_t)(int64_t)(int32_t)(byte_of(hw, 2 + k) << (((7u - k) * 8u) & 31u));
    return x;
}

// Frame f of a descriptor-indexed batch: its header at hdr_off[f], which must
// end (header + payload) by the next header offset (the wire's end for the
// last).  The (at most 14) header bytes come from ONE pair of aligned 16-byte
// loads, funnel-shifted into a register word, when both words lie inside the
// wire; headers within 32 bytes of its end are read byte by byte (same rules).
// Writes out_desc[f] = {payload offset, len, key (0 if unmasked)} -- error
// frames get len 0 and set kStatusBadHeader -- and, when given, out_flags[f]
// (header byte 0 | mask << 8) and out_err[f] (WSError).  Returns the desc.
__device__ __forceinline__ kmws_desc unpack_one(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                                const uint64_t* __restrict__ hdr_off, uint32_t n, uint32_t f,
                                                int mode, kmws_desc* __restrict__ out_desc,
                                                uint16_t* __restrict__ out_flags, uint8_t* __restrict__ out_err,
                                                WsHead* __restrict__ head)
{
    const uint64_t h = hdr_off[f];
    const uint64_t limit = f + 1 < n ? hdr_off[f + 1] : wire_len;  // this frame must end by the next header
    // the header window: bytes h .. h + 15 that lie inside the wire (avail of them)
    const uint64_t avail = h < wire_len ? (wire_len - h < 16 ? wire_len - h : 16) : 0;
    u32x4 hw = u32x4{0, 0, 0, 0};
    // aligned 16-byte words by absolute address: a word holding any wire byte is
    // readable (it cannot cross a page), whatever the wire's own alignment
    const uintptr_t a = reinterpret_cast<uintptr_t>(wire + h);
    const uintptr_t a16 = a & ~(uintptr_t)15;
    const uintptr_t end16 = (reinterpret_cast<uintptr_t>(wire) + wire_len + 15) & ~(uintptr_t)15;
    if (h < wire_len && a16 + 32 <= end16) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(a16);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(a16 + 16);
        hw = funnel16(lo, hi, (uint32_t)(a & 15u));
    } else {
        for (uint32_t k = 0; k < (uint32_t)avail; ++k) {
            const uint32_t b = wire[h + k];
            const uint32_t sh = 8u * (k & 3u);
            if ((k >> 2) == 0) hw.x |= b << sh;
            else if ((k >> 2) == 1) hw.y |= b << sh;
            else if ((k >> 2) == 2) hw.z |= b << sh;
            else hw.w |= b << sh;
        }
    }
    uint8_t err = KMWS_WS_NOERR;
    uint32_t len = 0, key = 0, hl = 2;
    uint32_t b0 = 0, b1 = 0;
    if (h + 2 > wire_len || limit < h || limit > wire_len) {
        err = h + 2 > wire_len ? KMWS_WS_NEED_MORE_DATA : KMWS_WS_INVALID_FRAME;
    } else {
        b0 = hw.x & 0xFFu;
        b1 = (hw.x >> 8) & 0xFFu;
        const uint32_t fin = b0 >> 7, op = b0 & 0x0F, mask = b1 >> 7, plen = b1 & 0x7F;
        if (!fin && op >= 8) {
            err = KMWS_WS_PROTOCOL_ERROR;                     // :126-130
        } else if (op >= 8 && plen > 125) {
            err = KMWS_WS_PROTOCOL_ERROR;                     // :145-149
        } else {
            const uint32_t ext = plen == 126 ? 2u : (plen == 127 ? 8u : 0u);
            hl = 2 + ext + (mask ? 4u : 0u);
            if (h + 2 + ext > wire_len) {
                err = KMWS_WS_NEED_MORE_DATA;
            } else if (plen == 126) {                          // :159-175
                len = (byte_of(hw, 2) << 8) | byte_of(hw, 3);
                if (len < 126) err = KMWS_WS_INVALID_LENGTH;
            } else if (plen == 127) {                          // :176-197, x86-64 shift quirk
                const uint64_t x = ext_len127(hw);
                if ((x >> 63) != 0) err = KMWS_WS_INVALID_LENGTH;
                else {
                    len = (uint32_t)x;
                    if (len > KMWS_MAX_FRAME_DATA_LENGTH) err = KMWS_WS_INVALID_LENGTH;
                }
            } else {
                len = plen;
            }
            if (err == KMWS_WS_NOERR) {
                if (mask && mode == KMWS_MODE_CLIENT) err = KMWS_WS_PROTOCOL_ERROR;          // :208-212
                else if (!mask && mode == KMWS_MODE_SERVER && len > 0) err = KMWS_WS_PROTOCOL_ERROR;  // :225-229
                else if (h + hl > wire_len) err = KMWS_WS_NEED_MORE_DATA;
                else if (mask) {  // key bytes verbatim at hl - 4 (2, 4 or 10)
                    const uint32_t k0 = hl - 4;
                    key = byte_of(hw, k0) | (byte_of(hw, k0 + 1) << 8) | (byte_of(hw, k0 + 2) << 16) |
                          (byte_of(hw, k0 + 3) << 24);
                }
                if (err == KMWS_WS_NOERR) {
                    if (h + hl + len > wire_len) err = KMWS_WS_NEED_MORE_DATA;
                    else if (h + hl + len > limit) err = KMWS_WS_INVALID_FRAME;  // offsets disagree with the stream
                }
            }
            if (err == KMWS_WS_NOERR && !mask) key = 0;
        }
    }
    kmws_desc o;
    if (err == KMWS_WS_NOERR) {
        o.off = h + hl;
        o.len = len;
        o.key = key;
    } else {  // error frames carry no payload (nothing downstream touches them)
        o.off = h;
        o.len = 0;
        o.key = 0;
        atomicOr(&head->status, kStatusBadHeader);
    }
    out_desc[f] = o;
    if (out_flags) out_flags[f] = (uint16_t)((b0 & 0xFFu) | ((b1 >> 7) << 8));
    if (out_err) out_err[f] = err;
    return o;
}


}  // namespace kmws
