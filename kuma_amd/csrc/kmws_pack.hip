// Batched frame-header pack/unpack and out-of-place mask-copy for MI355X.
//
// Encode (kmws_encode_batch) = for every frame, WSHandler::encodeFrameHeader
// (src/ws/WSHandler.cpp:46-106) followed by the masked payload
// (WebSocket::Impl::sendWsFrame, src/ws/WebSocketImpl.cpp:381-404): the wire
// image is header_0 payload_0 header_1 payload_1 ...  Kernels:
//   1. scan_reduce / scan_partials / scan_emit: exclusive scan of the wire
//      size (2/4/10 + 4*mask + len) of every frame -> wire_off[0..n]
//      (wave prefix sums with __shfl_up, one LDS round across the 4 waves);
//   2. dst_map: tile -> first frame over the output byte space;
//   3. mask_copy: every 16-byte output word is produced by exactly one lane:
//      header bytes come from a 14-byte header built in registers, payload
//      bytes from the source (funnel-shifted when source and destination are
//      misaligned) XOR the rotated key.  Outputs are written once, with no
//      read-modify-write.
// Decode (descriptor-indexed): kmws_unpack_headers parses and
// validates one header per frame with the reference's rules
// (WSHandler.cpp:118-234, including the 127-length quirk); the payload is then
// unmasked in place (kmws_unmask_batch) or gathered + unmasked into a dense
// arena by the same mask_copy kernel (kmws_gather_unmask).
#include "kmws_common.hpp"

namespace kmws {

constexpr int kScanItems = 8;                      // frames per lane in the scan
constexpr int kScanTile = kBlock * kScanItems;     // 2048 frames per block
constexpr int kCopyV = 4;                          // 16-byte words per lane
constexpr uint64_t kCopyTile = (uint64_t)kBlock * kCopyV * 16;  // 16 KiB of output per block
constexpr int kCopyCap = kBlock;                   // frames staged per LDS round

__host__ __device__ __forceinline__ uint32_t hdr_len(uint32_t len, uint32_t mask)
{
    return (len <= 125 ? 2u : (len <= 0xFFFFu ? 4u : 10u)) + (mask ? 4u : 0u);
}

// Header bytes of WSHandler::encodeFrameHeader as two little-endian u64
// (byte k of the header = byte k of h[k >> 3]).
__device__ __forceinline__ void build_header(uint32_t len, uint32_t flags, uint32_t key, uint64_t& h0,
                                             uint64_t& h1)
{
    const uint64_t b0 = flags & 0xFFu;
    const uint32_t mask = (flags >> 8) & 1u;
    const uint64_t m = mask ? 0x80u : 0u;
    uint64_t lo = b0, hi = 0;
    int n;
    if (len <= 125) {
        lo |= (m | len) << 8;
        n = 2;
    } else if (len <= 0xFFFFu) {
        lo |= (m | 126u) << 8;
        lo |= (uint64_t)(len >> 8) << 16;
        lo |= (uint64_t)(len & 0xFFu) << 24;
        n = 4;
    } else {  // 127: four zero bytes, then the 32-bit length big-endian (bytes 6..9)
        lo |= (m | 127u) << 8;
        lo |= (uint64_t)(len >> 24) << 48;
        lo |= (uint64_t)((len >> 16) & 0xFFu) << 56;
        hi |= (uint64_t)((len >> 8) & 0xFFu);
        hi |= (uint64_t)(len & 0xFFu) << 8;
        n = 10;
    }
    if (mask) {  // maskey bytes verbatim after the length (:101-104)
        for (int k = 0; k < 4; ++k) {
            const uint64_t kb = (key >> (8 * k)) & 0xFFu;
            const int p = n + k;
            if (p < 8) lo |= kb << (8 * p); else hi |= kb << (8 * (p - 8));
        }
    }
    h0 = lo;
    h1 = hi;
}

// ------------------------------ scan ------------------------------
// size(f) for the two users: encode (header + payload) and gather (payload).
struct WireSize {
    const kmws_desc* d;
    const uint16_t* flags;
    __device__ uint64_t operator()(uint32_t f) const
    {
        const uint32_t len = d[f].len;
        return (uint64_t)hdr_len(len, (flags[f] >> 8) & 1u) + len;
    }
};
struct PayloadSize {
    const kmws_desc* d;
    __device__ uint64_t operator()(uint32_t f) const { return d[f].len; }
};

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    return x;
}

// Block-wide exclusive scan of one value per lane; returns the block total too.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t x, uint64_t* s_wave, uint64_t& total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t inc = wave_incl_scan(x);
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint64_t before = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const uint64_t v = s_wave[w];
        if (w < wave) before += v;
        total += v;
    }
    __syncthreads();
    return before + inc - x;
}

template <class Size>
__global__ void __launch_bounds__(kBlock) scan_reduce_kernel(Size size, uint32_t n, uint64_t* __restrict__ partials)
{
    __shared__ uint64_t s_wave[kBlock / 64];
    const uint32_t f0 = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i)
        if (f0 + i < n) s += size(f0 + i);
    uint64_t total;
    block_excl_scan(s, s_wave, total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// One block scans the per-block totals in place (exclusive) and writes the grand total.
__global__ void __launch_bounds__(kBlock) scan_partials_kernel(uint64_t* __restrict__ partials, uint32_t nb,
                                                               uint64_t* __restrict__ total_out)
{
    __shared__ uint64_t s_wave[kBlock / 64];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nb; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t x = i < nb ? partials[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan(x, s_wave, tot);
        if (i < nb) partials[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total_out = carry;
}

template <class Size>
__global__ void __launch_bounds__(kBlock) scan_emit_kernel(Size size, uint32_t n, const uint64_t* __restrict__ partials,
                                                           uint64_t* __restrict__ out)
{
    __shared__ uint64_t s_wave[kBlock / 64];
    const uint32_t f0 = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint64_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        v[i] = f0 + i < n ? size(f0 + i) : 0;
        s += v[i];
    }
    uint64_t total;
    uint64_t run = partials[blockIdx.x] + block_excl_scan(s, s_wave, total);
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        if (f0 + i < n) out[f0 + i] = run;
        run += v[i];
    }
}

// ------------------------------ tile map over the output space ------------------------------
// Frame f's region in the output is [start[f], start[f+1]); tiles whose first
// byte falls in it get map = f.  start[n] is the total.
__global__ void __launch_bounds__(kBlock) dst_map_kernel(const uint64_t* __restrict__ start, uint32_t n,
                                                         uint64_t cap, uint32_t* __restrict__ map,
                                                         WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    const uint64_t total = start[n];
    if (total > cap) {
        if (f == 0) atomicOr(&head->status, kStatusBadDesc);
        return;
    }
    const uint64_t lo = f == 0 ? 0 : start[f];
    const uint64_t hi = start[f + 1];
    for (uint64_t b = (lo + kCopyTile - 1) / kCopyTile; b < (hi + kCopyTile - 1) / kCopyTile; ++b) map[b] = (uint32_t)f;
}

// ------------------------------ mask-copy emit ------------------------------
// Output word w (16 bytes at dst + a) for frames staged in LDS:
//   region j: [s_dst[j], s_dst[j] + s_hl[j] + s_len[j]) of the output,
//   header bytes first (s_hl[j] = 0 for a payload-only gather), then payload
//   bytes read from src + s_src[j] XOR key byte.
struct CopyLds {
    uint64_t end[kCopyCap];  // region end (payload end) in the output: the search key
    uint64_t dst[kCopyCap];  // region start (header start)
    uint64_t p0[kCopyCap];   // payload start in the output
    uint64_t sdel[kCopyCap]; // src offset - p0: source byte of output byte a is a + sdel
    uint64_t h0[kCopyCap];
    uint64_t h1[kCopyCap];
    uint32_t key[kCopyCap];
};

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

// W[k] = h[k - s] (0 where k - s is outside 0..15), s in [-15, 15].
__device__ __forceinline__ u32x4 shift_in(const u32x4& h, int s)
{
    const u32x4 z = u32x4{0, 0, 0, 0};
    if (s == 0) return h;
    return s > 0 ? funnel16(z, h, (uint32_t)(16 - s)) : funnel16(h, z, (uint32_t)(-s));
}

__device__ __forceinline__ u32x4 byte_range(int lo, int hi)
{
    return u32x4{dword_byte_mask(lo, hi, 0), dword_byte_mask(lo, hi, 1), dword_byte_mask(lo, hi, 2),
                 dword_byte_mask(lo, hi, 3)};
}

// Fill a CopyLds row for frame fi; returns the region end.
template <bool HEADERS>
__device__ __forceinline__ void load_frame(CopyLds& L, int row, uint32_t fi, const uint64_t* __restrict__ start,
                                           const kmws_desc* __restrict__ d, const uint16_t* __restrict__ flags)
{
    const kmws_desc x = d[fi];
    const uint64_t r0 = start[fi];
    uint32_t hl = 0;
    if (HEADERS) {
        const uint32_t fl = flags[fi];
        const uint32_t mask = (fl >> 8) & 1u;
        uint64_t h0, h1;
        build_header(x.len, fl, x.key, h0, h1);
        L.h0[row] = h0;
        L.h1[row] = h1;
        hl = hdr_len(x.len, mask);
        L.key[row] = mask ? x.key : 0u;
    } else {
        L.h0[row] = L.h1[row] = 0;
        L.key[row] = x.key;
    }
    L.dst[row] = r0;
    L.p0[row] = r0 + hl;
    L.end[row] = r0 + hl + x.len;
    L.sdel[row] = x.off - (r0 + hl);  // wraps modulo 2^64; a + sdel is exact
}

template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) mask_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                           const uint64_t* __restrict__ start,
                                                           const kmws_desc* __restrict__ d,
                                                           const uint16_t* __restrict__ flags, uint32_t n,
                                                           const uint32_t* __restrict__ map,
                                                           const WsHead* __restrict__ head, uint32_t tile_base)
{
    __shared__ CopyLds L;
    const uint32_t tile = tile_base + blockIdx.x;
    const uint64_t total = start[n];
    const uint64_t tile_lo = (uint64_t)tile * kCopyTile;
    if (tile_lo >= total || head->status != 0) return;  // uniform
    const uint64_t tile_hi = tile_lo + kCopyTile < total ? tile_lo + kCopyTile : total;
    const int tid = threadIdx.x;
    uint32_t f = map[tile];

    // Fast path: the whole tile is payload of one frame (uniform scalars).
    {
        const uint64_t r0 = start[f];
        const kmws_desc x = d[f];
        const uint32_t hl = HEADERS ? hdr_len(x.len, (flags[f] >> 8) & 1u) : 0u;
        const uint64_t p0 = r0 + hl;
        const bool masked = HEADERS ? ((flags[f] >> 8) & 1u) != 0 : true;
        if (tile_lo + kCopyTile <= total && p0 <= tile_lo && p0 + x.len >= tile_lo + kCopyTile) {
            const uint32_t rk = masked ? rot_key(x.key, p0) : 0u;
            // source byte of output byte a: x.off + (a - p0); shift = its misalignment
            const uint64_t sbase = x.off + (tile_lo - p0);
            const uint32_t delta = (uint32_t)(sbase & 15u);
            const uint8_t* s0 = src + (sbase - delta);
            u32x4 lo[kCopyV], hi[kCopyV];
#pragma unroll
            for (int i = 0; i < kCopyV; ++i) {
                const uint64_t w = (uint64_t)(tid + kBlock * i);
                lo[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s0 + 16 * w));
            }
            if (delta != 0) {
                // the next aligned word: from lane+1 by a cross-lane move, lane 63 loads it
                const int lane = tid & 63;
#pragma unroll
                for (int i = 0; i < kCopyV; ++i) {
                    const uint64_t w = (uint64_t)(tid + kBlock * i);
                    u32x4 nx;
                    nx.x = __shfl_down(lo[i].x, 1, 64);
                    nx.y = __shfl_down(lo[i].y, 1, 64);
                    nx.z = __shfl_down(lo[i].z, 1, 64);
                    nx.w = __shfl_down(lo[i].w, 1, 64);
                    if (lane == 63) nx = *reinterpret_cast<const u32x4*>(s0 + 16 * (w + 1));
                    hi[i] = nx;
                }
            }
#pragma unroll
            for (int i = 0; i < kCopyV; ++i) {
                const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
                const u32x4 v = delta ? funnel16(lo[i], hi[i], delta) : lo[i];
                __builtin_nontemporal_store(v ^ rk, reinterpret_cast<u32x4*>(dst + a));
            }
            return;
        }
    }

    // General path: stage every frame overlapping the tile, compose bytes.
    u32x4 out[kCopyV];
#pragma unroll
    for (int i = 0; i < kCopyV; ++i) out[i] = u32x4{0, 0, 0, 0};
    for (;;) {
        const uint32_t fi = f + (uint32_t)tid;
        int valid = 0;
        if (fi < n && start[fi] < tile_hi) {
            load_frame<HEADERS>(L, tid, fi, start, d, flags);
            valid = 1;
        }
        const int cnt = __syncthreads_count(valid);
#pragma unroll
        for (int i = 0; i < kCopyV; ++i) {
            const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
            if (a >= tile_hi) continue;
            // first staged frame whose region ends after a
            int lo = 0, hi = cnt;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (L.end[mid] <= a) lo = mid + 1; else hi = mid;
            }
            for (int j = lo; j < cnt; ++j) {
                const uint64_t r0 = L.dst[j];
                if (r0 >= a + 16) break;
                const uint64_t p0 = L.p0[j], r1 = L.end[j];
                // header bytes [r0, p0) of frame j that fall in this word
                if (HEADERS && p0 > a) {
                    const int s = (int)((int64_t)r0 - (int64_t)a);
                    const uint64_t h0 = L.h0[j], h1 = L.h1[j];
                    const u32x4 H = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
                    const int he = (int)(p0 - r0) + s;
                    out[i] |= shift_in(H, s) & byte_range(s < 0 ? 0 : s, he > 16 ? 16 : he);
                }
                // payload bytes [max(a, p0), min(a + 16, r1)) of frame j
                if (r1 > p0 && p0 < a + 16 && r1 > a) {
                    const uint64_t lo_b = p0 > a ? p0 : a, hi_b = r1 < a + 16 ? r1 : a + 16;
                    const uint64_t sdel = L.sdel[j];
                    const uint64_t slo = lo_b + sdel, shi = hi_b + sdel;
                    const uint64_t w0 = slo & ~(uint64_t)15, w1 = (shi - 1) & ~(uint64_t)15;
                    const u32x4 W0 = *reinterpret_cast<const u32x4*>(src + w0);
                    const u32x4 W1 = w1 != w0 ? *reinterpret_cast<const u32x4*>(src + w1) : W0;
                    const int dd = (int)((int64_t)(a + sdel) - (int64_t)w0);  // in [-15, 15]
                    const u32x4 V = dd >= 0 ? funnel16(W0, W1, (uint32_t)dd)
                                            : funnel16(u32x4{0, 0, 0, 0}, W0, (uint32_t)(16 + dd));
                    out[i] |= (V ^ rot_key(L.key[j], p0)) & byte_range((int)(lo_b - a), (int)(hi_b - a));
                }
            }
        }
        if (cnt < kCopyCap) break;
        f += kCopyCap;
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < kCopyV; ++i) {
        const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
        if (a + 16 <= tile_hi) {
            __builtin_nontemporal_store(out[i], reinterpret_cast<u32x4*>(dst + a));
        } else if (a < tile_hi) {  // last partial word of the output: byte stores
            const u32x4 o = out[i];
            for (uint64_t p = a; p < tile_hi; ++p) {
                const uint32_t k = (uint32_t)(p - a);
                const uint32_t dw = (k & 8u) ? ((k & 4u) ? o.w : o.z) : ((k & 4u) ? o.y : o.x);
                dst[p] = (uint8_t)(dw >> (8 * (k & 3u)));
            }
        }
    }
}

// ------------------------------ header unpack / validate ------------------------------
// One lane per frame: the reference's HDR1..MASKEY rules (WSHandler.cpp:118-234).
__global__ void __launch_bounds__(kBlock) unpack_headers_kernel(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                                                const uint64_t* __restrict__ hdr_off, uint32_t n,
                                                                int mode, kmws_desc* __restrict__ out_desc,
                                                                uint16_t* __restrict__ out_flags,
                                                                uint8_t* __restrict__ out_err,
                                                                WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    const uint64_t h = hdr_off[f];
    const uint64_t limit = f + 1 < n ? hdr_off[f + 1] : wire_len;  // this frame must end by the next header
    uint8_t err = KMWS_WS_NOERR;
    uint32_t len = 0, key = 0, hl = 2;
    uint32_t b0 = 0, b1 = 0;
    if (h + 2 > wire_len || limit < h || limit > wire_len) {
        err = h + 2 > wire_len ? KMWS_WS_NEED_MORE_DATA : KMWS_WS_INVALID_FRAME;
    } else {
        b0 = wire[h];
        b1 = wire[h + 1];
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
                len = ((uint32_t)wire[h + 2] << 8) | wire[h + 3];
                if (len < 126) err = KMWS_WS_INVALID_LENGTH;
            } else if (plen == 127) {                          // :176-197, x86-64 shift quirk
                uint64_t x = 0;
                for (uint32_t k = 0; k < 8; ++k) {
                    const uint32_t sh = ((7u - k) * 8u) & 31u;
                    x |= (uint64_t)(int64_t)(int32_t)((uint32_t)wire[h + 2 + k] << sh);
                }
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
                else if (mask) {
                    key = (uint32_t)wire[h + hl - 4] | ((uint32_t)wire[h + hl - 3] << 8) |
                          ((uint32_t)wire[h + hl - 2] << 16) | ((uint32_t)wire[h + hl - 1] << 24);
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
}

// ------------------------------ host launchers ------------------------------
struct CopyWs {
    WsHead* head;
    uint64_t* partials;
    uint32_t* map;
};

static uint64_t n_scan_blocks(uint32_t n) { return ((uint64_t)n + kScanTile - 1) / kScanTile; }

static size_t copy_ws_size(uint32_t n, uint64_t cap)
{
    const uint64_t nb = n_scan_blocks(n) + 1;
    const uint64_t nt = (cap + kCopyTile - 1) / kCopyTile;
    return sizeof(WsHead) + ((nb * 8 + 15) & ~15ull) + nt * 4;
}

static bool carve(void* ws, size_t ws_bytes, uint32_t n, uint64_t cap, CopyWs& c)
{
    if (!ws || ws_bytes < copy_ws_size(n, cap)) return false;
    char* p = static_cast<char*>(ws);
    c.head = reinterpret_cast<WsHead*>(p);
    c.partials = reinterpret_cast<uint64_t*>(p + sizeof(WsHead));
    const uint64_t nb = n_scan_blocks(n) + 1;
    c.map = reinterpret_cast<uint32_t*>(p + sizeof(WsHead) + ((nb * 8 + 15) & ~15ull));
    return true;
}

template <class Size>
static kmws_status launch_scan(Size size, uint32_t n, uint64_t* out, uint64_t* partials, hipStream_t s)
{
    const uint32_t nb = (uint32_t)n_scan_blocks(n);
    if (nb == 0) return hip_status(hipMemsetAsync(out, 0, sizeof(uint64_t), s));
    hipLaunchKernelGGL(scan_reduce_kernel<Size>, dim3(nb), dim3(kBlock), 0, s, size, n, partials);
    hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kBlock), 0, s, partials, nb, out + n);
    hipLaunchKernelGGL(scan_emit_kernel<Size>, dim3(nb), dim3(kBlock), 0, s, size, n, partials, out);
    return hip_status(hipGetLastError());
}

template <bool HEADERS>
static kmws_status launch_copy(const uint8_t* src, uint8_t* dst, uint64_t cap, const uint64_t* start,
                               const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c, hipStream_t s)
{
    hipLaunchKernelGGL(dst_map_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, start, n, cap, c.map,
                       c.head);
    const uint64_t ntiles = (cap + kCopyTile - 1) / kCopyTile;
    constexpr uint64_t kMaxBlocks = (1ull << 32) / kBlock / 2;
    for (uint64_t t0 = 0; t0 < ntiles; t0 += kMaxBlocks) {
        const uint64_t nb = ntiles - t0 < kMaxBlocks ? ntiles - t0 : kMaxBlocks;
        hipLaunchKernelGGL(mask_copy_kernel<HEADERS>, dim3((uint32_t)nb), dim3(kBlock), 0, s, src, dst, start, d,
                           flags, n, c.map, c.head, (uint32_t)t0);
    }
    return hip_status(hipGetLastError());
}

}  // namespace kmws

using namespace kmws;

extern "C" {

size_t kmws_copy_workspace_size(uint32_t n, uint64_t dst_cap) { return copy_ws_size(n, dst_cap); }

kmws_status kmws_encode_batch(const uint8_t* src, const kmws_desc* descs, const uint16_t* flags, uint32_t n,
                              uint8_t* dst, uint64_t dst_cap, uint64_t* wire_off, void* workspace,
                              size_t workspace_bytes, void* stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    CopyWs c;
    if (!wire_off || (n && (!src || !descs || !flags || !dst)) || (reinterpret_cast<uintptr_t>(dst) & 15u) ||
        (reinterpret_cast<uintptr_t>(src) & 15u) || !carve(workspace, workspace_bytes, n, dst_cap, c))
        return workspace && workspace_bytes < copy_ws_size(n, dst_cap) ? KMWS_ERR_BUFFER_TOO_SMALL
                                                                       : KMWS_ERR_INVALID_PARAM;
    if (hipMemsetAsync(c.head, 0, sizeof(WsHead), s) != hipSuccess) return KMWS_ERR_FAILED;
    kmws_status st = launch_scan(WireSize{descs, flags}, n, wire_off, c.partials, s);
    if (st != KMWS_OK || n == 0) return st;
    return launch_copy<true>(src, dst, dst_cap, wire_off, descs, flags, n, c, s);
}

kmws_status kmws_gather_unmask(const uint8_t* src, const kmws_desc* descs, uint32_t n, uint8_t* dst,
                               uint64_t dst_cap, uint64_t* dst_off, void* workspace, size_t workspace_bytes,
                               void* stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    CopyWs c;
    if (!dst_off || (n && (!src || !descs || !dst)) || (reinterpret_cast<uintptr_t>(dst) & 15u) ||
        (reinterpret_cast<uintptr_t>(src) & 15u) || !carve(workspace, workspace_bytes, n, dst_cap, c))
        return workspace && workspace_bytes < copy_ws_size(n, dst_cap) ? KMWS_ERR_BUFFER_TOO_SMALL
                                                                       : KMWS_ERR_INVALID_PARAM;
    if (hipMemsetAsync(c.head, 0, sizeof(WsHead), s) != hipSuccess) return KMWS_ERR_FAILED;
    kmws_status st = launch_scan(PayloadSize{descs}, n, dst_off, c.partials, s);
    if (st != KMWS_OK || n == 0) return st;
    return launch_copy<false>(src, dst, dst_cap, dst_off, descs, nullptr, n, c, s);
}

size_t kmws_unpack_workspace_size(void) { return sizeof(WsHead); }

kmws_status kmws_unpack_headers(const uint8_t* wire, uint64_t wire_len, const uint64_t* hdr_off, uint32_t n,
                                int mode, kmws_desc* out_desc, uint16_t* out_flags, uint8_t* out_err,
                                void* workspace, size_t workspace_bytes, void* stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!workspace || workspace_bytes < sizeof(WsHead) || (n && (!wire || !hdr_off || !out_desc)) ||
        (mode != KMWS_MODE_CLIENT && mode != KMWS_MODE_SERVER))
        return KMWS_ERR_INVALID_PARAM;
    WsHead* head = static_cast<WsHead*>(workspace);
    if (hipMemsetAsync(head, 0, sizeof(WsHead), s) != hipSuccess) return KMWS_ERR_FAILED;
    if (n == 0) return KMWS_OK;
    hipLaunchKernelGGL(unpack_headers_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, wire, wire_len,
                       hdr_off, n, mode, out_desc, out_flags, out_err, head);
    return hip_status(hipGetLastError());
}

}  // extern "C"
