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

// ------------------------------ frame-major mask-copy ------------------------------
// Output space [0, total) = regions back to back; region f = header (hl bytes,
// 0 for a payload-only gather) then payload (len bytes) read from
// src + descs[f].off and XORed with the rotated key.  Output words (16 B,
// aligned) split into
//   interior words: fully inside one payload -> interior_kernel, one wave per
//     unit of 256 words (4 KiB), the source shift uniform per frame, so each
//     lane loads one aligned word and takes the next from its neighbour;
//   boundary words: the rest (a word whose first byte lies in a header, or
//     the word straddling a payload end) -> boundary_kernel, owned by the one
//     frame whose region holds the word's first byte, composed byte-exactly.
// Every output byte in [0, total) is written exactly once.
constexpr int kUnitWords = 256;  // interior words per wave unit (4 words per lane)

struct FrameGeom {
    uint64_t r0, p0, r1;  // region start, payload start, region end (= payload end)
    uint64_t sdel;        // source offset - p0 (mod 2^64): source byte of output byte a = a + sdel
    uint32_t key;         // key to apply (0 = none)
    uint32_t len;
};

template <bool HEADERS>
__device__ __forceinline__ FrameGeom geom(uint32_t f, const uint64_t* __restrict__ start,
                                          const kmws_desc* __restrict__ d, const uint16_t* __restrict__ flags)
{
    const kmws_desc x = d[f];
    FrameGeom g;
    g.r0 = start[f];
    uint32_t hl = 0;
    g.key = x.key;
    if (HEADERS) {
        const uint32_t mask = (flags[f] >> 8) & 1u;
        hl = hdr_len(x.len, mask);
        if (!mask) g.key = 0;
    }
    g.p0 = g.r0 + hl;
    g.r1 = g.p0 + x.len;
    g.sdel = x.off - g.p0;
    g.len = x.len;
    return g;
}

// Interior word range [wlo, whi) of a frame and its number of wave units.
__device__ __forceinline__ void interior(const FrameGeom& g, uint64_t& wlo, uint64_t& whi)
{
    wlo = (g.p0 + 15) >> 4;
    whi = g.r1 >> 4;
    if (whi < wlo) whi = wlo;
}

template <bool HEADERS>
struct UnitCount {
    const uint64_t* start;
    const kmws_desc* d;
    const uint16_t* flags;
    __device__ uint64_t operator()(uint32_t f) const
    {
        const FrameGeom g = geom<HEADERS>(f, start, d, flags);
        uint64_t wlo, whi;
        interior(g, wlo, whi);
        return (whi - wlo + kUnitWords - 1) / kUnitWords;
    }
};

// One record per interior unit, written by the unit's frame: everything a
// wave needs in one 32-byte scalar load.
struct UnitRec {
    uint64_t dst;     // output byte of the unit's first word (16-B aligned)
    uint64_t src;     // source byte of that word (any alignment)
    uint32_t nwords;  // 1..kUnitWords
    uint32_t rk;      // rotated key for the unit's aligned output words (0 = no mask)
    uint64_t pad;
};
static_assert(sizeof(UnitRec) == 32, "UnitRec is one s_load_dwordx8");

// Per-unit records; also the capacity check (status set if total > cap).
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) unit_rec_kernel(const uint64_t* __restrict__ start,
                                                          const kmws_desc* __restrict__ d,
                                                          const uint16_t* __restrict__ flags,
                                                          const uint64_t* __restrict__ unit_off, uint32_t n,
                                                          uint64_t cap, UnitRec* __restrict__ rec,
                                                          WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    if (start[n] > cap) {
        if (f == 0) atomicOr(&head->status, kStatusBadDesc);
        return;
    }
    const FrameGeom g = geom<HEADERS>(f, start, d, flags);
    uint64_t wlo, whi;
    interior(g, wlo, whi);
    const uint32_t rk = g.key ? rot_key(g.key, g.p0) : 0u;
    uint64_t w = wlo;
    for (uint64_t u = unit_off[f]; u < unit_off[f + 1]; ++u, w += kUnitWords) {
        UnitRec r;
        r.dst = 16u * w;
        r.src = 16u * w + g.sdel;
        r.nwords = (uint32_t)(whi - w < (uint64_t)kUnitWords ? whi - w : (uint64_t)kUnitWords);
        r.rk = rk;
        r.pad = 0;
        rec[u] = r;
    }
}

// One wave per interior unit: 4 words per lane, 1 KiB per wave-instruction.
__global__ void __launch_bounds__(kBlock) interior_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          const uint64_t* __restrict__ unit_off, uint32_t n,
                                                          const UnitRec* __restrict__ rec,
                                                          const WsHead* __restrict__ head, uint64_t unit_base)
{
    const int lane = threadIdx.x & 63;
    // wave id through readfirstlane: provably uniform, so the record is one scalar load
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t u = unit_base + (uint64_t)blockIdx.x * (kBlock / 64) + wave;
    // record, unit count and status are independent scalar loads (one latency
    // level); records past the count lie inside the workspace and are ignored
    const UnitRec r = rec[u];
    const uint64_t total_units = unit_off[n];
    const uint32_t st = head->status;
    // no early exit between these loads and their uses (the compiler would sink
    // the record load below the count's wait): an out-of-range wave has 0 words
    const uint32_t nwords = (u < total_units && st == 0) ? r.nwords : 0u;
    const uint32_t delta = (uint32_t)(r.src & 15u);   // same for every word of the unit
    if (nwords == 0) return;                            // wave-uniform, after the record's wait
    const uint8_t* s0 = src + (r.src - delta);
    const uint32_t last = nwords - 1;
    constexpr int kW = kUnitWords / 64;
    // Every load is issued before the first store (vmcnt also counts stores, so
    // a load issued after a store would make its wait cover that store too).
    // Addresses are clamped to the unit instead of predicating the loads.
    u32x4 lo[kW], ex[kW];
#pragma unroll
    for (int i = 0; i < kW; ++i) {
        const uint32_t k = lane + 64 * i;
        lo[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s0 + 16u * (k < last ? k : last)));
    }
    if (delta) {
        // the next aligned source word comes from lane + 1, except on lane 63
        // and on the unit's last word, which load it themselves
#pragma unroll
        for (int i = 0; i < kW; ++i) {
            const uint32_t k = lane + 64 * i;
            if (lane == 63 || k >= last)
                ex[i] = *reinterpret_cast<const u32x4*>(s0 + 16u * ((k < last ? k : last) + 1));
        }
    }
    u32x4 out[kW];
#pragma unroll
    for (int i = 0; i < kW; ++i) {
        const uint32_t k = lane + 64 * i;
        u32x4 v = lo[i];
        if (delta) {
            u32x4 hi;
            hi.x = __shfl_down(lo[i].x, 1, 64);
            hi.y = __shfl_down(lo[i].y, 1, 64);
            hi.z = __shfl_down(lo[i].z, 1, 64);
            hi.w = __shfl_down(lo[i].w, 1, 64);
            if (lane == 63 || k >= last) hi = ex[i];
            v = funnel16(lo[i], hi, delta);
        }
        out[i] = v ^ r.rk;
    }
#pragma unroll
    for (int i = 0; i < kW; ++i) {
        const uint32_t k = lane + 64 * i;
        if (k < nwords) __builtin_nontemporal_store(out[i], reinterpret_cast<u32x4*>(dst + r.dst + 16u * k));
    }
}

// One lane per frame: the boundary words whose first byte lies in this frame's
// region: [ceil(r0/16), ceil(p0/16)) (header words) and the word straddling the
// payload end, composed from every frame that overlaps them.
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) boundary_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          const uint64_t* __restrict__ start,
                                                          const kmws_desc* __restrict__ d,
                                                          const uint16_t* __restrict__ flags, uint32_t n,
                                                          const WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n || head->status != 0) return;
    const uint64_t total = start[n];
    const FrameGeom g = geom<HEADERS>(f, start, d, flags);
    const uint64_t a_hdr0 = (g.r0 + 15) >> 4, a_hdr1 = (g.p0 + 15) >> 4;
    const uint64_t b0 = (g.r1 >> 4) > a_hdr1 ? (g.r1 >> 4) : a_hdr1, b1 = (g.r1 + 15) >> 4;
    for (int part = 0; part < 2; ++part) {
        const uint64_t wa = part == 0 ? a_hdr0 : b0, wb = part == 0 ? a_hdr1 : b1;
        for (uint64_t w = wa; w < wb; ++w) {
            const uint64_t a = 16u * w;
            u32x4 out = u32x4{0, 0, 0, 0};
            for (uint32_t j = f; j < n; ++j) {
                const FrameGeom h = j == f ? g : geom<HEADERS>(j, start, d, flags);
                if (h.r0 >= a + 16) break;
                if (HEADERS && h.p0 > a && h.p0 > h.r0) {  // header bytes [r0, p0)
                    const kmws_desc x = d[j];
                    uint64_t h0, h1;
                    build_header(x.len, flags[j], x.key, h0, h1);
                    const int s = (int)((int64_t)h.r0 - (int64_t)a);
                    const u32x4 H = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
                    const int he = (int)(h.p0 - h.r0) + s;
                    out |= shift_in(H, s) & byte_range(s < 0 ? 0 : s, he > 16 ? 16 : he);
                }
                if (h.r1 > h.p0 && h.p0 < a + 16 && h.r1 > a) {  // payload bytes
                    const uint64_t lo_b = h.p0 > a ? h.p0 : a, hi_b = h.r1 < a + 16 ? h.r1 : a + 16;
                    const uint64_t slo = lo_b + h.sdel, shi = hi_b + h.sdel;
                    const uint64_t s0 = slo & ~(uint64_t)15, s1 = (shi - 1) & ~(uint64_t)15;
                    const u32x4 W0 = *reinterpret_cast<const u32x4*>(src + s0);
                    const u32x4 W1 = s1 != s0 ? *reinterpret_cast<const u32x4*>(src + s1) : W0;
                    const int dd = (int)((int64_t)(a + h.sdel) - (int64_t)s0);  // in [-15, 15]
                    const u32x4 V = dd >= 0 ? funnel16(W0, W1, (uint32_t)dd)
                                            : funnel16(u32x4{0, 0, 0, 0}, W0, (uint32_t)(16 + dd));
                    const uint32_t rk = h.key ? rot_key(h.key, h.p0) : 0u;
                    out |= (V ^ rk) & byte_range((int)(lo_b - a), (int)(hi_b - a));
                }
            }
            if (a + 16 <= total) {
                *reinterpret_cast<u32x4*>(dst + a) = out;
            } else {  // last partial word of the output: byte stores
                for (uint64_t p = a; p < total; ++p) {
                    const uint32_t k = (uint32_t)(p - a);
                    const uint32_t dwv = (k & 8u) ? ((k & 4u) ? out.w : out.z) : ((k & 4u) ? out.y : out.x);
                    dst[p] = (uint8_t)(dwv >> (8 * (k & 3u)));
                }
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
    uint64_t* unit_off;
    UnitRec* rec;
};

static uint64_t n_scan_blocks(uint32_t n) { return ((uint64_t)n + kScanTile - 1) / kScanTile; }
static uint64_t max_units(uint32_t n, uint64_t cap) { return (cap + kUnitWords * 16 - 1) / (kUnitWords * 16) + n; }
static uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }

static size_t copy_ws_size(uint32_t n, uint64_t cap)
{
    return sizeof(WsHead) + r16((n_scan_blocks(n) + 1) * 8) + r16(((uint64_t)n + 1) * 8) +
           max_units(n, cap) * sizeof(UnitRec);
}

static bool carve(void* ws, size_t ws_bytes, uint32_t n, uint64_t cap, CopyWs& c)
{
    if (!ws || ws_bytes < copy_ws_size(n, cap)) return false;
    char* p = static_cast<char*>(ws);
    c.head = reinterpret_cast<WsHead*>(p);
    p += sizeof(WsHead);
    c.partials = reinterpret_cast<uint64_t*>(p);
    p += r16((n_scan_blocks(n) + 1) * 8);
    c.unit_off = reinterpret_cast<uint64_t*>(p);
    p += r16(((uint64_t)n + 1) * 8);
    c.rec = reinterpret_cast<UnitRec*>(p);
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
    kmws_status st = launch_scan(UnitCount<HEADERS>{start, d, flags}, n, c.unit_off, c.partials, s);
    if (st != KMWS_OK) return st;
    const uint32_t fb = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(unit_rec_kernel<HEADERS>, dim3(fb), dim3(kBlock), 0, s, start, d, flags, c.unit_off, n, cap,
                       c.rec, c.head);
    const uint64_t units = max_units(n, cap);  // upper bound; surplus waves exit at once
    constexpr uint64_t kWavesPerBlock = kBlock / 64;
    constexpr uint64_t kMaxUnitsPerLaunch = ((1ull << 32) / kBlock / 2) * kWavesPerBlock;
    for (uint64_t u0 = 0; u0 < units; u0 += kMaxUnitsPerLaunch) {
        const uint64_t nu = units - u0 < kMaxUnitsPerLaunch ? units - u0 : kMaxUnitsPerLaunch;
        hipLaunchKernelGGL(interior_kernel, dim3((uint32_t)((nu + kWavesPerBlock - 1) / kWavesPerBlock)),
                           dim3(kBlock), 0, s, src, dst, c.unit_off, n, c.rec, c.head, u0);
    }
    hipLaunchKernelGGL(boundary_kernel<HEADERS>, dim3(fb), dim3(kBlock), 0, s, src, dst, start, d, flags, n, c.head);
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
