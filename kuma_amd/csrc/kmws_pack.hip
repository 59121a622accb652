// Batched frame-header pack/unpack and out-of-place mask-copy for MI355X.
//
// Encode (kmws_encode_batch) = for every frame, WSHandler::encodeFrameHeader
// (src/ws/WSHandler.cpp:46-106) followed by the masked payload
// (WebSocket::Impl::sendWsFrame, src/ws/WebSocketImpl.cpp:381-404): the wire
// image is header_0 payload_0 header_1 payload_1 ...  Kernels:
//   1. reduce_kernel, 2048 frames per block: two per-frame values -- the wire
//      size (2/4/10 + 4*mask + len) and an upper bound on the frame's wave
//      units -- summed per 256-frame row and per tile; scan_tiles_kernel
//      (one block) scans the tile totals;
//   2. prologue_kernel, 256 frames per block: each frame's wire offset and
//      first unit slot (row prefix + block scan), the few words around its
//      boundaries (header bytes, the next frame's first bytes), composed
//      byte-exactly, and one 32-byte record per wave unit;
//   3. copy_kernel: one wave per unit of a frame's owned 64-byte granules;
//      interior words are loaded, funnel-shifted and XORed with the rotated
//      key, edge words are merged in; every granule is written once, by one
//      store instruction.
// Decode (descriptor-indexed): kmws_unpack_headers parses and
// validates one header per frame with the reference's rules
// (WSHandler.cpp:118-234, including the 127-length quirk); the payload is then
// unmasked in place (kmws_unmask_batch) or gathered + unmasked into a dense
// arena by the same copy kernels (kmws_gather_unmask).
// Header-only pack (kmws_pack_headers, kuma's iovec form): each header into a
// 16-byte slot, with the wire offsets after reduce_kernel.  Boundary discovery on the
// device (kmws_find_headers_streams): the serial header-chain walk, one lane
// per stream.
#include "kmws_common.hpp"
#include "kmws_frame_parse.hpp"

namespace kmws {

constexpr int kScanItems = 8;                      // frames per lane in reduce_kernel
constexpr int kScanTile = kBlock * kScanItems;     // 2048 frames per block

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
// One pass scans two per-frame quantities: the region size (header + payload
// for encode, payload for gather) -> region offsets, and an upper bound on the
// frame's wave units (it depends on the region size only) -> unit slot bases.
struct V2 {
    uint64_t a, b;
};
__device__ __forceinline__ V2 operator+(V2 x, V2 y) { return V2{x.a + y.a, x.b + y.b}; }

// Output words per wave unit: 4 per lane (4 KiB).  2, 3, 5, 6 and 8 words per
// lane measured the same or slower on cfg3/cfg4/64 KiB frames (round 1); again
// this round, 5 and 6 words per lane (one unit per 4 KiB fragment instead of
// two): cfg4 encode 0.57 / 0.60 against 0.73 (profiles/r03aq_unit_words_ab.txt).
constexpr int kUnitWords = 64 * 4;
// The unit copy grid's parts: 2 / 4 / 16 / XCD runs all slower on cfg4 and
// cfg3 (profiles/r03bi_copy_split_ab.txt).
constexpr uint32_t kCopySplit = 8;
constexpr uint32_t kChunkSplit = 4;  // the chunk grid's parts (r04r: 4 > 8 > 16 on cfg4)
constexpr uint64_t kUnitAlign = 64;  // unit bases: 1 KiB aligned in the output
constexpr uint64_t kLineBytes = 64;  // ownership granule: 64 B keeps a frame edge at 1 + 4 words
constexpr uint64_t kLineWords = kLineBytes / 16;
constexpr int kEdgeWords = 1 + (int)kLineWords;   // owned non-interior words per frame (at most)

// Wave units of a region of R bytes, whatever its offset: a region holds at most
// ceil(R/kLineBytes) granule starts, and the first unit's base lies at most
// 64 - kLineWords words below the first owned word.
__host__ __device__ __forceinline__ uint64_t unit_bound(uint64_t R)
{
    if (R == 0) return 0;
    return (kLineWords * ((R + kLineBytes - 1) / kLineBytes) + (kUnitAlign - kLineWords) + kUnitWords - 1) /
           kUnitWords;
}

// Per-frame quantities: load() reads what they depend on, value() computes
// them (split so a caller can issue many frames' loads before one wait).
struct SizeRaw {
    uint32_t len, fl;
};
struct WireSize {
    static constexpr bool kHeaders = true;
    static constexpr bool kClearsStatus = true;  // reduce_kernel clears the status word
    const kmws_desc* d;
    const uint16_t* flags;
    __device__ SizeRaw load(uint32_t f) const { return SizeRaw{d[f].len, flags[f]}; }
    __device__ V2 value(SizeRaw x) const
    {
        const uint64_t r = (uint64_t)hdr_len(x.len, (x.fl >> 8) & 1u) + x.len;
        return V2{r, unit_bound(r)};
    }
};
struct PayloadSize {
    static constexpr bool kHeaders = false;
    static constexpr bool kClearsStatus = true;
    const kmws_desc* d;
    __device__ SizeRaw load(uint32_t f) const { return SizeRaw{d[f].len, 0u}; }
    __device__ V2 value(SizeRaw x) const { return V2{x.len, unit_bound(x.len)}; }
};
// The descriptor-indexed decode fused into the gather's scan
// (kmws_unpack_gather): load() parses frame f's header where it lies in the
// wire (unpack_one: the frame's descriptor, flags and WSError are written for
// the prologue and copy kernels that follow) and yields its payload length.
// A header error ORs the status word during the kernel, so the word is
// cleared by a launch before it, not by reduce_kernel.
struct HeaderPayloadSize {
    static constexpr bool kHeaders = false;
    static constexpr bool kClearsStatus = false;
    const uint8_t* wire;
    uint64_t wire_len;
    const uint64_t* hdr_off;
    uint32_t n;
    int mode;
    kmws_desc* out_desc;
    uint16_t* out_flags;
    uint8_t* out_err;
    WsHead* head;
    __device__ SizeRaw load(uint32_t f) const
    {
        const kmws_desc o = unpack_one(wire, wire_len, hdr_off, n, f, mode, out_desc, out_flags, out_err, head);
        return SizeRaw{o.len, 0u};
    }
    __device__ V2 value(SizeRaw x) const { return V2{x.len, unit_bound(x.len)}; }
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t x)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// Two-level scan.  reduce_kernel: a block sums 2048 frames (8 rows of 256,
// read row-striped so every load is coalesced) and writes each row's exclusive
// prefix inside the tile to grp[] and the tile's total to tiles[];
// scan_tiles_kernel (one block) turns tiles[] into exclusive prefixes and
// writes the grand totals.  The per-frame offsets are emitted by the kernel
// that reads each 256-frame row next (the prologue, or the header-slot kernel):
// two loads give the row's prefix, a block scan the frame's.  Measured on 4 M
// frames: a decoupled look-back scan (one launch, tiles publishing aggregates
// and inclusive prefixes through device-scope atomics) 95-115 us; the reduce
// with the last block scanning the totals (a device-scope fence per block
// before its counter increment, i.e. an L2 write-back) 65-94 us.
constexpr int kRowsPerTile = kScanItems;  // 256-frame rows per 2048-frame tile

// Exclusive scan over the block (256 threads); `total` = the block's sum.
// s_w: 4 entries of LDS, free on entry (the caller syncs before reusing them).
__device__ __forceinline__ V2 block_excl_scan(V2 v, V2* __restrict__ s_w, V2& total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const V2 inc{wave_incl_scan(v.a), wave_incl_scan(v.b)};
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    V2 before{0, 0};
    total = V2{0, 0};
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        const V2 t = s_w[w];
        if (w < wave) before = before + t;
        total = total + t;
    }
    return V2{before.a + inc.a - v.a, before.b + inc.b - v.b};
}

// Loads are coalesced (row-striped: frame i * 256 + thread, all 16 issued
// before one wait) and staged in LDS; each thread then sums 8 consecutive
// frames, and a row's total is one 32-lane reduction (a wave-wide 64-bit
// reduction per row and quantity -- 16 per thread -- made the kernel ALU-bound:
// 24-36 us on 4 M frames).
constexpr uint32_t kPastEnd = 1u << 31;  // SizeRaw.fl: a slot past the batch
template <class Size>
__global__ void __launch_bounds__(kBlock) reduce_kernel(Size size, uint32_t n, V2* __restrict__ tiles,
                                                        V2* __restrict__ grp, WsHead* __restrict__ head)
{
    __shared__ SizeRaw s_raw[kScanTile];
    __shared__ V2 s_row[kRowsPerTile];
    const uint32_t t = threadIdx.x;
    // the batch's status word starts clear (set only by the kernels after this one)
    if constexpr (Size::kClearsStatus)
        if (blockIdx.x == 0 && t == 0) head->status = 0;
    const uint64_t F = (uint64_t)blockIdx.x * kScanTile;
    SizeRaw raw[kRowsPerTile];
#pragma unroll
    for (int i = 0; i < kRowsPerTile; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        raw[i] = size.load((uint32_t)__builtin_elementwise_min(f, (uint64_t)n - 1));
    }
#pragma unroll
    for (int i = 0; i < kRowsPerTile; ++i) {
        if (F + (uint64_t)i * kBlock + t >= n) raw[i].fl |= kPastEnd;
        s_raw[i * kBlock + t] = raw[i];
    }
    __syncthreads();
    V2 sum{0, 0};  // frames 8t .. 8t + 7 of the tile: row t / 32
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const SizeRaw r = s_raw[kScanItems * t + k];
        if (!(r.fl & kPastEnd)) sum = sum + size.value(r);
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
        sum.a += __shfl_xor(sum.a, o, 64);
        sum.b += __shfl_xor(sum.b, o, 64);
    }
    if ((t & 31u) == 0) s_row[t >> 5] = sum;
    __syncthreads();
    if (t <= (unsigned)kRowsPerTile) {  // thread i < 8: row i's prefix; thread 8: the tile's total
        V2 pre{0, 0};
#pragma unroll
        for (uint32_t r = 0; r < (uint32_t)kRowsPerTile; ++r)
            if (r < t) pre = pre + s_row[r];
        const uint64_t g = (uint64_t)blockIdx.x * kRowsPerTile + t;
        if (t == (unsigned)kRowsPerTile) tiles[blockIdx.x] = pre;
        else if (g * kBlock < n) grp[g] = pre;
    }
}

// tiles[0, ntiles) -> exclusive prefixes, tiles[ntiles] = the totals (also
// out_a[n]: the caller's offsets array has n + 1 entries).  One block.
__global__ void __launch_bounds__(kBlock) scan_tiles_kernel(V2* __restrict__ tiles, uint32_t ntiles,
                                                            uint64_t* __restrict__ out_a, uint32_t n)
{
    __shared__ V2 s_w[kBlock / 64];
    constexpr int K = 8;
    V2 carry{0, 0};
    for (uint64_t c = 0; c < ntiles; c += (uint64_t)kBlock * K) {
        V2 t[K], sum{0, 0};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t j = c + (uint64_t)threadIdx.x * K + k;
            t[k] = j < ntiles ? tiles[j] : V2{0, 0};
            sum = sum + t[k];
        }
        V2 tot;
        V2 run = carry + block_excl_scan(sum, s_w, tot);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t j = c + (uint64_t)threadIdx.x * K + k;
            if (j < ntiles) tiles[j] = run;
            run = run + t[k];
        }
        carry = carry + tot;
        __syncthreads();  // s_w is reused
    }
    if (threadIdx.x == 0) {
        tiles[ntiles] = carry;
        out_a[n] = carry.a;
    }
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

// ------------------------------ mask-copy ------------------------------
// Output space [0, total) = regions back to back; region f = header (hl bytes,
// none for a payload-only gather) then payload (len bytes) read from
// src + descs[f].off and XORed with the rotated key.
//
// Ownership: every 64-byte output granule belongs to the frame whose region
// holds the granule's first byte.  A frame's owned granules are cut into wave
// units of kUnitWords words (4 KiB) whose bases are 1 KiB aligned, so a granule is
// written by ONE store instruction of one wave (a line written piecewise by
// different waves at different times -- e.g. a separate edge kernel -- goes to
// memory as partial writes: unaligned units measured 15 % slower).  Only the line holding
// a frame boundary is shared, by two adjacent units.  Inside a unit
//   interior words (inside the frame's payload) take the fast path: the source
//     shift is uniform, each lane loads one aligned word and takes the next one
//     from its neighbour;
//   edge words -- at most one holding the header's end, and the words after the
//     payload's end up to the granule's end (the next frames' first bytes) --
//     are composed byte-exactly beforehand (edge_block), one thread per word,
//     into a per-frame buffer; the wave loads them (one lane per word) and moves
//     them into their store lanes with a lane permute.
// Every output byte in [0, total) is written exactly once.

struct FrameGeom {
    uint64_t r0, p0, r1;  // region start, payload start, region end (= payload end)
    uint64_t sdel;        // source offset - p0 (mod 2^64): source byte of output byte a = a + sdel
    uint32_t key;         // key to apply (0 = none)
    uint32_t len;
};

// Output words of a frame: owned [olo, ohi), interior [ilo, ihi) inside them,
// and its units (bases b0, b0 + 256, ...).
struct FrameWords {
    uint64_t olo, ohi, ilo, ihi, b0, units;
};

__device__ __forceinline__ FrameWords frame_words(const FrameGeom& g, uint64_t total_words)
{
    FrameWords w;
    w.olo = kLineWords * ((g.r0 + kLineBytes - 1) / kLineBytes);
    uint64_t ohi = kLineWords * ((g.r1 + kLineBytes - 1) / kLineBytes);
    if (ohi > total_words) ohi = total_words;  // the output's last line
    w.ohi = ohi > w.olo ? ohi : w.olo;
    uint64_t ilo = (g.p0 + 15) >> 4, ihi = g.r1 >> 4;  // words inside the payload
    ilo = ilo > w.olo ? ilo : w.olo;
    ihi = ihi < w.ohi ? ihi : w.ohi;
    w.ilo = ilo < w.ohi ? ilo : w.ohi;
    w.ihi = ihi > w.ilo ? ihi : w.ilo;
    w.b0 = w.olo & ~(kUnitAlign - 1);
    w.units = w.ohi > w.olo ? (w.ohi - w.b0 + kUnitWords - 1) / kUnitWords : 0;
    return w;
}

// One record per unit slot: everything a wave needs in one 32-byte scalar load.
struct UnitRec {
    uint64_t dst;       // output byte of the unit's base word
    uint64_t src;       // source byte of that word (any alignment)
    uint32_t f;         // owning frame
    uint32_t rk;        // rotated key for the unit's aligned output words (0 = no mask)
    uint32_t own;       // owned words [klo, khi) of the unit: klo | head_f << 12 | khi << 16 (khi == 0:
                        // empty slot); head_f = the frame's edge words before its interior
    uint32_t inner;     // interior words [ilo, ihi): ilo | ihi << 16, klo <= ilo <= ihi <= khi
};
static_assert(sizeof(UnitRec) == 32, "UnitRec is one s_load_dwordx8");

// Geometry of frame j given where its region starts (regions lie back to back:
// frame j+1 starts where frame j's payload ends).
template <bool HEADERS>
__device__ __forceinline__ FrameGeom geom_at(const kmws_desc& x, uint32_t fl, uint64_t r0)
{
    const uint32_t mask = HEADERS ? (fl >> 8) & 1u : 1u;
    FrameGeom g;
    g.r0 = r0;
    g.p0 = r0 + (HEADERS ? hdr_len(x.len, mask) : 0u);
    g.r1 = g.p0 + x.len;
    g.sdel = x.off - g.p0;
    g.key = mask ? x.key : 0u;
    g.len = x.len;
    return g;
}

// Descriptors (and flags) of frames f, f+1, f+2 -- the frames a word starting in
// frame f overlaps in all but tiny-frame batches -- loaded at once (indices
// clamped instead of branches, so the loads issue together).
constexpr int kPre = 3;
template <bool HEADERS>
__device__ __forceinline__ void load_descs(uint32_t f, uint32_t n, kmws_desc (&x)[kPre], uint32_t (&fl)[kPre],
                                           const kmws_desc* __restrict__ d, const uint16_t* __restrict__ flags)
{
#pragma unroll
    for (int i = 0; i < kPre; ++i) {
        const uint32_t j = f + i < n ? f + i : n - 1;
        x[i] = d[j];
        fl[i] = HEADERS ? flags[j] : 0u;
    }
}

// Output word [a, a + 16) composed byte by byte from every frame from f on that
// overlaps it -- the rare word three or more regions reach into (frames shorter
// than a word); few registers, one frame's geometry at a time (frame j+1's
// region starts where frame j's ends).
template <bool HEADERS>
__device__ __attribute__((noinline)) u32x4 compose_word_bytes(uint64_t a, uint32_t f, uint32_t n,
                                                              const uint8_t* __restrict__ src, FrameGeom h,
                                                              uint32_t flj, const kmws_desc* __restrict__ d,
                                                              const uint16_t* __restrict__ flags)
{
    u32x4 out = u32x4{0, 0, 0, 0};
    uint32_t j = f;
    for (uint32_t b = 0; b < 16; ++b) {
        const uint64_t x = a + b;
        while (x >= h.r1 && j + 1 < n) {
            ++j;
            flj = HEADERS ? flags[j] : 0u;
            h = geom_at<HEADERS>(d[j], flj, h.r1);
        }
        if (x < h.r0 || x >= h.r1) continue;  // past the last region
        uint32_t v;
        if (x < h.p0) {  // header byte x - r0
            uint64_t h0, h1;
            build_header(h.len, flj, h.key, h0, h1);
            const uint32_t k = (uint32_t)(x - h.r0);
            v = (uint32_t)((k < 8 ? h0 >> (8 * k) : h1 >> (8 * (k - 8))) & 0xFFu);
        } else {  // payload byte: data[i] ^ key[i % 4]
            v = src[x + h.sdel] ^ ((h.key >> (8 * ((x - h.p0) & 3u))) & 0xFFu);
        }
        const uint32_t sh = 8u * (b & 3u), q = b >> 2;
        if (q == 0) out.x |= v << sh;
        else if (q == 1) out.y |= v << sh;
        else if (q == 2) out.z |= v << sh;
        else out.w |= v << sh;
    }
    return out;
}

// Payload source words of frame h for the output word [a, a + 16): the aligned
// words holding its first and last payload byte there (src + 0 when it has none).
__device__ __forceinline__ void pay_words(bool live, const FrameGeom& h, uint64_t a, const uint8_t* __restrict__ src,
                                          u32x4& W0, u32x4& W1)
{
    const bool pay = live && h.r0 < a + 16 && h.r1 > h.p0 && h.p0 < a + 16 && h.r1 > a;
    const uint64_t lo_b = h.p0 > a ? h.p0 : a, hi_b = h.r1 < a + 16 ? h.r1 : a + 16;
    const uint64_t s0 = pay ? (lo_b + h.sdel) & ~(uint64_t)15 : 0;
    const uint64_t s1 = pay ? (hi_b + h.sdel - 1) & ~(uint64_t)15 : 0;
    W0 = *reinterpret_cast<const u32x4*>(src + s0);
    W1 = *reinterpret_cast<const u32x4*>(src + s1);
}

// Frame h's bytes (header, then masked payload) in [a, a + 16), its payload
// words W0/W1 from pay_words.
template <bool HEADERS>
__device__ __forceinline__ void put_frame(u32x4& out, uint64_t a, const FrameGeom& h, uint32_t fl, const u32x4& W0,
                                          const u32x4& W1)
{
    if (h.r0 >= a + 16) return;
    if (HEADERS && h.p0 > a && h.p0 > h.r0) {  // header bytes [r0, p0)
        uint64_t h0, h1;
        build_header(h.len, fl, h.key, h0, h1);
        const int s = (int)((int64_t)h.r0 - (int64_t)a);
        const u32x4 H = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
        const int he = (int)(h.p0 - h.r0) + s;
        out |= shift_in(H, s) & byte_range(s < 0 ? 0 : s, he > 16 ? 16 : he);
    }
    if (h.r1 > h.p0 && h.p0 < a + 16 && h.r1 > a) {  // payload bytes
        const uint64_t lo_b = h.p0 > a ? h.p0 : a, hi_b = h.r1 < a + 16 ? h.r1 : a + 16;
        const uint64_t s0 = (lo_b + h.sdel) & ~(uint64_t)15;
        const int dd = (int)((int64_t)(a + h.sdel) - (int64_t)s0);  // in [-15, 15]
        const u32x4 V = dd >= 0 ? funnel16(W0, W1, (uint32_t)dd) : funnel16(u32x4{0, 0, 0, 0}, W0, (uint32_t)(16 + dd));
        const uint32_t rk = h.key ? rot_key(h.key, h.p0) : 0u;
        out |= (V ^ rk) & byte_range((int)(lo_b - a), (int)(hi_b - a));
    }
}

// A frame's unit geometry for the slot-parallel record pass (LDS), word
// indices relative to its first unit base b0.
struct FrameUnits {
    uint64_t b0, sdel;
    uint32_t olo, ohi, ilo, ihi;  // owned and interior words - b0
    uint32_t rk, units, head_f, nedge;
};

// Everything the copy waves need of 256 frames, one block (after
// reduce_kernel: the row's prefix and a block scan give each frame's region
// offset, written to start[], and its first unit slot):
//   edge words -- a frame's owned words outside its interior: q < head_f at
//     olo + q, then the tail at ihi + (q - head_f) -- one thread per frame,
//     into LDS, then written out over one contiguous run edge[F0 * kEdgeWords ...]
//     (coalesced; 128-byte lines without a live word are skipped);
//   unit records, slot-parallel: slot s of the block finds its frame by a
//     binary search over the block's slot bases in LDS (slots past a frame's
//     exact unit count are marked empty); consecutive threads write
//     consecutive records.
// Edge words: the head word (q = 0 if head_f) holds the frame's header end and
// first payload bytes; the tail words (q = head_f + i) hold its last payload
// bytes (i = 0 only), then frame f+1's header and payload.  Every source word
// is loaded before anything is composed (one latency level): frame f's words
// of the head and first tail word, and a window of 5 consecutive source words
// of frame f+1 from which every tail word funnels its payload bytes (window
// indices clamped to f+1's payload; clamped words only feed bytes outside it,
// which are masked off).  The rare word a third region reaches into (a frame
// ending inside it) is composed byte by byte.  Frame f+1's region starts where
// frame f's ends, so only frame f's offset is read.  Owned words past the end
// of the output (the last frame's last granule) are composed as zero and never
// stored by the copy waves, which clip at the total.  Also the capacity check
// (status set if the output exceeds cap; nothing is written then).
//
// The prologue's per-row part (prologue_kernel; round 4's rejected fused row
// kernel shared it, profiles/r04i_pack_rows_ab.txt):
// row `row`'s frame offsets (written to start[]), its frames' unit geometry
// (s_fu, unit slot bases s_ub relative to the row's first slot) and edge words
// (s_edge, live counts s_ne), all in LDS.  Returns false (block-uniform) when
// the output exceeds cap: the status is set and nothing may be written.
struct RowLds {
    FrameUnits fu[kBlock];
    uint32_t ub[kBlock + 1];
    u32x4 edge[kBlock * kEdgeWords];
    uint8_t ne[kBlock];  // live edge words per frame
    V2 w[kBlock / 64];
};
struct RowInfo {
    uint64_t F0, S0, total;
    uint32_t nf;
};
template <bool HEADERS>
__device__ __forceinline__ bool row_prologue(uint32_t rid, const uint8_t* __restrict__ src,
                                             const kmws_desc* __restrict__ d, const uint16_t* __restrict__ flags,
                                             uint32_t n, uint64_t cap, WsHead* __restrict__ head,
                                             const V2* __restrict__ tiles, uint32_t ntiles,
                                             const V2* __restrict__ grp, uint64_t* __restrict__ start, RowLds& L,
                                             RowInfo& ri)
{
    FrameUnits* s_fu = L.fu;
    uint32_t* s_ub = L.ub;
    u32x4* s_edge = L.edge;
    uint8_t* s_ne = L.ne;
    V2* s_w = L.w;
    const uint32_t t = threadIdx.x;
    const uint64_t F0 = (uint64_t)rid * kBlock;
    const uint32_t nf = n - F0 < (uint64_t)kBlock ? (uint32_t)(n - F0) : (uint32_t)kBlock;
    const uint32_t f = (uint32_t)(F0 + (t < nf ? t : nf - 1));
    // totals, the row's prefix and the three frames' descriptors: one latency level
    const V2 tot = tiles[ntiles];
    const V2 pre = tiles[rid / kRowsPerTile] + grp[rid];
    const uint64_t total = tot.a;
    kmws_desc x[kPre];
    uint32_t fl[kPre];
    load_descs<HEADERS>(f, n, x, fl, d, flags);
    // this frame's region offset and first unit slot
    V2 row;
    const uint64_t rsz = (uint64_t)(HEADERS ? hdr_len(x[0].len, (fl[0] >> 8) & 1u) : 0u) + x[0].len;
    const V2 off = pre + block_excl_scan(t < nf ? V2{rsz, unit_bound(rsz)} : V2{0, 0}, s_w, row);
    const uint64_t r0 = off.a, uf = off.b, S0 = pre.b, uend = pre.b + row.b;
    if (t < nf) start[f] = r0;
    ri.F0 = F0;
    ri.S0 = S0;
    ri.total = total;
    ri.nf = nf;
    if (total > cap) {  // records would not fit the workspace; the copy waves see the status (block-uniform)
        if (F0 == 0 && t == 0) atomicOr(&head->status, kStatusBadDesc);
        return false;
    }
    FrameGeom g[kPre];
    g[0] = geom_at<HEADERS>(x[0], fl[0], r0);
#pragma unroll
    for (int i = 1; i < kPre; ++i) {
        g[i] = geom_at<HEADERS>(x[i], fl[i], g[i - 1].r1);
        if ((uint64_t)f + i >= n) g[i].r0 = ~0ull;  // past the last frame: overlaps nothing
    }
    if (t < nf) {
        const FrameWords w = frame_words(g[0], ~0ull >> 4);  // unclipped: the copy waves clip at the total
        uint32_t head_f = (uint32_t)(w.ilo - w.olo);
        uint32_t nedge = head_f + (uint32_t)(w.ohi - w.ihi);
        if (nedge > (uint32_t)kEdgeWords || w.olo - w.b0 >= kUnitAlign) {  // cannot happen
            atomicOr(&head->status, kStatusBadDesc);
            nedge = head_f = 0;
        }
        s_ub[t] = (uint32_t)(uf - S0);
        if (t == nf - 1) s_ub[nf] = (uint32_t)(uend - S0);
        FrameUnits fu;
        fu.b0 = w.b0;
        fu.sdel = g[0].sdel;
        fu.olo = (uint32_t)(w.olo - w.b0);
        fu.ohi = (uint32_t)(w.ohi - w.b0);
        fu.ilo = (uint32_t)(w.ilo - w.b0);
        fu.ihi = (uint32_t)(w.ihi - w.b0);
        fu.rk = g[0].key ? rot_key(g[0].key, g[0].p0) : 0u;
        fu.units = (uint32_t)w.units;
        fu.head_f = head_f;
        fu.nedge = nedge;
        s_ne[t] = (uint8_t)nedge;
        s_fu[t] = fu;

        const FrameGeom& F = g[0];
        const FrameGeom& N = g[1];
        const uint32_t ntail = nedge - head_f;
        const uint64_t ah = 16u * w.olo, at = 16u * w.ihi;
        u32x4 H0, H1, T0, T1, S[kLineWords + 1];
        pay_words(head_f != 0 && nedge != 0, F, ah, src, H0, H1);
        pay_words(ntail != 0, F, at, src, T0, T1);
        const bool nlive = ntail != 0 && N.r0 < at + 16 * kLineWords && N.r1 > N.p0;
        const uint64_t soff = N.p0 + N.sdel;  // f+1's source offset
        const int64_t wb = (int64_t)(at + N.sdel) >> 4, wlo = (int64_t)(soff >> 4),
                      whi = (int64_t)((soff + N.len - 1) >> 4);
        const uint32_t delta = (uint32_t)((at + N.sdel) & 15u);
#pragma unroll
        for (int j = 0; j <= (int)kLineWords; ++j) {
            int64_t k = wb + j;
            k = k < wlo ? wlo : (k > whi ? whi : k);
            S[j] = *reinterpret_cast<const u32x4*>(src + (nlive ? 16 * (uint64_t)k : 0));
        }
        u32x4* my = s_edge + t * kEdgeWords;
        uint32_t third = 0;
        if (head_f && nedge) {
            if (F.r1 < ah + 16 && (uint64_t)f + 1 < n) {
                third |= 1u;
            } else {
                u32x4 out = u32x4{0, 0, 0, 0};
                put_frame<HEADERS>(out, ah, F, fl[0], H0, H1);
                my[0] = out;
            }
        }
        const uint32_t rkN = N.key ? rot_key(N.key, N.p0) : 0u;
#pragma unroll
        for (int i = 0; i < (int)kLineWords; ++i) {
            const uint64_t a = at + 16u * i;
            const uint32_t q = head_f + i;
            if ((uint32_t)i >= ntail) break;
            if (N.r0 < a + 16 && N.r1 < a + 16 && (uint64_t)f + 2 < n) {
                third |= 1u << q;
                continue;
            }
            u32x4 out = u32x4{0, 0, 0, 0};
            if (i == 0) put_frame<HEADERS>(out, a, F, fl[0], T0, T1);
            if (N.r0 < a + 16) {
                if (HEADERS && N.p0 > a && N.p0 > N.r0) {  // f+1's header bytes [r0, p0)
                    uint64_t h0, h1;
                    build_header(N.len, fl[1], N.key, h0, h1);
                    const int sh = (int)((int64_t)N.r0 - (int64_t)a);
                    const u32x4 Hw = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
                    const int he = (int)(N.p0 - N.r0) + sh;
                    out |= shift_in(Hw, sh) & byte_range(sh < 0 ? 0 : sh, he > 16 ? 16 : he);
                }
                if (N.r1 > N.p0 && N.p0 < a + 16 && N.r1 > a) {  // f+1's payload bytes
                    const uint64_t lo_b = N.p0 > a ? N.p0 : a, hi_b = N.r1 < a + 16 ? N.r1 : a + 16;
                    out |= (funnel16(S[i], S[i + 1], delta) ^ rkN) & byte_range((int)(lo_b - a), (int)(hi_b - a));
                }
            }
            my[q] = out;
        }
#pragma clang loop unroll(disable)
        for (int q = 0; third != 0; ++q, third >>= 1) {
            if (third & 1u) {
                const uint64_t a = 16u * ((uint32_t)q < head_f ? w.olo + q : w.ihi + (q - head_f));
                my[q] = compose_word_bytes<HEADERS>(a, f, n, src, g[0], fl[0], d, flags);
            }
        }
    }
    __syncthreads();
    return true;
}

// A unit record from its frame's geometry: unit m of frame F0 + j.
__device__ __forceinline__ UnitRec make_rec(const FrameUnits& fu, uint32_t m, uint32_t f, WsHead* __restrict__ head)
{
    UnitRec r;
    const uint32_t b = m * (uint32_t)kUnitWords;  // unit base - b0
    auto rel = [&](uint32_t x) -> uint32_t {
        return x <= b ? 0u : (x - b >= (uint32_t)kUnitWords ? (uint32_t)kUnitWords : x - b);
    };
    r.dst = 16u * (fu.b0 + b);
    r.src = 16u * (fu.b0 + b) + fu.sdel;
    r.f = f;
    r.rk = fu.rk;
    const uint32_t klo = rel(fu.olo), khi = rel(fu.ohi), ilo = rel(fu.ilo), ihi = rel(fu.ihi);
    r.own = klo | fu.head_f << 12 | khi << 16;
    r.inner = ilo | ihi << 16;
    if (ilo - klo > fu.head_f)  // cannot happen
        atomicOr(&head->status, kStatusBadDesc);
    return r;
}

template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) prologue_kernel(const uint8_t* __restrict__ src,
                                                          const kmws_desc* __restrict__ d,
                                                          const uint16_t* __restrict__ flags, uint32_t n,
                                                          uint64_t cap, WsHead* __restrict__ head,
                                                          const V2* __restrict__ tiles, uint32_t ntiles,
                                                          const V2* __restrict__ grp, uint64_t* __restrict__ start,
                                                          UnitRec* __restrict__ rec, u32x4* __restrict__ edge)
{
    __shared__ RowLds L;
    RowInfo ri;
    const uint32_t t = threadIdx.x;
    if (!row_prologue<HEADERS>(blockIdx.x, src, d, flags, n, cap, head, tiles, ntiles, grp, start, L, ri)) return;
    const uint64_t F0 = ri.F0, S0 = ri.S0;
    const uint32_t nf = ri.nf;
    const FrameUnits* s_fu = L.fu;
    const uint32_t* s_ub = L.ub;
    const u32x4* s_edge = L.edge;
    const uint8_t* s_ne = L.ne;
    // edge words of the block's frames: one contiguous run, whole 128-byte lines
    // (the run starts on one: 256 frames x 80 B), skipping lines without a live
    // word (a line written in part costs more than writing it whole)
    u32x4* eout = edge + F0 * kEdgeWords;
    const uint32_t nw = nf * (uint32_t)kEdgeWords;
    for (uint32_t i = t; i < nw; i += kBlock) {
        // the line [l0, l0 + 8) meets frames j0..j1 (at most 3); frame j's live
        // words are [5j, 5j + nedge_j), and every frame after j0 starts inside the line
        const uint32_t l0 = i & ~7u, j0 = l0 / kEdgeWords, j1 = (l0 + 7) / kEdgeWords;
        bool live = kEdgeWords * j0 + s_ne[j0] > l0;
        if (j0 + 1 < nf && j0 + 1 <= j1) live |= s_ne[j0 + 1] != 0;
        if (j0 + 2 < nf && j0 + 2 <= j1) live |= s_ne[j0 + 2] != 0;
        if (live) eout[i] = s_edge[i];  // dead words of a live line: any value (never read)
    }
    // unit records, slot-parallel
    const uint32_t ns = s_ub[nf];
    for (uint32_t sl = t; sl < ns; sl += kBlock) {
        uint32_t lo = 0, hi = nf;  // s_ub[lo] <= sl < s_ub[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_ub[mid] <= sl) lo = mid; else hi = mid;
        }
        const FrameUnits fu = s_fu[lo];
        const uint32_t m = sl - s_ub[lo];
        UnitRec r;
        if (m < fu.units) {
            r = make_rec(fu, m, (uint32_t)F0 + lo, head);
        } else {
            r.dst = r.src = 0;
            r.f = r.rk = 0;
            r.own = r.inner = 0;
        }
        rec[S0 + sl] = r;
    }
}

__device__ __forceinline__ u32x4 shfl16(const u32x4& v, int lane)
{
    return u32x4{(uint32_t)__shfl((int)v.x, lane, 64), (uint32_t)__shfl((int)v.y, lane, 64),
                 (uint32_t)__shfl((int)v.z, lane, 64), (uint32_t)__shfl((int)v.w, lane, 64)};
}

// A unit's record decoded into wave-uniform scalars.
struct UnitInfo {
    uint64_t dst;       // output byte of the unit's base word
    const uint8_t* s0;  // aligned source word of the base word
    uint32_t f, rk, delta, klo, khi, ilo, ihi, head_f, last;
    bool fast;          // the unit has interior words
};

__device__ __forceinline__ UnitInfo decode_unit(const UnitRec& r, bool live, const uint8_t* __restrict__ src)
{
    UnitInfo x;  // a dead unit (past the count, or a bad batch) owns, loads and stores nothing
    const uint32_t own = live ? r.own : 0u, inner = live ? r.inner : 0u;
    x.khi = own >> 16;
    x.klo = own & 0x1FFu;
    x.head_f = (own >> 12) & 0xFu;
    x.ilo = inner & 0xFFFFu;
    x.ihi = inner >> 16;
    x.delta = (uint32_t)(r.src & 15u);  // same for every word of the unit
    x.s0 = src + (r.src - x.delta);
    x.dst = r.dst;
    x.f = live ? r.f : 0u;
    x.rk = r.rk;
    x.fast = x.ihi > x.ilo;
    x.last = x.fast ? x.ihi - 1 : x.ilo;
    return x;
}

// Source loads of the copy waves: non-temporal (streaming) by default.  A
// shifted source run of 1 KiB per wave instruction starts mid-line, so two
// instructions (or two waves) share its edge lines.
constexpr int kUnitW = kUnitWords / 64;  // words per lane
struct UnitRegs {
    u32x4 lo[kUnitW];  // aligned source word of each of the lane's output words
    u32x4 ex;          // the source word after the last interior word (every lane: one address)
    u32x4 sv;          // this lane's edge word, if any
};

// Issues every load of a unit, and nothing else, in straight-line code (no
// branch around a load: the wait before the unit's stores then counts exactly
// the loads issued after them, so a later unit's loads could stay in flight
// unit's loads in flight).  Interior words: one aligned source word per lane,
// addresses clamped to [ilo, ihi - 1] (a unit without interior words reads
// src's first word instead); the next source word comes from the neighbour
// lane, lane 63 takes it from lane 0 of the next instruction, and the last
// interior word from `ex`.  Edge words (composed by edge_block: [klo, ilo)
// then [ihi, khi)): one per lane, index clamped.
// fedge: the owning frame's kEdgeWords edge words (global: edge + f * kEdgeWords,
// or an LDS copy of them).
__device__ __forceinline__ void unit_issue(const UnitInfo& x, int lane, const uint8_t* __restrict__ src,
                                           const u32x4* __restrict__ fedge, UnitRegs& R)
{
    const uint8_t* s0 = x.fast ? x.s0 : src;
    const uint32_t lo_k = x.fast ? x.ilo : 0u, hi_k = x.fast ? x.last : 0u;
#pragma unroll
    for (int i = 0; i < kUnitW; ++i) {
        const uint32_t k = lane + 64 * i;
        const uint32_t kk = k < lo_k ? lo_k : (k < hi_k ? k : hi_k);
        R.lo[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s0 + 16u * kk));
    }
    // word last + 1 holds payload bytes only when the source is shifted (delta != 0)
    uint32_t xk = x.fast && x.delta ? x.last + 1 : hi_k;
    asm("" : "+v"(xk));  // a vector load (a uniform address would become a scalar load: lgkmcnt)
    R.ex = *reinterpret_cast<const u32x4*>(s0 + 16u * xk);
    const uint32_t nhead = x.ilo - x.klo;
    uint32_t q = (uint32_t)lane < nhead ? lane : x.head_f + (lane - nhead);
    q = q < (uint32_t)kEdgeWords ? q : (uint32_t)kEdgeWords - 1;
    R.sv = fedge[q];
}

__device__ __forceinline__ u32x4 readlane0(const u32x4& v)
{
    return u32x4{(uint32_t)__builtin_amdgcn_readlane((int)v.x, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.y, 0),
                 (uint32_t)__builtin_amdgcn_readlane((int)v.z, 0), (uint32_t)__builtin_amdgcn_readlane((int)v.w, 0)};
}

// Composes and stores a unit whose loads unit_issue issued: every owned word of
// the unit, each 64-byte granule by one store instruction.
__device__ __forceinline__ void unit_finish(const UnitInfo& x, int lane, uint8_t* __restrict__ dst, uint64_t total,
                                            const UnitRegs& R)
{
    // Every register the unit loaded is consumed here on every path, so the wait
    // for them is a counted one and no load into these registers stays pending
    // (a pending one would force a full wait before the registers are reused).
#pragma unroll
    for (int i = 0; i < kUnitW; ++i) asm volatile("" ::"v"(R.lo[i]));
    asm volatile("" ::"v"(R.ex), "v"(R.sv));
    const uint32_t nhead = x.ilo - x.klo, nslow = nhead + (x.khi - x.ihi);
    if (nslow && lane < (int)nslow) {
        const uint32_t k = (uint32_t)lane < nhead ? x.klo + lane : x.ihi + (lane - nhead);
        const uint64_t a = x.dst + 16u * k;
        if (a + 16 > total) {  // the output's last, partial word: byte stores
#pragma clang loop vectorize(disable) unroll(disable)
            for (uint64_t p = a; p < total; ++p) {
                const uint32_t b = (uint32_t)(p - a);
                const uint32_t v = (b & 8u) ? ((b & 4u) ? R.sv.w : R.sv.z) : ((b & 4u) ? R.sv.y : R.sv.x);
                dst[p] = (uint8_t)(v >> (8 * (b & 3u)));
            }
        }
    }
    u32x4 out[kUnitW];
#pragma unroll
    for (int i = 0; i < kUnitW; ++i) {
        const uint32_t k = lane + 64 * i;
        u32x4 v = R.lo[i];
        if (x.fast && x.delta) {
            u32x4 hi;
            hi.x = __shfl_down(R.lo[i].x, 1, 64);
            hi.y = __shfl_down(R.lo[i].y, 1, 64);
            hi.z = __shfl_down(R.lo[i].z, 1, 64);
            hi.w = __shfl_down(R.lo[i].w, 1, 64);
            if (i + 1 < kUnitW) {  // word 64 (i + 1) for lane 63 (the unit's last word is never below last)
                const u32x4 nx = readlane0(R.lo[i + 1 < kUnitW ? i + 1 : i]);
                if (lane == 63) hi = nx;
            }
            if (k == x.last) hi = R.ex;
            v = funnel16(R.lo[i], hi, x.delta);
        }
        out[i] = v ^ x.rk;
        // composed words of this instruction's 64 (wave-uniform test)
        const uint32_t c0 = 64u * i, c1 = c0 + 64u;
        if ((x.klo < x.ilo && x.klo < c1 && x.ilo > c0) || (x.ihi < x.khi && x.ihi < c1 && x.khi > c0)) {
            const bool slow = (k >= x.klo && k < x.ilo) || (k >= x.ihi && k < x.khi);
            const int from = (int)(k < x.ilo ? k - x.klo : nhead + (k - x.ihi)) & 63;
            const u32x4 w = shfl16(R.sv, from);
            if (slow) out[i] = w;
        }
    }
#pragma unroll
    for (int i = 0; i < kUnitW; ++i) {
        const uint32_t k = lane + 64 * i;
        const uint64_t a = x.dst + 16u * k;
        if (k >= x.klo && k < x.khi && a + 16 <= total)
            __builtin_nontemporal_store(out[i], reinterpret_cast<u32x4*>(dst + a));
    }
}

// One wave per unit: kUnitW words per lane, 1 KiB per wave-instruction.
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                      const V2* __restrict__ tot,
                                                      const UnitRec* __restrict__ rec,
                                                      const u32x4* __restrict__ edge,
                                                      const WsHead* __restrict__ head, uint64_t unit_base,
                                                      uint32_t split)
{
    const int lane = threadIdx.x & 63;
    // wave id through readfirstlane: provably uniform, so the record is one scalar load
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // consecutive blocks dealt over `split` parts of the unit slots, so the
    // blocks in flight stream that many windows of the output far apart
    // (split >= 1000: runs of split - 1000 blocks per XCD residue instead)
    uint32_t b = blockIdx.x;
    if (split >= 1000u) {
        const uint32_t c = split - 1000u, run = 8u * c;
        if (b < gridDim.x / run * run) b = (b / 8u / c) * run + (b % 8u) * c + (b / 8u) % c;
    } else {
        const uint32_t q = gridDim.x / split;
        if (b < q * split) b = (b % split) * q + b / split;
    }
    const uint64_t u = unit_base + (uint64_t)b * (kBlock / 64) + wave;
    // record, slot count, status and total are independent scalar loads (one
    // latency level); slots past the count lie inside the workspace and are ignored
    const UnitRec r = rec[u];
    const uint64_t total_units = tot->b;
    const uint32_t st = head->status;
    const uint64_t total = tot->a;
    // no early exit between these loads and their uses (the compiler would sink
    // the record load below the count's wait): an out-of-range wave owns no words
    // a bad header (fused decode) leaves the other frames to copy; a bad descriptor
    // or an output past cap stops every store
    const UnitInfo x = decode_unit(r, u < total_units && (st & kStatusBadDesc) == 0, src);
    // keep every field's load above the exit (one wait for all of them)
    asm volatile("" ::"s"(r.dst), "s"(r.src), "s"(r.f), "s"(r.rk), "s"(r.inner), "s"(total));
    if (x.khi == 0) return;  // wave-uniform, after the record's wait
    // Every load is issued before the first store (vmcnt also counts stores, so
    // a load issued after a store would make its wait cover that store too).
    UnitRegs R;
    unit_issue(x, lane, src, edge + (uint64_t)x.f * kEdgeWords, R);
    unit_finish(x, lane, dst, total, R);
}

__device__ __forceinline__ u32x4 shfl16_down1(const u32x4& v)
{
    return u32x4{(uint32_t)__shfl_down((int)v.x, 1, 64), (uint32_t)__shfl_down((int)v.y, 1, 64),
                 (uint32_t)__shfl_down((int)v.z, 1, 64), (uint32_t)__shfl_down((int)v.w, 1, 64)};
}

// ------------------------------ chunk copy ------------------------------
// The product form of encode and gather: output-stationary.  The output is cut
// into 4 KiB chunks on 4 KiB boundaries, one wave each, so every output line is
// written by one store instruction of one wave, and nothing per frame or per
// wave passes through memory between the kernels but the region offsets and
// one 4-byte entry per chunk (the frame holding its first byte).  A chunk's
// frames -- up to 64, one lane each -- go into a wave-private table in LDS;
// each of its words finds its frame there and is either an interior word
// (inside one payload: two aligned source words, funnel-shifted and XORed with
// the rotated key) or a boundary word (header bytes, a payload's end, the next
// frame's start).  Boundary words are listed per wave and composed byte-parallel
// (one lane per byte), from source lines the same wave reads for its interior
// words anyway -- round 3's prologue read them in a pass of its own (0.97 GiB
// more fetched on cfg4) and wrote 80 B of edge words and two
// 32 B unit records per 4 KiB frame; here their values join the chunk's four
// full-width stores through LDS.
// 4 words per lane (8 measured slower: 103 VGPRs, 4 waves per SIMD, 0.715 on cfg4)
constexpr uint32_t kChunkW = 4;
constexpr uint32_t kChunkWords = 64 * kChunkW;
constexpr uint64_t kChunkBytes = 16ull * kChunkWords;
constexpr uint32_t kSlowShift = 9;  // boundary-list entry: word | table frame << kSlowShift
constexpr uint32_t kSlowWord = (1u << kSlowShift) - 1;
static_assert(kChunkW == 4 || kChunkW == 8, "chunk: 4 or 8 words per lane");
constexpr uint32_t kChunkFrames = 64;           // a chunk's frame table, one lane per frame

__host__ __device__ __forceinline__ uint64_t chunk_count(uint64_t bytes) { return (bytes + kChunkBytes - 1) / kChunkBytes; }

// 256 frames per block, after the scan: each frame's region offset (start[f])
// and, for every chunk whose first byte lies in the block's regions, the frame
// holding it (cmap[c]).  Also the capacity check (status set, nothing stored).
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) chunk_map_kernel(const kmws_desc* __restrict__ d,
                                                           const uint16_t* __restrict__ flags, uint32_t n, uint64_t cap,
                                                           WsHead* __restrict__ head, const V2* __restrict__ tiles,
                                                           uint32_t ntiles, const V2* __restrict__ grp,
                                                           uint64_t* __restrict__ start, uint32_t* __restrict__ cmap)
{
    __shared__ uint64_t s_r0[kBlock + 1];
    __shared__ V2 s_w[kBlock / 64];
    const uint32_t t = threadIdx.x;
    const uint64_t F0 = (uint64_t)blockIdx.x * kBlock;
    const uint32_t nf = n - F0 < (uint64_t)kBlock ? (uint32_t)(n - F0) : (uint32_t)kBlock;
    const uint32_t f = (uint32_t)(F0 + (t < nf ? t : nf - 1));
    const V2 tot = tiles[ntiles];
    const V2 pre = tiles[blockIdx.x / kRowsPerTile] + grp[blockIdx.x];
    const kmws_desc x = d[f];
    const uint32_t fl = HEADERS ? flags[f] : 0u;
    const uint64_t rsz = (uint64_t)(HEADERS ? hdr_len(x.len, (fl >> 8) & 1u) : 0u) + x.len;
    if (blockIdx.x == 0 && t == 0) head->pad[0] = 0;  // chunk_copy_kernel's dense-chunk count
    V2 row;
    const V2 off = block_excl_scan(t < nf ? V2{rsz, 0} : V2{0, 0}, s_w, row);
    const uint64_t r0 = pre.a + off.a;
    if (t < nf) {
        start[f] = r0;
        s_r0[t] = r0;
    }
    if (t == 0) s_r0[nf] = pre.a + row.a;
    if (tot.a > cap) {  // block-uniform; the copy waves see the status and store nothing
        if (blockIdx.x == 0 && t == 0) atomicOr(&head->status, kStatusBadDesc);
        return;
    }
    __syncthreads();
    const uint64_t c0 = chunk_count(pre.a), c1 = chunk_count(pre.a + row.a);
    for (uint64_t c = c0 + t; c < c1; c += kBlock) {
        const uint64_t xb = c * kChunkBytes;
        uint32_t lo = 0, hi = nf;  // s_r0[lo] <= xb < s_r0[hi]: the last region starting at or before xb
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_r0[mid] <= xb) lo = mid; else hi = mid;
        }
        cmap[c] = (uint32_t)F0 + lo;
    }
}

// One frame of a chunk's table (LDS), 48 B: its geometry relative to the
// chunk's first byte A0 (clamped to +-2^30: only offsets within a few bytes of
// the chunk matter), its source pointer per output offset, the rotated key of
// its aligned output words (byte x & 3 of it masks output byte x), and the
// header bytes.
struct ChunkFrame {
    int32_t r0, p0, r1;  // region start, payload start, region end - A0
    uint32_t rk;         // rot_key(key, p0) (0: no mask)
    uint64_t sbase;      // source byte of output offset o = sbase + o
    uint8_t h[16];       // the header's bytes (encode)
    uint64_t pad;
};
static_assert(sizeof(ChunkFrame) == 48, "ChunkFrame is three 16-byte LDS loads");

__device__ __forceinline__ int32_t rel32(uint64_t x, uint64_t A0)
{
    const int64_t d = (int64_t)(x - A0);
    return d < -(1 << 30) ? -(1 << 30) : (d > (1 << 30) ? (1 << 30) : (int32_t)d);
}

// LDS written by some lanes of a wave and read by others: DS instructions of
// one wave execute in order; this keeps the compiler from reordering them.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t bal)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
}

// The output's last, partial word: bytes [a, total) only.
__device__ __forceinline__ void store_word_bytes(uint8_t* __restrict__ dst, uint64_t a, uint64_t total, const u32x4& v)
{
#pragma clang loop vectorize(disable) unroll(disable)
    for (uint64_t p = a; p < total; ++p) {
        const uint32_t b = (uint32_t)(p - a);
        const uint32_t w = (b & 8u) ? ((b & 4u) ? v.w : v.z) : ((b & 4u) ? v.y : v.x);
        dst[p] = (uint8_t)(w >> (8 * (b & 3u)));
    }
}

// The chunk copy's source loads: non-temporal (streaming) for every batch.
__device__ __forceinline__ u32x4 copy_src_load(const uint8_t* p)
{
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

// One wave per 4 KiB output chunk (4 words per lane, 1 KiB per instruction).
// A chunk meeting more than kChunkFrames frames is listed for chunk_dense_kernel.
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) chunk_copy_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            const kmws_desc* __restrict__ d,
                                                            const uint16_t* __restrict__ flags, uint32_t n,
                                                            const uint64_t* __restrict__ start,
                                                            const uint32_t* __restrict__ cmap,
                                                            const V2* __restrict__ tot, WsHead* __restrict__ head,
                                                            uint32_t* __restrict__ dense, uint64_t chunk_base,
                                                            uint32_t split)
{
    __shared__ ChunkFrame s_tab[kBlock / 64][kChunkFrames];
    __shared__ uint16_t s_slow[kBlock / 64][kChunkWords];  // boundary words: word | frame << kSlowShift
    __shared__ u32x4 s_val[kBlock / 64][64 + 16];  // boundary words 0..63, then 16 scratch slots
    const int lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // consecutive blocks dealt over `split` parts of the output: with split 8,
    // XCD x (blocks are dispatched round-robin over the 8 XCDs) streams part x
    uint32_t b = blockIdx.x;
    const uint32_t q = gridDim.x / split;
    if (b < q * split) b = (b % split) * q + b / split;
    const uint64_t c = chunk_base + (uint64_t)b * (kBlock / 64) + wave;
    const uint64_t total = tot->a;
    const uint32_t st = head->status;
    const uint64_t nch = chunk_count(total);
    // a bad batch, or offsets from a look-back that timed out: nothing is stored
    if (c >= nch || (st & (kStatusBadDesc | kStatusLookbackTimeout))) return;  // wave-uniform
    const uint32_t f0 = cmap[c];
    const uint32_t f1 = c + 1 < nch ? cmap[c + 1] : n - 1;  // holds the next chunk's first byte
    const uint32_t nfr = f1 - f0 + 1;
    const uint64_t A0 = c * kChunkBytes;
    if (nfr > kChunkFrames) {
        if (lane == 0) dense[atomicAdd(&head->pad[0], 1u)] = (uint32_t)c;
        return;
    }
    ChunkFrame* tab = s_tab[wave];
    if ((uint32_t)lane < nfr) {
        const uint32_t j = f0 + lane;
        const kmws_desc x = d[j];
        const uint32_t fl = HEADERS ? flags[j] : 0u;
        const uint32_t mask = HEADERS ? (fl >> 8) & 1u : 1u;
        const uint64_t r0 = start[j], p0 = r0 + (HEADERS ? hdr_len(x.len, mask) : 0u);
        const uint32_t key = mask ? x.key : 0u;
        ChunkFrame e;
        e.r0 = rel32(r0, A0);
        e.p0 = rel32(p0, A0);
        e.r1 = rel32(p0 + x.len, A0);
        e.rk = key ? rot_key(key, p0) : 0u;
        e.sbase = (uint64_t)(uintptr_t)src + x.off - (p0 - A0);
        uint64_t h0 = 0, h1 = 0;
        if (HEADERS) build_header(x.len, fl, key, h0, h1);
        __builtin_memcpy(e.h, &h0, 8);
        __builtin_memcpy(e.h + 8, &h1, 8);
        tab[lane] = e;
    }
    wave_lds_sync();
    const int32_t trel = total - A0 < kChunkBytes ? (int32_t)(total - A0) : (int32_t)kChunkBytes;  // live bytes
    // Pass 1: each word's frame (binary search over the table) and kind.  An
    // interior word lies inside one payload; it takes its second source word
    // from the next word's lane (lane 63: lane 0 of the next round) when that
    // word is interior to the same payload, else from one extra load per lane
    // (the chunk's last word, the last word of a payload; a lane whose words
    // need two lists the second).  Every other live word -- header bytes, a
    // payload's first or last bytes -- is listed as a boundary word.
    uint16_t* sl = s_slow[wave];
    uint64_t jbits = 0;
    uint32_t slowbits = 0, nslow = 0, exr = kChunkW;  // exr: the round of the lane's extra load
#pragma unroll
    for (int i = 0; i < (int)kChunkW; ++i) {
        const uint32_t k = 64u * i + lane;
        const int32_t a = 16 * (int32_t)k;
        uint32_t lo = 0, hi = nfr;  // tab[lo].r0 <= a < tab[hi].r0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (tab[mid].r0 <= a) lo = mid; else hi = mid;
        }
        const int32_t p0 = tab[lo].p0, r1 = tab[lo].r1;
        const bool live = a < trel;
        const bool inner = live && a >= p0 && a + 16 <= r1;
        const uint32_t delta = ((uint32_t)tab[lo].sbase + (uint32_t)a) & 15u;
        const bool nb = delta == 0 || (a + 32 <= r1 && (i + 1 < (int)kChunkW || lane != 63));
        const bool ex = inner && !nb && exr == kChunkW;
        if (ex) exr = i;
        const bool fast = inner && (nb || ex);
        const bool slow = live && !fast;
        const uint64_t bal = __ballot(slow);
        if (slow) sl[nslow + lanes_below(bal)] = (uint16_t)(k | lo << kSlowShift);
        jbits |= (uint64_t)lo << (6 * i);
        slowbits |= slow ? 1u << i : 0u;
        nslow += (uint32_t)__builtin_popcountll(bal);
    }
    wave_lds_sync();
    // Boundary words are composed byte-parallel: one lane per byte, 16 words
    // per batch (four per instruction).  Each byte's frame is found from its
    // word's first frame on; the byte is a header byte (from the table) or a
    // masked source byte.  The first batch's source bytes are loaded before the
    // interior words' (pass 2), so one latency covers both.  Words are
    // assembled in LDS: the first 64 join the stores of pass 4, later ones
    // (chunks of many small frames) are stored by their batch.
    uint8_t* sb = reinterpret_cast<uint8_t*>(&s_val[wave][0]);
    uint32_t hv[4], sv[4];
    auto batch_issue = [&](uint32_t g0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t qi = g0 + 4u * u + ((uint32_t)lane >> 4);
            const uint32_t ent = qi < nslow ? sl[qi] : 0u;
            uint32_t m = ent >> kSlowShift;
            const int32_t x = 16 * (int32_t)(ent & kSlowWord) + (lane & 15);
            while (m + 1 < nfr && tab[m + 1].r0 <= x) ++m;
            const ChunkFrame& e = tab[m];
            const bool live = qi < nslow && x < trel;
            const bool hdr = HEADERS && x < e.p0;
            if (hdr)  // header byte x - r0 (< 14); bit 8: no source byte
                hv[u] = 0x100u | e.h[live ? (uint32_t)(x - e.r0) & 15u : 0u];
            else  // the key byte of output byte x
                hv[u] = (e.rk >> (8 * (x & 3))) & 0xFFu;
            sv[u] = *reinterpret_cast<const uint8_t*>(live && !hdr ? e.sbase + (int64_t)x : (uint64_t)(uintptr_t)src);
        }
    };
    auto batch_put = [&](uint32_t g0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t qi = g0 + 4u * u + ((uint32_t)lane >> 4);
            const uint32_t v = (hv[u] & 0x100u) ? hv[u] : (sv[u] ^ hv[u]);
            if (qi < nslow) sb[16u * (qi < 64 ? qi : 64 + 4u * u + ((uint32_t)lane >> 4)) + (lane & 15)] = (uint8_t)v;
        }
        if (g0 >= 64) {  // wave-uniform: sixteen words past the first 64, stored now
            wave_lds_sync();
            if (lane < 16 && g0 + lane < nslow) {
                const uint64_t a = A0 + 16ull * (sl[g0 + lane] & kSlowWord);
                const u32x4 v = s_val[wave][64 + lane];
                if (a + 16 <= total) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + a));
                else store_word_bytes(dst, a, total, v);
            }
            wave_lds_sync();  // the scratch slots are reused
        }
    };
    if (nslow) batch_issue(0);
    // Pass 2: interior words' source words, one aligned word each (all four
    // rounds issued before anything waits).
    u32x4 L0[kChunkW], X;
    uint32_t rk[kChunkW], dl = 0;
    uint64_t xa = (uint64_t)(uintptr_t)src;
#pragma unroll
    for (int i = 0; i < (int)kChunkW; ++i) {
        const int32_t a = 16 * (int32_t)(64u * i + lane);
        const ChunkFrame& e = tab[(uint32_t)(jbits >> (6 * i)) & 63u];
        const bool inner = a < trel && a >= e.p0 && a + 16 <= e.r1;
        const uint64_t sa = e.sbase + (int64_t)a;
        L0[i] = copy_src_load(inner ? reinterpret_cast<const uint8_t*>(sa & ~15ull) : src);
        if (exr == (uint32_t)i) xa = (sa + 15) & ~15ull;  // the aligned word holding the word's last source byte
        dl |= (uint32_t)(sa & 15u) << (4 * i);
        rk[i] = e.rk;
    }
    X = copy_src_load(reinterpret_cast<const uint8_t*>(xa));
    // Pass 3: the boundary words
    if (nslow) batch_put(0);
    for (uint32_t g0 = 16; g0 < nslow; g0 += 16) {  // wave-uniform
        batch_issue(g0);
        batch_put(g0);
    }
    wave_lds_sync();
    // Pass 4: the four full-width stores, boundary words merged in.
    uint32_t seen = 0;
#pragma unroll
    for (int i = 0; i < (int)kChunkW; ++i) {
        const uint32_t k = 64u * i + lane;
        const uint64_t a = A0 + 16ull * k;
        u32x4 hi = shfl16_down1(L0[i]);
        if (i + 1 < (int)kChunkW) {
            const u32x4 nx = readlane0(L0[i + 1 < (int)kChunkW ? i + 1 : i]);
            if (lane == 63) hi = nx;
        }
        if (exr == (uint32_t)i) hi = X;
        u32x4 out = funnel16(L0[i], hi, (dl >> (4 * i)) & 15u) ^ rk[i];
        const bool slow = (slowbits >> i) & 1u;
        const uint64_t bal = __ballot(slow);
        bool mine = true;
        if (bal) {  // wave-uniform
            const uint32_t pos = seen + lanes_below(bal);
            if (slow) {
                mine = pos < 64;
                if (mine) out = s_val[wave][pos];
            }
            seen += (uint32_t)__builtin_popcountll(bal);
        }
        if (mine && a + 16 <= total) __builtin_nontemporal_store(out, reinterpret_cast<u32x4*>(dst + a));
        else if (mine && a < total) store_word_bytes(dst, a, total, out);
    }
}

// The chunks chunk_copy_kernel listed (more than kChunkFrames frames: regions
// averaging under 64 bytes): every word byte by byte, its first frame by a
// binary search over start[].  Correct for any batch, fast only where it does
// not matter; a batch of small frames takes the unit form instead (below).
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) chunk_dense_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                             const kmws_desc* __restrict__ d,
                                                             const uint16_t* __restrict__ flags, uint32_t n,
                                                             const uint64_t* __restrict__ start,
                                                             const uint32_t* __restrict__ cmap,
                                                             const V2* __restrict__ tot,
                                                             const WsHead* __restrict__ head,
                                                             const uint32_t* __restrict__ dense)
{
    if (head->status & (kStatusBadDesc | kStatusLookbackTimeout)) return;
    const uint32_t cnt = head->pad[0];
    const uint64_t total = tot->a, nch = chunk_count(total);
    const int lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * (kBlock / 64);
    for (uint32_t i = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); i < cnt; i += nw) {
        const uint64_t c = dense[i];
        const uint32_t f0 = cmap[c], f1 = c + 1 < nch ? cmap[c + 1] : n - 1;
        for (uint32_t k = lane; k < kChunkWords; k += 64) {
            const uint64_t a = c * kChunkBytes + 16ull * k;
            if (a >= total) break;
            uint32_t lo = f0, hi = f1 + 1;  // start[lo] <= a < start[hi] (start[n] = total)
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (start[mid] <= a) lo = mid; else hi = mid;
            }
            const uint32_t fl = HEADERS ? flags[lo] : 0u;
            const FrameGeom g = geom_at<HEADERS>(d[lo], fl, start[lo]);
            const u32x4 v = compose_word_bytes<HEADERS>(a, lo, n, src, g, fl, d, flags);
            if (a + 16 <= total) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + a));
            else store_word_bytes(dst, a, total, v);
        }
    }
}

// ------------------------------ header unpack / validate ------------------------------
// One lane per frame: the reference's HDR1..MASKEY rules (parse_frame_header,
// kmws_frame_parse.hpp).
__global__ void __launch_bounds__(kBlock) unpack_headers_kernel(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                                                const uint64_t* __restrict__ hdr_off, uint32_t n,
                                                                int mode, kmws_desc* __restrict__ out_desc,
                                                                uint16_t* __restrict__ out_flags,
                                                                uint8_t* __restrict__ out_err,
                                                                WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    unpack_one(wire, wire_len, hdr_off, n, f, mode, out_desc, out_flags, out_err, head);
}

// ------------------------------ header pack only ------------------------------
// One lane per frame: the header bytes of WSHandler::encodeFrameHeader in a
// 16-byte slot (one coalesced store per lane) and its length (no wire offsets:
// those come from pack_headers_chain_kernel below).
__global__ void __launch_bounds__(kBlock) pack_headers_kernel(const kmws_desc* __restrict__ d,
                                                              const uint16_t* __restrict__ flags, uint32_t n,
                                                              u32x4* __restrict__ hdr, uint8_t* __restrict__ hl_out)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    const kmws_desc x = d[f];
    const uint32_t fl = flags[f];
    uint64_t h0, h1;
    build_header(x.len, fl, x.key, h0, h1);
    hdr[f] = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
    if (hl_out) hl_out[f] = (uint8_t)hdr_len(x.len, (fl >> 8) & 1u);
}

// ------------------------------ header pack, one pass ------------------------------
// kmws_pack_headers with wire offsets as ONE pass over the descriptors: a
// chained scan (decoupled look-back) over 2048-frame tiles, tile = blockIdx.x.
// A block loads its tile's {len, key} and flags once, publishes its tile's
// aggregate, writes the header slots, resolves its prefix from its
// predecessors' published states and writes the wire offsets.  (The
// three-pass form -- reduce, scan the tile totals, emit -- reads the
// descriptors twice and pays two kernel boundaries: 17-19 + 5 + 27 us on 4 M
// frames, r03w_pack_kernel_trace.txt.)
//
// Measured on 4 M frames (2048 tiles; wall time per call, 20 calls back to
// back; profiles/r03ak_pack_headers_ab.txt, r03ax_pack_headers_ab.txt): this
// kernel 39.5-41 us; without the dependency 34 us (the floor of the design).
// Per-tile timestamps (s_memrealtime) showed what the look-back costs: not the
// wait itself but its reads -- every block reading a 512-tile window (two states
// per thread) delayed the other tiles' descriptor loads (the last tile's loads
// landed at 31.6 us instead of 20.9 without the dependency; 46-47 us per call),
// a 256-tile window 44.5 us, this 64-tile window read by one wave, no block
// barrier, 39.5-41 us (last loads at 22.9 us).  Also measured: the aggregate
// published after the header-slot stores (queued ahead of it in the in-order
// vector memory queue) 53 us; header slots after the look-back 74 us; a
// persistent grid of 512 blocks taking tiles in order 50 us; prefixes from
// per-64-tile group counters instead of a chain 169 us (every waiting block
// polled the same few words); the round's first look-back scan (c527e0f: tiles
// from one atomic ticket counter, which serves ~88 atomics per us --
// MI355X_MICROARCH.md "dequeue" -- and a 64-tile window) 95-115 us of kernel.
//
// Tile state: one 64-bit word, value << 2 | flag (0 none, 1 aggregate, 2
// inclusive prefix), written and read with agent-scope atomics (the XCDs' L2s
// are not coherent for plain accesses); zeroed by a kernel before each call.  A
// block waits only on lower-indexed blocks, which the dispatcher placed before
// it, so the wait always ends; the spin is bounded all
// the same, far beyond any real wait (2^24 polls of >= 8 x 64 cycles plus a
// load: seconds), and a state that never arrives sets kStatusLookbackTimeout --
// its own status bit, not the bad-input one -- instead of hanging; wire_off is
// then invalid.  A test build lowers the bound and skips one tile's publish
// (KMWS_TEST_SKIP_PUBLISH_TILE, tests/test_gpu_pack.py).
constexpr uint64_t kStAgg = 1ull, kStInc = 2ull;
#ifndef KMWS_LOOKBACK_SPIN_LIMIT
#define KMWS_LOOKBACK_SPIN_LIMIT (1u << 24)
#endif
constexpr uint32_t kLookSpinLimit = KMWS_LOOKBACK_SPIN_LIMIT;
// Does this tile publish its state?  Always, except in the test build, where
// one tile never does (a successor must time out).
__device__ __forceinline__ bool tile_publishes(uint32_t tile)
{
#ifdef KMWS_TEST_SKIP_PUBLISH_TILE
    return tile != (uint32_t)(KMWS_TEST_SKIP_PUBLISH_TILE);
#else
    (void)tile;
    return true;
#endif
}

__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS accesses,
// not for its outstanding global stores (__syncthreads would wait for every
// header-slot store of the tile first).
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One wave: the exclusive prefix of tile `tile` (> 0).  Lane 0 first polls the
// nearest predecessor; then lane l looks at the tile at distance l below
// `base`: the states up to and including the nearest inclusive one are summed
// (tiles below 0 count as an inclusive zero), states still missing below it
// are re-read alone; a 64-tile window of aggregates is summed whole and the
// next one read.  No block barrier inside; the nearest inclusive state is
// usually a few tiles away.
__device__ uint64_t look_back(const uint64_t* __restrict__ st, uint32_t tile, WsHead* __restrict__ head)
{
    const uint32_t lane = threadIdx.x & 63;
    uint64_t pre = 0;
    uint32_t spins = 0;
    if (lane == 0) {
        while ((ld_agent(st + tile - 1) & 3u) == 0 && ++spins < kLookSpinLimit) __builtin_amdgcn_s_sleep(8);
    }
    for (int64_t base = (int64_t)tile - 1;; base -= 64) {
        const int64_t j = base - (int64_t)lane;
        uint64_t v = j >= 0 ? ld_agent(st + j) : kStInc;
        for (;;) {
            const uint64_t inc = __ballot((v & 3u) == kStInc);
            const uint32_t dmin = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
            const bool missing = lane < dmin && (v & 3u) == 0;
            if (__ballot(missing) == 0) {
                pre += wave_sum(lane <= dmin ? v >> 2 : 0);
                if (dmin < 64) return pre;
                break;
            }
            if (++spins >= kLookSpinLimit) {  // every lower tile publishes: only a stalled or broken predecessor
                if (lane == 0) atomicOr(&head->status, kStatusLookbackTimeout);
                return pre;
            }
            __builtin_amdgcn_s_sleep(8);
            if (missing) v = ld_agent(st + j);
        }
    }
}

__global__ void __launch_bounds__(kBlock, 8) pack_headers_chain_kernel(const kmws_desc* __restrict__ d,
                                                                       const uint16_t* __restrict__ flags, uint32_t n,
                                                                       u32x4* __restrict__ hdr,
                                                                       uint8_t* __restrict__ hl_out,
                                                                       uint64_t* __restrict__ out,
                                                                       uint64_t* __restrict__ st,
                                                                       WsHead* __restrict__ head)
{
    __shared__ uint64_t s_sz[kScanTile];  // region sizes, then wire offsets
    __shared__ uint64_t s_w[kBlock / 64];
    __shared__ uint64_t s_a[kBlock / 64];
    __shared__ uint64_t s_pre;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t tile = blockIdx.x;
    const uint64_t F = (uint64_t)tile * kScanTile;
    // frames F + i * 256 + t: every load and store coalesced, all loads issued at once
    // (only {len, key}, the descriptor's second 8 bytes, and the flags)
    uint64_t lk[kScanItems];
    uint32_t fl[kScanItems];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        const uint32_t j = (uint32_t)__builtin_elementwise_min(f, (uint64_t)n - 1);
        lk[i] = reinterpret_cast<const uint64_t*>(d + j)[1];
        fl[i] = flags[j];
    }
    // the tile's aggregate first (a plain block sum: one barrier), published at once
    uint64_t part = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        const uint32_t len = (uint32_t)lk[i];
        part += f < n ? (uint64_t)hdr_len(len, (fl[i] >> 8) & 1u) + len : 0;
    }
    part = wave_sum(part);
    if (lane == 0) s_a[wave] = part;
    lds_barrier();
    uint64_t agg = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) agg += s_a[w];
    const bool first = tile == 0;
    const bool publish = tile_publishes(tile);
    if (t == 0 && publish) st_agent(st + tile, first ? agg << 2 | kStInc : agg << 2 | kStAgg);
    // then the header slots (they need no offset; stores issued ahead of the
    // publish would delay it: the vector memory queue is in order) and the sizes
    // for the per-frame scan
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        const uint32_t len = (uint32_t)lk[i], key = (uint32_t)(lk[i] >> 32);
        const uint32_t hl = hdr_len(len, (fl[i] >> 8) & 1u);
        s_sz[i * kBlock + t] = f < n ? (uint64_t)hl + len : 0;
        if (f < n) {
            uint64_t h0, h1;
            build_header(len, fl[i], key, h0, h1);
            hdr[f] = u32x4{(uint32_t)h0, (uint32_t)(h0 >> 32), (uint32_t)h1, (uint32_t)(h1 >> 32)};
            if (hl_out) hl_out[f] = (uint8_t)hl;
        }
    }
    lds_barrier();
    // thread t: frames 8t .. 8t + 7 of the tile (only thread t reads or writes
    // these entries until the barrier before the stores)
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) sum += s_sz[kScanItems * t + k];
    const uint64_t inc = wave_incl_scan(sum);
    if (lane == 63) s_w[wave] = inc;
    lds_barrier();
    uint64_t before = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w)
        if (w < (int)wave) before += s_w[w];
    uint64_t pre = 0;
    if (!first) {
        if (wave == 0) {
            const uint64_t p = look_back(st, tile, head);
            if (lane == 0) s_pre = p;
        }
        lds_barrier();
        pre = s_pre;
        if (t == 0 && publish) st_agent(st + tile, (pre + agg) << 2 | kStInc);
    }
    if (t == 0 && F + kScanTile >= n) out[n] = pre + agg;  // the last tile: the total
    uint64_t run = pre + before + inc - sum;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint64_t r = s_sz[kScanItems * t + k];
        s_sz[kScanItems * t + k] = run;
        run += r;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        if (f < n) out[f] = s_sz[i * kBlock + t];
    }
}

__global__ void __launch_bounds__(kBlock) zero_words_kernel(uint64_t* __restrict__ p, uint64_t words)
{
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < words; i += (uint64_t)gridDim.x * kBlock)
        p[i] = 0;
}

// The chunk form's front in ONE pass: a 2048-frame
// tile per block, the scan by decoupled look-back (the header-only pack's
// machinery above), then the tile's region offsets and its chunks' first
// frames -- in place of reduce_kernel + scan_tiles_kernel + chunk_map_kernel,
// which read the descriptors twice.  The tile states, the status word and the
// dense count are zeroed by the launch before it.  The last tile writes the
// total (start[n] and tot) and the capacity check; every tile clips its chunk
// map to the capacity, so an oversized batch writes nothing out of bounds.
template <bool HEADERS>
__global__ void __launch_bounds__(kBlock) chunk_scan_kernel(const kmws_desc* __restrict__ d,
                                                            const uint16_t* __restrict__ flags, uint32_t n,
                                                            uint64_t cap, WsHead* __restrict__ head,
                                                            uint64_t* __restrict__ st, V2* __restrict__ tot,
                                                            uint64_t* __restrict__ start, uint32_t* __restrict__ cmap)
{
    __shared__ uint64_t s_sz[kScanTile];  // region sizes, then offsets
    __shared__ uint64_t s_w[kBlock / 64];
    __shared__ uint64_t s_a[kBlock / 64];
    __shared__ uint64_t s_pre;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t tile = blockIdx.x;
    const uint64_t F = (uint64_t)tile * kScanTile;
    uint32_t len[kScanItems], fl[kScanItems];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        const uint32_t j = (uint32_t)__builtin_elementwise_min(f, (uint64_t)n - 1);
        len[i] = d[j].len;
        fl[i] = HEADERS ? flags[j] : 0u;
    }
    uint64_t part = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        const uint64_t r = (uint64_t)(HEADERS ? hdr_len(len[i], (fl[i] >> 8) & 1u) : 0u) + len[i];
        part += f < n ? r : 0;
        s_sz[i * kBlock + t] = f < n ? r : 0;
    }
    part = wave_sum(part);
    if (lane == 0) s_a[wave] = part;
    lds_barrier();
    uint64_t agg = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) agg += s_a[w];
    const bool publish = tile_publishes(tile);
    if (t == 0 && publish) st_agent(st + tile, tile == 0 ? agg << 2 | kStInc : agg << 2 | kStAgg);
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) sum += s_sz[kScanItems * t + k];
    const uint64_t inc = wave_incl_scan(sum);
    if (lane == 63) s_w[wave] = inc;
    lds_barrier();
    uint64_t before = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w)
        if (w < (int)wave) before += s_w[w];
    uint64_t pre = 0;
    if (tile != 0) {
        if (wave == 0) {
            const uint64_t p = look_back(st, tile, head);
            if (lane == 0) s_pre = p;
        }
        lds_barrier();
        pre = s_pre;
        if (t == 0 && publish) st_agent(st + tile, (pre + agg) << 2 | kStInc);
    }
    uint64_t run = pre + before + inc - sum;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint64_t r = s_sz[kScanItems * t + k];
        s_sz[kScanItems * t + k] = run;
        run += r;
    }
    lds_barrier();
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t f = F + (uint64_t)i * kBlock + t;
        if (f < n) start[f] = s_sz[i * kBlock + t];
    }
    const uint64_t T0 = pre, T1 = pre + agg;
    if (t == 0 && F + kScanTile >= n) {  // the last tile: the total and the capacity check
        start[n] = T1;
        tot->a = T1;
        tot->b = 0;
        if (T1 > cap) atomicOr(&head->status, kStatusBadDesc);
    }
    const uint32_t nf = n - F < (uint64_t)kScanTile ? (uint32_t)(n - F) : (uint32_t)kScanTile;
    const uint64_t cap_chunks = chunk_count(cap);
    uint64_t c1 = chunk_count(T1);
    c1 = c1 < cap_chunks ? c1 : cap_chunks;
    for (uint64_t c = chunk_count(T0) + t; c < c1; c += kBlock) {
        const uint64_t xb = c * kChunkBytes;
        uint32_t lo = 0, hi = nf;  // s_sz[lo] <= xb < s_sz[hi] (s_sz[nf] stands for T1)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_sz[mid] <= xb) lo = mid; else hi = mid;
        }
        cmap[c] = (uint32_t)(F + lo);
    }
}

// ------------------------------ header-chain walk, many streams ------------------------------
// One lane per stream, the rules of kmws_find_headers (kmws_codec.cpp) /
// the header states of WSHandler::decodeFrame (WSHandler.cpp:118-197): each
// step reads the (at most 10) bytes it needs from one pair of aligned 16-byte
// loads (byte loads near the wire's end), decodes the length class (with the
// 127-class shift quirk) and jumps over the payload.
// One step of the walk at p (already recorded): false = stop after this frame
// (truncated, invalid length, CLOSE); else p = done = the next header.
__device__ __forceinline__ bool walk_step(const uint8_t* __restrict__ wire, uintptr_t end16, uint64_t hi, uint64_t& p,
                                          uint64_t& done)
{
    if (p + 2 > hi) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(wire + p), a16 = a & ~(uintptr_t)15;
    u32x4 hw = u32x4{0, 0, 0, 0};
    if (a16 + 32 <= end16) {
        hw = funnel16(*reinterpret_cast<const u32x4*>(a16), *reinterpret_cast<const u32x4*>(a16 + 16),
                      (uint32_t)(a & 15u));
    } else {
        const uint64_t avail = hi - p < 10 ? hi - p : 10;
        for (uint32_t k = 0; k < (uint32_t)avail; ++k) {
            const uint32_t b = wire[p + k], sh = 8u * (k & 3u);
            if ((k >> 2) == 0) hw.x |= b << sh;
            else if ((k >> 2) == 1) hw.y |= b << sh;
            else hw.z |= b << sh;
        }
    }
    const uint32_t b0 = hw.x & 0xFFu, b1 = (hw.x >> 8) & 0xFFu;
    const uint32_t plen = b1 & 0x7F, mask = b1 >> 7;
    const uint64_t ext = plen == 126 ? 2 : (plen == 127 ? 8 : 0);
    if (p + 2 + ext > hi) return false;
    uint64_t L;
    if (plen == 126) {
        L = (byte_of(hw, 2) << 8) | byte_of(hw, 3);
    } else if (plen == 127) {
        const uint64_t x = ext_len127(hw);
        if ((x >> 63) != 0 || (uint32_t)x > KMWS_MAX_FRAME_DATA_LENGTH) return false;
        L = (uint32_t)x;
    } else {
        L = plen;
    }
    const uint64_t e = p + 2 + ext + (mask ? 4 : 0) + L;
    if (e > hi) return false;
    p = done = e;
    return (b0 & 0x0F) != KMWS_OP_CLOSE;
}

__global__ void __launch_bounds__(kBlock) walk_headers_kernel(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                                              const uint64_t* __restrict__ stream_off,
                                                              uint32_t n_streams, uint64_t* __restrict__ hdr_off,
                                                              uint32_t cap, uint32_t* __restrict__ n_out,
                                                              uint64_t* __restrict__ consumed)
{
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n_streams) return;
    // a stream is clamped to the wire (bad offsets walk nothing instead of reading past it)
    const uint64_t hi = stream_off[s + 1] < wire_len ? stream_off[s + 1] : wire_len;
    const uint64_t lo = stream_off[s] < hi ? stream_off[s] : hi;
    const uintptr_t end16 = (reinterpret_cast<uintptr_t>(wire) + wire_len + 15) & ~(uintptr_t)15;
    uint64_t* out = hdr_off + (uint64_t)s * cap;
    uint64_t p = lo, done = lo;
    uint32_t n = 0;
    bool stop = false;
    // Offsets are kept in registers and written 16 at a time (128 bytes, a whole
    // line per lane): one 8-byte store per lane and step left partial lines of
    // thousands of streams in flight, and the L2 wrote them back piecewise.
    while (!stop) {
        uint64_t buf[16];
        uint32_t cnt = 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (!stop) {
                if (p >= hi || n >= cap) {
                    stop = true;
                } else {
                    buf[j] = p;
                    cnt = j + 1;
                    ++n;
                    stop = !walk_step(wire, end16, hi, p, done);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j)
            if ((uint32_t)j < cnt) out[n - cnt + j] = buf[j];
    }
    n_out[s] = n;
    if (consumed) consumed[s] = done - lo;
}

// ------------------------------ host launchers ------------------------------
// The copy form, by the mean region bound cap / n: below kChunkFormBelow
// bytes the chunk form (chunk_map + chunk_copy), from it the unit form
// (prologue: edge words, unit records; copy_kernel).  Measured on one box
// (profiles/r04p_chunk_ab.txt): cfg4 (4 KiB frames) 0.748 / 0.772 chunk against
// 0.722 / 0.741 units, 8 M frames of 1-300 B 0.38 / 0.48 against 0.055 /
// 0.058, cfg3 (Zipf, 37 KiB mean, 97 % of the bytes in frames >= 16 KiB)
// 0.733 / 0.776 against 0.775 / 0.797 (encode / gather).
constexpr uint64_t kChunkFormBelow = 16384;
static bool use_chunks(uint32_t n, uint64_t cap) { return n && cap / n < kChunkFormBelow; }
// The chunk copy loads its source non-temporally for every batch (cfg4 0.77 /
// 0.79 against 0.76 / 0.76 encode / gather with ordinary loads,
// profiles/r04o_chunk_ab.txt) and runs without an LDS cap on its occupancy (5
// blocks per CU, the unit form's large-frame setting, ran 0.61 against 0.75 on
// cfg3).
struct CopyWs {
    WsHead* head;
    V2* tiles;  // ntiles + 1: tile prefixes, then the totals
    V2* grp;    // one per 256-frame row: its prefix inside the tile
    UnitRec* rec;
    u32x4* edge;
    uint32_t* cmap;   // chunk -> frame holding its first byte
    uint32_t* dense;  // chunks chunk_copy_kernel left to chunk_dense_kernel
};

static uint64_t n_tiles(uint32_t n) { return ((uint64_t)n + kScanTile - 1) / kScanTile; }
static uint64_t n_rows(uint32_t n) { return ((uint64_t)n + kBlock - 1) / kBlock; }
// sum of unit_bound(R_f) <= total / (16 U) + n (1 + 63 / U) (and total <= cap)
// (rounded up to whole blocks: every wave of the copy grid reads its record)
static uint64_t max_units(uint32_t n, uint64_t cap)
{
    // unit_bound(R) <= R / (16 U) + 1 + 63 / U per frame (U = kUnitWords)
    const uint64_t u = (cap + kUnitWords * 16 - 1) / (kUnitWords * 16) + n + (63ull * n + kUnitWords - 1) / kUnitWords + 1;
    return (u + kBlock / 64 - 1) / (kBlock / 64) * (kBlock / 64);
}
static uint64_t r16(uint64_t x) { return (x + 15) & ~15ull; }
static uint64_t r256(uint64_t x) { return (x + 255) & ~255ull; }

// head, tile prefixes, row prefixes (the scan's scratch)
static size_t scan_ws_size(uint32_t n)
{
    return r16(sizeof(WsHead)) + (n_tiles(n) + 1) * sizeof(V2) + n_rows(n) * sizeof(V2);
}
static void carve_scan(char* p, uint32_t n, CopyWs& c)
{
    c.head = reinterpret_cast<WsHead*>(p);
    c.tiles = reinterpret_cast<V2*>(p + r16(sizeof(WsHead)));
    c.grp = c.tiles + n_tiles(n) + 1;
}

static size_t copy_ws_size(uint32_t n, uint64_t cap)
{
    if (!use_chunks(n, cap))
        return r256(scan_ws_size(n)) + r256((uint64_t)n * kEdgeWords * 16) + max_units(n, cap) * sizeof(UnitRec);
    return r256(scan_ws_size(n)) + r256((chunk_count(cap) + 1) * sizeof(uint32_t)) +
           r256(chunk_count(cap) * sizeof(uint32_t));
}

static bool carve(void* ws, size_t ws_bytes, uint32_t n, uint64_t cap, CopyWs& c)
{
    if (!ws || ws_bytes < copy_ws_size(n, cap)) return false;
    char* p = static_cast<char*>(ws);
    carve_scan(p, n, c);
    p += r256(scan_ws_size(n));  // edge words and records (or the chunk map) on whole lines
    c.edge = reinterpret_cast<u32x4*>(p);
    c.cmap = reinterpret_cast<uint32_t*>(p);
    c.dense = c.cmap + r256((chunk_count(cap) + 1) * sizeof(uint32_t)) / sizeof(uint32_t);
    p += r256((uint64_t)n * kEdgeWords * 16);
    c.rec = reinterpret_cast<UnitRec*>(p);
    return true;
}

// reduce_kernel (which also clears the status word), scan_tiles_kernel (n > 0).
template <class Size>
static kmws_status launch_reduce(Size size, uint32_t n, uint64_t* out, CopyWs& c, hipStream_t s)
{
    const uint32_t nt = (uint32_t)n_tiles(n);
    hipLaunchKernelGGL(reduce_kernel<Size>, dim3(nt), dim3(kBlock), 0, s, size, n, c.tiles, c.grp, c.head);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(kBlock), 0, s, c.tiles, nt, out, n);
    return hip_status(hipGetLastError());
}

// Encode / gather: reduce (row and tile totals), scan the tile totals, the
// prologue (offsets, edge words, unit records), the copy grid.  Four launches,
// stream-ordered, nothing on the host in between.
template <bool HEADERS>
static kmws_status launch_copy_tail(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                    const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c, hipStream_t s);

// The chunk form's front: one look-back pass (chunk_scan_kernel) in place of
// reduce + scan + chunk_map (which the fused unpack-gather keeps: its scan
// parses the headers).  Same box (profiles/r04aq_chunk_one_pass_ab.txt): cfg4
// 0.752-0.767 / 0.774-0.779 against 0.749-0.766 / 0.772-0.777, 1-300 B frames
// 0.35-0.40 / 0.45-0.49 against 0.34-0.39 / 0.44-0.48 (encode / gather).
template <bool HEADERS>
static kmws_status launch_chunks_one_pass(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                          const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c,
                                          hipStream_t s);
template <bool HEADERS>
static kmws_status launch_copy(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start, const kmws_desc* d,
                               const uint16_t* flags, uint32_t n, CopyWs& c, hipStream_t s)
{
    if (n == 0) {
        if (launch_zero(c.head, sizeof(WsHead), s) != KMWS_OK) return KMWS_ERR_FAILED;
        return launch_zero(start, sizeof(uint64_t), s);
    }
    if (use_chunks(n, cap)) return launch_chunks_one_pass<HEADERS>(src, dst, cap, start, d, flags, n, c, s);
    const kmws_status st = HEADERS ? launch_reduce(WireSize{d, flags}, n, start, c, s)
                                   : launch_reduce(PayloadSize{d}, n, start, c, s);
    if (st != KMWS_OK) return st;
    return launch_copy_tail<HEADERS>(src, dst, cap, start, d, flags, n, c, s);
}

// The chunk form after the scan: chunk_map, the chunk copy grid, the dense
// chunks (usually none: the grid of chunk_dense_kernel exits at once).
template <bool HEADERS>
static kmws_status launch_chunk_copy(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                     const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c, uint32_t nt,
                                     hipStream_t s);
template <bool HEADERS>
static kmws_status launch_chunks(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start, const kmws_desc* d,
                                 const uint16_t* flags, uint32_t n, CopyWs& c, uint32_t nt, hipStream_t s)
{
    hipLaunchKernelGGL(chunk_map_kernel<HEADERS>, dim3((uint32_t)n_rows(n)), dim3(kBlock), 0, s, d, flags, n, cap,
                       c.head, c.tiles, nt, c.grp, start, c.cmap);
    return launch_chunk_copy<HEADERS>(src, dst, cap, start, d, flags, n, c, nt, s);
}

// The chunk form's front in one pass:
// zero the head, the totals and the tile states, then chunk_scan_kernel.
template <bool HEADERS>
static kmws_status launch_chunks_one_pass(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                          const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c,
                                          hipStream_t s)
{
    const uint32_t nt = (uint32_t)n_tiles(n);
    // head | tile totals (nt + 1) | the row-prefix area, whose first nt words hold the states
    const uint64_t words = (r16(sizeof(WsHead)) + (uint64_t)(nt + 1) * sizeof(V2) + (uint64_t)nt * 8) / 8;
    const uint64_t zb = (words + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(zero_words_kernel, dim3((uint32_t)(zb < 1024 ? zb : 1024)), dim3(kBlock), 0, s,
                       reinterpret_cast<uint64_t*>(c.head), words);
    hipLaunchKernelGGL(chunk_scan_kernel<HEADERS>, dim3(nt), dim3(kBlock), 0, s, d, flags, n, cap, c.head,
                       reinterpret_cast<uint64_t*>(c.grp), c.tiles + nt, start, c.cmap);
    return launch_chunk_copy<HEADERS>(src, dst, cap, start, d, flags, n, c, nt, s);
}

// The chunk copy grid and the dense chunks.
template <bool HEADERS>
static kmws_status launch_chunk_copy(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                     const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c, uint32_t nt,
                                     hipStream_t s)
{
    const uint64_t chunks = chunk_count(cap);  // upper bound; waves past the total exit at once
    constexpr uint64_t kWaves = kBlock / 64;
    constexpr uint64_t kMaxChunksPerLaunch = ((1ull << 32) / kBlock / 2) * kWaves;
    for (uint64_t c0 = 0; c0 < chunks; c0 += kMaxChunksPerLaunch) {
        const uint64_t nc = chunks - c0 < kMaxChunksPerLaunch ? chunks - c0 : kMaxChunksPerLaunch;
        const dim3 grid((uint32_t)((nc + kWaves - 1) / kWaves));
        hipLaunchKernelGGL(chunk_copy_kernel<HEADERS>, grid, dim3(kBlock), 0, s, src, dst, d, flags, n, start, c.cmap,
                           c.tiles + nt, c.head, c.dense, c0, kChunkSplit);
    }
    const uint32_t dense_blocks = (uint32_t)(chunks / kWaves < 512 ? chunks / kWaves + 1 : 512);
    hipLaunchKernelGGL(chunk_dense_kernel<HEADERS>, dim3(dense_blocks), dim3(kBlock), 0, s, src, dst, d, flags, n, start,
                       c.cmap, c.tiles + nt, c.head, c.dense);
    return hip_status(hipGetLastError());
}

// The copy form after the scan: chunks (small mean) or the prologue and the
// unit copy grid.
template <bool HEADERS>
static kmws_status launch_copy_tail(const uint8_t* src, uint8_t* dst, uint64_t cap, uint64_t* start,
                                    const kmws_desc* d, const uint16_t* flags, uint32_t n, CopyWs& c, hipStream_t s)
{
    const uint32_t nt = (uint32_t)n_tiles(n);
    if (use_chunks(n, cap)) return launch_chunks<HEADERS>(src, dst, cap, start, d, flags, n, c, nt, s);
    hipLaunchKernelGGL(prologue_kernel<HEADERS>, dim3((uint32_t)n_rows(n)), dim3(kBlock), 0, s, src, d, flags, n, cap,
                       c.head, c.tiles, nt, c.grp, start, c.rec, c.edge);
    // Occupancy: runs of large frames stream faster with 5 blocks per CU (fewer
    // concurrent DRAM streams; capped by 32 KiB of dynamic LDS per block),
    // batches of small frames need every wave slot to hide their per-unit
    // latency.  cap / n bounds the mean region size from above.
    const unsigned lds_pad = cap / n >= 16384 ? 32768u : 0u;
    const uint64_t units = max_units(n, cap);  // upper bound; surplus waves exit at once
    constexpr uint64_t kWavesPerBlock = kBlock / 64;
    constexpr uint64_t kMaxUnitsPerLaunch = ((1ull << 32) / kBlock / 2) * kWavesPerBlock;
    for (uint64_t u0 = 0; u0 < units; u0 += kMaxUnitsPerLaunch) {
        const uint64_t nu = units - u0 < kMaxUnitsPerLaunch ? units - u0 : kMaxUnitsPerLaunch;
        hipLaunchKernelGGL(copy_kernel<HEADERS>, dim3((uint32_t)((nu + kWavesPerBlock - 1) / kWavesPerBlock)),
                           dim3(kBlock), lds_pad, s, src, dst, c.tiles + nt, c.rec, c.edge, c.head, u0, kCopySplit);
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
    kmws::note_device_batch(2 * dst_cap, s);
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
    kmws::note_device_batch(2 * dst_cap, s);
    return launch_copy<false>(src, dst, dst_cap, dst_off, descs, nullptr, n, c, s);
}

// Header parse fused into the gather: status cleared, reduce over the parsed
// payload lengths (writing the descriptors), scan, prologue, copy -- the
// kmws_unpack_headers launch and its status clear are gone.
kmws_status kmws_unpack_gather(const uint8_t* wire, uint64_t wire_len, const uint64_t* hdr_off, uint32_t n, int mode,
                               kmws_desc* out_desc, uint16_t* out_flags, uint8_t* out_err, uint8_t* dst,
                               uint64_t dst_cap, uint64_t* dst_off, void* workspace, size_t workspace_bytes,
                               void* stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    CopyWs c;
    if (!dst_off || (n && (!wire || !hdr_off || !out_desc || !dst)) || (reinterpret_cast<uintptr_t>(dst) & 15u) ||
        (reinterpret_cast<uintptr_t>(wire) & 15u) || (mode != KMWS_MODE_CLIENT && mode != KMWS_MODE_SERVER) ||
        !carve(workspace, workspace_bytes, n, dst_cap, c))
        return workspace && workspace_bytes < copy_ws_size(n, dst_cap) ? KMWS_ERR_BUFFER_TOO_SMALL
                                                                       : KMWS_ERR_INVALID_PARAM;
    if (launch_zero(c.head, sizeof(WsHead), s) != KMWS_OK) return KMWS_ERR_FAILED;
    if (n == 0) return launch_zero(dst_off, sizeof(uint64_t), s);
    kmws::note_device_batch(wire_len + dst_cap, s);
    kmws_status st = launch_reduce(HeaderPayloadSize{wire, wire_len, hdr_off, n, mode, out_desc, out_flags, out_err,
                                                     c.head},
                                   n, dst_off, c, s);
    if (st != KMWS_OK) return st;
    return launch_copy_tail<false>(wire, dst, dst_cap, dst_off, out_desc, nullptr, n, c, s);
}

// head, then one 64-bit state per 2048-frame tile (pack_headers_chain_kernel)
size_t kmws_pack_headers_workspace_size(uint32_t n) { return r16(sizeof(WsHead)) + n_tiles(n) * sizeof(uint64_t); }

kmws_status kmws_pack_headers(const kmws_desc* descs, const uint16_t* flags, uint32_t n, uint8_t* hdr,
                              uint8_t* hl_out, uint64_t* wire_off, void* workspace, size_t workspace_bytes,
                              void* stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if ((n && (!descs || !flags || !hdr)) || (reinterpret_cast<uintptr_t>(hdr) & 15u) ||
        (wire_off && !workspace))
        return KMWS_ERR_INVALID_PARAM;
    u32x4* h = reinterpret_cast<u32x4*>(hdr);
    if (wire_off) {
        if (workspace_bytes < kmws_pack_headers_workspace_size(n)) return KMWS_ERR_BUFFER_TOO_SMALL;
        WsHead* head = static_cast<WsHead*>(workspace);
        uint64_t* st = reinterpret_cast<uint64_t*>(static_cast<char*>(workspace) + r16(sizeof(WsHead)));
        if (n == 0) {
            if (launch_zero(head, sizeof(WsHead), s) != KMWS_OK) return KMWS_ERR_FAILED;
            return launch_zero(wire_off, sizeof(uint64_t), s);
        }
        // two launches: zero the head and the tile states, then the one-pass kernel
        const uint64_t words = kmws_pack_headers_workspace_size(n) / 8;
        const uint64_t zb = (words + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(zero_words_kernel, dim3((uint32_t)(zb < 1024 ? zb : 1024)), dim3(kBlock), 0, s,
                           reinterpret_cast<uint64_t*>(head), words);
        hipLaunchKernelGGL(pack_headers_chain_kernel, dim3((uint32_t)n_tiles(n)), dim3(kBlock), 0, s, descs, flags, n, h,
                           hl_out, wire_off, st, head);
        return hip_status(hipGetLastError());
    }
    if (n == 0) return KMWS_OK;
    hipLaunchKernelGGL(pack_headers_kernel, dim3((uint32_t)n_rows(n)), dim3(kBlock), 0, s, descs, flags, n, h, hl_out);
    return hip_status(hipGetLastError());
}

kmws_status kmws_find_headers_streams(const uint8_t* wire, uint64_t wire_len, const uint64_t* stream_off,
                                      uint32_t n_streams, uint64_t* hdr_off, uint32_t cap, uint32_t* n_out,
                                      uint64_t* consumed, void* stream)
{
    if (n_streams && (!stream_off || !n_out || (cap && !hdr_off) || (wire_len && !wire))) return KMWS_ERR_INVALID_PARAM;
    if (n_streams == 0) return KMWS_OK;
    hipLaunchKernelGGL(walk_headers_kernel, dim3((n_streams + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), wire, wire_len, stream_off, n_streams, hdr_off, cap, n_out,
                       consumed);
    return hip_status(hipGetLastError());
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
    if (launch_zero(head, sizeof(WsHead), s) != KMWS_OK) return KMWS_ERR_FAILED;
    if (n == 0) return KMWS_OK;
    hipLaunchKernelGGL(unpack_headers_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, wire, wire_len,
                       hdr_off, n, mode, out_desc, out_flags, out_err, head);
    return hip_status(hipGetLastError());
}

}  // extern "C"
