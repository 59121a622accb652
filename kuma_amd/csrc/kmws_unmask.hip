// Batched in-place WebSocket payload unmask for MI355X (gfx950).
//
// Replaces the per-frame scalar loop WSHandler::handleDataMask
// (src/ws/WSHandler.cpp:303-310; gate :291-301) with one stream-ordered pass
// over a whole descriptor batch.  Byte semantics are identical: payload byte
// j of a frame is XORed with maskey[j % 4]; key phase restarts per frame.
//
// Layout: the payload address space [0, span) of `base` is cut into fixed
// tiles of kTile bytes.  A prep kernel writes, for every tile, the index of
// the frame whose region (its offset up to the next frame's offset) contains
// the tile start, so a tile block finds its frames with one load.  The main
// kernel block (256 lanes) issues its 16-byte loads first, then stages the
// descriptors of the frames overlapping its tile in LDS and builds a per-word
// mask (a rotated key splatted over the payload bytes of the word; header or
// gap bytes get 0), XORs and stores whole 16-byte words.  HBM-bound: 2 bytes
// of traffic per payload byte + 16 B per descriptor; no MFMA.
#include "kmws_common.hpp"


// Uncapped split grids (batches of frames shorter than a tile, the LDS-staged
// path) load the tile's descriptors before its payload: cfg4's in-place unmask
// 80.3-80.4 -> 81.7-82.2 % (profiles/r02bt_unmask_desc_prefetch_ab.txt).  0 = off.
#ifndef KMWS_UNMASK_PRE
#define KMWS_UNMASK_PRE 1
#endif

namespace kmws {

// Payload store of a tile word: non-temporal (streams past the L2; the
// default) or temporal (NT = false: the line stays in L2 and is written back
// on eviction).  Which one streams faster depends on the batch's layout: on an
// aligned arena temporal stores ran +0.3-1.0 points, on a packed wire image
// they lost 1.6-7 (profiles/r02bz_unmask_store_policy_ab.txt), so the policy
// is part of the schedule the autotune times on the caller's batch.
template <bool NT>
__device__ __forceinline__ void store_word(const u32x4& val, u32x4* p)
{
    if constexpr (NT) __builtin_nontemporal_store(val, p);
    else *p = val;
}

// Each lane owns V consecutive-block words: word w = tid + kBlock * i.
template <int V>
struct UnmaskCfg {
    static constexpr int kWords = kBlock * V;
    static constexpr uint64_t kTile = (uint64_t)kWords * 16u;
    static constexpr int kCap = kBlock;  // descriptors staged per LDS round
};

// Tile -> first frame map.  Frame f owns tile starts in [start_f, next_f)
// where start_0 = 0, start_f = off_f, next_f = off_{f+1} (span for the last).
// Validates sortedness / non-overlap / bounds on the fly.
__global__ void __launch_bounds__(kBlock) tile_map_kernel(const kmws_desc* __restrict__ d, uint32_t n,
                                                          uint64_t span, uint32_t tile_shift,
                                                          uint32_t* __restrict__ map,
                                                          WsHead* __restrict__ head)
{
    const uint32_t f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= n) return;
    const kmws_desc df = d[f];
    const uint64_t next = (f + 1 < n) ? d[f + 1].off : span;
    if (df.off > span || df.off + (uint64_t)df.len > next) {
        atomicOr(&head->status, kStatusBadDesc);
        return;
    }
    const uint64_t start = f == 0 ? 0 : df.off;
    const uint64_t T = 1ull << tile_shift;
    const uint64_t b0 = (start + T - 1) >> tile_shift;
    const uint64_t b1 = (next + T - 1) >> tile_shift;
    for (uint64_t b = b0; b < b1; ++b) map[b] = f;
    if (f == n - 1) map[b1] = f;  // sentinel after the last tile: "next tile's frame" of the last tile
}

// Issue every payload load of a tile.  Full tiles load unconditionally so the
// loads stay back to back.  Payload is touched once: non-temporal loads and
// stores (measured +6 % on MI355X for this in-place stream, tools/membw_probe.hip).
template <int V, bool FULL>
__device__ __forceinline__ void load_tile(const uint8_t* __restrict__ base, uint64_t tile_lo, uint64_t tile_hi,
                                          u32x4 (&v)[V])
{
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
        if (FULL || a < tile_hi) v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + a));
        else v[i] = u32x4{0, 0, 0, 0};
    }
}

// Mask and store a loaded tile.  f = the tile-map frame, ok = plan status clean.
template <int V, bool FULL, bool TWO = false, bool NT = true>
__device__ __forceinline__ void finish_tile(uint8_t* __restrict__ base, uint64_t tile_lo, uint64_t tile_hi,
                                            const kmws_desc* __restrict__ d, uint32_t n,
                                            const uint32_t* __restrict__ map, uint32_t tile, bool ok,
                                            const u32x4 (&v)[V], uint64_t* s_off, uint64_t* s_end, uint32_t* s_key,
                                            const u32x4* pre = nullptr)
{
    using Cfg = UnmaskCfg<V>;
    const int tid = threadIdx.x;
    // frames [f, flast] are the only ones that can overlap the tile: flast's
    // region holds the next tile's start (the map's last entry is a sentinel)
    uint32_t f = map[tile];
    const uint32_t flast = map[tile + 1];

    // Fast path: one frame covers the whole tile (every tile of a 64 KiB-frame
    // arena).  The test reads block-uniform scalars only, so the branch is
    // uniform and needs no LDS or barrier.
    const kmws_desc d0 = d[f < n ? f : 0];
    if (FULL && f < n && d0.off <= tile_lo && d0.off + d0.len >= tile_hi) {
        const uint32_t r = rot_key(d0.key, d0.off);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
            if (ok) store_word<NT>(v[i] ^ r, reinterpret_cast<u32x4*>(base + a));
        }
        return;
    }

    // Two frames at most (a frame boundary inside the tile, e.g. a packed wire
    // image of frames longer than a tile): both descriptors are block-uniform
    // scalars, each word's mask is built from them directly -- no LDS, no
    // barrier (at 2 blocks per CU a barrier's latency is not hidden; TWO: the
    // capped launches; uncapped, the LDS path measured faster on 4 KiB frames).
    // Every mask is built before the first store, so the mask ALU runs while
    // the payload loads are still in flight (built word by word between the
    // stores, it delayed each boundary tile's stores by ~12 %: the two-frame
    // path replaced by a plain XOR ran the packed wire at the aligned rate,
    // profiles/r02bj_unmask_two_frame_ab.txt).  Words whose mask is zero (headers,
    // gaps) are not stored.
    if (TWO && FULL && flast <= f + 1 && f < n) {
        const kmws_desc d1 = flast > f && flast < n ? d[flast] : kmws_desc{~0ull, 0u, 0u};
        const uint32_t r0 = rot_key(d0.key, d0.off), r1 = rot_key(d1.key, d1.off);
        // payload extents relative to the tile, clamped to [0, kTile]: block-uniform
        // scalars, so each per-word test is one 32-bit compare
        constexpr uint32_t T = (uint32_t)Cfg::kTile;
        auto rel = [&](uint64_t x) -> uint32_t {
            return x <= tile_lo ? 0u : (x - tile_lo >= T ? T : (uint32_t)(x - tile_lo));
        };
        const uint32_t s0 = rel(d0.off), t0 = rel(d0.off + d0.len);
        const uint32_t s1 = rel(d1.off), t1 = d1.len ? rel(d1.off + d1.len) : s1;
        u32x4 m[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint32_t x = 16u * (uint32_t)(tid + kBlock * i);
            u32x4 mm = u32x4{0, 0, 0, 0};
            if (s0 <= x && t0 >= x + 16) {
                mm = u32x4{r0, r0, r0, r0};
            } else if (s1 <= x && t1 >= x + 16) {
                mm = u32x4{r1, r1, r1, r1};
            } else {  // a word holding a frame edge: byte-exact
                // each frame's bytes of the word, clamped to [0, 16] (empty if none)
                auto cl = [&](uint32_t y) -> int { return y <= x ? 0 : (y - x >= 16u ? 16 : (int)(y - x)); };
                mm = (word_byte_range(cl(s0), cl(t0)) & r0) | (word_byte_range(cl(s1), cl(t1)) & r1);
            }
            m[i] = mm;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
            if (ok && (m[i].x | m[i].y | m[i].z | m[i].w) != 0u)
                store_word<NT>(v[i] ^ m[i], reinterpret_cast<u32x4*>(base + a));
        }
        return;
    }

    // General path: stage the descriptors of frames overlapping the tile in
    // LDS, kCap per round, and build a byte-exact mask per 16-byte word.
    u32x4 m[V];
#pragma unroll
    for (int i = 0; i < V; ++i) m[i] = u32x4{0, 0, 0, 0};
    // One round: lane tid holds descriptor f + tid (`have`: it exists and can
    // overlap the tile); returns how many were staged.
    auto round = [&](bool have, const u32x4& x) -> int {
        int valid = 0;
        if (have) {
            const uint64_t off = (uint64_t)x.x | ((uint64_t)x.y << 32);
            if (off < tile_hi) {
                valid = 1;
                s_off[tid] = off;
                s_end[tid] = off + x.z;
                s_key[tid] = x.w;
            }
        }
        const int cnt = __syncthreads_count(valid);  // sorted => a prefix
#pragma unroll
        for (int i = 0; i < V; ++i) {
            const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
            int lo = 0, hi = cnt;  // first staged frame with end > a
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_end[mid] <= a) lo = mid + 1; else hi = mid;
            }
            for (int j = lo; j < cnt; ++j) {
                const uint64_t o = s_off[j];
                if (o >= a + 16) break;
                const uint64_t e = s_end[j];
                const uint32_t r = rot_key(s_key[j], o);
                if (o <= a && e >= a + 16) {
                    m[i] |= u32x4{r, r, r, r};
                } else {
                    const int blo = o > a ? (int)(o - a) : 0;
                    const int bhi = e < a + 16 ? (int)(e - a) : 16;
                    m[i].x |= r & dword_byte_mask(blo, bhi, 0);
                    m[i].y |= r & dword_byte_mask(blo, bhi, 1);
                    m[i].z |= r & dword_byte_mask(blo, bhi, 2);
                    m[i].w |= r & dword_byte_mask(blo, bhi, 3);
                }
            }
        }
        __syncthreads();  // every lane done reading this round's LDS (also before a next tile reuses it)
        return cnt;
    };
    // no descriptor loads past the tile's last frame; the first round's may
    // have been issued before the payload loads (`pre`): then no wait here
    // covers the payload
    auto have_f = [&]() { return f + (uint32_t)tid < n && f + (uint32_t)tid <= flast; };
    auto load_f = [&]() { return have_f() ? *reinterpret_cast<const u32x4*>(d + f + tid) : u32x4{0, 0, 0, 0}; };
    int cnt = pre ? round(have_f(), *pre) : round(have_f(), load_f());
    while (cnt == Cfg::kCap) {
        f += Cfg::kCap;
        cnt = round(have_f(), load_f());
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint64_t a = tile_lo + 16u * (uint64_t)(tid + kBlock * i);
        const u32x4 mm = m[i];
        if (ok && (FULL || a < tile_hi) && (mm.x | mm.y | mm.z | mm.w) != 0u)
            store_word<NT>(v[i] ^ mm, reinterpret_cast<u32x4*>(base + a));
    }
}

// One block per tile.  W = minimum waves per SIMD the register allocation must
// allow (1 = unconstrained; the tuning variants test 6 and 8).
template <int V, int W = 1, bool TWO = false>
__global__ void __launch_bounds__(kBlock, W) unmask_tiles_kernel(uint8_t* __restrict__ base, uint64_t span,
                                                              const kmws_desc* __restrict__ d, uint32_t n,
                                                              const uint32_t* __restrict__ map,
                                                              const WsHead* __restrict__ head, uint32_t tile_base)
{
    using Cfg = UnmaskCfg<V>;
    __shared__ uint64_t s_off[Cfg::kCap];
    __shared__ uint64_t s_end[Cfg::kCap];
    __shared__ uint32_t s_key[Cfg::kCap];
    const uint32_t tile = tile_base + blockIdx.x;
    const uint64_t tile_lo = (uint64_t)tile * Cfg::kTile;
    u32x4 v[V];
    // Metadata comes after the payload loads, with no early exit between the
    // loads and their uses, so the compiler cannot sink the loads below the
    // scalar metadata waits.  A bad plan (status != 0) stores nothing.
    if (tile_lo + Cfg::kTile <= span) {
        load_tile<V, true>(base, tile_lo, tile_lo + Cfg::kTile, v);
        __builtin_amdgcn_sched_barrier(0);
        finish_tile<V, true, TWO>(base, tile_lo, tile_lo + Cfg::kTile, d, n, map, tile, head->status == 0, v, s_off,
                             s_end, s_key);
    } else {
        load_tile<V, false>(base, tile_lo, span, v);
        __builtin_amdgcn_sched_barrier(0);
        finish_tile<V, false>(base, tile_lo, span, d, n, map, tile, head->status == 0, v, s_off, s_end, s_key);
    }
}

// One block per full tile like unmask_tiles_kernel, blocks dealt over `k`
// equal parts of the span: block b takes tile (b mod k) * (nfull / k) + b / k,
// so the blocks in flight stream k windows far apart instead of one (the
// blocks past k * (nfull / k) take the remaining tiles in order).  With c > 0
// the span is cut into runs of c tiles instead, dealt round-robin to the k
// residues of b (blocks go round-robin over the 8 XCDs: k = 8 gives each XCD
// its own runs).
template <int V, bool TWO = false, bool NT = true>
__global__ void __launch_bounds__(kBlock) unmask_split_kernel(uint8_t* __restrict__ base,
                                                              const kmws_desc* __restrict__ d, uint32_t n,
                                                              const uint32_t* __restrict__ map,
                                                              const WsHead* __restrict__ head, uint32_t nfull,
                                                              uint32_t k, uint32_t c, uint32_t b0, uint32_t w)
{
    using Cfg = UnmaskCfg<V>;
    __shared__ uint64_t s_off[Cfg::kCap];
    __shared__ uint64_t s_end[Cfg::kCap];
    __shared__ uint32_t s_key[Cfg::kCap];
    const uint32_t b = b0 + blockIdx.x;
    uint32_t tile = b;
    if (c == 0) {  // k equal parts
        const uint32_t q = nfull / k;
        if (b < q * k) tile = (b % k) * q + b / k;
    } else if (w <= 1) {  // runs of c tiles dealt round-robin over the k residues of b mod k
        const uint64_t run = (uint64_t)k * c;
        if (b < nfull / run * run) {
            const uint32_t x = b % k, i = b / k;
            tile = (i / c) * (uint32_t)run + x * c + i % c;
        }
    } else {  // residues split into w groups, each group's runs inside its own far-apart window
        const uint32_t kg = k / w;                      // residues per group
        const uint64_t run = (uint64_t)kg * c;          // tiles per round of a group's runs
        const uint64_t per = (uint64_t)nfull / w / run * run;
        if (b < per * w) {
            const uint32_t x = b % k, i = b / k;
            const uint32_t g = x % w, xi = x / w;
            tile = (uint32_t)(g * per) + (i / c) * (uint32_t)run + xi * c + i % c;
        }
    }
    const uint64_t lo = (uint64_t)tile * Cfg::kTile;
    u32x4 v[V];
#if KMWS_UNMASK_PRE
    if constexpr (!TWO) {
        // the tile's descriptors first: their wait then counts only them, not the
        // payload loads issued after them (vmcnt is one in-order queue)
        const uint32_t f = map[tile], fl = map[tile + 1];
        const uint32_t fi = f + threadIdx.x;
        u32x4 pre = u32x4{0, 0, 0, 0};
        if (fi < n && fi <= fl) pre = *reinterpret_cast<const u32x4*>(d + fi);
        load_tile<V, true>(base, lo, lo + Cfg::kTile, v);
        __builtin_amdgcn_sched_barrier(0);
        finish_tile<V, true, TWO, NT>(base, lo, lo + Cfg::kTile, d, n, map, tile, head->status == 0, v, s_off, s_end,
                                      s_key, &pre);
        return;
    }
#endif
    load_tile<V, true>(base, lo, lo + Cfg::kTile, v);
    __builtin_amdgcn_sched_barrier(0);
    finish_tile<V, true, TWO, NT>(base, lo, lo + Cfg::kTile, d, n, map, tile, head->status == 0, v, s_off, s_end,
                                  s_key);
}

// Grid-stride over the full tiles [0, nfull): block b takes tiles b, b+G, ...
// and issues the next tile's loads before finishing the current one.
template <int V>
__global__ void __launch_bounds__(kBlock) unmask_persist_kernel(uint8_t* __restrict__ base,
                                                                const kmws_desc* __restrict__ d, uint32_t n,
                                                                const uint32_t* __restrict__ map,
                                                                const WsHead* __restrict__ head, uint32_t nfull)
{
    using Cfg = UnmaskCfg<V>;
    __shared__ uint64_t s_off[Cfg::kCap];
    __shared__ uint64_t s_end[Cfg::kCap];
    __shared__ uint32_t s_key[Cfg::kCap];
    uint32_t t = blockIdx.x;
    if (t >= nfull) return;
    const bool ok = head->status == 0;
    u32x4 v[V];
    load_tile<V, true>(base, (uint64_t)t * Cfg::kTile, 0, v);
    for (;;) {
        const uint32_t tn = t + gridDim.x;
        u32x4 w[V];
        if (tn < nfull) load_tile<V, true>(base, (uint64_t)tn * Cfg::kTile, 0, w);
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t lo = (uint64_t)t * Cfg::kTile;
        finish_tile<V, true>(base, lo, lo + Cfg::kTile, d, n, map, t, ok, v, s_off, s_end, s_key);
        if (tn >= nfull) break;
#pragma unroll
        for (int i = 0; i < V; ++i) v[i] = w[i];
        t = tn;
    }
}

// Grid-stride like unmask_persist_kernel, software-pipelined for real: two
// register sets used in turn (a copy from one to the other waits for the loads
// in flight), and a loop with one exit at the bottom -- both steps run every
// trip, a step past the end loads a clamped tile and stores nothing -- so the
// wait before a tile's stores counts only that tile's loads.
template <int V>
__global__ void __launch_bounds__(kBlock) unmask_pipe_kernel(uint8_t* __restrict__ base,
                                                             const kmws_desc* __restrict__ d, uint32_t n,
                                                             const uint32_t* __restrict__ map,
                                                             const WsHead* __restrict__ head, uint32_t nfull)
{
    using Cfg = UnmaskCfg<V>;
    __shared__ uint64_t s_off[Cfg::kCap];
    __shared__ uint64_t s_end[Cfg::kCap];
    __shared__ uint32_t s_key[Cfg::kCap];
    uint32_t t = blockIdx.x;
    if (t >= nfull) return;
    const bool ok = head->status == 0;
    const uint32_t last = nfull - 1;
    u32x4 va[V], vb[V];
    load_tile<V, true>(base, (uint64_t)t * Cfg::kTile, 0, va);
    auto step = [&](const u32x4(&vc)[V], u32x4(&vn)[V]) __attribute__((always_inline)) {
        const uint32_t tn = t + gridDim.x;
        const bool more = tn < nfull;
        load_tile<V, true>(base, (uint64_t)(more ? tn : last) * Cfg::kTile, 0, vn);
        __builtin_amdgcn_sched_barrier(0);
        const bool live = t < nfull;
        const uint32_t tt = live ? t : last;
        const uint64_t lo = (uint64_t)tt * Cfg::kTile;
        finish_tile<V, true>(base, lo, lo + Cfg::kTile, d, n, map, tt, ok && live, vc, s_off, s_end, s_key);
        __builtin_amdgcn_sched_barrier(0);
        t = tn;
        return more;
    };
    for (;;) {
        const bool a = step(va, vb);
        const bool b = step(vb, va);
        if (!(a & b)) break;
    }
}

// Small host batches: the decoder's payloads of one socket read or one loop
// iteration, produced by its own parser (disjoint, in range: nothing to
// validate).  A plan + apply per read costs more than the bytes, so these go
// in ONE launch: block b unmasks piece pieces[b] -- up to kPieceWords words of
// one frame's aligned hull -- with descriptors and piece list read from
// host-visible memory.  A hull's first and last words may hold bytes of other
// frames (or headers): those words are written byte by byte, the frame's own
// bytes only, so blocks of neighbouring frames never write the same byte.
__global__ void __launch_bounds__(kBlock) unmask_pieces_kernel(uint8_t* __restrict__ base,
                                                               const kmws_desc* __restrict__ d,
                                                               const PieceRec* __restrict__ pieces)
{
    constexpr int V = kPieceWords / kBlock;
    const PieceRec pr = pieces[blockIdx.x];
    const kmws_desc x = d[pr.frame];
    const uint64_t end = x.off + x.len;
    const uint64_t w0 = (x.off >> 4) + (uint64_t)pr.piece * kPieceWords;
    const uint64_t wh = (end + 15) >> 4;
    const uint64_t w1 = wh < w0 + kPieceWords ? wh : w0 + kPieceWords;
    const uint32_t r = rot_key(x.key, x.off);
    u32x4 v[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint64_t w = w0 + threadIdx.x + (uint64_t)kBlock * i;
        v[i] = w < w1 ? *reinterpret_cast<const u32x4*>(base + 16 * w) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const uint64_t w = w0 + threadIdx.x + (uint64_t)kBlock * i;
        if (w >= w1) continue;
        const uint64_t a = 16 * w;
        if (a >= x.off && a + 16 <= end) {
            *reinterpret_cast<u32x4*>(base + a) = v[i] ^ r;
        } else {  // the hull's first or last word: own bytes only
            const uint64_t lo = a > x.off ? a : x.off, hi = a + 16 < end ? a + 16 : end;
            for (uint64_t q = lo; q < hi; ++q) {
                const uint32_t b = (uint32_t)(q - a);
                const uint32_t dw = (b & 8u) ? ((b & 4u) ? v[i].w : v[i].z) : ((b & 4u) ? v[i].y : v[i].x);
                base[q] = (uint8_t)((dw ^ r) >> (8 * (b & 3u)));
            }
        }
    }
}

// ---- synthetic fill: byte i = byte (i & 7) of splitmix64(seed + (i >> 3)) ----
__global__ void __launch_bounds__(kBlock) fill_synthetic_kernel(uint8_t* __restrict__ base, uint64_t bytes,
                                                                uint64_t seed)
{
    const uint64_t nw = bytes >> 4;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < nw; w += stride) {
        const uint64_t a = splitmix64(seed + 2 * w), b = splitmix64(seed + 2 * w + 1);
        *reinterpret_cast<u32x4*>(base + 16 * w) =
            u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
    }
    if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) {
        const uint64_t i = (nw << 4) + threadIdx.x;
        base[i] = (uint8_t)(splitmix64(seed + (i >> 3)) >> (8 * (i & 7)));
    }
}

__global__ void __launch_bounds__(kBlock) uniform_descs_kernel(kmws_desc* __restrict__ d, uint32_t n,
                                                               uint64_t stride, uint32_t len, uint64_t key_seed)
{
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    kmws_desc x;
    x.off = (uint64_t)i * stride;
    x.len = len;
    x.key = (uint32_t)splitmix64(key_seed + i);
    d[i] = x;
}

// ---- independent checker: simple byte-wise restatement, not the product path ----
constexpr int kCheckBytes = 4096;  // bytes per checker block

__global__ void __launch_bounds__(kBlock) check_unmasked_kernel(const uint8_t* __restrict__ base, uint64_t bytes,
                                                                uint64_t seed, const kmws_desc* __restrict__ d,
                                                                uint32_t n, unsigned long long* mismatches)
{
    __shared__ uint32_t s_first;
    const uint64_t nblk = (bytes + kCheckBytes - 1) / kCheckBytes;
    unsigned long long bad = 0;
    for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const uint64_t blk_lo = blk * kCheckBytes;
    __syncthreads();
    if (threadIdx.x == 0) {
        // first frame with off + len > blk_lo (binary search over sorted descs)
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (d[mid].off + d[mid].len <= blk_lo) lo = mid + 1; else hi = mid;
        }
        s_first = lo;
    }
    __syncthreads();
    uint32_t f = s_first;
    const uint64_t p0 = blk_lo + 16u * threadIdx.x;
    for (int k = 0; k < 16; ++k) {
        const uint64_t p = p0 + k;
        if (p >= bytes) break;
        while (f < n && d[f].off + d[f].len <= p) ++f;
        uint8_t expect = (uint8_t)(splitmix64(seed + (p >> 3)) >> (8 * (p & 7)));
        if (f < n && d[f].off <= p) {
            const uint32_t key = d[f].key;
            expect ^= (uint8_t)(key >> (8 * ((p - d[f].off) & 3)));
        }
        bad += base[p] != expect;
    }
    }
    if (bad) atomicAdd(mismatches, bad);
}

// Tile geometry used by the product path (tuned on MI355X).
constexpr int kUnmaskV = 4;

// Apply schedule per device (codes: launch_schedule).  Where the blocks in
// flight are decides the rate: the in-order grid streams one 16 MiB window
// (74.5-75 % of HBM peak everywhere); dealing blocks over 8 parts of the span
// streams 8 windows far apart (82-83 % on some 64 GiB placements in HBM, 76 %
// on others); runs of 16 tiles per XCD hold 78-79 % on every placement; two
// groups of 4 XCDs, each with runs of 16 in its own half of the span, match
// the better of the two on every placement measured and lead on 4 KiB frames
// (82 %) (profiles/r01f_unmask_placement.txt).  Default: the grouped runs;
// kmws_unmask_autotune picks per device on the caller's batch.
constexpr int kMaxDevices = 64;
static uint32_t g_schedule[kMaxDevices];
using ProdCfg = UnmaskCfg<kUnmaskV>;

// Blocks of an apply grid resident per CU.  Fewer blocks in flight stream HBM
// better: 2 blocks of 256 lanes per CU (32 KiB of loads in flight per CU) run
// the 64 GiB batch at 84.5-84.8 % of peak against 82.4-82.9 % with the 6 the
// registers allow, 3 blocks at 83.4 %, 1 block at 65-75 %
// (profiles/r02ag_unmask_occupancy.txt).  The cap is dynamic LDS the kernel does
// not use: a block asks for just over a third of the CU's LDS.
// KMWS_UNMASK_BLOCKS_PER_CU overrides it for every batch (0 = no cap; tuning).
constexpr uint32_t kUnmaskBlocksPerCU = 2;
constexpr uint32_t kUnmaskStaticLds = UnmaskCfg<4>::kCap * (8 + 8 + 4);  // s_off, s_end, s_key
static unsigned unmask_lds_pad_device();
// The cap pays where tiles take the one- or two-frame paths (regions of a tile
// or more: 16 KiB frames ran 85.5 % capped vs 79-83 % uncapped); batches of
// smaller frames (several per tile: the LDS-staged path, whose barriers need the
// latency hiding of a full CU) keep every block: 8 KiB frames ran 54.8 % capped
// vs 83 %, 4 KiB frames 47.6 % vs 80 % (profiles/r02at_unmask_framelen_occupancy.txt).
// Mean region >= 1 tile selects.
static unsigned unmask_lds_pad(uint64_t span, uint32_t n)
{
    static const bool forced = getenv("KMWS_UNMASK_BLOCKS_PER_CU") != nullptr;  // tuning: the cap on every batch
    return forced || (n && span / n >= UnmaskCfg<4>::kTile) ? unmask_lds_pad_device() : 0u;
}
static unsigned unmask_lds_pad_device()
{
    static thread_local int dev_cached = -1;
    static thread_local unsigned pad = 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (dev != dev_cached) {
        static const int want = [] {
            const char* e = getenv("KMWS_UNMASK_BLOCKS_PER_CU");
            return e ? atoi(e) : (int)kUnmaskBlocksPerCU;
        }();
        int lds = 0;
        pad = 0;
        if (want > 0 && hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) ==
                            hipSuccess && lds > 0) {
            const unsigned per_block = (unsigned)lds / (unsigned)(want + 1) + 1;  // want + 1 blocks do not fit
            pad = per_block > kUnmaskStaticLds ? per_block - kUnmaskStaticLds : 0u;
        }
        dev_cached = dev;
    }
    return pad;
}

static uint32_t ilog2_u64(uint64_t x)
{
    uint32_t r = 0;
    while ((1ull << r) < x) ++r;
    return r;
}

template <int V>
static kmws_status check_ws(uint64_t span, size_t ws_bytes, uint64_t* ntiles_out)
{
    using Cfg = UnmaskCfg<V>;
    const uint64_t ntiles = (span + Cfg::kTile - 1) / Cfg::kTile;
    if (ntiles > 0x7FFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    if (ws_bytes < sizeof(WsHead) + (ntiles + 1) * sizeof(uint32_t)) return KMWS_ERR_BUFFER_TOO_SMALL;
    *ntiles_out = ntiles;
    return KMWS_OK;
}

template <int V>
static kmws_status launch_plan(uint64_t span, const kmws_desc* descs, uint32_t n, void* workspace,
                               size_t ws_bytes, hipStream_t s)
{
    uint64_t ntiles = 0;
    kmws_status st = check_ws<V>(span, ws_bytes, &ntiles);
    if (st != KMWS_OK) return st;
    WsHead* head = static_cast<WsHead*>(workspace);
    if (launch_zero(head, sizeof(WsHead), s) != KMWS_OK) return KMWS_ERR_FAILED;
    if (n == 0 || span == 0) return KMWS_OK;
    hipLaunchKernelGGL(tile_map_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, descs, n, span,
                       ilog2_u64(UnmaskCfg<V>::kTile), reinterpret_cast<uint32_t*>(head + 1), head);
    return hip_status(hipGetLastError());
}

template <int V, int W = 1>
static kmws_status launch_apply(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                const void* workspace, size_t ws_bytes, hipStream_t s)
{
    uint64_t ntiles = 0;
    kmws_status st = check_ws<V>(span, ws_bytes, &ntiles);
    if (st != KMWS_OK) return st;
    if (n == 0 || span == 0) return KMWS_OK;
    const WsHead* head = static_cast<const WsHead*>(workspace);
    // A launch may hold at most 2^32 work-items: split huge spans into pieces.
    constexpr uint64_t kMaxBlocks = (1ull << 32) / kBlock / 2;
    for (uint64_t t0 = 0; t0 < ntiles; t0 += kMaxBlocks) {
        const uint64_t nb = ntiles - t0 < kMaxBlocks ? ntiles - t0 : kMaxBlocks;
        const unsigned pad = unmask_lds_pad(span, n);
        if (pad)
            hipLaunchKernelGGL((unmask_tiles_kernel<V, W, true>), dim3((uint32_t)nb), dim3(kBlock), pad, s, base, span,
                               descs, n, reinterpret_cast<const uint32_t*>(head + 1), head, (uint32_t)t0);
        else
            hipLaunchKernelGGL((unmask_tiles_kernel<V, W>), dim3((uint32_t)nb), dim3(kBlock), 0, s, base, span, descs,
                               n, reinterpret_cast<const uint32_t*>(head + 1), head, (uint32_t)t0);
    }
    return hip_status(hipGetLastError());
}

template <int V>
static kmws_status launch_apply_persist(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                        const void* workspace, size_t ws_bytes, hipStream_t s, uint32_t grid)
{
    using Cfg = UnmaskCfg<V>;
    uint64_t ntiles = 0;
    kmws_status st = check_ws<V>(span, ws_bytes, &ntiles);
    if (st != KMWS_OK) return st;
    if (n == 0 || span == 0) return KMWS_OK;
    const WsHead* head = static_cast<const WsHead*>(workspace);
    const uint32_t* map = reinterpret_cast<const uint32_t*>(head + 1);
    const uint64_t nfull = span / Cfg::kTile;
    if (nfull > 0xFFFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    if (nfull) {
        const uint32_t g = (uint32_t)(nfull < grid ? nfull : grid);
        hipLaunchKernelGGL(unmask_persist_kernel<V>, dim3(g), dim3(kBlock), 0, s, base, descs, n, map, head,
                           (uint32_t)nfull);
    }
    if (ntiles > nfull)  // the partial last tile
        hipLaunchKernelGGL(unmask_tiles_kernel<V>, dim3(1), dim3(kBlock), 0, s, base, span, descs, n, map, head,
                           (uint32_t)nfull);
    return hip_status(hipGetLastError());
}

template <int V>
static kmws_status launch_apply_pipe(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                     const void* workspace, size_t ws_bytes, hipStream_t s, uint32_t grid)
{
    using Cfg = UnmaskCfg<V>;
    uint64_t ntiles = 0;
    kmws_status st = check_ws<V>(span, ws_bytes, &ntiles);
    if (st != KMWS_OK) return st;
    if (n == 0 || span == 0) return KMWS_OK;
    const WsHead* head = static_cast<const WsHead*>(workspace);
    const uint32_t* map = reinterpret_cast<const uint32_t*>(head + 1);
    const uint64_t nfull = span / Cfg::kTile;
    if (nfull > 0xFFFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    if (nfull) {
        const uint32_t g = (uint32_t)(nfull < grid ? nfull : grid);
        hipLaunchKernelGGL(unmask_pipe_kernel<V>, dim3(g), dim3(kBlock), 0, s, base, descs, n, map, head,
                           (uint32_t)nfull);
    }
    if (ntiles > nfull)  // the partial last tile
        hipLaunchKernelGGL(unmask_tiles_kernel<V>, dim3(1), dim3(kBlock), 0, s, base, span, descs, n, map, head,
                           (uint32_t)nfull);
    return hip_status(hipGetLastError());
}

// Resident blocks of a kernel on the current device (CUs x blocks per CU).
static uint32_t resident_blocks(const void* kernel)
{
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess) return 0;
    return (uint32_t)(cus * per);
}

template <int V, bool NT = true>
static kmws_status launch_apply_split(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                      const void* workspace, size_t ws_bytes, hipStream_t s, uint32_t k,
                                      uint32_t c = 0, uint32_t w = 1)
{
    using Cfg = UnmaskCfg<V>;
    uint64_t ntiles = 0;
    kmws_status st = check_ws<V>(span, ws_bytes, &ntiles);
    if (st != KMWS_OK) return st;
    if (n == 0 || span == 0) return KMWS_OK;
    const WsHead* head = static_cast<const WsHead*>(workspace);
    const uint32_t* map = reinterpret_cast<const uint32_t*>(head + 1);
    const uint64_t nfull = span / Cfg::kTile;
    if (nfull > 0x7FFFFFFFull) return KMWS_ERR_INVALID_PARAM;
    // a launch may hold at most 2^32 work-items: huge spans go in pieces of blocks
    constexpr uint64_t kMaxBlocks = (1ull << 32) / kBlock / 2;
    const unsigned lds_pad = unmask_lds_pad(span, n);
    for (uint64_t b0 = 0; b0 < nfull; b0 += kMaxBlocks) {
        const uint64_t nb = nfull - b0 < kMaxBlocks ? nfull - b0 : kMaxBlocks;
        if (lds_pad)
            hipLaunchKernelGGL((unmask_split_kernel<V, true, NT>), dim3((uint32_t)nb), dim3(kBlock), lds_pad, s, base,
                               descs, n, map, head, (uint32_t)nfull, k, c, (uint32_t)b0, w);
        else
            hipLaunchKernelGGL((unmask_split_kernel<V, false, NT>), dim3((uint32_t)nb), dim3(kBlock), 0, s, base, descs,
                               n, map, head, (uint32_t)nfull, k, c, (uint32_t)b0, w);
    }
    if (ntiles > nfull)  // the partial last tile
        hipLaunchKernelGGL(unmask_tiles_kernel<V>, dim3(1), dim3(kBlock), 0, s, base, span, descs, n, map, head,
                           (uint32_t)nfull);
    return hip_status(hipGetLastError());
}

template <int V>
static kmws_status launch_unmask(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                 void* workspace, size_t ws_bytes, hipStream_t s)
{
    kmws_status st = launch_plan<V>(span, descs, n, workspace, ws_bytes, s);
    if (st != KMWS_OK) return st;
    return launch_apply<V>(base, span, descs, n, workspace, ws_bytes, s);
}

// Flag on schedule codes 0, 2, 3, 4, 5: payload stores temporal instead of
// non-temporal (store_word).
constexpr uint32_t kSchedTemporal = 1u << 30;

// Schedule code, one block per 16 KiB tile: the XCDs in 2 groups of 4, each
// group dealing runs of 16 tiles to its XCDs inside its own half of the span
// (0, the default), in order (1), tiles dealt over 2 parts of the span (2) or
// over 8 parts (3), runs of 16 tiles per XCD in one window (4); codes >= 64: a
// persistent grid of that many blocks, grid-stride (even) or software-pipelined
// (odd, grid = code - 1).
static kmws_status launch_schedule(uint32_t code, uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                   const void* workspace, size_t ws_bytes, hipStream_t s)
{
    if (code & kSchedTemporal) {  // the same split schedules with temporal payload stores
        switch (code & ~kSchedTemporal) {
        case 0: return launch_apply_split<kUnmaskV, false>(base, span, descs, n, workspace, ws_bytes, s, 8u, 16u, 2u);
        case 2: return launch_apply_split<kUnmaskV, false>(base, span, descs, n, workspace, ws_bytes, s, 2u);
        case 3: return launch_apply_split<kUnmaskV, false>(base, span, descs, n, workspace, ws_bytes, s, 8u);
        case 4: return launch_apply_split<kUnmaskV, false>(base, span, descs, n, workspace, ws_bytes, s, 8u, 16u);
        case 5: return launch_apply_split<kUnmaskV, false>(base, span, descs, n, workspace, ws_bytes, s, 4u);
        default: return KMWS_ERR_INVALID_PARAM;
        }
    }
    if (code == 0) return launch_apply_split<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, 8u, 16u, 2u);
    if (code == 4) return launch_apply_split<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, 8u, 16u);
    if (code == 1) return launch_apply<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s);
    if (code == 2) return launch_apply_split<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, 2u);
    if (code == 3) return launch_apply_split<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, 8u);
    if (code == 5) return launch_apply_split<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, 4u);
    if (code < 64) return KMWS_ERR_INVALID_PARAM;
    if (code & 1u) return launch_apply_pipe<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, code & ~1u);
    return launch_apply_persist<kUnmaskV>(base, span, descs, n, workspace, ws_bytes, s, code);
}

static uint32_t current_schedule()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 0;
    return __atomic_load_n(&g_schedule[dev], __ATOMIC_RELAXED);
}

static bool bad_args(const uint8_t* base, const kmws_desc* descs, uint32_t n, const void* ws)
{
    return !ws || (n && (!base || !descs)) || (reinterpret_cast<uintptr_t>(base) & 15u);
}

__global__ void __launch_bounds__(64) zero_kernel(uint64_t* __restrict__ p, uint32_t words)
{
    for (uint32_t i = threadIdx.x; i < words; i += 64) p[i] = 0;
}

kmws_status launch_zero(void* p, uint32_t bytes, hipStream_t s)
{
    if (!p || (bytes & 7u) || bytes > 4096) return KMWS_ERR_INVALID_PARAM;
    hipLaunchKernelGGL(zero_kernel, dim3(1), dim3(64), 0, s, static_cast<uint64_t*>(p), bytes / 8);
    return hip_status(hipGetLastError());
}

kmws_status launch_unmask_pieces(uint8_t* base, const kmws_desc* descs, const PieceRec* pieces, uint32_t np,
                                 hipStream_t s)
{
    if (np == 0) return KMWS_OK;
    if (!base || !descs || !pieces) return KMWS_ERR_INVALID_PARAM;
    hipLaunchKernelGGL(unmask_pieces_kernel, dim3(np), dim3(kBlock), 0, s, base, descs, pieces);
    return hip_status(hipGetLastError());
}
}  // namespace kmws

using namespace kmws;

extern "C" {

size_t kmws_unmask_workspace_size(uint64_t span)
{
    // sized for the smallest tile any variant uses (8 KiB: variants 40, 41)
    const uint64_t ntiles = (span + UnmaskCfg<2>::kTile - 1) / UnmaskCfg<2>::kTile;
    return sizeof(WsHead) + (size_t)(ntiles + 1) * sizeof(uint32_t);  // + the map's sentinel
}

kmws_status kmws_unmask_batch(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                              void* workspace, size_t workspace_bytes, void* stream)
{
    if (bad_args(base, descs, n, workspace)) return KMWS_ERR_INVALID_PARAM;
    kmws_status st = launch_plan<kUnmaskV>(span, descs, n, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
    if (st != KMWS_OK) return st;
    return kmws_unmask_apply(base, span, descs, n, workspace, workspace_bytes, stream);
}

kmws_status kmws_unmask_plan(uint64_t span, const kmws_desc* descs, uint32_t n, void* workspace,
                             size_t workspace_bytes, void* stream)
{
    if (!workspace || (n && !descs)) return KMWS_ERR_INVALID_PARAM;
    return launch_plan<kUnmaskV>(span, descs, n, workspace, workspace_bytes, static_cast<hipStream_t>(stream));
}

kmws_status kmws_unmask_apply(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                              const void* workspace, size_t workspace_bytes, void* stream)
{
    if (bad_args(base, descs, n, workspace)) return KMWS_ERR_INVALID_PARAM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    return launch_schedule(current_schedule(), base, span, descs, n, workspace, workspace_bytes, s);
}

int kmws_unmask_schedule(void) { return (int)current_schedule(); }

int kmws_unmask_resident_blocks(void)
{
    return (int)resident_blocks(reinterpret_cast<const void*>(kmws::unmask_pipe_kernel<kUnmaskV>));
}

// Times each schedule on the caller's batch, twice per schedule (XOR applied
// twice is the identity, so the payload is unchanged on return), and keeps the
// fastest as this device's kmws_unmask_apply schedule.  Synchronizes.
int kmws_unmask_autotune(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n, void* workspace,
                         size_t workspace_bytes, void* stream)
{
    if (bad_args(base, descs, n, workspace)) return KMWS_ERR_INVALID_PARAM;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return KMWS_ERR_FAILED;
    hipStream_t s = static_cast<hipStream_t>(stream);
    kmws_status st = launch_plan<kUnmaskV>(span, descs, n, workspace, workspace_bytes, s);
    if (st != KMWS_OK) return st;
    // grouped XCD runs, 4 parts, 8 parts, XCD runs, 2 parts, in order: which wins
    // depends on where the batch lies in HBM, on its frame layout and on the
    // blocks in flight (profiles/r01f_unmask_placement.txt; at 2 blocks per CU
    // 4 parts led with 85.3 %, profiles/r02al_unmask_schedules_2bpc.txt)
    // (+ the split schedules with temporal stores: faster on aligned arenas,
    // slower on packed wire images, profiles/r02bz_unmask_store_policy_ab.txt;
    // with them split 2 leads on the aligned arena, r02cj_unmask_ts_candidates_ab.txt)
    static const uint32_t cand[] = {0u, 5u, 3u, 4u, 2u, 1u, 5u | kSchedTemporal, 3u | kSchedTemporal,
                                    2u | kSchedTemporal, 0u | kSchedTemporal, 4u | kSchedTemporal};
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess) return KMWS_ERR_FAILED;
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return KMWS_ERR_FAILED;
    }
    float best = 1e30f;
    uint32_t pick = 0;
    for (int rep = 0; rep < 2; ++rep) {
        for (uint32_t g : cand) {
            if (hipEventRecord(e0, s) != hipSuccess) { st = KMWS_ERR_FAILED; break; }
            for (int k = 0; k < 2 && st == KMWS_OK; ++k)
                st = launch_schedule(g, base, span, descs, n, workspace, workspace_bytes, s);
            if (st != KMWS_OK || hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) {
                st = st != KMWS_OK ? st : KMWS_ERR_FAILED;
                break;
            }
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep == 1 && ms < best) {  // rep 0 warms every schedule up
                best = ms;
                pick = g;
            }
        }
        if (st != KMWS_OK) break;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (st != KMWS_OK) return st;
    __atomic_store_n(&g_schedule[dev], pick, __ATOMIC_RELAXED);
    return (int)pick;
}

// Tuning entry: same contract as kmws_unmask_batch with an explicit tile
// variant (0: 16 KiB, 1: 32 KiB, 2: 64 KiB).  Used by bench/tune scripts.
kmws_status kmws_unmask_batch_variant(uint8_t* base, uint64_t span, const kmws_desc* descs, uint32_t n,
                                      void* workspace, size_t workspace_bytes, void* stream, int variant)
{
    if (bad_args(base, descs, n, workspace)) return KMWS_ERR_INVALID_PARAM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (variant) {
    case 0: return launch_unmask<4>(base, span, descs, n, workspace, workspace_bytes, s);
    case 1: return launch_unmask<8>(base, span, descs, n, workspace, workspace_bytes, s);
    case 2: return launch_unmask<16>(base, span, descs, n, workspace, workspace_bytes, s);
    case 3:
    case 4:
    case 5:
    case 6:
    case 7: {  // 16 KiB tiles, persistent grid-stride with next-tile prefetch: 4096 .. 16384 blocks
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        static const uint32_t grids[] = {8192u, 16384u, 24576u, 32768u, 65536u};
        const uint32_t grid = grids[variant - 3];
        return launch_apply_persist<4>(base, span, descs, n, workspace, workspace_bytes, s, grid);
    }
    case 8:
    case 9: {  // 16 KiB tiles, registers capped for 6 (8) or 8 (9) waves per SIMD
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        return variant == 8 ? launch_apply<4, 6>(base, span, descs, n, workspace, workspace_bytes, s)
                            : launch_apply<4, 8>(base, span, descs, n, workspace, workspace_bytes, s);
    }
    case 10:
    case 11:
    case 12: {  // 16 KiB tiles, pipelined persistent grid: 16384 / 32768 / 65536 blocks
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        static const uint32_t grids[] = {16384u, 32768u, 65536u};
        return launch_apply_pipe<4>(base, span, descs, n, workspace, workspace_bytes, s, grids[variant - 10]);
    }
    case 21:
    case 22:
    case 23:
    case 24: {  // 16 KiB tiles, one block per tile, blocks dealt over 2 / 4 / 8 / 16 parts of the span
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        return launch_apply_split<4>(base, span, descs, n, workspace, workspace_bytes, s, 2u << (variant - 21));
    }
    case 25:
    case 26:
    case 27:
    case 28:
    case 29: {  // 16 KiB tiles, one block per tile, runs of 4 / 8 / 16 / 32 / 128 tiles per XCD residue
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        static const uint32_t runs[] = {4u, 8u, 16u, 32u, 128u};
        return launch_apply_split<4>(base, span, descs, n, workspace, workspace_bytes, s, 8u, runs[variant - 25]);
    }
    case 30:
    case 31:
    case 32:
    case 33: {  // 16 KiB tiles, one block per tile, blocks dealt over 3 / 6 / 12 / 32 parts of the span
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        static const uint32_t ks[] = {3u, 6u, 12u, 32u};
        return launch_apply_split<4>(base, span, descs, n, workspace, workspace_bytes, s, ks[variant - 30]);
    }
    case 34:
    case 35: {  // 32 KiB tiles, one block per tile, blocks dealt over 2 / 8 parts of the span
        kmws_status st = launch_plan<8>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        return launch_apply_split<8>(base, span, descs, n, workspace, workspace_bytes, s, variant == 34 ? 2u : 8u);
    }
    case 36:
    case 37:
    case 38: {  // XCD runs of 16 tiles, the 8 residues in 2 / 4 / 8 groups, each group in its own window
        kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        return launch_apply_split<4>(base, span, descs, n, workspace, workspace_bytes, s, 8u, 16u,
                                     2u << (variant - 36));
    }
    case 40:
    case 41: {  // 8 KiB tiles, one block per tile: split 8 / XCD runs of 32 tiles
        kmws_status st = launch_plan<2>(span, descs, n, workspace, workspace_bytes, s);
        if (st != KMWS_OK) return st;
        return variant == 40 ? launch_apply_split<2>(base, span, descs, n, workspace, workspace_bytes, s, 8u)
                             : launch_apply_split<2>(base, span, descs, n, workspace, workspace_bytes, s, 8u, 32u);
    }
    default:
        if (variant >= 64) {  // a raw schedule code (kmws_unmask_schedule's encoding)
            kmws_status st = launch_plan<4>(span, descs, n, workspace, workspace_bytes, s);
            if (st != KMWS_OK) return st;
            return launch_schedule((uint32_t)variant, base, span, descs, n, workspace, workspace_bytes, s);
        }
        return KMWS_ERR_INVALID_PARAM;
    }
}

kmws_status kmws_read_status(const void* workspace, uint32_t* status_out, void* stream)
{
    if (!workspace || !status_out) return KMWS_ERR_INVALID_PARAM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemcpyAsync(status_out, workspace, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return hip_status(e);
}

void* kmws_arena_alloc(uint64_t bytes, int device, int* contiguous)
{
    if (contiguous) *contiguous = 0;
    if (bytes == 0) return nullptr;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return nullptr;
    if (device != prev && hipSetDevice(device) != hipSuccess) return nullptr;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) == hipSuccess && p) {
        if (contiguous) *contiguous = 1;
    } else {
        (void)hipGetLastError();
        p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
        }
    }
    if (device != prev) (void)hipSetDevice(prev);
    return p;
}

void kmws_arena_free(void* p, int device)
{
    if (!p) return;
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return;
    if (device != prev) (void)hipSetDevice(device);
    (void)hipFree(p);
    if (device != prev) (void)hipSetDevice(prev);
}

int64_t kmws_arena_place(uint8_t* arena, uint64_t arena_bytes, uint64_t span, uint64_t step, void* stream,
                         float* frac_out, uint32_t max_out)
{
    // Offsets 0, step, 2 step, ... with offset + span <= arena_bytes.  The probe
    // batch: uniform 64 KiB frames over the span (contents are whatever the arena
    // holds; XOR applied twice leaves them unchanged); an offset scores the better
    // of the split-4 and split-8 schedules (codes 5, 3: which one leads depends
    // on the placement, and kmws_unmask_autotune then picks among all).
    constexpr uint64_t kFrame = 65536;
    if (!arena || span == 0 || span > arena_bytes || step == 0 || (step & 15u) ||
        (reinterpret_cast<uintptr_t>(arena) & 15u) || span / kFrame > 0xFFFFFFFFull)
        return KMWS_ERR_INVALID_PARAM;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint32_t n = (uint32_t)((span + kFrame - 1) / kFrame);
    const size_t ws_bytes = kmws_unmask_workspace_size(span);
    kmws_desc* d = nullptr;
    void* ws = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int64_t result = KMWS_ERR_FAILED;
    if (hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * sizeof(kmws_desc)) != hipSuccess ||
        hipMalloc(&ws, ws_bytes) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess) {
        (void)hipGetLastError();
    } else {
        hipLaunchKernelGGL(uniform_descs_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, d, n, kFrame,
                           (uint32_t)kFrame, 0x706c6163ull);
        // the last frame ends at the span (uniform_descs gives every frame kFrame bytes)
        const uint32_t last_len = (uint32_t)(span - (uint64_t)(n - 1) * kFrame);
        kmws_status st = hip_status(hipMemcpyAsync(&d[n - 1].len, &last_len, sizeof(last_len),
                                                   hipMemcpyHostToDevice, s));
        if (st == KMWS_OK) st = hip_status(hipStreamSynchronize(s));
        float best = 1e30f;
        uint64_t pick = 0;
        uint32_t k = 0;
        for (uint64_t off = 0; st == KMWS_OK && off + span <= arena_bytes; off += step, ++k) {
            float t = 1e30f;
            for (int rep = 0; rep < 4 && st == KMWS_OK; ++rep) {  // min of two pairs per schedule
                st = launch_plan<kUnmaskV>(span, d, n, ws, ws_bytes, s);
                if (st == KMWS_OK) st = hip_status(hipEventRecord(e0, s));
                for (int i = 0; i < 2 && st == KMWS_OK; ++i)
                    st = launch_schedule(rep & 1 ? 3u : 5u, arena + off, span, d, n, ws, ws_bytes, s);
                if (st == KMWS_OK) st = hip_status(hipEventRecord(e1, s));
                if (st == KMWS_OK) st = hip_status(hipEventSynchronize(e1));
                float ms = 0;
                if (st == KMWS_OK && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms < t) t = ms;
            }
            if (st != KMWS_OK) break;
            // fraction of the 8 TB/s HBM peak: 2 passes x (2 span + 16 n) bytes
            if (frac_out && k < max_out) frac_out[k] = (float)(2.0 * (2.0 * span + 16.0 * n) / (t * 1e-3) / 8e12);
            if (t < best) {
                best = t;
                pick = off;
            }
        }
        uint32_t status = 0;
        if (st == KMWS_OK) st = hip_status(hipMemcpy(&status, ws, sizeof(status), hipMemcpyDeviceToHost));
        result = st != KMWS_OK ? (int64_t)st : (status != 0 ? (int64_t)KMWS_ERR_FAILED : (int64_t)pick);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (ws) (void)hipFree(ws);
    if (d) (void)hipFree(d);
    return result;
}

kmws_status kmws_fill_synthetic(uint8_t* base, uint64_t bytes, uint64_t seed, void* stream)
{
    if (!base && bytes) return KMWS_ERR_INVALID_PARAM;
    if ((reinterpret_cast<uintptr_t>(base) & 15u)) return KMWS_ERR_INVALID_PARAM;
    if (bytes == 0) return KMWS_OK;
    hipLaunchKernelGGL(fill_synthetic_kernel, dim3(8192), dim3(kBlock), 0, static_cast<hipStream_t>(stream), base,
                       bytes, seed);
    return hip_status(hipGetLastError());
}

kmws_status kmws_fill_uniform_descs(kmws_desc* descs, uint32_t n, uint64_t stride, uint32_t len,
                                    uint64_t key_seed, void* stream)
{
    if (!descs && n) return KMWS_ERR_INVALID_PARAM;
    if (n == 0) return KMWS_OK;
    hipLaunchKernelGGL(uniform_descs_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), descs, n, stride, len, key_seed);
    return hip_status(hipGetLastError());
}

kmws_status kmws_check_unmasked(const uint8_t* base, uint64_t bytes, uint64_t seed, const kmws_desc* descs,
                                uint32_t n, unsigned long long* mismatches, void* stream)
{
    if ((!base && bytes) || !mismatches) return KMWS_ERR_INVALID_PARAM;
    if (bytes == 0) return KMWS_OK;
    uint64_t nb = (bytes + kCheckBytes - 1) / kCheckBytes;
    if (nb > 65536) nb = 65536;  // grid-stride beyond this
    hipLaunchKernelGGL(check_unmasked_kernel, dim3((uint32_t)nb), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       base, bytes, seed, descs, n, mismatches);
    return hip_status(hipGetLastError());
}

int kmws_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) ++good;
    }
    return good;
}

}  // extern "C"
