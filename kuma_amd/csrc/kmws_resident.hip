// Resident unmask worker: the synchronous host entries without a kernel launch
// per call, concurrent across the process's event-loop threads.
//
// kuma calls WSHandler::handleData once per <= 64 KiB socket read
// (TcpConnection.cpp:229-233 -> WebSocketImpl.cpp:225-246) and
// WSHandler::handleDataMask once per send (WebSocketImpl.cpp:388, :414), and
// expects the payload unmasked when the call returns -- on every loop thread
// (10 in kuma's test client, test/client/main.cpp:20; 5 in its server,
// test/server/main.cpp:22).  A stream launch plus an event wait costs 13-15 us
// per call, about what kuma's byte loop (WSHandler.cpp:303-310) spends on a
// whole 64 KiB read.  Here ONE grid of kResSlots workgroups (1024 lanes each)
// stays resident per device, on one greatest-priority stream: workgroup b
// serves mailbox slot b, and a host thread claims a slot once (lock-free) and
// keeps it until it exits.  Each slot is polled from pinned host memory by its
// own workgroup: the thread writes a job (up to kResMaxDescs payloads, each a
// device-visible address, a length and a key) and bumps the slot's job
// number; the workgroup sees it over PCIe, unmasks every payload in place
// there (zero-copy, 4 x 16-byte words per lane in flight: 64 KiB per round),
// makes its stores visible system-wide and writes the job number back; the
// thread spins on that word.  No launch, no completion signal, no interrupt,
// no lock: threads on different slots run their jobs at the same time.  A
// thread that finds no free slot launches on its own stream instead; it never
// waits for another thread.  (One grid, not a worker per thread: two workers'
// greatest-priority streams shared a hardware queue, so one thread's job
// waited for the other's worker to leave -- round 4, r04x.)
//
// The grid exits by itself after kResIdleUs (200 us) without a job in any
// slot, after a lease of kResLeaseUs (1 ms) however busy it is, and a
// workgroup leaves on its slot's quit bit (process exit; a job past its
// timeout): every wave reaches the exit, the grid drains, and a host thread
// that stops feeding never leaves a kernel behind.  The next job relaunches
// it.  The stream is non-blocking and of the greatest priority, so work on
// other streams -- the legacy default stream included -- does not queue behind
// it, and the lease bounds the wait of any kernel that still shares its
// hardware queue (tests/test_gpu_decoder.py).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "kmws_bench.h"
#include "kmws_host_util.hpp"

namespace kmws {

constexpr int kResBlock = 1024;  // 16 waves: 4 words each = 64 KiB of loads in flight
constexpr int kResWords = 4;
// Jobs of up to this many 16-byte words store write-through (sc0 sc1) and end
// without a release; larger ones store into the L2 and end with one
// system-scope release (a buffer_wbl2 of the XCD's L2) -- unless a device
// batch of this library is running on the device (kmws::note_device_batch):
// then every job writes through.  A release per job at a million small jobs a
// second slowed a device batch beside the grid (tools/grid_interference.cpp),
// and with 64 KiB jobs 1.36x against 1.11x written through (r06az); write-
// through stores of 64 KiB generations halved 8 loopback connections' decode
// (18.6 -> 8.6-10.9 GiB/s, r06an-ap).  The thread decides (kWriteThroughBit).
constexpr int kResWriteThroughWords = 1024;
// Slots per device: one per loop thread that uses the synchronous entries
// (kuma's test client runs 10 loop threads, its server 5).  Unclaimed slots'
// workgroups poll one word every few microseconds; a claimed slot's workgroup
// polls its job word and 31 descriptor slots (512 B) back to back.
constexpr int kResSlots = 16;
// Workgroups per slot: one CU moves ~13 GB/s of a job's PCIe traffic (the misses
// it keeps in flight to host memory bound it, not its lanes), so a job of at
// least 2 x kPartWords words is split over up to kResParts workgroups, each
// polling the slot's job word itself.
constexpr int kResParts = 4;
constexpr uint32_t kPartWords = 1024;  // 16 KiB: the least a part takes
// Idle exit: short.  The runtime maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4 on the box), so a kernel launched on a stream that
// shares the worker's queue waits until the worker leaves; and
// hipDeviceSynchronize (torch.cuda.synchronize) waits for every stream, the
// worker's included (measured: a device synchronize behind a 50 ms-idle worker
// took 50 ms; the loopback "gpu" mode, whose batches keep several streams, fell
// from 2.0 to 0.57 GiB/s with a 5 ms idle).  A loop thread under load feeds far
// more often than this; a worker that idled out costs one launch at the next
// job, the price of every call without it.
constexpr uint32_t kResIdleUs = 200;
// Lease: an incarnation also leaves after kResLeaseUs of life however busy it
// is, before it takes the next job (the host relaunches it for that job).  A
// thread that feeds back to back would otherwise keep the worker resident for
// good, and a kernel on another stream that shares its hardware queue would
// wait for as long (measured: up to 6.9 s behind a feeder thread).  The
// relaunch it costs (~10-15 us) is spread over the ~100 jobs of one lease.
constexpr uint32_t kResLeaseUs = 1000;
// A job not done after kResTimeoutMs is withdrawn: the slot's quit bit asks
// its workgroup to leave, and the thread waits up to kResDrainMs more for it.
// Only when the workgroup has left (or finished the job) does the call return
// without KMWS_ERR_TIMEOUT -- nothing writes the payloads after that.  The
// test build shortens both (kuma_amd/build.py).
#ifndef KMWS_RESIDENT_TIMEOUT_MS
#define KMWS_RESIDENT_TIMEOUT_MS 2000
#endif
#ifndef KMWS_RESIDENT_DRAIN_MS
#define KMWS_RESIDENT_DRAIN_MS 2000
#endif
// A job whose workgroup left while the rest of the grid still runs (it is
// closing, or another workgroup is stuck in a job) is withdrawn after this long
// and launched by the caller.
constexpr uint32_t kResOrphanUs = 200;

static inline void cpu_relax()
{
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
    __builtin_ia32_pause();
#endif
}

struct ResDesc {  // one payload: device-visible address, bytes, LE key of its first byte
    uint64_t addr;
    uint32_t len;
    uint32_t key;
};
static_assert(sizeof(ResDesc) == 16, "ResDesc is one 16-byte load");

// The polled word of a slot: job number (bits 0-39), payload count (40-47),
// parts - 1 (48-49: the workgroups the job is split over), cancelled (61: a
// job its thread withdrew -- no workgroup runs it), claimed (62: a thread holds
// the slot, so its part-0 workgroup polls the descriptors too) and quit (63).
// The first kPollDescs descriptor slots follow it and are read with it at
// every poll of part 0, so a job of up to kPollDescs payloads costs one PCIe
// round trip to notice and none more to read its descriptors.  The host
// rewrites every one of those slots for every job (unused ones with length 0),
// each as two 8-byte stores tagged with the job's low bits (address bits
// 48-63; length bits 21-31 in the half that also holds the key): a half read
// before the host's write landed carries the previous job's tag, and the job's
// descriptors are then read again after the word.
constexpr uint64_t kJobMask = (1ull << 40) - 1;
constexpr int kPartShift = 48;
constexpr uint64_t kWriteThroughBit = 1ull << 50;  // the job's stores write through (no release)
constexpr uint64_t kCancelBit = 1ull << 61;
constexpr uint64_t kClaimedBit = 1ull << 62;
constexpr uint64_t kQuitBit = 1ull << 63;
// word + 31 slots: a slot's first 512 bytes, one 16-byte load per lane of
// wave 0 -- a cfg1 read (16 frames of 4 KiB, and a partial one) fits
constexpr int kPollDescs = 31;
static_assert(kPollDescs < 64, "one lane of wave 0 per polled slot");
constexpr uint64_t kAddrMask = (1ull << 48) - 1;
constexpr uint32_t kLenMask = (1u << 21) - 1;  // kResMaxBytes fits
static_assert(kResMaxBytes <= kLenMask && kResMaxBytesAsync <= kLenMask, "tagged length");
__host__ __device__ __forceinline__ ResDesc tag_desc(ResDesc x, uint64_t job)
{
    x.addr |= (job & 0xFFFFull) << 48;
    x.len |= (uint32_t)(job & 0x7FFu) << 21;
    return x;
}
__host__ __device__ __forceinline__ bool desc_tagged(const ResDesc& x, uint64_t job)
{
    return (x.addr >> 48) == (job & 0xFFFFull) && (x.len >> 21) == (uint32_t)(job & 0x7FFu);
}
__host__ __device__ __forceinline__ ResDesc untag_desc(ResDesc x)
{
    x.addr &= kAddrMask;
    x.len &= kLenMask;
    return x;
}
// Words of a payload's 16-byte aligned hull.
__host__ __device__ __forceinline__ uint32_t hull_words(uint64_t addr, uint32_t len)
{
    return len ? (uint32_t)(((addr + len + 15) >> 4) - (addr >> 4)) : 0u;
}

// Pinned host memory.  Host-written and device-written words sit in different
// 128-byte lines.
struct alignas(256) ResSlot {
    uint64_t word;  // job | ndesc << 40 | (parts - 1) << 48 | cancel << 61 | claimed << 62 | quit << 63
    uint64_t pad1;
    ResDesc desc[kResMaxDescs];  // desc[i] at 16 + 16 i
    alignas(128) uint64_t done[kResParts];  // per part: last job number finished (release: its bytes visible)
    uint64_t gone[kResParts];               // per part: incarnation whose workgroup has left
    alignas(128) uint64_t pad2;
};
struct ResMailbox {
    ResSlot slot[kResSlots];
    alignas(128) uint64_t exited;  // incarnation whose last workgroup has left (device)
    alignas(128) uint64_t resize;  // (host) incarnations up to this one leave: a slot was claimed outside them
    alignas(128) uint64_t pad3;
};
// Why a workgroup left: its lease ran out, another workgroup found the grid
// idle (closing), a thread asked for a resize, it found the grid idle itself,
// its slot's quit bit.
constexpr int kResExitReasons = 5;
// Device memory, shared by the grid's workgroups.  Counters and marks are
// compared with the incarnation number, so nothing is cleared between launches.
struct ResCtl {
    uint64_t closing;   // max incarnation that is leaving (idle or lease)
    uint64_t exits;     // workgroups exited, all incarnations (each adds the grid size)
    uint64_t idle;      // workgroups of the running incarnation idle 200 us (or gone on their quit bit)
    uint64_t pad;
    uint64_t why[kResExitReasons];  // workgroup exits by reason (kmws_resident_exit_reasons)
};

// Loads of host-written words bypass every cache (and are never scalar loads).
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Write-through (sc0 sc1: system scope) stores of a small job's payload
// bytes (kResWriteThroughWords).  Complete -- written through to host memory
// -- once the storing wave's vmcnt drains, so the done word needs no release:
// a system-scope release is a buffer_wbl2 of the whole XCD L2, which at a
// million small jobs a second stalled a device batch running beside the grid
// (tools/grid_interference.cpp).  A lane's four words go in ONE asm
// statement: the compiler waits for every access in flight before an inline
// asm, so four statements made each store wait for the one before.  Flat
// stores: a lane with nothing to store aims its words at its own 16 bytes of
// LDS (no memory traffic).  8-byte stores the compiler could count instead
// wrote half of every 16 bytes per instruction and ran 10x slower (r06ao).
__device__ __forceinline__ void st_sys16x4(uint64_t a0, u32x4 v0, uint64_t a1, u32x4 v1, uint64_t a2, u32x4 v2,
                                           uint64_t a3, u32x4 v3)
{
    asm volatile(
        "flat_store_dwordx4 %0, %1 sc0 sc1\n\t"
        "flat_store_dwordx4 %2, %3 sc0 sc1\n\t"
        "flat_store_dwordx4 %4, %5 sc0 sc1\n\t"
        "flat_store_dwordx4 %6, %7 sc0 sc1\n\t"
        "s_nop 1" ::"v"(a0),
        "v"(v0), "v"(a1), "v"(v1), "v"(a2), "v"(v2), "v"(a3), "v"(v3)
        : "memory");
}
// A small job's hull edge bytes, written through: stores the compiler counts
// (no wait between them).
__device__ __forceinline__ void st_sys1(uint64_t a, uint32_t v)
{
    __hip_atomic_store(reinterpret_cast<__attribute__((address_space(1))) uint8_t*>(a), (uint8_t)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}
// ResCtl lives in uncached device memory (ResidentWorker::init), so a plain
// load of a word other XCDs update is never served stale from this XCD's L2
// (a read-modify-write would be coherent too, but 64 workgroups doing one on
// the same word every fourth poll serialized at the atomic unit).
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// nslots x kResParts workgroups (slots 0 .. nslots - 1: those claimed when
// the incarnation was launched), persistent until idle: workgroup blockIdx.x
// serves part p = blockIdx.x / nslots of slot (blockIdx.x - p) mod nslots, i.e.
// part p of slot s sits at p * nslots + (s + p) mod nslots.  Workgroups are
// dealt to the 8 XCDs by blockIdx.x mod 8, so slot s's part 0 (all a small job
// uses) is on XCD s mod 8 and its four parts on four different XCDs: with
// blockIdx.x mod nslots as the slot, 8 or 16 slots put a slot's parts on one
// XCD, and slot-major numbering put every part 0 on XCDs 0 and 4 (16 threads'
// 4 KiB masks 2.2 -> 1.6 M calls/s, r05bk; the diagonal keeps 2.2 M and gives 8
// loopback connections' one-end runs 0-10 % more, r05bl).  A job's hull words are split evenly over its parts;
// each part polls the slot's job word itself -- no hand-off between
// workgroups -- runs its words and writes its own done word.  `inc` = this
// incarnation's number (from 1); `exit_base` = the workgroups of every
// earlier incarnation (the exit counter's value once they all left).
__global__ void __launch_bounds__(kResBlock) resident_unmask_kernel(ResMailbox* mb, ResCtl* ctl, uint64_t inc,
                                                                    uint32_t nslots, uint64_t exit_base,
                                                                    uint64_t idle_ticks, uint64_t lease_ticks)
{
    __shared__ ResDesc s_d[kResMaxDescs];
    __shared__ uint32_t s_pre[kResMaxDescs + 1];  // word prefix over the payload hulls
    __shared__ uint64_t s_cmd;
    __shared__ uint32_t s_have;  // descriptors taken from the poll
    __shared__ u32x4 s_sink[kResBlock];  // per lane: where a lane with no whole word stores its words
    const int t = threadIdx.x;
    const uint32_t part = blockIdx.x / nslots;
    ResSlot* sl = &mb->slot[(blockIdx.x % nslots + nslots - part % nslots) % nslots];
    const uint64_t born = wall_clock64();
    const uint64_t my_sink = reinterpret_cast<uint64_t>(static_cast<void*>(&s_sink[t]));  // a flat (LDS) address
    // lane l <= kPollDescs of wave 0 of part 0 polls bytes [16 l, 16 l + 16)
    // of the slot: the job word (lane 0) and descriptor slot l - 1; other
    // parts, and part 0 while the slot is unclaimed, load the word only (one
    // request)
    const uint64_t* pw0 = &sl->word;
    const uint64_t* pw = pw0 + 2 * (t <= kPollDescs ? t : 0);
    // Idle exit without comparing clocks across workgroups: a workgroup whose
    // slot has had no job for idle_ticks counts itself in ctl->idle (and out
    // again at the slot's next job, whichever part it is for); the one whose
    // count completes the grid closes it.  Before, each compared its clock with
    // a device-wide "last job" time other workgroups wrote, and under load read
    // it stale or skewed: 16 busy threads' grids closed as idle every ~0.3 ms
    // (r05as / r05at: 650-1,199 idle decisions in 25 ms; 1.26 M calls/s).
    uint64_t last = 0, t_act = born;  // (wave 0) job seen last; this slot's latest job
    bool idle = false;                // (wave 0) counted in ctl->idle
    bool full = part == 0;            // (wave 0) poll the descriptors too
    uint32_t why = 0;                 // (wave 0) the exit reason (ResCtl::why)
    if (t < 64) last = ld_sys(&sl->done[part]);
    for (;;) {
        if (t < 64) {  // wave 0, uniform control flow
            uint64_t cmd = 0, v0 = 0, v1 = 0;
            bool polled_full = false;
            for (uint32_t it = 0;; ++it) {
                const uint64_t now = wall_clock64();
                const uint64_t* a = full ? pw : pw0;
                v0 = ld_sys(a);
                v1 = ld_sys(a + 1);
                // with the word's loads in flight: is the grid leaving (idle;
                // every 4th poll) or asked to (a thread claimed a slot it does
                // not serve, and the relaunch will; every 16th poll -- every 4th,
                // 64 workgroups reading that one host word slowed 16 threads'
                // jobs to 1.4 M/s at an 11 us median, against 2.1 M/s at 6.5 us,
                // r05av)?  A posted job waits for the relaunch, as at the lease.
                uint64_t closing = 0, resize = 0;
                if ((it & 3u) == 0) closing = ld_agent(&ctl->closing);
                if ((it & 15u) == 0) resize = ld_sys(&mb->resize);
                if ((uint64_t)(now - born) > lease_ticks || closing >= inc || resize >= inc) {
                    why = closing >= inc ? 1u : resize >= inc ? 2u : 0u;
                    cmd = 0;
                    break;
                }
                polled_full = full;
                const uint64_t w = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v0) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v0 >> 32)) << 32;
                // (lane 0's job word; each half through uint32_t: readfirstlane is signed)
                if (w & kQuitBit) {  // this slot only: the rest of the grid serves on
                    why = 4;
                    break;
                }
                if ((w & kJobMask) != last) {  // a job on this slot: activity, whichever part it is for
                    t_act = now;
                    if (idle) {
                        if (t == 0) __hip_atomic_fetch_sub(&ctl->idle, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        idle = false;
                    }
                    const uint32_t parts = (uint32_t)(w >> kPartShift & 3u) + 1u;
                    if (part >= parts || (w & kCancelBit)) {
                        last = w & kJobMask;  // not this workgroup's (no done word: nobody waits for it)
                        continue;
                    }
                    cmd = w;
                    break;
                }
                const bool claimed = (w & kClaimedBit) != 0;
                full = part == 0 && claimed;
                if (!idle && (uint64_t)(now - t_act) > idle_ticks) {  // idle here: counted
                    uint64_t before = 0;
                    if (t == 0) before = __hip_atomic_fetch_add(&ctl->idle, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    before = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)before) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(before >> 32)) << 32;
                    idle = true;
                    if (before + 1 >= gridDim.x) {  // every workgroup idle: the grid leaves
                        if (t == 0) __hip_atomic_fetch_max(&ctl->closing, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        why = 3;
                        break;
                    }
                }
                if (claimed) __builtin_amdgcn_s_sleep(2);
                else __builtin_amdgcn_s_sleep(127);  // ~4 us: an unclaimed slot gets a job rarely
            }
            uint32_t have = 0;
            if (cmd) {
                const uint32_t nd = (uint32_t)(cmd >> 40) & 0xFFu;
                const ResDesc x = ResDesc{v0, (uint32_t)v1, (uint32_t)(v1 >> 32)};
                const bool mine = polled_full && t >= 1 && t <= (int)nd && t <= kPollDescs;
                const bool ok = desc_tagged(x, cmd & kJobMask);
                if (mine && ok) s_d[t - 1] = untag_desc(x);
                // every descriptor of the job came with the word: no second round trip
                const uint64_t bad = __ballot(mine && !ok);
                have = polled_full && nd <= (uint32_t)kPollDescs && bad == 0 ? nd : 0u;
                // acquire at system scope (the CU's vector L1 and the L2): the
                // payloads (and descriptors) the host wrote before the job word
                // are read fresh; the other waves load after the barrier below
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
            if (t == 0) {
                s_cmd = cmd;
                s_have = have;
            }
        }
        __syncthreads();
        const uint64_t cmd = s_cmd;
        if (cmd == 0) break;  // every wave leaves together
        const uint32_t nd = (uint32_t)(cmd >> 40) & 0xFFu;
        const uint32_t n = nd < (uint32_t)kResMaxDescs ? nd : (uint32_t)kResMaxDescs;
        const uint32_t parts = (uint32_t)(cmd >> kPartShift & 3u) + 1u;
        if (s_have == 0 && t < (int)n) {
            const uint64_t* q = reinterpret_cast<const uint64_t*>(&sl->desc[t]);
            const uint64_t lo = ld_sys(q), hi = ld_sys(q + 1);  // each half one 8-byte load
            s_d[t] = untag_desc(ResDesc{lo, (uint32_t)hi, (uint32_t)(hi >> 32)});
        }
        __syncthreads();
#ifdef KMWS_TEST_RESIDENT_STALL_KEY
        // test build only (kuma_amd/build.py): a job whose first payload's key
        // has these upper 24 bits stalls the workgroup for (key & 0xFF) x 10 ms,
        // then is dropped if its thread withdrew it meanwhile (the quit bit)
        if ((s_d[0].key & 0xFFFFFF00u) == (uint32_t)(KMWS_TEST_RESIDENT_STALL_KEY)) {
            const uint64_t t0 = wall_clock64(), ticks = lease_ticks / kResLeaseUs * 10000u * (s_d[0].key & 0xFFu);
            while ((uint64_t)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(127);
            if (t == 0 && (ld_sys(pw0) & kQuitBit)) s_cmd = 0;
            __syncthreads();
            if (s_cmd == 0) {
                why = 4;  // gone on its quit bit
                break;
            }
        }
#endif
        if (t == 0) {
            uint32_t w = 0;
            for (uint32_t i = 0; i < n; ++i) {
                s_pre[i] = w;
                w += hull_words(s_d[i].addr, s_d[i].len);
            }
            s_pre[n] = w;
        }
        __syncthreads();
        const uint32_t total = s_pre[n];
        const bool wt = (cmd & kWriteThroughBit) != 0;
        // this part's words: an even share, in job order
        const uint32_t wb = (uint32_t)((uint64_t)total * part / parts), we = (uint32_t)((uint64_t)total * (part + 1) / parts);
        for (uint32_t w0 = wb; w0 < we; w0 += kResBlock * kResWords) {
            if (w0 + (uint32_t)(t & ~63) >= we) break;  // nothing left for this wave (uniform)
            u32x4 v[kResWords];
            uint32_t di[kResWords];
#pragma unroll
            for (int i = 0; i < kResWords; ++i) {
                // a lane past the part's end loads nothing (clamped to the
                // part's last word, many waves reading one host word stalled
                // the grid: 4 KiB jobs ran at 48 us, r06ao; a load from its
                // LDS sink instead cost a device batch beside the grid 1.08x
                // against 1.02x, r06ay).  One asm statement takes every store,
                // so the compiler's wait for these loads costs nothing more.
                const uint32_t w = w0 + t + kResBlock * i;
                uint32_t lo = 0, hi = n;  // last payload whose first word is <= w
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_pre[mid] <= w) lo = mid; else hi = mid;
                }
                di[i] = lo;
                const ResDesc x = s_d[lo];
                v[i] = u32x4{0, 0, 0, 0};
                if (w < we) v[i] = *reinterpret_cast<const u32x4*>(((x.addr >> 4) + (w - s_pre[lo])) << 4);
            }
            // each word XORed with its payload's rotated key (the loads' registers
            // free from here: fewer live VGPRs leave more of each SIMD to a device
            // batch sharing the CU -- 96 against 82 cost that batch 1.07-1.08x
            // against 1.02x, r06bq)
            u32x4 sv[kResWords];
            uint64_t sa[kResWords];
            uint32_t edge = 0;  // bit i: word i is a hull's edge word of this part
#pragma unroll
            for (int i = 0; i < kResWords; ++i) {
                const uint32_t w = w0 + t + kResBlock * i;
                const ResDesc x = s_d[di[i]];
                const uint64_t a = ((x.addr >> 4) + (w - s_pre[di[i]])) << 4;
                sv[i] = v[i] ^ rot_key(x.key, x.addr);
                sa[i] = a;
                // no short-circuit: with `&&` the compiler (ROCm 7.2, gfx950)
                // branched around the descriptor's length and lost the sink
                // for the last word of a payload on word 0 -- it stored the
                // whole word, over the next frame's header (r06ap)
                const bool in = w < we, whole = in & (a >= x.addr) & (a + 16 <= x.addr + x.len);
                edge |= (uint32_t)(in & !whole) << i;
                if (wt) sa[i] = whole ? a : my_sink;
                else if (whole) *reinterpret_cast<u32x4*>(a) = sv[i];  // into the L2 (the release follows)
            }
            // write-through: the four words in one asm statement
            static_assert(kResWords == 4, "st_sys16x4 stores four words");
            if (wt) st_sys16x4(sa[0], sv[0], sa[1], sv[1], sa[2], sv[2], sa[3], sv[3]);
            // a hull's edge words: this payload's bytes only
#pragma unroll
            for (int i = 0; i < kResWords; ++i) {
                if (!(edge >> i & 1u)) continue;
                const ResDesc x = s_d[di[i]];
                const uint64_t a = sa[i] == my_sink ? ((x.addr >> 4) + (w0 + t + kResBlock * i - s_pre[di[i]])) << 4 : sa[i];
                const uint64_t end = x.addr + x.len;
                const uint64_t lo = a > x.addr ? a : x.addr, hi = a + 16 < end ? a + 16 : end;
                for (uint64_t q = lo; q < hi; ++q) {
                    const uint32_t b = (uint32_t)(q - a);
                    const uint32_t dw = (b & 8u) ? ((b & 4u) ? sv[i].w : sv[i].z) : ((b & 4u) ? sv[i].y : sv[i].x);
                    const uint32_t o = dw >> (8 * (b & 3u));
                    if (wt) st_sys1(q, o);
                    else *reinterpret_cast<uint8_t*>(q) = (uint8_t)o;
                }
            }
        }
        // every wave waits for its own stores, then ONE lane writes the
        // part's done word: a small job's stores were written through (in
        // host memory once vmcnt drains), so no release; a large job's sit in
        // the L2 and that lane's release writes them back (one release: in all
        // 16 waves it cost 2.7 us more per 64 KiB job, tools/zc_probe.hip,
        // profiles/r05n_zc_probe.jsonl)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0) {
            if (wt) __hip_atomic_store(&sl->done[part], cmd & kJobMask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            else __hip_atomic_store(&sl->done[part], cmd & kJobMask, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (t < 64) {
            last = cmd & kJobMask;
            t_act = wall_clock64();  // the slot was busy until now (a long job is not idle time)
        }
    }
    if (t == 0) {
        __hip_atomic_fetch_add(&ctl->why[why < kResExitReasons ? why : 0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (why == 4 && !idle) {  // gone on its quit bit: idle for the rest of the incarnation
            const uint64_t b = __hip_atomic_fetch_add(&ctl->idle, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (b + 1 >= gridDim.x) __hip_atomic_fetch_max(&ctl->closing, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __hip_atomic_store(&sl->gone[part], inc, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t before = __hip_atomic_fetch_add(&ctl->exits, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (before + 1 == exit_base + gridDim.x) {  // the grid's last workgroup: the next starts with none idle
            (void)__hip_atomic_exchange(&ctl->idle, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&mb->exited, inc, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

namespace {

void quit_all_workers();

template <class T>
T ld_acq(const T* p)
{
    return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

// Is job s of a slot finished, given the slot's done word?  Jobs of a slot run
// one at a time in number order (40-bit, wrapping), so a done word at or past
// s means s has run -- a ticket may be waited for after a later job of the
// same slot finished.
inline bool job_done(uint64_t done, uint64_t s) { return ((done - s) & kJobMask) < (1ull << 39); }

using Clock = std::chrono::steady_clock;

// One per device, shared by every host thread.  Slots are claimed with one
// atomic on a bit mask; a job on a slot needs no lock (the slot's thread is
// its only writer).  launch_mu_ is taken only to relaunch the grid or to
// withdraw a job no workgroup can take any more.  Never freed: releasing
// pinned memory from a static destructor can run after the HIP runtime was
// torn down.  At process exit an atexit handler -- registered after the HIP
// runtime's own, so it runs before the runtime's teardown -- asks every
// workgroup to quit and waits (bounded) until the grid has exited.
class ResidentWorker {
public:
    explicit ResidentWorker(int device) : device_(device) {}

    // A free slot for the calling thread (its owner token `me`, never 0), or
    // -1 (all taken, or unusable).
    int claim(uint64_t me)
    {
        if (!usable()) return -1;
        uint32_t m = ld_acq(&claimed_);
        for (;;) {
            if (m == 0xFFFFFFFFu >> (32 - kResSlots)) return -1;
            const int b = __builtin_ctz(~m);
            if (__atomic_compare_exchange_n(&claimed_, &m, m | (1u << b), false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
                __atomic_store_n(&hs_[b].owner, me, __ATOMIC_RELEASE);
                // the workgroup polls the descriptors from now on (no job: same number)
                __atomic_fetch_or(&mb_->slot[b].word, kClaimedBit, __ATOMIC_RELEASE);
                // a running incarnation without this slot's workgroups is asked
                // to leave; the next job relaunches a grid that serves it
                const uint64_t cur = ld_acq(&inc_);
                if (cur && (uint32_t)b >= ld_acq(&nslots_)) request_resize(cur);
                return b;
            }
        }
    }
    // The thread `me` gives slot b back (thread exit, or it switched the worker
    // off).  Its last job -- an rx / tx batch's submit may still be running --
    // is first waited for: finished (its batch's poll then sees it done), or
    // withdrawn unrun (the poll sees that and launches it).  Only then may
    // another thread claim the slot and post on it: a job number the slot's
    // next holder reuses can no longer be mistaken for this thread's.  False:
    // the job neither finished nor left in time -- the slot stays taken.
    bool release(int b, uint64_t me)
    {
        if (b < 0 || b >= kResSlots || !mb_) return true;
        if (__atomic_load_n(&hs_[b].owner, __ATOMIC_ACQUIRE) != me) return true;  // not this thread's
        const uint64_t s = hs_[b].seq;
        if (s && hs_[b].cancelled != s && !all_done(mb_->slot[b], s, hs_[b].parts)) {
            __atomic_fetch_add(&drained_, 1, __ATOMIC_RELAXED);
            if (wait(b, s) == KMWS_ERR_TIMEOUT) return false;
        }
        __atomic_store_n(&hs_[b].owner, 0ull, __ATOMIC_RELEASE);
        if (!__atomic_load_n(&exiting_, __ATOMIC_ACQUIRE))
            __atomic_fetch_and(&mb_->slot[b].word, ~kClaimedBit, __ATOMIC_RELEASE);
        __atomic_fetch_and(&claimed_, ~(1u << b), __ATOMIC_ACQ_REL);
        return true;
    }
    // A thread whose slots were given back at its exit asked for a job: it
    // launches instead (counted).
    void note_late_post() { __atomic_fetch_add(&late_posts_, 1, __ATOMIC_RELAXED); }

    // Ask every workgroup to leave at its next poll and wait for the grid (atexit).
    void quit_and_wait()
    {
        __atomic_store_n(&exiting_, true, __ATOMIC_RELEASE);
        if (!mb_) return;
        std::lock_guard<std::mutex> lk(launch_mu_);
        state_ = -1;  // no relaunch from here on
        for (int b = 0; b < kResSlots; ++b) __atomic_fetch_or(&mb_->slot[b].word, kQuitBit, __ATOMIC_RELEASE);
        const uint64_t cur = ld_acq(&inc_);
        const auto t0 = Clock::now();
        while (cur && ld_acq(&mb_->exited) != cur && Clock::now() - t0 < std::chrono::milliseconds(500)) cpu_relax();
    }

    // created on first use: a process whose threads all switched the worker
    // off creates nothing (no stream, no mailbox)
    bool usable()
    {
        int s = ld_acq(&state_);
        if (s == 0) {
            std::lock_guard<std::mutex> lk(launch_mu_);
            if (state_ == 0) state_ = init() == KMWS_OK ? 1 : -1;
            s = state_;
        }
        return s == 1;
    }

    // Posts one job of n <= kResMaxDescs payloads on slot b (held by the
    // calling thread) and returns without waiting; *job = its number.
    // KMWS_ERR_NOT_SUPPORTED: the slot's previous job is still running, or the
    // worker cannot be (re)launched -- nothing was posted.
    kmws_status post(int b, uint64_t me, const ResDesc* d, uint32_t n, uint64_t* job)
    {
        if (n == 0 || n > (uint32_t)kResMaxDescs || !usable()) return KMWS_ERR_NOT_SUPPORTED;
        for (uint32_t i = 0; i < n; ++i)
            if ((d[i].addr >> 48) != 0 || d[i].len > kLenMask) return KMWS_ERR_NOT_SUPPORTED;
        // only the slot's holder writes its descriptors and job word: a post
        // from any other thread is refused (and counted -- never expected)
        if (__atomic_load_n(&hs_[b].owner, __ATOMIC_ACQUIRE) != me) {
            __atomic_fetch_add(&unowned_posts_, 1, __ATOMIC_RELAXED);
            return KMWS_ERR_NOT_SUPPORTED;
        }
        ResSlot& sl = mb_->slot[b];
        const uint64_t prev = hs_[b].seq;
        uint64_t cur = ld_acq(&inc_);
        if (hs_[b].cancelled != prev && !all_done(sl, prev, hs_[b].parts)) {  // busy: the caller launches
            // (a job a previous holder left posted: a grid that left is relaunched for it)
            if (cur && ld_acq(&mb_->exited) == cur) (void)relaunch(cur);
            return KMWS_ERR_NOT_SUPPORTED;
        }
        if (cur == 0 || ld_acq(&mb_->exited) == cur) cur = relaunch(cur);
        if (cur == 0) return KMWS_ERR_NOT_SUPPORTED;
        // a slot claimed after the running incarnation was launched has no
        // workgroups in it: that incarnation was asked to leave (claim); launch
        // until it has, and the next post relaunches
        if ((uint32_t)b >= ld_acq(&nslots_)) {
            request_resize(cur);
            return KMWS_ERR_NOT_SUPPORTED;
        }
        const uint64_t s = (prev + 1) & kJobMask;
        uint64_t words = 0;
        for (uint32_t i = 0; i < n; ++i) words += hull_words(d[i].addr, d[i].len);
        const uint32_t parts = (uint32_t)std::min<uint64_t>(kResParts, std::max<uint64_t>(1, words / kPartWords));
        const bool wt = words <= (uint64_t)kResWriteThroughWords || device_batch_running(device_);
        __atomic_fetch_add(wt ? &wt_jobs_ : &released_jobs_, 1, __ATOMIC_RELAXED);
        // every polled slot is rewritten, so a stale half always carries job s - 1's tag
        for (uint32_t i = 0; i < n || i < (uint32_t)kPollDescs; ++i) {
            const ResDesc x = tag_desc(i < n ? d[i] : ResDesc{0, 0, 0}, s);
            uint64_t* q = reinterpret_cast<uint64_t*>(&sl.desc[i]);
            __atomic_store_n(q, x.addr, __ATOMIC_RELAXED);
            __atomic_store_n(q + 1, (uint64_t)x.len | (uint64_t)x.key << 32, __ATOMIC_RELAXED);
        }
        __atomic_store_n(&hs_[b].parts, parts, __ATOMIC_RELAXED);
        __atomic_store_n(&hs_[b].seq, s, __ATOMIC_RELEASE);
        __atomic_store_n(&hs_[b].jobs, hs_[b].jobs + 1, __ATOMIC_RELAXED);  // (a withdrawn job is taken off again)
        __atomic_store_n(&sl.word,
                         s | (uint64_t)n << 40 | (uint64_t)(parts - 1) << kPartShift | (wt ? kWriteThroughBit : 0) |
                             kClaimedBit,
                         __ATOMIC_RELEASE);
        *job = s;
        return KMWS_OK;
    }

    // 1 when job s of slot b is done, 0 while it runs (relaunching a grid that
    // left before taking it), KMWS_ERR_NOT_SUPPORTED when it was withdrawn
    // (never run: the caller launches it).
    int test(int b, uint64_t s)
    {
        ResSlot& sl = mb_->slot[b];
        if (withdrawn_job(b, s)) return KMWS_ERR_NOT_SUPPORTED;
        if (finished(b, s)) return 1;
        const uint64_t cur = ld_acq(&inc_);
        if (ld_acq(&mb_->exited) == cur) {
            if (finished(b, s)) return 1;
            if (relaunch(cur) == 0 && withdraw(b, s, cur)) return KMWS_ERR_NOT_SUPPORTED;
        }
        (void)sl;
        return 0;
    }

    // Waits for job s of slot b.  KMWS_OK: done.  KMWS_ERR_NOT_SUPPORTED:
    // withdrawn without having run (payloads untouched; the caller launches).
    // KMWS_ERR_TIMEOUT: the workgroup holding it neither finished nor left
    // within the bounds -- the device may still write its payloads.
    kmws_status wait(int b, uint64_t s)
    {
        ResSlot& sl = mb_->slot[b];
        if (withdrawn_job(b, s)) return KMWS_ERR_NOT_SUPPORTED;  // (by its thread's release at exit)
        const auto t0 = Clock::now();
        Clock::time_point orphan{};
        for (uint32_t spin = 0;; ++spin) {
            if (finished(b, s)) return KMWS_OK;
            cpu_relax();
            if ((spin & 255) != 255) continue;
            const uint64_t cur = ld_acq(&inc_);
            if (ld_acq(&mb_->exited) == cur) {  // the whole grid left: relaunch (the new one takes job s)
                if (finished(b, s)) return KMWS_OK;
                if (relaunch(cur) == 0) {
                    if (withdraw(b, s, cur)) return KMWS_ERR_NOT_SUPPORTED;
                    continue;
                }
                orphan = Clock::time_point{};
            } else if (part_left(sl, s, hs_[b].parts, cur)) {  // a part's workgroup left, others run on
                if (finished(b, s)) return KMWS_OK;
                const auto now = Clock::now();
                if (orphan == Clock::time_point{}) orphan = now;
                else if (now - orphan > std::chrono::microseconds(kResOrphanUs) && withdraw(b, s, cur))
                    return KMWS_ERR_NOT_SUPPORTED;
            } else {
                orphan = Clock::time_point{};
            }
            if (Clock::now() - t0 > std::chrono::milliseconds(KMWS_RESIDENT_TIMEOUT_MS)) return timed_out(b, s);
        }
    }

    uint64_t jobs() const
    {
        uint64_t n = 0;
        for (const SlotHost& h : hs_) n += __atomic_load_n(&h.jobs, __ATOMIC_RELAXED);
        return n;
    }
    uint64_t launches() const { return ld_acq(&inc_); }
    uint64_t timeouts() const { return ld_acq(&timeouts_); }
    uint64_t withdrawn() const { return ld_acq(&withdrawn_); }
    uint64_t unowned_posts() const { return ld_acq(&unowned_posts_); }
    uint64_t late_posts() const { return ld_acq(&late_posts_); }
    uint64_t drained() const { return ld_acq(&drained_); }
    uint64_t wt_jobs() const { return ld_acq(&wt_jobs_); }
    uint64_t released_jobs() const { return ld_acq(&released_jobs_); }
    int claimed() const { return __builtin_popcount(ld_acq(&claimed_)); }
    // Workgroup exits so far by reason (ResCtl::why), read from device memory.
    kmws_status exit_reasons(uint64_t* out, int n)
    {
        if (!dctl_) {
            for (int i = 0; i < n; ++i) out[i] = 0;
            return KMWS_OK;
        }
        uint64_t w[kResExitReasons] = {};
        DevGuard g(device_);
        if (hipMemcpy(w, dctl_->why, sizeof w, hipMemcpyDeviceToHost) != hipSuccess) {
            (void)hipGetLastError();
            return KMWS_ERR_FAILED;
        }
        for (int i = 0; i < n; ++i) out[i] = i < kResExitReasons ? w[i] : 0;
        return KMWS_OK;
    }
    int running() const
    {
        const uint64_t cur = ld_acq(&inc_);
        return mb_ && cur && ld_acq(&mb_->exited) != cur ? 1 : 0;
    }

private:
    // Every part of job s finished?  (A part's done word at or past s.)
    static bool all_done(const ResSlot& sl, uint64_t s, uint32_t parts)
    {
        for (uint32_t j = 0; j < parts; ++j)
            if (!job_done(ld_acq(&sl.done[j]), s)) return false;
        return true;
    }
    // Job s of slot b finished -- or the slot has moved on (a later job is
    // posted only once s was finished or withdrawn, by s's own waiter).
    // (Read by the job's poller, which after a release at thread exit may not
    // be the slot's holder any more: atomic loads.)
    bool finished(int b, uint64_t s) const
    {
        return ld_acq(&hs_[b].seq) != s || all_done(mb_->slot[b], s, ld_acq(&hs_[b].parts));
    }
    // Job s of slot b was withdrawn unrun (by its waiter, or by the release at
    // its thread's exit): its caller launches it.
    bool withdrawn_job(int b, uint64_t s) const { return ld_acq(&hs_[b].cancelled) == s; }
    // Has the workgroup of an unfinished part of job s left grid `cur`?
    static bool part_left(const ResSlot& sl, uint64_t s, uint32_t parts, uint64_t cur)
    {
        for (uint32_t j = 0; j < parts; ++j)
            if (!job_done(ld_acq(&sl.done[j]), s) && ld_acq(&sl.gone[j]) == cur) return true;
        return false;
    }

    // Takes job s of slot b back if no workgroup ran any of it and none can
    // take it any more: the grid `cur` is still the latest (no relaunch can
    // start while launch_mu_ is held) and the workgroup of every part has left.
    // The word keeps the job number with the cancel bit (and the quit bit
    // cleared), so no workgroup -- of this grid or a later one -- runs it; the
    // slot's next job takes the next number.  False: a part ran (or runs), or
    // a newer grid will take it.
    bool withdraw(int b, uint64_t s, uint64_t cur)
    {
        ResSlot& sl = mb_->slot[b];
        std::lock_guard<std::mutex> lk(launch_mu_);
        if (ld_acq(&inc_) != cur || hs_[b].seq != s) return false;
        const bool all_left = ld_acq(&mb_->exited) == cur;
        for (uint32_t j = 0; j < hs_[b].parts; ++j) {
            if (job_done(ld_acq(&sl.done[j]), s)) return false;
            if (!all_left && ld_acq(&sl.gone[j]) != cur) return false;
        }
        __atomic_store_n(&sl.word, (ld_acq(&sl.word) | kCancelBit) & ~kQuitBit, __ATOMIC_RELEASE);
        __atomic_store_n(&hs_[b].cancelled, s, __ATOMIC_RELEASE);
        __atomic_fetch_add(&withdrawn_, 1, __ATOMIC_RELAXED);
        __atomic_store_n(&hs_[b].jobs, hs_[b].jobs - 1, __ATOMIC_RELAXED);
        return true;
    }

    // Past the timeout: the quit bit asks slot b's workgroup to leave (it may
    // be inside the job, or stuck); wait, bounded, until it has.
    kmws_status timed_out(int b, uint64_t s)
    {
        ResSlot& sl = mb_->slot[b];
        const uint32_t parts = hs_[b].parts;
        __atomic_fetch_add(&timeouts_, 1, __ATOMIC_RELAXED);
        __atomic_fetch_or(&sl.word, kQuitBit, __ATOMIC_RELEASE);
        const auto t0 = Clock::now();
        for (uint32_t spin = 0;; ++spin) {
            if (finished(b, s)) {
                std::lock_guard<std::mutex> lk(launch_mu_);
                __atomic_fetch_and(&sl.word, ~kQuitBit, __ATOMIC_RELEASE);
                return KMWS_OK;
            }
            cpu_relax();
            if ((spin & 255) != 255) continue;
            const uint64_t cur = ld_acq(&inc_);
            const bool all_left = ld_acq(&mb_->exited) == cur;
            bool settled = true;  // every part finished, or its workgroup left
            for (uint32_t j = 0; j < parts; ++j)
                settled &= job_done(ld_acq(&sl.done[j]), s) || all_left || ld_acq(&sl.gone[j]) == cur;
            if (settled) {
                if (withdraw(b, s, cur)) return KMWS_ERR_NOT_SUPPORTED;  // no part ran: the caller launches
                // some parts ran: the others run in the next grid (the quit bit cleared)
                {
                    std::lock_guard<std::mutex> lk(launch_mu_);
                    __atomic_fetch_and(&sl.word, ~kQuitBit, __ATOMIC_RELEASE);
                }
                if (all_left) (void)relaunch(cur);
            }
            if (Clock::now() - t0 > std::chrono::milliseconds(KMWS_RESIDENT_DRAIN_MS)) break;
        }
        // still held by a workgroup that does not leave: the payloads stay the
        // device's, and no job is posted on this device's worker again
        std::lock_guard<std::mutex> lk(launch_mu_);
        state_ = -1;
        return KMWS_ERR_TIMEOUT;
    }

    kmws_status init()  // under launch_mu_
    {
        if (device_ < 0 || kmws_device_count() <= device_) return KMWS_ERR_NOT_SUPPORTED;
        DevGuard g(device_);
        void* p = nullptr;
        if (hipHostMalloc(&p, sizeof(ResMailbox), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            return KMWS_ERR_FAILED;
        }
        mb_ = static_cast<ResMailbox*>(p);
        std::memset(static_cast<void*>(mb_), 0, sizeof(ResMailbox));
        dmb_ = static_cast<ResMailbox*>(device_view(mb_));
        if (!dmb_) return KMWS_ERR_FAILED;
        // uncached: every XCD's workgroups read and update these words
        if (hipExtMallocWithFlags(reinterpret_cast<void**>(&dctl_), sizeof(ResCtl), hipDeviceMallocUncached) !=
            hipSuccess) {
            (void)hipGetLastError();
            dctl_ = nullptr;
            if (hipMalloc(reinterpret_cast<void**>(&dctl_), sizeof(ResCtl)) != hipSuccess) {
                (void)hipGetLastError();
                return KMWS_ERR_FAILED;
            }
        }
        // A non-blocking stream: the legacy default stream (torch's current stream
        // unless the caller picked another) waits for every blocking stream's
        // work, which would include this kernel -- measured: a kernel on the null
        // stream behind a CU-masked (blocking) worker stream waited out its idle
        // time, 5.02 ms each time.  At the greatest priority: the runtime keeps
        // separate hardware queues per priority, so the worker does not share a
        // queue with the process's ordinary streams unless those ask for the
        // same priority (the lease bounds the wait when they do).
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
            (void)hipGetLastError();
            greatest = least = 0;
        }
        // The grid runs on the SECOND greatest-priority stream this worker makes:
        // on the first one, a device batch beside the grid ran 1.33-1.40x slower
        // (cfg2, 0.82 -> 0.59 of HBM peak) whatever the grid did -- its jobs, its
        // polls, its block size, its lease (every such variant measured, and a
        // probe kernel of the grid's shape on a stream of its own slowed nothing);
        // with a greatest-priority stream made before it the same grid cost
        // 1.02x under 16 threads' 4 KiB masks (tools/grid_interference.cpp,
        // tools/priority_probe.hip, profiles/r06ag_*).  The spare stays unused.
        if (hipStreamCreateWithPriority(&spare_stream_, hipStreamNonBlocking, greatest) != hipSuccess ||
            hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest) != hipSuccess) {
            (void)hipGetLastError();
            return KMWS_ERR_FAILED;
        }
        // cleared on the worker's own stream: a device-wide synchronize here
        // would wait for every stream of the process (a long kernel elsewhere),
        // with launch_mu_ held
        if (hipMemsetAsync(dctl_, 0, sizeof(ResCtl), stream_) != hipSuccess ||
            hipStreamSynchronize(stream_) != hipSuccess) {
            (void)hipGetLastError();
            return KMWS_ERR_FAILED;
        }
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || khz <= 0)
            khz = 100000;  // gfx9 constant clock: 100 MHz
        idle_ticks_ = (uint64_t)khz * kResIdleUs / 1000u;
        lease_ticks_ = (uint64_t)khz * kResLeaseUs / 1000u;
        // registered after the HIP runtime initialised (the calls above), so at
        // exit it runs before the runtime's own teardown
        static std::once_flag once;
        std::call_once(once, [] { std::atexit(quit_all_workers); });
        return KMWS_OK;
    }

    // Incarnations up to `cur` leave at their next few polls (monotonic).
    void request_resize(uint64_t cur)
    {
        uint64_t r = ld_acq(&mb_->resize);
        while (r < cur && !__atomic_compare_exchange_n(&mb_->resize, &r, cur, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        }
    }

    // Launches the next incarnation once `seen` (0: none yet) has left
    // entirely; returns the incarnation now serving, or 0 if the worker is
    // unusable (nothing launched).
    uint64_t relaunch(uint64_t seen)
    {
        std::lock_guard<std::mutex> lk(launch_mu_);
        if (state_ != 1) return 0;
        const uint64_t cur = inc_;
        if (cur != seen) return cur;                                   // another thread relaunched
        if (cur != 0 && ld_acq(&mb_->exited) != cur) return cur;      // still running
        // the slots claimed now, up to the highest (a slot claimed later is
        // served from the next incarnation on; its jobs launch until then)
        const uint32_t m = ld_acq(&claimed_);
        const uint32_t nslots = m ? 32u - (uint32_t)__builtin_clz(m) : 1u;
        DevGuard g(device_);
        hipLaunchKernelGGL(resident_unmask_kernel, dim3(nslots * kResParts), dim3(kResBlock), 0, stream_, dmb_, dctl_,
                           cur + 1, nslots, exit_base_, idle_ticks_, lease_ticks_);
        if (hipGetLastError() != hipSuccess) {
            state_ = -1;
            return 0;
        }
        exit_base_ += (uint64_t)nslots * kResParts;
        __atomic_store_n(&nslots_, nslots, __ATOMIC_RELEASE);
        __atomic_store_n(&inc_, cur + 1, __ATOMIC_RELEASE);
        return cur + 1;
    }

    int device_;
    std::mutex launch_mu_;
    int state_ = 0;  // 0 untried, 1 ready, -1 unusable
    bool exiting_ = false;
    uint32_t claimed_ = 0;  // bit b: slot b held by a thread
    ResMailbox* mb_ = nullptr;
    ResMailbox* dmb_ = nullptr;
    ResCtl* dctl_ = nullptr;
    hipStream_t stream_ = nullptr;
    hipStream_t spare_stream_ = nullptr;  // made first, never used (see init)
    uint64_t idle_ticks_ = 0, lease_ticks_ = 0;
    uint64_t inc_ = 0;  // latest incarnation launched
    uint32_t nslots_ = 0;     // slots the latest incarnation serves
    uint64_t exit_base_ = 0;  // workgroups launched in all incarnations so far
    // Per slot, written by its holder thread (a withdraw by the holder too,
    // under launch_mu_), each on a cache line of its own: a thread spinning on
    // its job reads its own line only, and another thread's post does not
    // invalidate it (16 threads shared three arrays and one job counter before).
    struct alignas(64) SlotHost {
        uint64_t seq = 0;        // last job number posted
        uint64_t cancelled = 0;  // the last job withdrawn
        uint64_t jobs = 0;       // jobs posted and not withdrawn (summed by jobs())
        uint64_t owner = 0;      // owner token of the thread holding the slot (0: free)
        uint32_t parts = 0;      // parts of job `seq`
    };
    SlotHost hs_[kResSlots];
    alignas(64) uint64_t timeouts_ = 0;
    uint64_t withdrawn_ = 0;
    uint64_t unowned_posts_ = 0;  // posts refused: the caller did not hold the slot
    uint64_t wt_jobs_ = 0, released_jobs_ = 0;  // jobs posted by kind (kWriteThroughBit)
    uint64_t late_posts_ = 0;     // jobs asked for after the thread gave its slots back (launched)
    uint64_t drained_ = 0;        // releases that first waited for the slot's last job
};

// Every worker of the process (for the exit handler); never freed.
std::mutex g_all_mu;
std::vector<ResidentWorker*>* g_all = nullptr;

void quit_all_workers()
{
    std::lock_guard<std::mutex> lk(g_all_mu);
    if (g_all)
        for (ResidentWorker* w : *g_all) w->quit_and_wait();
}

constexpr int kMaxDevices = 64;
ResidentWorker* g_by_dev[kMaxDevices];  // set once under g_all_mu, read with acquire loads

ResidentWorker* worker(int device)
{
    if (device < 0 || device >= kMaxDevices) return nullptr;
    ResidentWorker* w = __atomic_load_n(&g_by_dev[device], __ATOMIC_ACQUIRE);
    if (w) return w;
    std::lock_guard<std::mutex> lk(g_all_mu);
    w = g_by_dev[device];
    if (!w) {
        w = new (std::nothrow) ResidentWorker(device);
        if (!w) return nullptr;
        if (!g_all) g_all = new std::vector<ResidentWorker*>();
        g_all->push_back(w);
        __atomic_store_n(&g_by_dev[device], w, __ATOMIC_RELEASE);
    }
    return w;
}

// The calling thread's slots, one per device.  Plain data -- zero-initialised,
// trivially destructible -- so it stays valid while the thread's other
// thread_local objects are destroyed, before and after ThreadExit below gives
// the slots back.  slot1[d] = slot + 1 (0: none held; -1: its job timed out,
// the slot is never given back).  kmws_resident_enable(0) makes the thread's
// calls launch instead (the A/B of the worker) and gives its slot back.
struct ThreadSlots {
    int8_t slot1[kMaxDevices];
    uint64_t off_mask;  // bit d: worker off for device d on this thread
    uint64_t token;     // this thread's owner token (0 until its first claim)
    bool gone;          // its slots were given back at thread exit: later jobs launch
};
thread_local ThreadSlots t_slots;

// Gives the thread's slots back when it exits.  Constructed at the thread's
// first claim (or by kmws_thread_attach), so C++'s reverse order of
// thread_local destruction runs it after every thread_local object that was
// complete by then -- and before those completed later.  VERDICT r05: a
// thread_local RxLoop / TxLoop made before the thread's first job was
// destroyed AFTER the slot had been given back, and its flush posted on a slot
// another thread might hold by then (both wrote the same job number).  Now
// such a flush finds `gone` set and launches; a loop that attached in its
// constructor is destroyed first and flushes on its slot.
struct ThreadExit {
    bool armed = false;
    ~ThreadExit()
    {
        t_slots.gone = true;
        for (int d = 0; d < kMaxDevices; ++d)
            if (t_slots.slot1[d] > 0)
                if (ResidentWorker* w = __atomic_load_n(&g_by_dev[d], __ATOMIC_ACQUIRE))
                    t_slots.slot1[d] = w->release(t_slots.slot1[d] - 1, t_slots.token) ? 0 : -1;
    }
};
thread_local ThreadExit t_exit;

uint64_t g_next_token = 0;

// The calling thread's slot on `device` (claimed on first use), or -1.
int thread_slot(int device, ResidentWorker** wout)
{
    if (device < 0 || device >= kMaxDevices || ((t_slots.off_mask >> device) & 1u)) return -1;
    ResidentWorker* w = worker(device);
    if (!w) return -1;
    *wout = w;
    if (t_slots.gone) {  // past this thread's ThreadExit: nothing is claimed any more
        w->note_late_post();
        return -1;
    }
    const int s1 = t_slots.slot1[device];
    if (s1 != 0) return s1 - 1;  // held (or -2: kept by a timed-out job)
    if (!t_slots.token) t_slots.token = __atomic_add_fetch(&g_next_token, 1, __ATOMIC_RELAXED);
    t_exit.armed = true;  // constructs it before the claim: the slot is given back at exit
    const int b = w->claim(t_slots.token);
    if (b >= 0) t_slots.slot1[device] = (int8_t)(b + 1);
    return b;
}

}  // namespace

// Posts the unmask of descs[0..n) over dev_base and descs2[0..n2) over
// dev_base2 (device views of pinned host memory, offsets relative to them) on
// the calling thread's slot; see kmws_common.hpp.
kmws_status resident_post(int device, const kmws_desc* descs, const uint8_t* dev_base, size_t n,
                          const kmws_desc* descs2, const uint8_t* dev_base2, size_t n2, ResidentJob* job,
                          uint64_t max_bytes)
{
    if (n + n2 == 0 || n + n2 > (size_t)kResMaxDescs) return KMWS_ERR_NOT_SUPPORTED;
    ResidentWorker* w = nullptr;
    const int b = thread_slot(device, &w);
    if (b < 0) return KMWS_ERR_NOT_SUPPORTED;
    ResDesc d[kResMaxDescs];
    uint64_t bytes = 0;
    size_t k = 0;
    for (size_t i = 0; i < n; ++i, ++k) {
        d[k] = ResDesc{(uint64_t)(uintptr_t)(dev_base + descs[i].off), descs[i].len, descs[i].key};
        bytes += descs[i].len;
    }
    for (size_t i = 0; i < n2; ++i, ++k) {
        d[k] = ResDesc{(uint64_t)(uintptr_t)(dev_base2 + descs2[i].off), descs2[i].len, descs2[i].key};
        bytes += descs2[i].len;
    }
    if (bytes > max_bytes || bytes > kResMaxBytesAsync) return KMWS_ERR_NOT_SUPPORTED;
    uint64_t s = 0;
    const kmws_status st = w->post(b, t_slots.token, d, (uint32_t)k, &s);
    if (st != KMWS_OK) return st;
    job->device = device;
    job->slot = b;
    job->seq = s;
    return KMWS_OK;
}

int resident_test(const ResidentJob& job)
{
    ResidentWorker* w = worker(job.device);
    return w ? w->test(job.slot, job.seq) : KMWS_ERR_INVALID_PARAM;
}

kmws_status resident_wait(const ResidentJob& job)
{
    ResidentWorker* w = worker(job.device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    const kmws_status st = w->wait(job.slot, job.seq);
    if (st == KMWS_ERR_TIMEOUT && job.device >= 0 && job.device < kMaxDevices &&
        t_slots.slot1[job.device] == job.slot + 1)
        t_slots.slot1[job.device] = -1;  // the slot stays the device's
    return st;
}

kmws_status resident_unmask(int device, const kmws_desc* descs, const uint8_t* dev_base, size_t n,
                            const kmws_desc* descs2, const uint8_t* dev_base2, size_t n2)
{
    ResidentJob job;
    const kmws_status st = resident_post(device, descs, dev_base, n, descs2, dev_base2, n2, &job);
    return st != KMWS_OK ? st : resident_wait(job);
}

}  // namespace kmws

extern "C" {

kmws_status kmws_resident_enable(int device, int on)
{
    if (device < 0 || device >= kmws::kMaxDevices) return KMWS_ERR_INVALID_PARAM;
    kmws::ThreadSlots& ts = kmws::t_slots;
    if (on) {
        ts.off_mask &= ~(1ull << device);
    } else {
        ts.off_mask |= 1ull << device;
        if (ts.slot1[device] > 0) {
            kmws::ResidentWorker* w = __atomic_load_n(&kmws::g_by_dev[device], __ATOMIC_ACQUIRE);
            ts.slot1[device] = !w || w->release(ts.slot1[device] - 1, ts.token) ? 0 : -1;
        }
    }
    return KMWS_OK;
}

kmws_status kmws_resident_info(int device, uint64_t* jobs, uint64_t* launches, int* running)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    if (jobs) *jobs = w->jobs();
    if (launches) *launches = w->launches();
    if (running) *running = w->running();
    return KMWS_OK;
}

kmws_status kmws_resident_counters(int device, int* thread_slot, int* slots_claimed, uint64_t* timeouts,
                                   uint64_t* withdrawn)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    if (thread_slot) *thread_slot = kmws::t_slots.slot1[device] > 0 ? kmws::t_slots.slot1[device] - 1 : -1;
    if (slots_claimed) *slots_claimed = w->claimed();
    if (timeouts) *timeouts = w->timeouts();
    if (withdrawn) *withdrawn = w->withdrawn();
    return KMWS_OK;
}

kmws_status kmws_resident_guard_counters(int device, uint64_t* unowned_posts, uint64_t* late_posts,
                                         uint64_t* drained_releases)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    if (unowned_posts) *unowned_posts = w->unowned_posts();
    if (late_posts) *late_posts = w->late_posts();
    if (drained_releases) *drained_releases = w->drained();
    return KMWS_OK;
}

kmws_status kmws_resident_store_counters(int device, uint64_t* write_through, uint64_t* released)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    if (write_through) *write_through = w->wt_jobs();
    if (released) *released = w->released_jobs();
    return KMWS_OK;
}

int kmws_device_batch_busy(int device) { return kmws::device_batch_running(device) ? 1 : 0; }

int kmws_thread_attach(int device)
{
    if (device == KMWS_DEVICE_AUTO) device = kmws_thread_device();
    if (device < 0 || device >= kmws::kMaxDevices || kmws_device_count() <= device) return KMWS_ERR_NOT_SUPPORTED;
    kmws::ResidentWorker* w = nullptr;
    const int b = kmws::thread_slot(device, &w);
    // even without a slot (all taken, worker off): the thread's exit hook now
    // exists, so a slot claimed later is still given back after this caller's
    // thread_local objects
    if (!kmws::t_slots.gone) kmws::t_exit.armed = true;
    return b;
}

kmws_status kmws_resident_exit_reasons(int device, uint64_t* counts, int n)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w || !counts || n < 0) return KMWS_ERR_INVALID_PARAM;
    return w->exit_reasons(counts, n);
}

}  // extern "C"
