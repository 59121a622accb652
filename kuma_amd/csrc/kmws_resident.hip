// Resident unmask worker: the synchronous host entries without a kernel launch
// per call.
//
// kuma calls WSHandler::handleData once per <= 64 KiB socket read
// (TcpConnection.cpp:229-233 -> WebSocketImpl.cpp:225-246) and
// WSHandler::handleDataMask once per send (WebSocketImpl.cpp:388, :414), and
// expects the payload unmasked when the call returns.  A stream launch plus an
// event wait costs 13-15 us per call -- about what kuma's byte loop
// (WSHandler.cpp:303-310) spends on a whole 64 KiB read -- so the synchronous
// drop-in lost to the reference.  Here one workgroup of 1024
// lanes stays resident on the GPU per device -- shared by the process's host
// threads, one job at a time under a spin lock (a worker per thread measured
// worse: two workers' streams share a hardware queue, so one thread's job
// waited for the other's worker to leave, up to its lease) -- and polls a
// mailbox in pinned host memory: the host writes a job (up to kResMaxDescs
// payloads, each a device-visible address, a length and a key) and bumps the
// job number; the worker sees it over PCIe, unmasks every payload in place
// there (zero-copy, 4 x 16-byte words per lane in flight: 64 KiB per round),
// makes its stores visible system-wide and writes the job number back; the
// host spins on that word.  No launch, no completion signal, no interrupt.
//
// The worker exits by itself after kResIdleUs (200 us) without a job, after a
// lease of kResLeaseUs (1 ms) however busy it is, and on quit:
// every wave reaches the exit, the grid drains, and a host thread that stops
// feeding never leaves a kernel behind.  The next job relaunches it.  It runs
// on a non-blocking stream of its own at the greatest priority, so work on
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
// Idle exit: short.  The runtime maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES, 4 on the box), so a kernel launched on a stream that
// shares the worker's queue waits until the worker leaves; and
// hipDeviceSynchronize (torch.cuda.synchronize) waits for every stream, the
// worker's included (measured: a device synchronize behind a 50 ms-idle worker
// took 50 ms; the loopback "gpu" mode, whose batches keep several streams, fell
// from 2.0 to 0.57 GiB/s with a 5 ms idle).  A loop thread under load feeds far
// more often than this; a worker that idled out costs one launch at the next
// job, the price of every call without it.
#ifndef KMWS_RESIDENT_IDLE_US
#define KMWS_RESIDENT_IDLE_US 200
#endif
constexpr uint32_t kResIdleUs = KMWS_RESIDENT_IDLE_US;
// Lease: an incarnation also leaves after kResLeaseUs of life however busy it
// is, before it takes the next job (the host relaunches it for that job).  A
// thread that feeds back to back would otherwise keep the worker resident for
// good, and a kernel on another stream that shares its hardware queue would
// wait for as long (measured: up to 6.9 s behind a feeder thread).  The
// relaunch it costs (~10-15 us) is spread over the ~100 jobs of one lease.
#ifndef KMWS_RESIDENT_LEASE_US
#define KMWS_RESIDENT_LEASE_US 1000
#endif
constexpr uint32_t kResLeaseUs = KMWS_RESIDENT_LEASE_US;

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

// Pinned host memory, polled by the worker.  Host-written and device-written
// words sit in different 128-byte lines.  The polled word carries the job
// number (bits 0-39), the payload count (40-47) and the quit bit (63); the
// first kPollDescs descriptor slots follow it and are read with it at every
// poll, so a job of up to kPollDescs payloads costs one PCIe round trip to
// notice and none more to read its descriptors.  The host rewrites every one
// of those slots for every job (unused ones with length 0), each half of a
// slot tagged with the job's low bits (address bits 48-63, length bits
// 21-31): a slot read before the host's write landed carries the previous
// job's tag, and the job's descriptors are then read again after the word.
constexpr uint64_t kJobMask = (1ull << 40) - 1;
constexpr uint64_t kQuitBit = 1ull << 63;
// word + 31 slots: the mailbox's first 512 bytes, one 16-byte load per lane
// of wave 0 -- a cfg1 read (16 frames of 4 KiB, and a partial one) fits
#ifndef KMWS_RESIDENT_POLL_DESCS
#define KMWS_RESIDENT_POLL_DESCS 31
#endif
constexpr int kPollDescs = KMWS_RESIDENT_POLL_DESCS;
static_assert(kPollDescs < 64, "one lane of wave 0 per polled slot");
constexpr uint64_t kAddrMask = (1ull << 48) - 1;
constexpr uint32_t kLenMask = (1u << 21) - 1;  // kResMaxBytes fits
static_assert(kResMaxBytes <= kLenMask, "tagged length");
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
struct alignas(256) ResMailbox {
    uint64_t word;  // job | ndesc << 40 | quit << 63, written last by the host (release)
    uint64_t pad1;
    ResDesc desc[kResMaxDescs];  // desc[i] at 16 + 16 i
    alignas(128) uint64_t done;    // job number finished (device, release: payloads visible)
    alignas(128) uint64_t exited;  // incarnation number of the worker that exited
    alignas(128) uint64_t pad2[16];
};

// Loads of host-written words bypass every cache (and are never scalar loads).
__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One block, persistent until idle.  `last` = the job number already done when
// it starts (jobs are numbered from 1); `inc` = this incarnation's number.
__global__ void __launch_bounds__(kResBlock) resident_unmask_kernel(ResMailbox* mb, uint64_t last, uint64_t inc,
                                                                    uint64_t idle_ticks, uint64_t lease_ticks)
{
    __shared__ ResDesc s_d[kResMaxDescs];
    __shared__ uint32_t s_pre[kResMaxDescs + 1];  // word prefix over the payload hulls
    __shared__ uint64_t s_cmd;
    __shared__ uint32_t s_have;  // descriptors taken from the poll
    const int t = threadIdx.x;
    const uint64_t born = wall_clock64();
    // lane l <= kPollDescs of wave 0 polls bytes [16 l, 16 l + 16) of the
    // mailbox: the job word (lane 0) and descriptor slot l - 1; the other
    // lanes load lane 0's address (one request)
    const uint64_t* pw = reinterpret_cast<const uint64_t*>(mb) + 2 * (t <= kPollDescs ? t : 0);
    for (;;) {
        if (t < 64) {  // wave 0, uniform control flow
            uint64_t cmd = 0, v0 = 0, v1 = 0;
            const uint64_t t0 = wall_clock64();
            for (;;) {
                if ((uint64_t)(wall_clock64() - born) > lease_ticks) break;  // a posted job waits for the relaunch
                v0 = ld_sys(pw);
                v1 = ld_sys(pw + 1);
                const uint64_t w = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v0) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v0 >> 32)) << 32;
                // (lane 0's job word; each half through uint32_t: readfirstlane is signed)
                if (w & kQuitBit) break;
                if ((w & kJobMask) != last) {
                    cmd = w;
                    break;
                }
                if ((uint64_t)(wall_clock64() - t0) > idle_ticks) break;
                __builtin_amdgcn_s_sleep(2);
            }
            uint32_t have = 0;
            if (cmd) {
                const uint32_t nd = (uint32_t)(cmd >> 40) & 0xFFu;
                const ResDesc x = ResDesc{v0, (uint32_t)v1, (uint32_t)(v1 >> 32)};
                const bool mine = t >= 1 && t <= (int)nd && t <= kPollDescs;
                const bool ok = desc_tagged(x, cmd & kJobMask);
                if (mine && ok) s_d[t - 1] = untag_desc(x);
                // every descriptor of the job came with the word: no second round trip
                const uint64_t bad = __ballot(mine && !ok);
                have = nd <= (uint32_t)kPollDescs && bad == 0 ? nd : 0u;
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
        if (s_have == 0 && t < (int)n) s_d[t] = untag_desc(mb->desc[t]);
        __syncthreads();
        if (t == 0) {
            uint32_t w = 0;
            for (uint32_t i = 0; i < n; ++i) {
                s_pre[i] = w;
                const ResDesc x = s_d[i];
                w += x.len ? (uint32_t)(((x.addr + x.len + 15) >> 4) - (x.addr >> 4)) : 0u;
            }
            s_pre[n] = w;
        }
        __syncthreads();
        const uint32_t total = s_pre[n];
        for (uint32_t w0 = 0; w0 < total; w0 += kResBlock * kResWords) {
            u32x4 v[kResWords];
            uint32_t di[kResWords];
#pragma unroll
            for (int i = 0; i < kResWords; ++i) {
                const uint32_t w = w0 + t + kResBlock * i;
                di[i] = 0;
                v[i] = u32x4{0, 0, 0, 0};
                if (w < total) {
                    uint32_t lo = 0, hi = n;  // last payload whose first word is <= w
                    while (hi - lo > 1) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_pre[mid] <= w) lo = mid; else hi = mid;
                    }
                    di[i] = lo;
                    const ResDesc x = s_d[lo];
                    v[i] = *reinterpret_cast<const u32x4*>(((x.addr >> 4) + (w - s_pre[lo])) << 4);
                }
            }
#pragma unroll
            for (int i = 0; i < kResWords; ++i) {
                const uint32_t w = w0 + t + kResBlock * i;
                if (w >= total) continue;
                const ResDesc x = s_d[di[i]];
                const uint64_t a = ((x.addr >> 4) + (w - s_pre[di[i]])) << 4;
                const uint64_t end = x.addr + x.len;
                const uint32_t r = rot_key(x.key, x.addr);
                if (a >= x.addr && a + 16 <= end) {
                    *reinterpret_cast<u32x4*>(a) = v[i] ^ r;
                } else {  // a hull's first or last word: this payload's bytes only
                    const uint64_t lo = a > x.addr ? a : x.addr, hi = a + 16 < end ? a + 16 : end;
                    for (uint64_t q = lo; q < hi; ++q) {
                        const uint32_t b = (uint32_t)(q - a);
                        const uint32_t dw = (b & 8u) ? ((b & 4u) ? v[i].w : v[i].z) : ((b & 4u) ? v[i].y : v[i].x);
                        *reinterpret_cast<uint8_t*>(q) = (uint8_t)((dw ^ r) >> (8 * (b & 3u)));
                    }
                }
            }
        }
        // release at system scope by every lane (each wave waits for its own
        // stores and writes the L2 back), then the job number: the host sees
        // every payload byte before it sees `done`
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __syncthreads();
        if (t == 0) __hip_atomic_store(&mb->done, cmd & kJobMask, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        last = cmd & kJobMask;
    }
    if (t == 0) __hip_atomic_store(&mb->exited, inc, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

namespace {

void quit_all_workers();

// One per device, shared by every host thread: a job holds the worker's spin
// lock from posting its descriptors to seeing it done (jobs take microseconds;
// the kernel serves one at a time anyway).  Never freed: releasing pinned
// memory from a static destructor can run after the HIP runtime was torn
// down.  At process exit an atexit handler -- registered after the HIP
// runtime's own, so it runs before the runtime's teardown -- asks every
// worker to quit and waits (bounded) until each running kernel has exited:
// the grid has drained before the process ends.  The idle exit ends a worker
// nobody feeds.
class ResidentWorker {
public:
    explicit ResidentWorker(int device) : device_(device) {}

    void lock()
    {
        for (;;) {
            if (!__atomic_exchange_n(&busy_, true, __ATOMIC_ACQUIRE)) return;
            while (__atomic_load_n(&busy_, __ATOMIC_RELAXED)) cpu_relax();
        }
    }
    void unlock() { __atomic_store_n(&busy_, false, __ATOMIC_RELEASE); }

    // Ask the kernel to leave at its next poll and wait for it (atexit).
    void quit_and_wait()
    {
        if (!mb_ || !running_) return;
        __atomic_store_n(&mb_->word, kQuitBit, __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        while (__atomic_load_n(&mb_->exited, __ATOMIC_ACQUIRE) != inc_ &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(500))
            cpu_relax();
    }

    // (under the lock) created on first use: a process whose threads all
    // switched the worker off creates nothing (no stream, no mailbox)
    bool usable()
    {
        if (state_ == 0) state_ = init() == KMWS_OK ? 1 : -1;
        return state_ == 1;
    }

    // One synchronous job of n <= kResMaxDescs payloads (under the lock).
    kmws_status run(const ResDesc* d, uint32_t n)
    {
        if (n == 0) return KMWS_OK;
        if (!usable() || n > (uint32_t)kResMaxDescs) return KMWS_ERR_NOT_SUPPORTED;
        const uint64_t inc_exited = __atomic_load_n(&mb_->exited, __ATOMIC_ACQUIRE);
        if (!running_ || inc_exited == inc_) {
            kmws_status st = launch(seq_ & kJobMask);  // every earlier job is done
            if (st != KMWS_OK) return st;
        }
        const uint64_t s = (seq_ + 1) & kJobMask;
        for (uint32_t i = 0; i < n; ++i)
            if ((d[i].addr >> 48) != 0 || d[i].len > kLenMask) return KMWS_ERR_NOT_SUPPORTED;
        // every polled slot is rewritten, so a stale one always carries job s - 1's tag
        for (uint32_t i = 0; i < n || i < (uint32_t)kPollDescs; ++i)
            mb_->desc[i] = tag_desc(i < n ? d[i] : ResDesc{0, 0, 0}, s);
        ++seq_;
        __atomic_store_n(&mb_->word, s | (uint64_t)n << 40, __ATOMIC_RELEASE);
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t spin = 0;; ++spin) {
            if (__atomic_load_n(&mb_->done, __ATOMIC_ACQUIRE) == s) break;
            cpu_relax();
            if ((spin & 255) != 255) continue;
            if (__atomic_load_n(&mb_->exited, __ATOMIC_ACQUIRE) == inc_) {
                // idle or lease exit raced with this job: done is written before exited
                if (__atomic_load_n(&mb_->done, __ATOMIC_ACQUIRE) == s) break;
                kmws_status st = launch((s - 1) & kJobMask);  // the new incarnation takes job s
                if (st != KMWS_OK) return st;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                // The job may still run later, so it is not retried (XOR twice is
                // the identity): the call fails, and this worker is never used
                // again (later calls launch kernels on their own streams).
                __atomic_store_n(&mb_->word, kQuitBit, __ATOMIC_RELEASE);
                state_ = -1;
                return KMWS_ERR_FAILED;
            }
        }
        ++jobs_;
        return KMWS_OK;
    }

    uint64_t jobs() const { return jobs_; }
    uint64_t launches() const { return inc_; }
    int running()
    {
        return running_ && __atomic_load_n(&mb_->exited, __ATOMIC_ACQUIRE) != inc_ ? 1 : 0;
    }

private:
    kmws_status init()
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
        if (hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest) != hipSuccess) {
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

    kmws_status launch(uint64_t last)
    {
        DevGuard g(device_);
        ++inc_;
        hipLaunchKernelGGL(resident_unmask_kernel, dim3(1), dim3(kResBlock), 0, stream_, dmb_, last, inc_,
                           idle_ticks_, lease_ticks_);
        if (hipGetLastError() != hipSuccess) {
            state_ = -1;
            return KMWS_ERR_FAILED;
        }
        running_ = true;
        return KMWS_OK;
    }

    int device_;
    bool busy_ = false;  // the spin lock
    int state_ = 0;      // 0 untried, 1 ready, -1 unusable
    bool running_ = false;
    ResMailbox* mb_ = nullptr;
    ResMailbox* dmb_ = nullptr;
    hipStream_t stream_ = nullptr;
    uint64_t idle_ticks_ = 0, lease_ticks_ = 0;
    uint64_t seq_ = 0, inc_ = 0, jobs_ = 0;
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

// kmws_resident_enable is per calling thread: a thread that switched the
// worker off launches its jobs (the A/B of the worker), others keep it.
thread_local uint64_t t_off_mask = 0;  // bit d: off for device d on this thread
bool off_here(int device) { return device >= 0 && device < kMaxDevices && ((t_off_mask >> device) & 1u); }

}  // namespace

// Synchronous unmask of host payloads (device-visible views of pinned memory)
// through the device's resident worker.  KMWS_ERR_NOT_SUPPORTED: the job does
// not fit a worker job (more than kResMaxDescs payloads or kResMaxBytes bytes),
// the calling thread switched the worker off, or it is unusable; the caller
// launches.
kmws_status resident_unmask(int device, const kmws_desc* descs, const uint8_t* dev_base, size_t n,
                            const kmws_desc* descs2, const uint8_t* dev_base2, size_t n2)
{
    if (n + n2 > (size_t)kResMaxDescs || off_here(device)) return KMWS_ERR_NOT_SUPPORTED;
    ResidentWorker* w = worker(device);
    if (!w) return KMWS_ERR_NOT_SUPPORTED;
    ResDesc job[kResMaxDescs];
    uint64_t bytes = 0;
    size_t k = 0;
    for (size_t i = 0; i < n; ++i, ++k) {
        job[k] = ResDesc{(uint64_t)(uintptr_t)(dev_base + descs[i].off), descs[i].len, descs[i].key};
        bytes += descs[i].len;
    }
    for (size_t i = 0; i < n2; ++i, ++k) {
        job[k] = ResDesc{(uint64_t)(uintptr_t)(dev_base2 + descs2[i].off), descs2[i].len, descs2[i].key};
        bytes += descs2[i].len;
    }
    if (bytes > kResMaxBytes) return KMWS_ERR_NOT_SUPPORTED;
    w->lock();
    const kmws_status st = w->run(job, (uint32_t)k);
    w->unlock();
    return st;
}

}  // namespace kmws

extern "C" {

kmws_status kmws_resident_enable(int device, int on)
{
    if (device < 0 || device >= kmws::kMaxDevices) return KMWS_ERR_INVALID_PARAM;
    if (on) kmws::t_off_mask &= ~(1ull << device);
    else kmws::t_off_mask |= 1ull << device;
    return KMWS_OK;
}

kmws_status kmws_resident_info(int device, uint64_t* jobs, uint64_t* launches, int* running)
{
    kmws::ResidentWorker* w = kmws::worker(device);
    if (!w) return KMWS_ERR_INVALID_PARAM;
    w->lock();
    if (jobs) *jobs = w->jobs();
    if (launches) *launches = w->launches();
    if (running) *running = w->running();
    w->unlock();
    return KMWS_OK;
}

}  // extern "C"
