// Device selection for the host-side objects (SURVEY.md sec.8 e): which GPU a
// kuma loop thread's decoders, rx / tx batches, pinned rings and pipelines use.
//
// kuma runs a pool of event-loop threads per process (10 in its test client,
// test/client/main.cpp:20; 5 in its server, test/server/main.cpp:22); every
// connection's bytes arrive on its loop thread (TcpConnection.cpp:229).  With
// every object on device 0, all loop threads of an 8-GPU node share one GPU's
// PCIe link -- about 30 GB/s each way at 8 loopback connections (DESIGN.md
// sec.5) -- while the other seven links idle.  Here every `device` argument of
// include/kmws_gpu.h also takes KMWS_DEVICE_AUTO, the calling thread's device:
//   - pinned by kmws_set_thread_device (an explicit map, e.g. loop i -> GPU i);
//   - else chosen once per thread, at its first AUTO call, by the process's
//     policy: NUMA (default) -- round robin over the GPUs on the NUMA node of the
//     CPU the thread runs on (its PCIe root, and the host DRAM its socket reads
//     land in), over all GPUs if that node has none; ROUND_ROBIN -- over all
//     GPUs in thread order; FIRST -- device 0 (the pre-round-6 behaviour).
// A thread's device never changes once chosen (its resident slot, stages and
// rings live there).  The choice is a pure function of (policy, node, the GPUs'
// nodes, a counter): kmws_device_policy_pick, which the CPU tests drive with
// synthetic topologies.  No environment variable is read.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <atomic>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"

namespace {

constexpr int kMaxDev = 64;
constexpr int kMaxNodes = 64;

struct Topology {
    int ngpus = 0;
    int gpu_node[kMaxDev];  // NUMA node of each gfx950 device's PCIe function (-1: unknown)
    std::vector<int> cpu_node;  // NUMA node per CPU (-1: unknown)
};

int read_int_file(const std::string& path, int dflt)
{
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return dflt;
    int v = dflt;
    if (std::fscanf(f, "%d", &v) != 1) v = dflt;
    std::fclose(f);
    return v;
}

// "0-3,8,10-11" -> each CPU's node
void parse_cpulist(const char* s, int node, std::vector<int>& out)
{
    while (*s) {
        char* e = nullptr;
        long a = std::strtol(s, &e, 10);
        if (e == s) break;
        long b = a;
        s = e;
        if (*s == '-') {
            b = std::strtol(s + 1, &e, 10);
            s = e;
        }
        for (long c = a; c <= b && c < 65536; ++c) {
            if ((size_t)c >= out.size()) out.resize((size_t)c + 1, -1);
            out[(size_t)c] = node;
        }
        while (*s == ',' || std::isspace((unsigned char)*s)) ++s;
    }
}

const Topology& topology()
{
    static Topology* t = [] {
        Topology* x = new Topology();
        x->ngpus = kmws_device_count();
        if (x->ngpus > kMaxDev) x->ngpus = kMaxDev;
        for (int d = 0; d < x->ngpus; ++d) {
            x->gpu_node[d] = -1;
            char bus[64] = {0};
            if (hipDeviceGetPCIBusId(bus, (int)sizeof bus - 1, d) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
            x->gpu_node[d] = read_int_file(std::string("/sys/bus/pci/devices/") + bus + "/numa_node", -1);
        }
        for (int n = 0; n < kMaxNodes; ++n) {
            const std::string path = "/sys/devices/system/node/node" + std::to_string(n) + "/cpulist";
            FILE* f = std::fopen(path.c_str(), "r");
            if (!f) continue;
            char buf[4096] = {0};
            if (std::fgets(buf, (int)sizeof buf, f)) parse_cpulist(buf, n, x->cpu_node);
            std::fclose(f);
        }
        return x;
    }();
    return *t;
}

int g_policy = KMWS_DEVICE_POLICY_NUMA;
uint32_t g_rr = 0;                // threads placed round robin so far
uint32_t g_node_rr[kMaxNodes + 1];  // per node (last: unknown node)

// Plain data, zero-initialised: device + 1 (0: not chosen yet).
thread_local int t_dev1;

}  // namespace

extern "C" {

int kmws_device_policy_pick(int policy, int thread_node, const int* gpu_nodes, int ngpus, uint32_t seq)
{
    if (ngpus <= 0) return KMWS_ERR_NOT_SUPPORTED;
    if (ngpus > kMaxDev) ngpus = kMaxDev;
    switch (policy) {
    case KMWS_DEVICE_POLICY_FIRST: return 0;
    case KMWS_DEVICE_POLICY_ROUND_ROBIN: return (int)(seq % (uint32_t)ngpus);
    case KMWS_DEVICE_POLICY_NUMA: {
        int cand[kMaxDev], nc = 0;
        if (thread_node >= 0 && gpu_nodes)
            for (int d = 0; d < ngpus; ++d)
                if (gpu_nodes[d] == thread_node) cand[nc++] = d;
        if (nc == 0) return (int)(seq % (uint32_t)ngpus);  // no GPU on this node (or unknown): all of them
        return cand[seq % (uint32_t)nc];
    }
    default: return KMWS_ERR_INVALID_PARAM;
    }
}

kmws_status kmws_set_device_policy(int policy)
{
    if (policy != KMWS_DEVICE_POLICY_NUMA && policy != KMWS_DEVICE_POLICY_ROUND_ROBIN &&
        policy != KMWS_DEVICE_POLICY_FIRST)
        return KMWS_ERR_INVALID_PARAM;
    __atomic_store_n(&g_policy, policy, __ATOMIC_RELEASE);
    return KMWS_OK;
}

kmws_status kmws_set_thread_device(int device)
{
    if (device == KMWS_DEVICE_AUTO) {
        t_dev1 = 0;
        return KMWS_OK;
    }
    if (device < 0 || device >= topology().ngpus) return device < 0 ? KMWS_ERR_INVALID_PARAM : KMWS_ERR_NOT_SUPPORTED;
    t_dev1 = device + 1;
    return KMWS_OK;
}

int kmws_thread_device(void)
{
    if (t_dev1 > 0) return t_dev1 - 1;
    const Topology& t = topology();
    if (t.ngpus <= 0) return KMWS_ERR_NOT_SUPPORTED;
    const int policy = __atomic_load_n(&g_policy, __ATOMIC_ACQUIRE);
    int node = -1;
    const int cpu = sched_getcpu();
    if (cpu >= 0 && (size_t)cpu < t.cpu_node.size()) node = t.cpu_node[(size_t)cpu];
    uint32_t seq = 0;
    if (policy == KMWS_DEVICE_POLICY_ROUND_ROBIN) {
        seq = __atomic_fetch_add(&g_rr, 1u, __ATOMIC_RELAXED);
    } else if (policy == KMWS_DEVICE_POLICY_NUMA) {
        bool on_node = false;
        for (int d = 0; d < t.ngpus && node >= 0; ++d) on_node |= t.gpu_node[d] == node;
        seq = __atomic_fetch_add(&g_node_rr[on_node && node < kMaxNodes ? node : kMaxNodes], 1u, __ATOMIC_RELAXED);
    }
    const int d = kmws_device_policy_pick(policy, node, t.gpu_node, t.ngpus, seq);
    if (d < 0) return d;
    t_dev1 = d + 1;
    return d;
}

kmws_status kmws_device_numa_node(int device, int* node)
{
    const Topology& t = topology();
    if (!node || device < 0 || device >= t.ngpus) return KMWS_ERR_INVALID_PARAM;
    *node = t.gpu_node[device];
    return KMWS_OK;
}

}  // extern "C"

namespace kmws {

int resolve_device(int device) { return device == KMWS_DEVICE_AUTO ? kmws_thread_device() : device; }

// Per device: steady-clock ns until which device batches are assumed to run.
// An estimate, not a completion signal (an event per batch would cost every
// resident job a HIP query): 20 us + the batch's bytes at 6 TB/s, queued
// batches back to back, so a batch on another stream only lengthens it.
constexpr int kBatchDevices = 64;
static std::atomic<uint64_t> g_batch_until[kBatchDevices];

static uint64_t steady_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void note_device_batch(uint64_t bytes, hipStream_t stream)
{
    hipDevice_t dev = -1;
    if (stream && hipStreamGetDevice(stream, &dev) != hipSuccess) {
        (void)hipGetLastError();
        dev = -1;
    }
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    if (dev < 0 || dev >= kBatchDevices) return;
    const uint64_t now = steady_ns(), est = 20000u + bytes / 6000u;
    uint64_t cur = g_batch_until[dev].load(std::memory_order_relaxed);
    while (!g_batch_until[dev].compare_exchange_weak(cur, (cur > now ? cur : now) + est, std::memory_order_relaxed)) {
    }
}

bool device_batch_running(int device)
{
    return device >= 0 && device < kBatchDevices &&
           steady_ns() < g_batch_until[device].load(std::memory_order_relaxed);
}

}  // namespace kmws
