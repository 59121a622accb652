// Thread exit with frames still queued, against threads that keep claiming
// resident slots.  kuma stops its loop pool with frames queued
// (test/server/main.cpp:150 loop_pool.stop()) while other threads live on.
//
// Each round starts `exiters` loop threads that queue masked frames on both
// sides and exit without flushing:
//   - "loop" threads use kmws::RxLoop::forThisThread / TxLoop::forThisThread
//     (which attach the thread's resident slot in their constructors, so their
//     destructors flush on it before the thread gives it back);
//   - "raw" threads hold an rx and a tx batch in a thread_local object made
//     BEFORE the thread's first resident job -- its destructor runs after the
//     thread's exit hook gave the slot back (the round-5 race): its flush must
//     find the slot gone and launch (counted as a late post).
// Meanwhile `maskers` threads run short-lived threads that each claim a slot,
// mask 4 KiB buffers (kmws_mask_host_chain) and exit.  Every received payload,
// every sent frame and every masked buffer is compared with kuma's codec
// restated in oracle/ (encodeFrameHeader + the byte-loop mask,
// WSHandler.cpp:46-106, 303-322); no post may land on a slot its thread does
// not hold (kmws_resident_guard_counters).  Test infrastructure:
// tests/test_abi_build.py.
//
// usage: thread_exit_check [rounds] [exiters] [maskers] [both|loop|raw]
#include <sys/uio.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"
#include "kmws_wshandler.hpp"

extern "C" {  // oracle/kmws_oracle.c (test infrastructure)
typedef struct orc_hdr {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, plen, _pad;
    uint64_t xpl64;
    uint8_t maskey[4];
    uint32_t length;
} orc_hdr;
void orc_mask(const uint8_t key[4], uint8_t* data, size_t len, size_t phase);
int orc_encode_header(const orc_hdr* h, uint8_t out[14]);
}

namespace {

uint64_t mix(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// One masked client frame (kuma's sendWsFrame bytes, :381-403) and its payload.
struct Frame {
    std::string payload;  // plain
    uint32_t key;
    std::string wire;     // header + masked payload (oracle)
};
Frame make_frame(uint64_t seed, size_t len)
{
    Frame f;
    f.payload.resize(len);
    for (size_t i = 0; i < len; ++i) f.payload[i] = (char)(mix(seed * 7919 + i / 8) >> (8 * (i & 7)));
    f.key = (uint32_t)mix(seed ^ 0xABCDEF);
    orc_hdr o;
    std::memset(&o, 0, sizeof o);
    o.fin = 1;
    o.opcode = KMWS_OP_BINARY;
    o.mask = 1;
    std::memcpy(o.maskey, &f.key, 4);
    o.length = (uint32_t)len;
    uint8_t hb[14];
    const int hl = orc_encode_header(&o, hb);
    std::string m = f.payload;
    orc_mask(o.maskey, reinterpret_cast<uint8_t*>(&m[0]), m.size(), 0);
    f.wire.assign(reinterpret_cast<const char*>(hb), (size_t)hl);
    f.wire += m;
    return f;
}

// What one exiting thread sent and received, checked by main after the join.
struct Out {
    std::vector<Frame> rx_in;   // frames fed to the receive side (masked wire)
    std::vector<std::string> rx_got;  // payloads delivered
    std::vector<Frame> tx_in;   // frames sent
    std::string tx_wire;        // bytes written by the send side
    int rx_pending_at_exit = 0, rx_inflight_at_exit = 0, tx_pending_at_exit = 0, tx_inflight_at_exit = 0;
    int err = 0;
};

constexpr int kFrames = 24;

void gen_frames(Out* o, uint64_t seed)
{
    for (int i = 0; i < kFrames; ++i) {
        const size_t len = 1 + (size_t)(mix(seed + (uint64_t)i) % 9000);
        o->rx_in.push_back(make_frame(seed * 1000 + (uint64_t)i, len));
        o->tx_in.push_back(make_frame(seed * 1000 + 500 + (uint64_t)i, len));
    }
}

// ---- "loop" exiters: kmws::RxLoop / TxLoop thread_locals ----

struct LoopHolder {  // made before the loops: destroyed after them (the RxLoop's flush delivers to h)
    std::unique_ptr<kmws::ws::WSHandler> h;
    ~LoopHolder()
    {
        if (h) h->setRxLoop(nullptr);  // its RxLoop is gone already: nothing to discard there
    }
};
LoopHolder& loop_holder()
{
    thread_local LoopHolder x;
    return x;
}

void loop_exiter(Out* o)
{
    LoopHolder& hold = loop_holder();
    std::vector<kmws::RxLoop::Task> tasks;  // the loop's posted tasks (run a few times, then dropped)
    kmws::RxLoop& rx = kmws::RxLoop::forThisThread([&tasks](kmws::RxLoop::Task t) { tasks.push_back(std::move(t)); });
    kmws::TxLoop& tx = kmws::TxLoop::forThisThread([&tasks](kmws::TxLoop::Task t) { tasks.push_back(std::move(t)); });
    if (!rx.valid() || !tx.valid()) {
        o->err = 1;
        return;
    }
    hold.h.reset(new kmws::ws::WSHandler(rx.device()));
    hold.h->setMode(kmws::ws::WSMode::SERVER);
    hold.h->setRxLoop(&rx);
    hold.h->setFrameCallback([o](kmws::ws::FrameHeader, kmws::ws::BufferChain& b) {
        o->rx_got.emplace_back(static_cast<const char*>(b.readPtr()), b.length());
        return 0;
    });
    kmws::TxLoop::Conn* c = tx.open([o](const iovec* v, int n) {
        for (int i = 0; i < n; ++i) o->tx_wire.append(static_cast<const char*>(v[i].iov_base), v[i].iov_len);
        return 0;
    });
    for (int i = 0; i < kFrames; ++i) {
        std::string w = o->rx_in[(size_t)i].wire;  // kuma's read buffer
        if ((int)hold.h->handleData(reinterpret_cast<uint8_t*>(&w[0]), w.size()) != 0) o->err = 2;
        const Frame& f = o->tx_in[(size_t)i];
        kmws_frame_hdr hdr;
        std::memset(&hdr, 0, sizeof hdr);
        hdr.fin = 1;
        hdr.opcode = KMWS_OP_BINARY;
        hdr.mask = 1;
        std::memcpy(hdr.maskey, &f.key, 4);
        if (tx.send(c, hdr, reinterpret_cast<const uint8_t*>(f.payload.data()), f.payload.size()) < 0) o->err = 3;
        if (i % 5 == 4 && i < kFrames - 6) {  // a loop iteration's tasks, except near the end
            std::vector<kmws::RxLoop::Task> now;
            now.swap(tasks);
            for (auto& t : now) t();
        }
    }
    // one more iteration: a generation goes in flight on the slot, then the
    // last frames are fed and sent -- and the thread exits without flushing
    {
        std::vector<kmws::RxLoop::Task> now;
        now.swap(tasks);
        for (auto& t : now) t();
    }
    o->rx_pending_at_exit = rx.pending();
    o->rx_inflight_at_exit = rx.inflight();
    o->tx_pending_at_exit = tx.pending();
    o->tx_inflight_at_exit = tx.inflight();
    rx.setPoster(nullptr);  // the loop is stopping: tasks are no longer run
    tx.setPoster(nullptr);
}

// ---- "raw" exiters: C-ABI batches in a thread_local made before the first job ----

int on_frame_raw(const kmws_frame_hdr*, uint8_t* payload, size_t len, void* user)
{
    static_cast<Out*>(user)->rx_got.emplace_back(reinterpret_cast<const char*>(payload), len);
    return 0;
}

struct RawHolder {
    Out* o = nullptr;
    kmws_rx_batch* rb = nullptr;
    kmws_decoder* dec = nullptr;
    kmws_tx_batch* tb = nullptr;
    std::vector<std::string> tx_bufs;  // payloads queued for masking (the caller's buffers)
    std::vector<std::string> tx_hdrs;
    ~RawHolder()
    {
        // destroyed after the thread's exit hook: these flushes find no slot
        if (rb) {
            if (kmws_rx_batch_flush(rb) < 0) o->err = 11;
            kmws_rx_batch_destroy(rb);
        }
        if (dec) kmws_decoder_destroy(dec);
        if (tb) {
            if (kmws_tx_batch_flush(tb) < 0) o->err = 12;
            kmws_tx_batch_destroy(tb);
            for (size_t i = 0; i < tx_bufs.size(); ++i) o->tx_wire += tx_hdrs[i] + tx_bufs[i];
        }
    }
};
RawHolder& raw_holder()
{
    thread_local RawHolder x;
    return x;
}

void raw_exiter(Out* o)
{
    // The batches first: the thread's first HIP calls set up the HIP runtime's
    // own per-thread state, which C++ then destroys AFTER the holder below (a
    // thread_local made before a thread's first HIP call must not call HIP from
    // its destructor: the runtime's per-thread objects are gone by then).
    kmws_rx_batch* rb = kmws_rx_batch_create(KMWS_DEVICE_AUTO);
    kmws_decoder* dec = kmws_decoder_create(KMWS_MODE_SERVER, KMWS_DEVICE_AUTO);
    kmws_tx_batch* tb = kmws_tx_batch_create(KMWS_DEVICE_AUTO);
    RawHolder& r = raw_holder();  // before any resident job: no exit hook yet
    r.o = o;
    r.rb = rb;
    r.dec = dec;
    r.tb = tb;
    if (!r.rb || !r.dec || !r.tb) {
        o->err = 10;
        return;
    }
    r.tx_bufs.reserve(kFrames);  // stable addresses: the batch masks them in place
    for (int i = 0; i < kFrames; ++i) {
        const std::string& w = o->rx_in[(size_t)i].wire;
        if (kmws_decoder_feed_deferred(r.dec, r.rb, reinterpret_cast<const uint8_t*>(w.data()), w.size(), on_frame_raw,
                                       o) != 0)
            o->err = 13;
        const Frame& f = o->tx_in[(size_t)i];
        kmws_frame_hdr hdr;
        std::memset(&hdr, 0, sizeof hdr);
        hdr.fin = 1;
        hdr.opcode = KMWS_OP_BINARY;
        hdr.mask = 1;
        std::memcpy(hdr.maskey, &f.key, 4);
        r.tx_bufs.push_back(f.payload);
        uint8_t* seg = reinterpret_cast<uint8_t*>(&r.tx_bufs.back()[0]);
        size_t len = f.payload.size();
        uint8_t hb[KMWS_MAX_HEADER_SIZE];
        const int hl = kmws_tx_batch_add(r.tb, &hdr, &seg, &len, 1, hb);
        if (hl < 0) o->err = 14;
        r.tx_hdrs.emplace_back(reinterpret_cast<const char*>(hb), hl > 0 ? (size_t)hl : 0);
        if (i == kFrames / 2) {  // asynchronous submits: the thread's first resident jobs (claims the slot)
            if (kmws_rx_batch_submit(r.rb) < 0 || kmws_tx_batch_submit(r.tb) < 0) o->err = 15;
        }
    }
    o->rx_pending_at_exit = kmws_rx_batch_pending(r.rb);
    o->rx_inflight_at_exit = kmws_rx_batch_inflight(r.rb);
    o->tx_pending_at_exit = kmws_tx_batch_pending(r.tb);
}

bool check(const Out& o, std::string* why)
{
    if (o.err) {
        *why = "error " + std::to_string(o.err);
        return false;
    }
    if (o.rx_got.size() != o.rx_in.size()) {
        *why = "rx frames " + std::to_string(o.rx_got.size());
        return false;
    }
    std::string want;
    for (size_t i = 0; i < o.rx_in.size(); ++i) {
        if (o.rx_got[i] != o.rx_in[i].payload) {
            *why = "rx payload " + std::to_string(i);
            return false;
        }
        want += o.tx_in[i].wire;
    }
    if (o.tx_wire != want) {
        *why = "tx bytes";
        return false;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 20;
    const int exiters = argc > 2 ? std::atoi(argv[2]) : 8;
    const int maskers = argc > 3 ? std::atoi(argv[3]) : 8;
    const std::string kinds = argc > 4 ? argv[4] : "both";
    if (kmws_device_count() < 1) {
        std::printf("{\"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    std::atomic<bool> stop{false};
    std::atomic<long> masks{0}, mask_bad{0}, masker_threads{0};
    std::vector<std::thread> mk;
    for (int m = 0; m < maskers; ++m)
        mk.emplace_back([&, m] {
            for (uint64_t gen = 0; !stop.load(std::memory_order_acquire); ++gen) {
                std::thread t([&, m, gen] {  // a short-lived thread: claims a slot, masks, exits
                    std::vector<uint8_t> a(4096), b;
                    for (int i = 0; i < 40; ++i) {
                        for (size_t j = 0; j < a.size(); ++j) a[j] = (uint8_t)mix((uint64_t)m * 131 + gen * 7 + (uint64_t)i + j);
                        b = a;
                        const uint32_t k32 = (uint32_t)mix(gen * 977 + (uint64_t)i + (uint64_t)m);
                        uint8_t key[4];
                        std::memcpy(key, &k32, 4);
                        uint8_t* seg = a.data();
                        size_t len = a.size();
                        if (kmws_mask_host_chain(key, &seg, &len, 1, KMWS_DEVICE_AUTO) != KMWS_OK) ++mask_bad;
                        orc_mask(key, b.data(), b.size(), 0);
                        if (a != b) ++mask_bad;
                        ++masks;
                    }
                });
                t.join();
                ++masker_threads;
            }
        });
    long bad = 0, exited = 0, loop_ex = 0, raw_ex = 0;
    long rx_pending = 0, rx_inflight = 0, tx_pending = 0, tx_inflight = 0;
    std::string first_why;
    for (int r = 0; r < rounds; ++r) {
        std::vector<Out> outs((size_t)exiters);
        for (int e = 0; e < exiters; ++e) gen_frames(&outs[(size_t)e], (uint64_t)r * 64 + (uint64_t)e + 1);
        std::vector<std::thread> th;
        for (int e = 0; e < exiters; ++e) {
            Out* o = &outs[(size_t)e];
            const bool loop = kinds == "loop" || (kinds == "both" && e % 2 == 0);
            if (loop) th.emplace_back([o] { loop_exiter(o); });
            else th.emplace_back([o] { raw_exiter(o); });
        }
        for (auto& t : th) t.join();
        for (int e = 0; e < exiters; ++e) {
            const Out& o = outs[(size_t)e];
            std::string why;
            if (!check(o, &why)) {
                ++bad;
                if (first_why.empty()) first_why = "round " + std::to_string(r) + " thread " + std::to_string(e) + ": " + why;
            }
            ++exited;
            ((kinds == "loop" || (kinds == "both" && e % 2 == 0)) ? loop_ex : raw_ex)++;
            rx_pending += o.rx_pending_at_exit;
            rx_inflight += o.rx_inflight_at_exit;
            tx_pending += o.tx_pending_at_exit;
            tx_inflight += o.tx_inflight_at_exit;
        }
    }
    stop.store(true, std::memory_order_release);
    for (auto& t : mk) t.join();
    uint64_t unowned = 0, late = 0, drained = 0;
    kmws_resident_guard_counters(0, &unowned, &late, &drained);
    uint64_t jobs = 0, launches = 0;
    kmws_resident_info(0, &jobs, &launches, nullptr);
    const bool ok = bad == 0 && mask_bad == 0 && unowned == 0;
    std::printf("{\"rounds\": %d, \"exited_threads\": %ld, \"loop_threads\": %ld, \"raw_threads\": %ld, "
                "\"frames_queued_at_exit\": {\"rx_pending\": %ld, \"rx_inflight_generations\": %ld, "
                "\"tx_pending\": %ld, \"tx_inflight_generations\": %ld}, "
                "\"masker_threads\": %ld, \"masks\": %ld, \"mask_bad\": %ld, \"bad_threads\": %ld, "
                "\"unowned_posts\": %llu, \"late_posts\": %llu, \"drained_releases\": %llu, "
                "\"resident_jobs\": %llu, \"grid_launches\": %llu, \"first_failure\": \"%s\", \"exact\": %s}\n",
                rounds, exited, loop_ex, raw_ex, rx_pending, rx_inflight, tx_pending, tx_inflight,
                masker_threads.load(), masks.load(), mask_bad.load(), bad, (unsigned long long)unowned,
                (unsigned long long)late, (unsigned long long)drained, (unsigned long long)jobs,
                (unsigned long long)launches, first_why.c_str(), ok ? "true" : "false");
    return ok ? 0 : 1;
}
