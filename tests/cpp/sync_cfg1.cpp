// The synchronous drop-in against kuma's codec, in
// process, on kuma's own call pattern:
//
//   decode  BASELINE configs[0]'s stream (1,000 x 4 KiB masked TEXT frames)
//           fed in 64 KiB reads from a pageable read buffer, one call per read
//           (TcpConnection.cpp:229-233 -> WebSocketImpl.cpp:225-246):
//             kuma    the oracle's restatement of WSHandler::handleData;
//             kmws    kmws::ws::WSHandler::handleData (kmws_decoder_feed) with
//                     the thread's resident worker (no launch per read);
//             views   the same, payloads delivered as views of the unmasked
//                     staging copy (kmws_decoder_set_in_place(0)): no copy back;
//             launch  the resident form with the worker switched off (a kernel
//                     launch and an event wait per read: round 3's form).
//   decode_sync_threads  the same decode on T = 1, 2, 4, 8 loop threads at
//           once (kuma runs 5-10 loop threads, test/server/main.cpp:22,
//           test/client/main.cpp:20), each with its own handler and read
//           buffer, `passes` passes of the stream each; aggregate GiB/s over
//           the wall time of all threads (the copy of each read into the
//           buffer is timed here, for every codec alike).  The resident form
//           gives each thread its own slot of the device's resident grid.
//   mask    WSHandler::handleDataMask(key, data, len) once per send
//           (WebSocketImpl.cpp:388), 1 KiB, 4 KiB and 64 KiB payloads in a
//           pageable buffer: the oracle's byte loop vs
//           kmws::ws::WSHandler::handleDataMask (resident worker / launch).
//   mask_sync_threads  handleDataMask of 4 KiB on T = 1, 2, 4, 8, 16 threads at
//           once (a slot each), `calls` calls per thread: the per-call median
//           and 99th percentile over every thread, and the aggregate calls/s;
//           with "idle": one thread masks while T - 1 others hold slots of the
//           grid without jobs (what the other slots' polling costs one job).
//
// Only the codec call is timed (the copy of the next read into the buffer,
// standing in for recv, is not); best of `reps` passes.  Every decoded payload
// and every masked buffer is checked.  One JSON line per case.  Test
// infrastructure (links the oracle): tests/test_abi_build.py, tools/bench_configs.py.
//
// usage: sync_cfg1 [reps] [only: mask_threads]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
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
typedef struct orc_decoder orc_decoder;
typedef int (*orc_frame_cb)(const orc_hdr* hdr, const uint8_t* payload, size_t len, void* user);
void orc_mask(const uint8_t key[4], uint8_t* data, size_t len, size_t phase);
int orc_encode_header(const orc_hdr* h, uint8_t out[14]);
orc_decoder* orc_decoder_create(int mode);
void orc_decoder_destroy(orc_decoder* d);
int orc_decoder_feed(orc_decoder* d, uint8_t* data, size_t len, orc_frame_cb cb, void* user);
}

namespace {

constexpr int kFrames = 1000;
constexpr size_t kLen = 4096;
constexpr size_t kRead = 64 * 1024;  // TcpConnection.cpp:229

uint64_t splitmix(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

using Clock = std::chrono::steady_clock;
double secs(Clock::duration d) { return std::chrono::duration<double>(d).count(); }

struct Check {
    const std::vector<uint8_t>* plain;
    int got = 0, bad = 0;
    void frame(const uint8_t* p, size_t len)  // frame got % kFrames of a pass
    {
        const size_t k = (size_t)(got % kFrames);
        if (len != kLen || std::memcmp(p, plain->data() + k * kLen, kLen) != 0) ++bad;
        ++got;
    }
};

int orc_cb(const orc_hdr*, const uint8_t* p, size_t len, void* user)
{
    static_cast<Check*>(user)->frame(p, len);
    return 0;
}

// Feeds the wire in 64 KiB reads; returns the best total seconds of the feed calls.
// pinned: the read buffer is pinned host memory (kmws_host_alloc) -- the
// in-chunk zero-copy path, no staging copies -- instead of pageable memory.
template <class Feed>
double time_decode(const std::vector<uint8_t>& wire, int reps, Feed&& feed, bool pinned = false)
{
    std::vector<uint8_t> vbuf(pinned ? 0 : kRead);  // the loop's read buffer (pageable, as kuma's stack buffer)
    uint8_t* pbuf = pinned ? static_cast<uint8_t*>(kmws_host_alloc(kRead, 0)) : nullptr;
    struct Span {
        uint8_t* p;
        uint8_t* data() { return p; }
    } buf{pinned ? pbuf : vbuf.data()};
    if (pinned && !pbuf) std::exit(3);
    double best = 1e30;
    for (int r = 0; r <= reps; ++r) {
        double t = 0;
        for (size_t i = 0; i < wire.size(); i += kRead) {
            const size_t n = std::min(kRead, wire.size() - i);
            std::memcpy(buf.data(), wire.data() + i, n);  // recv (untimed)
            const auto t0 = Clock::now();
            feed(buf.data(), n);
            t += secs(Clock::now() - t0);
        }
        if (r) best = std::min(best, t);  // pass 0 warms up (staging growth, worker launch)
    }
    if (pbuf) kmws_host_free(pbuf);
    return best;
}

void emit_decode(const char* codec, double t, size_t reads, const Check& c, int reps)
{
    std::printf("{\"case\": \"decode_sync\", \"codec\": \"%s\", \"frames\": %d, \"frame_len\": %zu, "
                "\"read_bytes\": %zu, \"reads\": %zu, \"best_of\": %d, \"GiB_s\": %.3f, \"us_per_read\": %.3f, "
                "\"verified\": %s}\n",
                codec, kFrames, kLen, kRead, reads, reps, (double)kFrames * kLen / t / (1u << 30), t / reads * 1e6,
                c.bad == 0 && c.got == kFrames * (reps + 1) ? "true" : "false");
}

// T threads, each: make(tid) -> a feed function (created on that thread, so a
// handler's resident slot belongs to it); one untimed warm-up pass, then
// `passes` passes of the wire in 64 KiB reads.  Returns wall seconds from the
// common start to the last thread's end.
double time_threads(int T, int passes, const std::vector<uint8_t>& wire,
                    const std::function<std::function<void(uint8_t*, size_t)>(int)>& make)
{
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::function<void(uint8_t*, size_t)> feed = make(t);
            std::vector<uint8_t> buf(kRead);
            auto pass = [&] {
                for (size_t i = 0; i < wire.size(); i += kRead) {
                    const size_t n = std::min(kRead, wire.size() - i);
                    std::memcpy(buf.data(), wire.data() + i, n);  // recv
                    feed(buf.data(), n);
                }
            };
            pass();
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (int p = 0; p < passes; ++p) pass();
        });
    while (ready.load() < T) std::this_thread::yield();
    const auto t0 = Clock::now();
    go.store(true, std::memory_order_release);
    for (auto& x : th) x.join();
    return secs(Clock::now() - t0);
}

// T threads masking `len` bytes per call with the drop-in's static handleDataMask
// (each thread its slot); active = how many of them mask (the others only hold a
// slot: one call, then they wait at the end).  Prints one JSON line; false on a
// wrong result.
bool mask_threads(int T, int active, size_t len, int calls)
{
    std::atomic<int> ready{0}, done{0};
    std::atomic<bool> go{false};
    std::vector<std::vector<double>> lat(T);
    std::vector<int> slot(T, -1);
    std::atomic<int> bad{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            std::vector<uint8_t> src(len), buf(len);
            for (size_t i = 0; i < len; ++i) src[i] = (uint8_t)splitmix(len * 131 + t * 7 + i);
            const uint8_t key[4] = {(uint8_t)(0x37 + t), 0xfa, 0x21, 0x3d};
            std::vector<uint8_t> want = src;
            orc_mask(key, want.data(), len, 0);
            buf = src;
            if (kmws::ws::WSHandler::handleDataMask(key, buf.data(), len) != KMWS_OK || buf != want) bad.fetch_add(1);
            buf = src;
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            if (t < active) {
                lat[t].reserve(calls);
                for (int i = 0; i < calls; ++i) {
                    const auto t0 = Clock::now();
                    kmws::ws::WSHandler::handleDataMask(key, buf.data(), len);
                    lat[t].push_back(secs(Clock::now() - t0));
                }
                if (buf != (calls % 2 ? want : src)) bad.fetch_add(1);
                kmws_resident_counters(0, &slot[t], nullptr, nullptr, nullptr);
                done.fetch_add(1);
            } else {  // holds its slot idle until the maskers are done
                while (done.load() < active) std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
        });
    while (ready.load() < T) std::this_thread::yield();
    uint64_t jobs0 = 0, jobs1 = 0, inc0 = 0, inc1 = 0, why0[5] = {}, why1[5] = {};
    kmws_resident_info(0, &jobs0, &inc0, nullptr);
    kmws_resident_exit_reasons(0, why0, 5);
    const auto t0 = Clock::now();
    go.store(true, std::memory_order_release);
    while (done.load() < active) std::this_thread::yield();
    kmws_resident_info(0, &jobs1, &inc1, nullptr);
    kmws_resident_exit_reasons(0, why1, 5);
    const double wall = secs(Clock::now() - t0);
    for (auto& x : th) x.join();
    std::vector<double> all;
    std::string per = "[";  // [slot, median us] per masking thread
    for (int t = 0; t < active; ++t) {
        std::vector<double> v = lat[t];
        std::sort(v.begin(), v.end());
        char b[48];
        std::snprintf(b, sizeof b, "%s[%d, %.2f]", t ? ", " : "", slot[t], v[v.size() / 2] * 1e6);
        per += b;
    }
    per += "]";
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    std::printf("{\"case\": \"mask_sync_threads\", \"codec\": \"kmws_resident\", \"threads\": %d, \"masking\": %d, "
                "\"len\": %zu, \"calls_per_thread\": %d, \"us_median\": %.3f, \"us_p99\": %.3f, "
                "\"calls_per_s\": %.0f, \"resident_jobs\": %llu, \"incarnations\": %llu, \"slot_median_us\": %s, "
                "\"exits_lease_closing_resize_idle_quit\": [%llu, %llu, %llu, %llu, %llu], \"verified\": %s}\n",
                T, active, len, calls, all[all.size() / 2] * 1e6, all[all.size() * 99 / 100] * 1e6,
                (double)active * calls / wall, (unsigned long long)(jobs1 - jobs0), (unsigned long long)(inc1 - inc0),
                per.c_str(), (unsigned long long)(why1[0] - why0[0]), (unsigned long long)(why1[1] - why0[1]),
                (unsigned long long)(why1[2] - why0[2]), (unsigned long long)(why1[3] - why0[3]),
                (unsigned long long)(why1[4] - why0[4]), bad.load() == 0 ? "true" : "false");
    std::fflush(stdout);
    return bad.load() == 0;
}

}  // namespace

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? std::max(1, std::atoi(argv[1])) : 10;
    if (kmws_device_count() < 1) {
        std::printf("{\"error\": \"no gfx950 device\"}\n");
        return 1;
    }
    if (argc > 2 && std::string(argv[2]) == "mask_threads") {
        bool ok = true;
        for (int T : {1, 2, 4, 8, 16}) ok &= mask_threads(T, T, 4096, 2000);
        for (int T : {2, 4, 8, 16}) ok &= mask_threads(T, 1, 4096, 2000);
        for (int T : {1, 4, 16}) ok &= mask_threads(T, T, 65536, 500);
        return ok ? 0 : 1;
    }
    // the cfg1 wire: n x (81 fe 10 00 <key>) + payload ^ key
    std::vector<uint8_t> plain((size_t)kFrames * kLen), wire;
    for (size_t i = 0; i < plain.size(); ++i) plain[i] = (uint8_t)(0x20 + splitmix(i) % 95);
    for (int f = 0; f < kFrames; ++f) {
        orc_hdr h;
        std::memset(&h, 0, sizeof h);
        h.fin = 1;
        h.opcode = 1;
        h.mask = 1;
        h.length = (uint32_t)kLen;
        const uint32_t key = (uint32_t)splitmix(0x6b756d61ull + f);
        std::memcpy(h.maskey, &key, 4);
        uint8_t hb[14];
        const int hl = orc_encode_header(&h, hb);
        wire.insert(wire.end(), hb, hb + hl);
        const size_t p0 = wire.size();
        wire.insert(wire.end(), plain.begin() + (size_t)f * kLen, plain.begin() + (size_t)(f + 1) * kLen);
        orc_mask(h.maskey, wire.data() + p0, kLen, 0);
    }
    const size_t reads = (wire.size() + kRead - 1) / kRead;
    bool ok = true;

    {  // kuma's decoder (oracle restatement), SERVER mode
        Check c{&plain};
        orc_decoder* d = orc_decoder_create(1);
        const double t = time_decode(wire, reps, [&](uint8_t* p, size_t n) { orc_decoder_feed(d, p, n, orc_cb, &c); });
        orc_decoder_destroy(d);
        emit_decode("kuma_oracle", t, reads, c, reps);
        ok &= c.bad == 0 && c.got == kFrames * (reps + 1);
    }
    for (const char* codec : {"kmws_resident", "kmws_resident_views", "kmws_resident_pinned_read_buffer", "kmws_launch"}) {  // the drop-in, synchronous
        const bool resident = std::string(codec) != "kmws_launch";
        const bool pinned = std::string(codec) == "kmws_resident_pinned_read_buffer";
        kmws_resident_enable(0, resident ? 1 : 0);
        Check c{&plain};
        kmws::ws::WSHandler h;
        h.setMode(kmws::ws::WSMode::SERVER);
        h.setInPlace(std::string(codec) != "kmws_resident_views");
        h.setFrameCallback([&](kmws::ws::FrameHeader, kmws::ws::BufferChain& b) {
            c.frame(static_cast<const uint8_t*>(b.readPtr()), b.length());
            return 0;
        });
        uint64_t jobs0 = 0, jobs1 = 0;
        kmws_resident_info(0, &jobs0, nullptr, nullptr);
        const double t = time_decode(wire, reps, [&](uint8_t* p, size_t n) {
            const kmws::ws::WSError e = h.handleData(p, n);
            if (e != kmws::ws::WSError::NOERR && e != kmws::ws::WSError::NEED_MORE_DATA) std::exit(4);
        }, pinned);
        kmws_resident_info(0, &jobs1, nullptr, nullptr);
        emit_decode(codec, t, reads, c, reps);
        ok &= c.bad == 0 && c.got == kFrames * (reps + 1) && (resident ? jobs1 > jobs0 : jobs1 == jobs0);
    }
    kmws_resident_enable(0, 1);

    // the decode on T loop threads at once
    const int passes = std::max(2, reps);
    for (const char* codec : {"kuma_oracle", "kmws_resident", "kmws_launch"}) {
        for (int T : {1, 2, 4, 8}) {
            std::vector<Check> checks(T, Check{&plain});
            std::vector<std::unique_ptr<kmws::ws::WSHandler>> hs(T);
            std::vector<orc_decoder*> ods(T, nullptr);
            const std::string c = codec;
            uint64_t jobs0 = 0, jobs1 = 0;
            kmws_resident_info(0, &jobs0, nullptr, nullptr);
            const double t = time_threads(T, passes, wire, [&](int tid) -> std::function<void(uint8_t*, size_t)> {
                Check* ck = &checks[tid];
                if (c == "kuma_oracle") {
                    ods[tid] = orc_decoder_create(1);
                    orc_decoder* d = ods[tid];
                    return [d, ck](uint8_t* p, size_t n) { orc_decoder_feed(d, p, n, orc_cb, ck); };
                }
                kmws_resident_enable(0, c == "kmws_resident" ? 1 : 0);  // this thread's calls
                hs[tid].reset(new kmws::ws::WSHandler());
                kmws::ws::WSHandler* h = hs[tid].get();
                h->setMode(kmws::ws::WSMode::SERVER);
                h->setFrameCallback([ck](kmws::ws::FrameHeader, kmws::ws::BufferChain& b) {
                    ck->frame(static_cast<const uint8_t*>(b.readPtr()), b.length());
                    return 0;
                });
                return [h](uint8_t* p, size_t n) {
                    const kmws::ws::WSError e = h->handleData(p, n);
                    if (e != kmws::ws::WSError::NOERR && e != kmws::ws::WSError::NEED_MORE_DATA) std::exit(4);
                };
            });
            kmws_resident_info(0, &jobs1, nullptr, nullptr);
            bool exact = true;
            for (const Check& ck : checks) exact &= ck.bad == 0 && ck.got == kFrames * (passes + 1);
            for (orc_decoder* d : ods)
                if (d) orc_decoder_destroy(d);
            hs.clear();
            const bool resident = c == "kmws_resident";
            exact &= c == "kuma_oracle" || (resident ? jobs1 > jobs0 : jobs1 == jobs0);
            ok &= exact;
            const double bytes = (double)kFrames * kLen * passes * T;
            std::printf("{\"case\": \"decode_sync_threads\", \"codec\": \"%s\", \"threads\": %d, \"passes\": %d, "
                        "\"frames_per_pass\": %d, \"read_bytes\": %zu, \"GiB_s\": %.3f, \"us_per_read_per_thread\": %.3f, "
                        "\"resident_jobs\": %llu, \"verified\": %s}\n",
                        codec, T, passes, kFrames, kRead, bytes / t / (1u << 30),
                        t / ((double)reads * passes) * 1e6, (unsigned long long)(jobs1 - jobs0), exact ? "true" : "false");
            std::fflush(stdout);
        }
    }

    // handleDataMask per send
    for (size_t len : {(size_t)1024, (size_t)4096, (size_t)65536}) {
        std::vector<uint8_t> src(len), buf(len), want(len);
        for (size_t i = 0; i < len; ++i) src[i] = (uint8_t)splitmix(len + i);
        const uint8_t key[4] = {0x37, 0xfa, 0x21, 0x3d};
        want = src;
        orc_mask(key, want.data(), len, 0);
        const int calls = (int)std::max<size_t>(64, (8u << 20) / len) & ~1;  // even: the buffer ends unmasked
        struct Leg {
            const char* codec;
            int mode;  // 0 oracle, 1 resident, 2 launch
        };
        for (Leg g : {Leg{"kuma_oracle", 0}, Leg{"kmws_resident", 1}, Leg{"kmws_launch", 2}}) {
            if (g.mode) kmws_resident_enable(0, g.mode == 1 ? 1 : 0);
            buf = src;
            bool exact = true;
            if (g.mode == 0) orc_mask(key, buf.data(), len, 0);
            else exact &= kmws::ws::WSHandler::handleDataMask(key, buf.data(), len) == KMWS_OK;
            exact &= buf == want;
            if (g.mode == 0) orc_mask(key, buf.data(), len, 0);
            else exact &= kmws::ws::WSHandler::handleDataMask(key, buf.data(), len) == KMWS_OK;
            double best = 1e30;
            for (int r = 0; r < 3; ++r) {
                const auto t0 = Clock::now();
                for (int i = 0; i < calls; ++i) {
                    if (g.mode == 0) orc_mask(key, buf.data(), len, 0);
                    else kmws::ws::WSHandler::handleDataMask(key, buf.data(), len);
                }
                best = std::min(best, secs(Clock::now() - t0));
            }
            exact &= buf == src;
            ok &= exact;
            std::printf("{\"case\": \"mask_sync\", \"codec\": \"%s\", \"len\": %zu, \"calls\": %d, \"best_of\": 3, "
                        "\"us_per_call\": %.3f, \"GiB_s\": %.3f, \"verified\": %s}\n",
                        g.codec, len, calls, best / calls * 1e6, (double)len * calls / best / (1u << 30),
                        exact ? "true" : "false");
        }
        kmws_resident_enable(0, 1);
    }
    return ok ? 0 : 1;
}
