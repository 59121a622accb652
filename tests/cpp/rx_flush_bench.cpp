// Isolated timing of one loop iteration's receive batch (no sockets, one
// thread): 16 masked 4 KiB frames in a pinned ring, fed with
// kmws_decoder_feed_deferred, then delivered by
//   flush       kmws_rx_batch_flush (submit with sync = the resident worker
//               when the job fits one, else a launch and a wait; then poll)
//   submitpoll  kmws_rx_batch_submit + kmws_rx_batch_poll(wait)
//   noresident  flush with this thread's resident worker switched off
// Prints one JSON line per mode: microseconds per iteration (median, mean).
// usage: rx_flush_bench [iterations] [frames] [frame_len]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kmws_bench.h"
#include "kmws_gpu.h"

namespace {

struct Sink {
    size_t frames = 0, bad = 0;
    const std::vector<uint8_t>* plain = nullptr;
    size_t frame_len = 0;
};

int on_frame(const kmws_frame_hdr* hdr, uint8_t* payload, size_t len, void* user)
{
    Sink* s = static_cast<Sink*>(user);
    (void)hdr;
    if (len != s->frame_len || std::memcmp(payload, s->plain->data(), len) != 0) ++s->bad;
    ++s->frames;
    return 0;
}

}  // namespace

int main(int argc, char** argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const size_t nfr = argc > 2 ? (size_t)std::atoll(argv[2]) : 16;
    const size_t L = argc > 3 ? (size_t)std::atoll(argv[3]) : 4096;
    if (kmws_device_count() <= 0) {
        std::fprintf(stderr, "no gfx950 device\n");
        return 2;
    }
    std::vector<uint8_t> plain(L);
    for (size_t i = 0; i < L; ++i) plain[i] = (uint8_t)(i * 131 + 7);
    // the masked wire: 0x82, 126, len (BE16), key, payload ^ key
    std::vector<uint8_t> wire;
    for (size_t f = 0; f < nfr; ++f) {
        const uint8_t key[4] = {(uint8_t)(0x11 + f), 0x22, (uint8_t)(0x33 ^ f), 0x44};
        const uint8_t h[8] = {0x82, 0xFE, (uint8_t)(L >> 8), (uint8_t)L, key[0], key[1], key[2], key[3]};
        wire.insert(wire.end(), h, h + 8);
        for (size_t i = 0; i < L; ++i) wire.push_back(plain[i] ^ key[i & 3]);
    }
    const size_t ring_bytes = wire.size() + 4096;
    uint8_t* ring = static_cast<uint8_t*>(kmws_host_alloc(ring_bytes, 0));
    kmws_rx_batch* b = kmws_rx_batch_create(0);
    kmws_decoder* d = kmws_decoder_create(KMWS_MODE_SERVER, 0);
    if (!ring || !b || !d || kmws_rx_batch_attach_ring(b, ring, ring_bytes) != KMWS_OK) return 3;
    Sink sink;
    sink.plain = &plain;
    sink.frame_len = L;
    const char* modes[] = {"flush", "submitpoll", "noresident", "flush", "submitpoll"};
    for (const char* mode : modes) {
        const bool nores = std::strcmp(mode, "noresident") == 0, sp = std::strcmp(mode, "submitpoll") == 0;
        kmws_resident_enable(0, nores ? 0 : 1);
        std::vector<double> us;
        sink.frames = sink.bad = 0;
        for (int it = 0; it < iters + 50; ++it) {
            std::memcpy(ring, wire.data(), wire.size());
            const auto t0 = std::chrono::steady_clock::now();
            if (kmws_decoder_feed_deferred(d, b, ring, wire.size(), on_frame, &sink) < 0) return 4;
            int r;
            if (sp) {
                r = kmws_rx_batch_submit(b);
                if (r >= 0) r = kmws_rx_batch_poll(b, 1);
            } else {
                r = kmws_rx_batch_flush(b);
            }
            if (r < 0) return 5;
            const double t = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (it >= 50) us.push_back(t);
        }
        std::sort(us.begin(), us.end());
        double mean = 0;
        for (double x : us) mean += x;
        mean /= (double)us.size();
        uint64_t jobs = 0, launches = 0;
        int running = 0;
        kmws_resident_info(0, &jobs, &launches, &running);
        std::printf("{\"mode\": \"%s\", \"frames\": %zu, \"frame_len\": %zu, \"iters\": %d, \"us_median\": %.2f, "
                    "\"us_mean\": %.2f, \"us_p90\": %.2f, \"bad\": %zu, \"delivered\": %zu, \"resident_jobs\": %llu, "
                    "\"resident_launches\": %llu}\n",
                    mode, nfr, L, iters, us[us.size() / 2], mean, us[us.size() * 9 / 10], sink.bad, sink.frames,
                    (unsigned long long)jobs, (unsigned long long)launches);
        std::fflush(stdout);
        if (sink.bad) return 6;
    }
    kmws_decoder_destroy(d);
    kmws_rx_batch_destroy(b);
    kmws_host_free(ring);
    return 0;
}
