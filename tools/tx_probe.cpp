// Dev probe: kmws_tx_batch_flush cost over a pinned send ring (kmws_host_alloc),
// one thread, with the payload rewritten by the CPU before each flush or not.
// build: g++ -std=c++17 -O2 -I include tools/tx_probe.cpp -L kuma_amd/lib -lkmws_gpu -Wl,-rpath,$PWD/kuma_amd/lib
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "kmws_gpu.h"

int main()
{
    const size_t L = 4096;
    for (int frames : {16, 250, 1000}) {
        for (int touch = 0; touch < 2; ++touch) {
            kmws_tx_batch* tx = kmws_tx_batch_create(0);
            uint8_t* ring = static_cast<uint8_t*>(kmws_host_alloc(frames * L, 0));
            std::vector<uint8_t> src(frames * L, 0x41);
            if (!tx || !ring || kmws_tx_batch_attach_ring(tx, ring, frames * L) != KMWS_OK) return 1;
            double best = 1e9;
            for (int rep = 0; rep < 20; ++rep) {
                if (touch) std::memcpy(ring, src.data(), frames * L);
                auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < frames; ++i) {
                    kmws_frame_hdr h;
                    std::memset(&h, 0, sizeof h);
                    h.fin = 1;
                    h.opcode = 1;
                    h.mask = 1;
                    h.maskey[0] = (uint8_t)i;
                    uint8_t* p = ring + (size_t)i * L;
                    size_t len = L;
                    uint8_t hb[14];
                    kmws_tx_batch_add(tx, &h, &p, &len, 1, hb);
                }
                const long r = (long)kmws_tx_batch_flush(tx);
                const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (r != frames) return 2;
                if (rep) best = t < best ? t : best;
            }
            std::printf("{\"frames\": %d, \"cpu_rewrites_payload\": %d, \"add+flush_ms\": %.4f, \"GiB_s\": %.2f}\n", frames,
                        touch, best * 1e3, frames * L / best / (1u << 30));
            kmws_tx_batch_destroy(tx);
            kmws_host_free(ring);
        }
    }
    return 0;
}
