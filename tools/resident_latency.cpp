// Where a synchronous resident job's time goes (diagnostic; links the timing
// variant, tools/patches/resident_job_timestamps.patch, which stamps part 0's
// wall clock -- 100 MHz, s_memrealtime -- when it notices a job, when its
// descriptors are ready, and just before it writes done).  For 1 / 4 / 64 KiB
// handleDataMask calls on one thread: the call's host time, the two memcpys
// the call does (staging in and out, timed alone), and the device's notice ->
// descriptors -> done intervals; what is left is noticing the job (a poll
// round trip after the post) and the host seeing done (the release's write
// crossing PCIe, then the host's spin).  Medians over 2,000 calls.
//
// build: g++ -O2 -I include tools/resident_latency.cpp -L <variant dir> -lkmws_gpu -lpthread
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "kmws_gpu.h"

extern "C" kmws_status kmws_resident_debug_times(int device, uint64_t* out3);

namespace {
using Clock = std::chrono::steady_clock;
double us(Clock::duration d) { return std::chrono::duration<double, std::micro>(d).count(); }
double med(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}
}  // namespace

int main()
{
    if (kmws_device_count() < 1) return 1;
    for (size_t len : {(size_t)1024, (size_t)4096, (size_t)65536}) {
        std::vector<uint8_t> buf(len, 0x5a), stage(len);
        const uint8_t key[4] = {1, 2, 3, 4};
        for (int i = 0; i < 200; ++i) kmws_mask_host_chain(key, std::vector<uint8_t*>{buf.data()}.data(), &len, 1, 0);
        std::vector<double> call, copies, notice_ready, ready_done;
        for (int i = 0; i < 2000; ++i) {
            uint8_t* seg = buf.data();
            const auto t0 = Clock::now();
            if (kmws_mask_host_chain(key, &seg, &len, 1, 0) != KMWS_OK) return 2;
            const auto t1 = Clock::now();
            uint64_t d[3] = {};
            if (kmws_resident_debug_times(0, d) != KMWS_OK) return 3;
            call.push_back(us(t1 - t0));
            notice_ready.push_back((double)(d[1] - d[0]) / 100.0);
            ready_done.push_back((double)(d[2] - d[1]) / 100.0);
            const auto c0 = Clock::now();  // the call's two copies, alone
            std::memcpy(stage.data(), buf.data(), len);
            std::memcpy(buf.data(), stage.data(), len);
            copies.push_back(us(Clock::now() - c0));
        }
        const double c = med(call), cp = med(copies), nr = med(notice_ready), rd = med(ready_done);
        std::printf("{\"len\": %zu, \"us_call\": %.3f, \"us_host_copies\": %.3f, \"us_device_notice_to_descs\": %.3f, "
                    "\"us_device_descs_to_done\": %.3f, \"us_rest_notice_and_done_signal\": %.3f}\n",
                    len, c, cp, nr, rd, c - cp - nr - rd);
        std::fflush(stdout);
    }
    return 0;
}
