// Shared device helpers for the kmws kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "kmws_gpu.h"

namespace kmws {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;          // 4 waves of 64 lanes

// First 16 bytes of every workspace: status word, zeroed by a kernel (not a memset node: see launch_zero) at the
// start of each batch call.
struct WsHead {
    uint32_t status;
    uint32_t pad[3];
};
constexpr uint32_t kStatusBadDesc = 1u;
constexpr uint32_t kStatusBadHeader = 2u;
constexpr uint32_t kStatusLookbackTimeout = 4u;  // a scan predecessor never published: outputs invalid

__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Mask word for an aligned dword whose first byte sits at (address - frame
// start) == -o (mod 4): byte j of the dword takes key byte (j - o) & 3, i.e.
// rotl32(key, 8*(o & 3)) with key = LE u32 of the wire key bytes.
__device__ __forceinline__ uint32_t rot_key(uint32_t key, uint64_t frame_off)
{
    return __builtin_rotateleft32(key, (uint32_t)(frame_off & 3u) * 8u);
}

// Byte-select mask for bytes [lo, hi) of dword d (0..3) of a 16-byte word.
__device__ __forceinline__ uint32_t dword_byte_mask(int lo, int hi, int d)
{
    int a = lo - 4 * d, b = hi - 4 * d;
    a = a < 0 ? 0 : a;
    b = b > 4 ? 4 : b;
    if (b <= a) return 0u;
    uint32_t hm = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
    uint32_t lm = (1u << (8 * a)) - 1u;
    return hm & ~lm;
}

// Bytes [lo, hi) of a 16-byte word as a lane mask, 0 <= lo, hi <= 16 (empty when
// hi <= lo): two 64-bit halves, a shift and a select each, no branches.
__device__ __forceinline__ uint64_t low_bytes64(int k)  // bytes [0, k) of 8, 0 <= k <= 8
{
    return k >= 8 ? ~0ull : ((1ull << (8 * k)) - 1ull);
}
__device__ __forceinline__ u32x4 word_byte_range(int lo, int hi)
{
    const int l0 = lo < 8 ? lo : 8, h0 = hi < 8 ? hi : 8;
    const int l1 = lo > 8 ? lo - 8 : 0, h1 = hi > 8 ? hi - 8 : 0;
    const uint64_t a = low_bytes64(h0) & ~low_bytes64(l0);
    const uint64_t b = low_bytes64(h1) & ~low_bytes64(l1);
    return u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
}

inline kmws_status hip_status(hipError_t e)
{
    return e == hipSuccess ? KMWS_OK : KMWS_ERR_FAILED;
}

// Zeroes `bytes` (a multiple of 8, at most 4 KiB) at an 8-byte aligned device
// address with one small kernel.  Used instead of hipMemsetAsync for the status
// word and scan totals: a call captured into a HIP graph then holds kernel nodes
// only (replayed memset nodes of this runtime were seen writing a pointer value
// instead of zero when the graph was replayed after other work on the device).
kmws_status launch_zero(void* p, uint32_t bytes, hipStream_t s);

// Small host batches (the decoder's staging, kmws_unmask.hip): one block per
// piece of at most kPieceWords 16-byte words of one frame's aligned hull.
constexpr uint32_t kPieceWords = 4 * kBlock;  // 16 KiB
struct PieceRec {
    uint32_t frame;  // index into the descriptor list
    uint32_t piece;  // piece of that frame's hull
};
// Pieces of a payload at byte offset `off`, `len` bytes (0 for an empty one).
inline uint64_t piece_count(uint64_t off, uint32_t len)
{
    if (len == 0) return 0;
    const uint64_t words = ((off + len + 15) >> 4) - (off >> 4);
    return (words + kPieceWords - 1) / kPieceWords;
}
// Unmasks the payloads of descs[] (device-visible, sorted or not, disjoint)
// in base[] with one launch over the np pieces; no plan, no validation (the
// caller produced the descriptors).
kmws_status launch_unmask_pieces(uint8_t* base, const kmws_desc* descs, const PieceRec* pieces, uint32_t np,
                                 hipStream_t s);

// KMWS_DEVICE_AUTO -> the calling thread's device (kmws_devmap.cpp; negative
// without a gfx950 device); any other value unchanged.
int resolve_device(int device);
// A device batch (an HBM-resident kernel over `bytes` of traffic) was just
// enqueued on `stream` (its device; the current device for the null stream):
// until about when it should
// have finished (queued batches add up), the resident grid on that device
// stores large jobs write-through instead of releasing the L2 once per job
// (kmws_resident.hip: kResWriteThroughWords).
void note_device_batch(uint64_t bytes, hipStream_t stream);
bool device_batch_running(int device);

// Resident worker (kmws_resident.hip): host jobs of at most kResMaxDescs
// payloads and kResMaxBytes bytes go to the calling thread's slot of a grid
// that stays on the GPU polling pinned memory, instead of a launch per call.
constexpr int kResMaxDescs = KMWS_RESIDENT_MAX_PAYLOADS;
// A job runs on up to four workgroups of its slot (one per 16 KiB of hull
// words): 256 KiB take ~11 us on the device (tools/zc_probe.hip), a launch of
// the pieces kernel alone ~20 us.  Synchronous (a flush, a feed, a mask) and
// asynchronous jobs (an rx / tx batch's submit) alike.
constexpr uint64_t kResMaxBytes = KMWS_RESIDENT_MAX_BYTES;
constexpr uint64_t kResMaxBytesAsync = kResMaxBytes;
struct ResidentJob {
    int device = -1;
    int slot = -1;
    uint64_t seq = 0;
};
// Posts the unmask of descs[0..n) over dev_base and descs2[0..n2) over
// dev_base2 (device views of pinned host memory, offsets relative to them) on
// the calling thread's slot and returns at once.  KMWS_ERR_NOT_SUPPORTED
// (nothing posted): too large for one job, no slot free, the thread switched
// the worker off, its slot still runs a job, or the worker is unusable -- the
// caller launches instead.
kmws_status resident_post(int device, const kmws_desc* descs, const uint8_t* dev_base, size_t n,
                          const kmws_desc* descs2, const uint8_t* dev_base2, size_t n2, ResidentJob* job,
                          uint64_t max_bytes = kResMaxBytes);
// 1: done; 0: running; KMWS_ERR_NOT_SUPPORTED: withdrawn, never run (launch it).
int resident_test(const ResidentJob& job);
// KMWS_OK: done.  KMWS_ERR_NOT_SUPPORTED: withdrawn, never run (launch it).
// KMWS_ERR_TIMEOUT: neither finished nor abandoned in time -- the device may
// still write the payloads, so their memory must not be reused.
kmws_status resident_wait(const ResidentJob& job);
// post + wait.
kmws_status resident_unmask(int device, const kmws_desc* descs, const uint8_t* dev_base, size_t n,
                            const kmws_desc* descs2, const uint8_t* dev_base2, size_t n2);

}  // namespace kmws
