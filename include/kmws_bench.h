/*
 * kmws_bench.h -- bench / test support entries of libkmws_gpu.so.
 *
 * Not part of the drop-in boundary (include/kmws_gpu.h): these allocate payload
 * arenas, generate synthetic batches on the device and check them there, so
 * bench.py and the GPU tests can build 64 GiB batches without host copies.
 * Same conventions as kmws_gpu.h (kmws_status returns, device pointers,
 * `void*` HIP streams).
 */
#ifndef KMWS_BENCH_H
#define KMWS_BENCH_H

#include "kmws_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- payload arenas ---- */

/* Device memory for a batch arena, physically contiguous when the device can
 * provide it (hipExtMallocWithFlags + hipDeviceMallocContiguous), else a plain
 * hipMalloc.  Where an allocation lands in HBM decides how well the unmask
 * schedule spreads its in-flight windows over the memory: contiguous arenas
 * held 81-83 % of peak, plain 64 GiB allocations 76-83 % depending on the
 * allocation.  *contiguous (optional) reports which one was
 * obtained.  Free with kmws_arena_free.  Returns NULL on failure. */
void* kmws_arena_alloc(uint64_t bytes, int device, int* contiguous);
void  kmws_arena_free(void* p, int device);

/* Placement probe for a long-lived batch region inside an arena: times in-place
 * split-4 and split-8 unmasks of `span` bytes (uniform 64 KiB probe frames, each
 * applied twice, so the arena's bytes are unchanged) at offsets 0, step, 2*step,
 * ... (offset + span <= arena_bytes) and returns the byte offset where the better
 * of the two is fastest, or a negative kmws_status.  The split schedules run 76 % or 82-85 % of HBM
 * peak depending on where the batch lies in physical HBM, which the kernel
 * cannot see (DESIGN.md sec.4 "Placement").  frac_out (optional, max_out
 * entries) receives each offset's rate as a fraction of 8 TB/s.  A setup call:
 * allocates its probe descriptors and workspace, synchronizes the stream. */
int64_t kmws_arena_place(uint8_t* arena, uint64_t arena_bytes, uint64_t span, uint64_t step, void* stream,
                         float* frac_out, uint32_t max_out);

/* ---- synthetic data + checks (bench / test support, device side) ---- */

/* base[i] for i < bytes := byte (i & 7) of splitmix64(seed + (i >> 3)). */
kmws_status kmws_fill_synthetic(uint8_t* base, uint64_t bytes, uint64_t seed, void* stream);

/* Uniform descriptors: desc i = {i*stride, len, key_i}, key_i = low 32 bits of
 * splitmix64(key_seed + i). */
kmws_status kmws_fill_uniform_descs(kmws_desc* descs, uint32_t n, uint64_t stride, uint32_t len,
                                    uint64_t key_seed, void* stream);

/* Independent byte-wise checker: counts bytes of base[0..bytes) that differ
 * from synthetic(seed) XOR (the key byte of the covering frame, if any) into
 * *mismatches (device u64, accumulated).  Descriptors must be sorted. */
kmws_status kmws_check_unmasked(const uint8_t* base, uint64_t bytes, uint64_t seed,
                                const kmws_desc* descs, uint32_t n,
                                unsigned long long* mismatches, void* stream);

/* The resident worker on `device` (kmws_resident.hip): one grid per device, up
 * to 16 mailbox slots of four workgroups each (a job's parts); a host thread
 * claims a slot at its first job and keeps it until it exits, so up to 16 loop
 * threads run their jobs at once (a thread finding no free slot launches
 * instead; an incarnation serves the slots claimed when it started).  It serves the host
 * entries' small jobs (kmws_decoder_feed, kmws_mask_host_chain, rx / tx batch
 * flushes and submits; <= 128 payloads and <= 256 KiB) without a launch per
 * call.  enable(0) makes the CALLING thread's calls launch a kernel per call
 * instead (the A/B of bench.py cfg1) and gives its slot back; info: jobs
 * served, launches (incarnations) so far, and whether it is on the GPU now (it
 * exits 200 us after the last job of any slot and after a 1 ms lease; until
 * then a device-wide synchronize such as torch.cuda.synchronize waits for
 * it); counters: the calling thread's slot (-1: none), slots held, jobs that
 * hit the timeout, jobs withdrawn unrun (and launched by their caller). */
kmws_status kmws_resident_enable(int device, int on);
kmws_status kmws_resident_info(int device, uint64_t* jobs, uint64_t* launches, int* running);
kmws_status kmws_resident_counters(int device, int* thread_slot, int* slots_claimed, uint64_t* timeouts,
                                   uint64_t* withdrawn);
/* Slot ownership guard: posts refused because the calling
 * thread did not hold the slot (never expected: 0), jobs asked for by a
 * thread after its exit hook gave its slots back (they launched), and slot
 * releases that first waited for the slot's last job (an async submit still
 * running when its thread exited or switched the worker off). */
kmws_status kmws_resident_guard_counters(int device, uint64_t* unowned_posts, uint64_t* late_posts,
                                         uint64_t* drained_releases);
/* Resident jobs posted so far by how their stores reach host memory: written
 * through (small jobs, and every job while a device batch of this library
 * runs on the device), or stored into the L2 and released once. */
kmws_status kmws_resident_store_counters(int device, uint64_t* write_through, uint64_t* released);
/* 1 while device batches enqueued through this library (kmws_unmask_*,
 * kmws_unpack_*, kmws_encode_batch, kmws_gather_unmask) are estimated to run
 * on `device` (20 us + their bytes at 6 TB/s, back to back), else 0. */
int kmws_device_batch_busy(int device);
/* Device selection (kmws_gpu.h KMWS_DEVICE_POLICY_*) as a pure function, for
 * tests: the device `policy` gives a thread on NUMA node `thread_node` (-1:
 * unknown) when the GPUs' nodes are gpu_nodes[0..ngpus) and `seq` threads
 * were placed before it on the same candidates. */
int kmws_device_policy_pick(int policy, int thread_node, const int* gpu_nodes, int ngpus, uint32_t seq);
/* NUMA node of a gfx950 device's PCIe function (sysfs; -1 unknown). */
kmws_status kmws_device_numa_node(int device, int* node);
/* Diagnostics: the worker's workgroup exits so far by reason, counts[0..n):
 * 0 its 1 ms lease ran out, 1 another workgroup found the grid idle, 2 a thread
 * claimed a slot outside the running incarnation (resize), 3 it found the grid
 * idle itself, 4 its slot's quit bit.  Reads device memory (synchronous). */
kmws_status kmws_resident_exit_reasons(int device, uint64_t* counts, int n);

#ifdef __cplusplus
}
#endif
#endif /* KMWS_BENCH_H */
