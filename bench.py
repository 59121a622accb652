#!/usr/bin/env python3
"""Headline benchmark: device-resident batched WebSocket unmask on MI355X.

Workload (BASELINE.json configs[1], SURVEY.md sec.8 d row 2): per GPU, N frames
of 64 KiB masked binary payload in an aligned HBM arena (frame i at
i * 65536) plus 16-byte descriptors {u64 off, u32 len, u32 key}; one step =
kmws_unmask_batch over the whole batch (plan kernel + unmask kernel), in
place.  Payload and keys are synthetic (counter-based splitmix64, generated
on device, untimed).  With --gpus N (torchrun, one rank per GPU) every rank
unmasks its own batch: a plain per-GPU frame partition (weak scaling), no
data-path collective; the barrier and the max-over-ranks timing use RCCL.
--job-frames J instead fixes the job (strong scaling, BASELINE configs[4]:
10,485,760 frames over 1/2/4/8 GPUs): a rank whose shard exceeds one
resident batch (--max-batch-frames, 80 GiB) runs it as sub-batches, each
generated on device untimed and timed like one batch; the step time is the
sum over sub-batches.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the formulas.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident WS frame mask/unmask, 64 KiB frames; % HBM peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak, MI355X_MICROARCH.md
DESC_BYTES = 16


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs (ranks) of this node. Without WORLD_SIZE in the environment bench.py starts the N "
                        "rank processes itself (one per GPU, before any GPU call); under torchrun WORLD_SIZE "
                        "must equal N")
    p.add_argument("--config", default="cfg2", choices=["cfg2", "cfg1", "e2e"],
                   help="cfg2 (default): the headline device-resident unmask; cfg1: kuma's CPU case "
                        "(1,000 x 4 KiB frames in 64 KiB reads) with its cpu_baseline; e2e: host-resident "
                        "frames end to end (pinned H2D -> kernel -> D2H), each rank its own shard through its "
                        "own pinned staging and kmws_pipeline (SURVEY 8 e), --e2e-gib per rank")
    p.add_argument("--cfg5-anchor", type=int, default=1,
                   help="N = 1 cfg2 run: also time BASELINE configs[4]'s whole job (cfg5_job key), the same-job "
                        "anchor of the N > 1 curve (0 = skip)")
    p.add_argument("--e2e-gib", type=float, default=4.0,
                   help="host-resident end-to-end shard per rank in GiB: the e2e_host key of a cfg2 run "
                        "(0 = skip), or the workload of --config e2e")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--frames", type=int, default=1 << 20, help="frames per GPU")
    p.add_argument("--job-frames", type=int, default=None,
                   help="strong scaling: a fixed job of this many frames split over the ranks (configs[4]: 10485760, "
                        "the default for N > 1); 0 = weak scaling, --frames per GPU (the default for N = 1: cfg2)")
    p.add_argument("--max-batch-frames", type=int, default=1310720,
                   help="largest resident batch per GPU (80 GiB of 64 KiB frames); larger shards run as sub-batches")
    p.add_argument("--frame-len", type=int, default=65536)
    p.add_argument("--schedule", type=int, default=-1,
                   help="pin an unmask schedule code (include/kmws_gpu.h KMWS_SCHED_*); -1 = autotune the batch")
    p.add_argument("--seed", type=int, default=0x6B756D61)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline budget (0 = skip)")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = the effective core count: os.sched_getaffinity capped by the cgroup CPU quota")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--no-autotune", action="store_true", help="skip kmws_unmask_autotune (keep the default schedule)")
    p.add_argument("--no-plain", action="store_true",
                   help="skip the second measurement of the same schedule on a plain torch.empty batch")
    p.add_argument("--placement", default="plain", choices=["probe", "plain"],
                   help="plain (default): the batch is torch.empty(span), the footprint a deployment has; "
                        "probe: carve it from a contiguous arena 96 GiB larger at the offset where a timed "
                        "unmask runs fastest (DESIGN.md sec.5), and measure the plain allocation beside it")
    p.add_argument("--placement-slack-gib", type=int, default=96, help="arena = batch + this many GiB (probe)")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="harness collectives (barrier, max time); nccl = RCCL. gloo lets several ranks share one "
                        "GPU to rehearse the N>1 path")
    return p.parse_args()


def host_cores():
    """(cores this process may run on, the cgroup CPU quota in cores or None)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def effective_cores() -> int:
    """Threads the host can actually run at once: the affinity set, capped by
    the cgroup CPU quota rounded up (256 affinity cores under a 16-core quota
    time-slice onto 16 cores' worth of CPU)."""
    import math
    aff, quota = host_cores()
    return max(1, min(aff, math.ceil(quota))) if quota else aff


def _time_unmask(orc, base, descs, threads: int, seconds: float):
    orc.unmask_batch(base, descs, threads)  # warm
    passes, t0 = 0, time.perf_counter()
    while True:
        orc.unmask_batch(base, descs, threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return passes, el


def cpu_baseline(seconds: float, threads: int, frame_len: int, seed: int):
    """Times the oracle (kuma's byte loop, WSHandler.cpp:303-310, restated in
    oracle/kmws_oracle.c) on host cores over a bounded sample of the same
    workload: 16384 x frame_len frames (1 GiB), repeated for ~`seconds` in
    all: ~3/4 of it on `threads` threads (the effective core count: affinity
    capped by the cgroup quota), the rest on one thread (SURVEY sec.6 quotes
    kuma per core)."""
    import numpy as np
    from oracle import oracle as orc
    n = 16384  # 1 GiB of 64 KiB frames: 4x the host's L3, so the sample streams from DRAM
    rng = np.random.default_rng(seed)
    base = np.frombuffer(rng.bytes(n * frame_len), dtype=np.uint8).copy()
    descs = np.zeros(n, dtype=orc.DESC_DTYPE)
    descs["off"] = np.arange(n, dtype=np.uint64) * frame_len
    descs["len"] = frame_len
    descs["key"] = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    passes, el = _time_unmask(orc, base, descs, threads, seconds * 0.75)
    p1, el1 = _time_unmask(orc, base, descs, 1, seconds * 0.25)
    gib = n * frame_len / 2**30
    aff, quota = host_cores()
    return {"value": round(passes * gib / el, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_core_GiB_s": round(p1 * gib / el1, 3),
            "affinity_cores": aff, "cgroup_cpu_quota_cores": quota,
            "sample": f"{n} x {frame_len} B frames ({n * frame_len >> 20} MiB), in-place unmask with the "
                      f"oracle's restatement of WSHandler::handleDataMask (scalar byte loop, gcc -O3), "
                      f"{threads} threads (affinity {aff} capped by the cgroup quota {quota}), {passes} passes "
                      f"in {el:.1f} s; 1 thread: {p1} passes in {el1:.1f} s. The port is not calibrated "
                      f"against a build of kuma's own src/ws: none is possible here (WSHandler.cpp needs "
                      f"libkev headers the reference does not carry; DESIGN.md sec.2)",
            "cpu_model": _cpu_model()}


def _cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


TEMPORAL_STORES, NT_STORES = 1 << 30, 1 << 29  # KMWS_SCHED_* store bits (include/kmws_gpu.h)
UNMASK_KERNEL = "unmask_split_kernel"


def schedule_name(schedule: int) -> str:
    kind = {0: "one block per 16 KiB tile, 2 groups of 4 XCDs, runs of 16 tiles per XCD in the group's half",
            1: "one block per 16 KiB tile, in order",
            2: "one block per 16 KiB tile, tiles dealt over 2 parts of the span",
            3: "one block per 16 KiB tile, tiles dealt over 8 parts of the span",
            4: "one block per 16 KiB tile, runs of 16 tiles per XCD",
            5: "one block per 16 KiB tile, tiles dealt over 4 parts of the span"}.get(schedule & 0xFF, "?")
    if schedule & TEMPORAL_STORES:
        return kind + ", temporal payload stores"
    if schedule & NT_STORES:
        return kind + ", non-temporal payload stores"
    return kind + ", automatic store policy (temporal on tile-aligned batches)"


def traffic_from_profile(frames: int, frame_len: int, kernel: str, schedule=None, profiles_dir=None):
    """HBM bytes per launch of the unmask kernel from the committed PMC passes
    (profiles/*traffic*.json, written by tools/pmc_traffic.py) measured on this
    exact configuration: the newest one (by the `measured_at` time each record
    carries) for this schedule if there is one, else the newest for the
    kernel; None if there is none."""
    import datetime
    import glob

    def when(t):
        try:
            return datetime.datetime.fromisoformat(t.get("measured_at", "")).timestamp()
        except ValueError:
            return float("-inf")
    same, any_ = [], []
    for path in glob.glob(os.path.join(profiles_dir or os.path.join(ROOT, "profiles"), "*traffic*.json")):
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        if t.get("frames") == frames and t.get("frame_len") == frame_len and t.get("kernel") == kernel:
            any_.append(t)
            if schedule is not None and t.get("schedule") == schedule:
                same.append(t)
    pool = same or any_
    return max(pool, key=when).get("hbm_bytes_per_launch") if pool else None


def cpu_baseline_cfg1(run) -> float:
    """cpu_baseline leg of cfg1: the oracle's restatement of kuma's decoder
    (WSHandler::handleData, state machine + byte loop) timed by the same
    driver as the product: best seconds for the whole stream."""
    import ctypes as C
    from oracle import oracle as orc
    O = orc.lib()
    return run(lambda: O.orc_decoder_create(1),
               lambda d, b, l: O.orc_decoder_feed(d, b, l, C.cast(None, orc.FRAME_CB), None),
               O.orc_decoder_destroy)


def tx_batch_cfg1(K, payload, keys, n, L, reps) -> dict:
    """Send side of cfg1: the 1,000 payloads queued as client frames with
    kmws_tx_batch_add (header packed per send) and masked by ONE
    kmws_tx_batch_flush; payloads in a pinned send ring (zero-copy) and in
    pageable buffers (staged).  The flush is timed; the per-send add cost is
    reported apart, since from Python it is mostly ctypes overhead."""
    import ctypes as C
    import time as _t
    import numpy as np
    import torch
    ring = torch.from_numpy(payload.copy()).pin_memory()
    page = bytearray(payload.tobytes())
    pbuf = (C.c_uint8 * len(page)).from_buffer(page)
    hdr_out = (C.c_uint8 * 14)()
    out = {}
    for name, base in (("pinned_ring", ring.data_ptr()), ("pageable", C.addressof(pbuf))):
        b = K.kmws_tx_batch_create(0)
        if name == "pinned_ring":
            assert K.kmws_tx_batch_attach_ring(b, ring.data_ptr(), ring.numel()) == 0
        best, add_best = 1e9, 1e9
        for rep in range(reps + 1):
            t0 = _t.perf_counter()
            for i in range(n):
                from kuma_amd.kmws import FrameHdr
                h = FrameHdr()
                h.fin, h.opcode, h.mask = 1, 1, 1
                kk = int(keys[i])
                for j in range(4):
                    h.maskey[j] = (kk >> (8 * j)) & 0xFF
                ptr = (C.c_void_p * 1)(base + i * L)
                ln = (C.c_size_t * 1)(L)
                assert K.kmws_tx_batch_add(b, C.byref(h), ptr, ln, 1, hdr_out) == 8
            t1 = _t.perf_counter()
            assert K.kmws_tx_batch_flush(b) == n
            t2 = _t.perf_counter()
            if rep:
                best, add_best = min(best, t2 - t1), min(add_best, (t1 - t0) / n)
        K.kmws_tx_batch_destroy(b)
        out[name] = {"flush_GiB_s": n * L / best / 2**30, "flush_ms": best * 1e3,
                     "add_us_per_send_from_python": add_best * 1e6}
    # reps + 1 flushes per buffer (odd or even): re-mask to compare with the oracle-free expectation
    kb = keys.view(np.uint8).reshape(n, 4)
    masked = payload.reshape(n, L) ^ np.tile(kb, L // 4)
    want = masked if (reps + 1) % 2 else payload.reshape(n, L)
    out["verified"] = bool(np.array_equal(ring.numpy().reshape(n, L), want) and
                           np.array_equal(np.frombuffer(page, dtype=np.uint8).reshape(n, L), want))
    return out


def run_cfg1(reps: int = 10) -> dict:
    """BASELINE configs[0] (test/client <-> test/server, 1,000 x 4 KiB masked
    TEXT frames; SURVEY 8 d row 1): the stream fed in 64 KiB reads, SERVER mode.
    CPU baseline = kuma's decoder restated in oracle/ on one core; product =
    kmws_decoder_feed (one GPU batch per read), the deferred batch (one GPU
    batch per loop iteration), the deferred batch over a pinned receive ring,
    and on the send side one kmws_tx_batch flush for the 1,000 frames."""
    import ctypes as C
    import numpy as np
    from kuma_amd import kmws
    SEED = 0x6B756D61

    def splitmix_keys(seed, cnt):
        with np.errstate(over="ignore"):
            z = np.arange(cnt, dtype=np.uint64) + np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
        return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)

    n, L = 1000, 4096
    rng = np.random.default_rng(SEED)
    keys = splitmix_keys(SEED, n)
    payload = (0x20 + rng.integers(0, 2**31, size=n * L) % 95).astype(np.uint8)
    # the wire image: n x (81 fe 10 00 <key>) + payload ^ key (masked TEXT, 16-bit length)
    kb = keys.view(np.uint8).reshape(n, 4)
    frames = np.empty((n, 8 + L), dtype=np.uint8)
    frames[:, :4] = np.array([0x81, 0xFE, L >> 8, L & 0xFF], dtype=np.uint8)
    frames[:, 4:8] = kb
    frames[:, 8:] = payload.reshape(n, L) ^ np.tile(kb, L // 4)
    wire = frames.tobytes()
    chunk = 64 * 1024

    # Every decoder / batch is long-lived, as on an event loop (one per
    # connection / loop thread): created once, warmed by one untimed pass (its
    # pinned staging grows to size), then the best of `reps` timed passes.
    def run(create, feed, destroy):
        d = create()
        bufs = [bytearray(wire[i:i + chunk]) for i in range(0, len(wire), chunk)]
        cbufs = [(C.c_uint8 * len(b)).from_buffer(b) for b in bufs]
        best = 1e9
        for rep in range(reps + 1):
            for i, b in enumerate(bufs):  # fresh masked bytes (the decoder unmasks in place)
                b[:] = wire[i * chunk:i * chunk + len(b)]
            t0 = time.perf_counter()
            for b, cb in zip(bufs, cbufs):
                r = feed(d, cb, len(b))
                assert r in (0, 1), r
            if rep:
                best = min(best, time.perf_counter() - t0)
        destroy(d)
        return best

    t_orc = cpu_baseline_cfg1(run)
    res = {"metric": "GiB/s decode+unmask, 1000 x 4 KiB masked TEXT frames fed in 64 KiB reads (cfg1)",
           "config": "cfg1", "frames": n, "frame_len": L, "wire_bytes": len(wire), "feed_chunk": chunk,
           "cpu_baseline": {"GiB_s": n * L / t_orc / 2**30, "us_per_frame": t_orc / n * 1e6, "cores": 1,
                            "kind": "port", "best_of": reps,
                            "sample": "the whole cfg1 stream through the oracle's restatement of "
                                      "WSHandler::handleData (state machine + byte loop), SERVER mode"}}
    if kmws.device_count() > 0:
        K = kmws.lib()
        for key, resident in (("product_decoder_sync", True), ("product_decoder_sync_launch", False)):
            kmws.resident_enable(resident)
            t_gpu = run(lambda: K.kmws_decoder_create(1, 0),
                        lambda d, b, l: K.kmws_decoder_feed(d, b, l, C.cast(None, kmws.FRAME_CB), None),
                        K.kmws_decoder_destroy)
            res[key] = {"GiB_s": n * L / t_gpu / 2**30, "us_per_frame": t_gpu / n * 1e6, "best_of": reps,
                        "note": "kmws_decoder_feed: host parse + one GPU unmask per 64 KiB read (pageable chunk -> "
                                "pinned staging, zero-copy over PCIe) " +
                                ("by the thread's resident worker (no launch per read)" if resident else
                                 "with the resident worker off: one HIP launch + event wait per read")}
        kmws.resident_enable(True)
        # deferred: every read of the burst fed, ONE flush (one GPU batch per loop iteration)
        nullcb = C.cast(None, kmws.FRAME_CB)
        bufs = [bytes(wire[i:i + chunk]) for i in range(0, len(wire), chunk)]
        cbufs = [(C.c_uint8 * len(x)).from_buffer_copy(x) for x in bufs]
        d = K.kmws_decoder_create(1, 0)
        b = K.kmws_rx_batch_create(0)
        best = 1e9
        for rep in range(reps + 1):
            t0 = time.perf_counter()
            for x, cb in zip(bufs, cbufs):
                r = K.kmws_decoder_feed_deferred(d, b, cb, len(x), nullcb, None)
                assert r in (0, 1), r
            got = K.kmws_rx_batch_flush(b)
            if rep:
                best = min(best, time.perf_counter() - t0)
            assert got == n, got
        K.kmws_rx_batch_destroy(b)
        K.kmws_decoder_destroy(d)
        res["product_decoder_deferred"] = {"GiB_s": n * L / best / 2**30, "us_per_frame": best / n * 1e6,
                                           "best_of": reps,
                                           "note": "kmws_decoder_feed_deferred per read + one kmws_rx_batch_flush"}
        # deferred + pinned receive ring: reads land in the ring (recv into the ring replaces
        # kuma's recv into a stack buffer, untimed here as in the CPU case), zero-copy unmask
        import torch
        ring = torch.empty(len(wire) + 64 * 128, dtype=torch.uint8).pin_memory()
        wire_t = torch.frombuffer(bytearray(wire), dtype=torch.uint8)
        d = K.kmws_decoder_create(1, 0)
        b = K.kmws_rx_batch_create(0)
        assert K.kmws_rx_batch_attach_ring(b, ring.data_ptr(), ring.numel()) == 0
        best = 1e9
        for rep in range(reps + 1):
            offs = []
            w = 0
            for i in range(0, len(wire), chunk):
                m = min(chunk, len(wire) - i)
                ring[w:w + m] = wire_t[i:i + m]
                offs.append((w, m))
                w += m + 64  # reads land at arbitrary ring positions
            base = ring.data_ptr()
            t0 = time.perf_counter()
            for o, m in offs:
                r = K.kmws_decoder_feed_deferred(d, b, base + o, m, nullcb, None)
                assert r in (0, 1), r
            got = K.kmws_rx_batch_flush(b)
            if rep:
                best = min(best, time.perf_counter() - t0)
            assert got == n, got
        K.kmws_rx_batch_destroy(b)
        K.kmws_decoder_destroy(d)
        res["product_decoder_deferred_ring"] = {"GiB_s": n * L / best / 2**30, "us_per_frame": best / n * 1e6,
                                                "best_of": reps,
                                                "note": "reads in a pinned ring attached to the batch; one flush"}
        # one loop iteration per 64 KiB read, asynchronous: every read is fed,
        # submitted and the finished generations polled (kmws::RxLoop's posted task)
        d = K.kmws_decoder_create(1, 0)
        b = K.kmws_rx_batch_create(0)
        assert K.kmws_rx_batch_attach_ring(b, ring.data_ptr(), ring.numel()) == 0
        best = 1e9
        for rep in range(reps + 1):
            base = ring.data_ptr()
            t0 = time.perf_counter()
            got = 0
            for o, m in offs:
                r = K.kmws_decoder_feed_deferred(d, b, base + o, m, nullcb, None)
                assert r in (0, 1), r
                assert K.kmws_rx_batch_submit(b) >= 0
                got += K.kmws_rx_batch_poll(b, 0)
            got += K.kmws_rx_batch_poll(b, 1)
            if rep:
                best = min(best, time.perf_counter() - t0)
            assert got == n, got
        K.kmws_rx_batch_destroy(b)
        K.kmws_decoder_destroy(d)
        res["product_decoder_async_per_read"] = {"GiB_s": n * L / best / 2**30, "us_per_frame": best / n * 1e6,
                                                 "best_of": reps,
                                                 "note": "reads in a pinned ring; per 64 KiB read: feed_deferred, "
                                                         "rx_batch_submit, rx_batch_poll(0) (one loop iteration per "
                                                         "read, GPU completion overlapping the next reads)"}
        res["product_tx_batch"] = tx_batch_cfg1(K, payload, keys, n, L, reps)
    return res




PLACEMENT_STEP = 16 << 30
CFG5_JOB_FRAMES = 10485760  # BASELINE configs[4]


def placement_slack(span: int, free: int, want: int) -> int:
    """Arena bytes beyond the batch for the placement probe: a multiple of
    16 GiB, at most `want`, at most 1.5 x the batch, and what fits beside the
    batch in free memory with 8 GiB to spare (< 16 GiB: no probe)."""
    st = PLACEMENT_STEP
    return max(0, min(want, span * 3 // 2 // st * st, (free - span - (8 << 30)) // st * st))


def place_batch(kmws, torch, dev, span, slack):
    """Carves the batch out of one physically contiguous arena of span + slack
    bytes, at the offset (multiples of 16 GiB) where two in-place split-8 unmask
    passes (payload unchanged) run fastest.  The rate of the split schedules
    depends on where the batch lies in physical HBM (75.5-76 % vs 82-83 %,
    profiles/r01f_unmask_placement.txt, r01h_offset192.txt); the kernel cannot
    see physical addresses, so the layout is chosen by measurement once, as a
    long-lived batch ring would be.  Returns (arena | None, batch view, record)."""
    free, _ = torch.cuda.mem_get_info(dev)
    slack = placement_slack(span, free, slack)
    if slack < PLACEMENT_STEP:
        return None, None, {"kind": "plain torch.empty", "why": "no room for a placement probe"}
    try:
        arena = kmws.Arena(span + slack, device=dev.index)
    except RuntimeError as e:
        return None, None, {"kind": "plain torch.empty", "why": str(e)}
    off, probe = kmws.arena_place(arena, span, PLACEMENT_STEP)  # kmws_arena_place: timed split-4/8 passes
    pick = off >> 30
    rec = {"kind": "offset in a contiguous arena, picked by kmws_arena_place (timed probe: best of split 4 and split 8 per offset)",
           "arena_GiB": (span + slack) >> 30, "contiguous": arena.contiguous, "offset_GiB": pick,
           "probe_frac_by_offset_GiB": {o >> 30: v for o, v in probe.items()}}
    return arena, arena.tensor[pick << 30:(pick << 30) + span], rec


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script (one
    per GPU) with the torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE,
    MASTER_ADDR=127.0.0.1, MASTER_PORT) and wait for all of them.  The parent
    never touches the GPU (it only forks children, no exec from a GPU process).
    Rank 0 prints the JSON line; returns the first non-zero exit status."""
    import subprocess
    import threading
    port = _free_port()
    procs, pumps = [], []

    def pump(r, stream):
        # only rank 0's JSON line goes to stdout (the contract's ONE line); anything
        # else the ranks or their libraries print (gloo's connection notices) to stderr
        for line in stream:
            out = sys.stdout if (r == 0 and line.startswith("{")) else sys.stderr
            out.write(line)
            out.flush()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             stdout=subprocess.PIPE, text=True, bufsize=1)
        procs.append(p)
        pumps.append(threading.Thread(target=pump, args=(r, p.stdout), daemon=True))
        pumps[-1].start()
    codes = [p.wait() for p in procs]
    for t in pumps:
        t.join()
    bad = [c for c in codes if c != 0]
    if bad:
        print(f"bench: rank exit codes {codes}", file=sys.stderr)
    return bad[0] if bad else 0


def time_steps(kmws, torch, stream, step, steps, world, dist):
    """Barrier + synchronize, `steps` timed steps with HIP events around each
    unmask launch on the launch stream, synchronize + barrier.  Returns (wall s,
    summed event ms)."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(*evs[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return time.perf_counter() - t0, sum(e0.elapsed_time(e1) for e0, e1 in evs)


def plain_rate(kmws, torch, dev, n, L, descs, ws, schedule, seed, steps, warmup, stream):
    """The same batch and schedule on a plain torch.empty allocation (no arena,
    no placement probe): fraction of the 8 TB/s peak from the HIP events of
    `steps` timed launches, every byte verified.  Also the autotune's pick on
    that allocation and its rate."""
    span = n * L
    base = torch.empty(span, dtype=torch.uint8, device=dev)
    kmws.fill_synthetic(base, seed)
    out = {}
    for label, tune in (("same_schedule", False), ("autotuned", True)):
        if tune:
            sched = kmws.unmask_autotune(base, descs, ws, span)
        else:
            kmws.unmask_set_schedule(ws, schedule)
            sched = schedule
        kmws.unmask_plan(descs, ws, span)
        for _ in range(warmup):
            kmws.unmask_apply(base, descs, ws, span)
        torch.cuda.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        for e0, e1 in evs:
            e0.record(stream)
            kmws.unmask_apply(base, descs, ws, span)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / steps
        out[label] = {"schedule": sched, "kernel_ms": round(ms, 4),
                      "frac": round(n * (2 * L + DESC_BYTES) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        if (warmup + steps) % 2 == 1:  # leave the batch masked, as generated
            kmws.unmask_apply(base, descs, ws, span)
    kmws.unmask_batch(base, descs, ws, span)
    mism = kmws.check_unmasked(base, seed, descs)
    kmws.unmask_set_schedule(ws, schedule)  # the placed batch's schedule, as before
    del base
    torch.cuda.empty_cache()
    out["byte_mismatches"] = mism
    return out


E2E_METRIC = ("GiB/s host-resident WS frame unmask end to end (pinned H2D -> unmask kernel -> D2H), "
              "64 KiB frames")
E2E_HDR = 14  # a masked 64 KiB frame's header (WSHandler.cpp:46-106: 2 + 8 + 4)


def _splitmix32(seed: int, n: int):
    import numpy as np
    with np.errstate(over="ignore"):
        z = np.arange(n, dtype=np.uint64) + np.uint64(seed & (2**64 - 1)) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def run_e2e(a, kmws, torch, dist, dev, coll_dev, rank, world, ndev, gib=None, steps=None, warmup=None):
    """The host-resident path on N GPUs (SURVEY 8 e, f-3).
    kuma's frames start and end in host memory (a socket read on a loop
    thread, TcpConnection.cpp:229).  Each rank holds its own shard -- `gib` GiB
    of masked 64 KiB frames in a pinned host wire image (14-byte headers between
    payloads, as they arrive) allocated with kmws_host_alloc on its own GPU --
    and unmasks it in place end to end through its own kmws_pipeline (a 3-slot
    SDMA ring: H2D || unmask kernel || D2H on three streams, 64 MiB chunks), so
    every rank's payload crosses its own GPU's PCIe link twice into its own
    staging.  No data-path collective; host DRAM is what the ranks share.
    value = all ranks' payload over the slowest rank's time (weak scaling: a
    fixed shard per rank).  Each rank also times raw pinned H2D and D2H copies
    of 1 GiB with every rank copying at once (its share of PCIe and host DRAM
    under the same concurrency).  Every byte of every shard is verified on the
    device after an odd number of passes (payload unmasked, headers untouched).
    Returns rank 0's record (None on other ranks)."""
    import ctypes as C
    import numpy as np
    gib = a.e2e_gib if gib is None else gib
    steps = a.steps if steps is None else steps
    warmup = a.warmup if warmup is None else warmup
    L, H = 65536, E2E_HDR
    stride = L + H
    n = max(1, int(gib * 2**30) // stride)
    span = n * stride
    seed = (a.seed ^ 0xE2E0) + rank * (span >> 3)  # the shards are slices of one job
    K = kmws.lib()
    ptr = K.kmws_host_alloc(span, dev.index)
    if not ptr:
        raise RuntimeError(f"kmws_host_alloc({span}) failed on rank {rank}")
    try:
        host = torch.from_numpy(np.ctypeslib.as_array((C.c_uint8 * span).from_address(ptr)))
        scratch = torch.empty(span, dtype=torch.uint8, device=dev)

        def barrier():
            if world > 1:
                dist.barrier()

        # raw pinned copies, every rank at once (before the shard is written)
        cb = min(1 << 30, span)
        rates = {}
        for name, (dst, src) in (("h2d", (scratch[:cb], host[:cb])), ("d2h", (host[:cb], scratch[:cb]))):
            best = 1e9
            for _ in range(3):
                barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            rates[name] = cb / best / 2**30
        # the shard: synthetic bytes everywhere, frame i's payload at i * stride + H
        kmws.fill_synthetic(scratch, seed)
        host.copy_(scratch)
        torch.cuda.synchronize()
        d = np.zeros(n, dtype=[("off", "<u8"), ("len", "<u4"), ("key", "<u4")])
        d["off"] = np.arange(n, dtype=np.uint64) * stride + H
        d["len"] = L
        d["key"] = _splitmix32((a.seed ^ 0x5EED) + rank * n, n)
        chunk = 64 << 20
        pipe = kmws.Pipeline(dev.index, chunk, 1 << 16, 3, transfer=kmws.Pipeline.COPY)
        for _ in range(warmup):
            pipe.unmask(host, d)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            pipe.unmask(host, d)
        elapsed = time.perf_counter() - t0
        barrier()
        passes = warmup + steps
        if passes % 2 == 0:  # an odd count leaves the payloads unmasked: what the checker expects
            pipe.unmask(host, d)
        scratch.copy_(host)
        descs = kmws.make_descs(d["off"].astype(np.int64), d["len"].astype(np.int64), d["key"].astype(np.int64),
                                device=dev)
        mism = kmws.check_unmasked(scratch, seed, descs)
        del pipe
    finally:
        torch.cuda.synchronize()
        scratch = host = None
        K.kmws_host_free(ptr)
        torch.cuda.empty_cache()
    me = {"rank": rank, "device": dev.index, "frames": n, "host_bytes": span, "elapsed_s": round(elapsed, 4),
          "payload_GiB_s": round(n * L * steps / elapsed / 2**30, 2), "raw_h2d_GiB_s": round(rates["h2d"], 2),
          "raw_d2h_GiB_s": round(rates["d2h"], 2), "byte_mismatches": mism}
    ranks = [me]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    if rank != 0:
        return None
    total_mism = sum(r["byte_mismatches"] for r in ranks)
    payload = n * L * world
    value = payload * steps / elapsed / 2**30
    raw = min(min(r["raw_h2d_GiB_s"], r["raw_d2h_GiB_s"]) for r in ranks)
    return {"metric": E2E_METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": steps,
            "warmup": warmup, "ms_per_step": round(elapsed * 1e3 / steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (device-generated splitmix64 bytes copied into pinned host memory, per-frame keys)",
            "config": {"workload": "host-resident end to end: per rank %d x 64 KiB masked frames in a pinned host "
                                   "wire image (14-B headers between payloads), in-place unmask through the rank's "
                                   "own kmws_pipeline (3-slot SDMA ring, H2D || kernel || D2H)" % n,
                       "frames_per_gpu": n, "host_bytes_per_gpu": span, "chunk_MiB": chunk >> 20,
                       "transfer": "copy (SDMA ring)", "ranks_share_one_gpu": world > ndev,
                       "parallelism": f"shard per rank x{world}, own PCIe link and pinned staging, no collective",
                       "dist_backend": a.dist_backend if world > 1 else None},
            "pcie": {"bytes_per_step_per_gpu": 2 * span, "note": "each shard crosses PCIe twice (H2D of the "
                     "chunk, D2H of its frames' extent: at most 2 x the wire image)",
                     "payload_frac_of_concurrent_raw_copy": round(value / world / raw, 3) if raw else None},
            "ranks": ranks, "verify": {"byte_mismatches": total_mism, "ok": total_mism == 0},
            "shared_limit": "host DRAM: every rank's H2D reads and D2H writes land in the same sockets' memory; "
                            "compare raw_h2d / raw_d2h per rank at N with N = 1"}


def run_job(a, kmws, torch, dist, dev, coll_dev, rank, world, job_frames, shared_gpu, with_plain=True):
    """One pass of the device-resident unmask over a job: `job_frames` frames
    split over the ranks (strong scaling, BASELINE configs[4]), or 0 = a.frames
    per rank (weak, configs[1]).  A rank's shard larger than one resident batch
    runs as sub-batches (the same count on every rank), each generated on the
    device untimed, then timed between barriers; the step time is the sum over
    sub-batches.  Returns the rank-0 facts (every rank returns them)."""
    from kuma_amd import shard
    L = a.frame_len
    # Rank g owns global frames [lo, hi) (kuma_amd/shard.py); payload and keys are
    # generated from global positions, so the shards are slices of one big job.
    job = job_frames if job_frames else a.frames * world
    g_lo, g_hi = shard.uniform_range(job, rank, world)
    n, batches = shard.sub_batches(job, rank, world, a.max_batch_frames)
    nb = len(batches)
    span = n * L
    descs = torch.empty((n, 2), dtype=torch.int64, device=dev)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span), device=dev)
    arena, placement = None, {"kind": "plain torch.empty"}
    if a.placement == "probe" and not shared_gpu:
        arena, base_all, placement = place_batch(kmws, torch, dev, span, a.placement_slack_gib << 30)
    elif shared_gpu:
        placement["why"] = f"{world} ranks share one GPU: rehearsal, no arena"
    arena_used = arena  # None: the timed batch is a plain allocation
    if arena is None:
        base_all = torch.empty(span, dtype=torch.uint8, device=dev)

    stream = torch.cuda.current_stream()
    schedule = a.schedule if a.schedule >= 0 else kmws.sched_default(span, n)
    elapsed, ev_ms, launches, alg_total, mismatches, st, done = 0.0, 0.0, 0, 0, 0, 0, 0
    ranges = []
    for j, (b_lo, b_hi) in enumerate(batches):
        bn = b_hi - b_lo
        bspan = bn * L
        base, bdescs = base_all[:bspan], descs[:bn]
        seed = a.seed + (b_lo * L >> 3)
        if bn:
            kmws.fill_uniform_descs(bdescs, L, L, (a.seed ^ 0x5EED) + b_lo)
            kmws.fill_synthetic(base, seed)
            if a.schedule >= 0:
                kmws.unmask_set_schedule(ws, a.schedule)
            elif j == 0 and not a.no_autotune:
                # untimed, payload unchanged: picks this batch's faster unmask schedule
                # (kept on ws, the host plan of the batches it serves)
                schedule = kmws.unmask_autotune(base, bdescs, ws, bspan)
            elif not a.no_autotune:
                kmws.unmask_set_schedule(ws, schedule)  # same layout as batch 0
        torch.cuda.synchronize()

        def step(ev0=None, ev1=None):
            if bn == 0:
                return
            kmws.unmask_plan(bdescs, ws, bspan)
            if ev0 is not None:
                ev0.record(stream)
            kmws.unmask_apply(base, bdescs, ws, bspan)
            if ev1 is not None:
                ev1.record(stream)

        for _ in range(a.warmup):
            step()
        torch.cuda.synchronize()
        wall, ms = time_steps(kmws, torch, stream, step, a.steps, world, dist)
        elapsed += wall
        if bn:
            ev_ms += ms
            launches += a.steps
            alg_total += a.steps * bn * (2 * L + DESC_BYTES)
        done += bn
        ranges.append([b_lo, b_hi])
        st |= ws.status()
        if not a.no_verify and bn:
            if (a.warmup + a.steps) % 2 == 0:  # XOR twice is the identity: bring the batch to the unmasked state
                kmws.unmask_batch(base, bdescs, ws, bspan)
            mismatches += kmws.check_unmasked(base, seed, bdescs)
    assert done == g_hi - g_lo
    # average unmask-kernel launch: duration and algorithmic bytes (every batch is
    # full, n frames, when nb divides the shard)
    kern_ms = ev_ms / max(launches, 1)
    alg_bytes = alg_total // max(launches, 1)

    plain = None
    if with_plain and world == 1 and not a.no_plain and arena is not None:
        # the same schedule on a plain allocation: the headline is not a best-of-placements number alone
        base_all = base = arena = None
        torch.cuda.empty_cache()
        b_lo, b_hi = batches[0]
        plain = plain_rate(kmws, torch, dev, b_hi - b_lo, L, descs[:b_hi - b_lo], ws, schedule,
                           a.seed + (b_lo * L >> 3), a.steps, a.warmup, stream)
        if not a.no_verify:
            mismatches += plain["byte_mismatches"]

    # gather per-rank facts on rank 0: elapsed, kernel time, mismatches, frame ranges
    per_rank = [{"rank": rank, "device": dev.index, "frames": [g_lo, g_hi], "sub_batches": ranges,
                 "elapsed_s": round(elapsed, 4), "kernel_ms": round(kern_ms, 4), "byte_mismatches": mismatches}]
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        t = torch.tensor([mismatches, st], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(t)
        mismatches, st = int(t[0]), int(t[1])
        gathered = [None] * world
        dist.all_gather_object(gathered, per_rank[0])
        per_rank = gathered
    base_all = base = descs = ws = arena = None  # the next job (cfg5_job, e2e_host) gets the HBM back
    torch.cuda.empty_cache()
    return {"job": job, "n": n, "nb": nb, "g_lo": g_lo, "g_hi": g_hi, "elapsed": elapsed, "kern_ms": kern_ms,
            "alg_bytes": alg_bytes, "mismatches": None if a.no_verify else mismatches, "status": st,
            "schedule": schedule, "placement": placement, "arena_used": arena_used is not None, "plain": plain,
            "ranks": per_rank,
            # payload GiB/s of the whole job (all ranks) over the slowest rank's time
            "value": job * L * a.steps / elapsed / 2**30, "ms_per_step": elapsed * 1e3 / a.steps}


def main():
    a = parse()
    if a.config == "cfg1":
        print(json.dumps(run_cfg1(max(a.steps, 10))), flush=True)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))
    world = int(env_world or "1")
    if world != a.gpus:
        raise SystemExit(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}: one rank per GPU, the two must agree")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    job_frames = a.job_frames if a.job_frames is not None else (CFG5_JOB_FRAMES if world > 1 else 0)

    import torch
    import torch.distributed as dist
    from kuma_amd import kmws

    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench: no GPU visible; the HIP path has no CPU fallback")
    dev = torch.device("cuda", local % ndev)  # one GPU per rank; modulo only when rehearsing on fewer GPUs
    shared_gpu = world > ndev  # a rehearsal: several ranks on one GPU (gloo)
    torch.cuda.set_device(dev)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    coll_dev = dev if a.dist_backend == "nccl" else torch.device("cpu")
    if kmws.device_count() < 1:
        raise SystemExit("bench: no gfx950 device visible; the HIP path has no CPU fallback")

    if a.config == "e2e":
        out = run_e2e(a, kmws, torch, dist, dev, coll_dev, rank, world, ndev)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if world > 1:
            dist.destroy_process_group()
        if out is not None and not out["verify"]["ok"]:
            raise SystemExit("bench: e2e verification failed")
        return

    L = a.frame_len
    # The host-resident leg first, in a fresh process (after the 64-80 GiB device
    # jobs the same 4 GiB shard ran at 36 instead of 44.7 GiB/s: r06ai vs r06aj).
    e2e = None
    if a.e2e_gib > 0:
        try:
            e2e = run_e2e(a, kmws, torch, dist, dev, coll_dev, rank, world, ndev, gib=a.e2e_gib,
                          steps=min(a.steps, 5), warmup=2)
        except Exception as ex:  # recorded, never masking the headline
            e2e = {"error": repr(ex)}
    r = run_job(a, kmws, torch, dist, dev, coll_dev, rank, world, job_frames, shared_gpu)
    # At N = 1 the headline is cfg2 (weak); the N > 1 lines run BASELINE
    # configs[4]'s fixed job (strong).  So that the 1 -> 8 curve has a same-job
    # anchor, N = 1 also times that job, its 8 resident
    # sub-batches timed exactly as N > 1 times its ranks' sub-batches.
    cfg5 = None
    if world == 1 and not job_frames and a.cfg5_anchor:
        c = run_job(a, kmws, torch, dist, dev, coll_dev, rank, world, CFG5_JOB_FRAMES, shared_gpu, with_plain=False)
        cfg5 = {"value": round(c["value"], 2), "unit": "GiB/s", "ms_per_step": round(c["ms_per_step"], 4),
                "total_frames": c["job"], "frame_len": L, "resident_batch_frames": c["n"], "sub_batches": c["nb"],
                "kernel_ms": round(c["kern_ms"], 4), "unmask_schedule": c["schedule"],
                "frac": round(c["alg_bytes"] / (c["kern_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "verify": {"status_word": c["status"], "byte_mismatches": c["mismatches"]}, "ranks": c["ranks"],
                "scaling": "strong",
                "note": "BASELINE configs[4]'s whole job on this one GPU, timed as bench.py --gpus N times it: "
                        "per sub-batch, generated on device untimed, barrier + synchronize around the timed "
                        "steps, step time = sum over sub-batches; the N > 1 lines' value over this value is "
                        "their speed-up"}

    ms_per_step = r["ms_per_step"]
    value = r["value"]  # = shard.aggregate_rate over ranks (elapsed = max)
    kern_ms, alg_bytes, schedule, plain = r["kern_ms"], r["alg_bytes"], r["schedule"], r["plain"]
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = traffic_from_profile(r["n"], L, UNMASK_KERNEL, schedule)
    mismatches, st = r["mismatches"], r["status"]
    if cfg5 is not None and mismatches is not None:
        mismatches += cfg5["verify"]["byte_mismatches"] or 0
        st |= cfg5["verify"]["status_word"]

    if rank == 0:
        cpu = None
        if a.cpu_seconds > 0 and world == 1:
            thr = a.cpu_threads or effective_cores()
            cpu = cpu_baseline(a.cpu_seconds, thr, L, a.seed)
        job = r["job"]
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "strong" if job_frames else "weak", "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (device-generated splitmix64 payload, per-frame random keys)",
            "config": {"workload": ("cfg5: fixed job of %d frames split over the GPUs (per-GPU frame partition), "
                                    "device-resident in-place unmask" % job) if job_frames else
                                   "cfg2: 1 GPU device-resident in-place unmask of masked binary frames "
                                   "(aligned arena); N GPUs = per-GPU frame partition",
                       "frames_per_gpu": r["g_hi"] - r["g_lo"], "frame_len": L, "total_frames": job,
                       "resident_batch_frames": r["n"], "sub_batches": r["nb"],
                       "layout": "aligned arena, frame i at i*frame_len",
                       "parallelism": f"frame-partition x{world} (no collective)",
                       "dist_backend": a.dist_backend if world > 1 else None,
                       "unmask_schedule": schedule, "unmask_schedule_name": schedule_name(schedule),
                       "placement": r["placement"]},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         # the headline itself when the batch is a plain allocation (the default)
                         "frac_plain": (plain["same_schedule"]["frac"] if plain else
                                        round(achieved / HBM_PEAK_GBS, 4) if not r["arena_used"] else None),
                         "traffic": traffic,
                         "kernel": UNMASK_KERNEL,
                         "kernel_ms": round(kern_ms, 4),
                         "algorithmic_bytes_per_launch": alg_bytes},
            "plain_allocation": plain,
            "hbm_frac_whole_step": round(job * L / world * (2 + DESC_BYTES / L) /
                                         (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "verify": {"status_word": st, "byte_mismatches": mismatches},
            "ranks": r["ranks"],
            "cfg5_job": cfg5,
            "e2e_host": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if st != 0 or (mismatches not in (None, 0)):
        raise SystemExit(f"bench: verification failed (status={st}, mismatches={mismatches})")


if __name__ == "__main__":
    main()
