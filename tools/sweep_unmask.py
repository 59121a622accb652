"""Interleaved A/B of unmask schedules in ONE process (one allocation):
cfg2 (1 M x 64 KiB frames, device-resident), every variant timed with HIP
events on the launch stream, `rounds` rounds of `reps` launches each.
usage: python tools/sweep_unmask.py <variant,variant,...> [rounds] [reps] [frames] [sync|b2b] [stride] [len]
(frame i's payload at i * stride, len bytes; default 64 KiB frames back to back)
sync: every launch timed alone (synchronized); b2b: `reps` launches queued back
to back and timed as one (as bench.py runs them), per-launch average.
Variant numbers as kmws_unmask_batch_variant; >= 64 = a raw schedule code
(grid size, +1 for the pipelined grid).  Prints one JSON line per variant."""
import json
import statistics
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kuma_amd import kmws
    variants = [int(v) for v in sys.argv[1].split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    n = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 20
    mode = sys.argv[5] if len(sys.argv) > 5 else "sync"
    stride = int(sys.argv[6]) if len(sys.argv) > 6 else 65536
    L = int(sys.argv[7]) if len(sys.argv) > 7 else stride
    span = n * stride
    base = torch.empty(span, dtype=torch.uint8, device="cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(base, 7)
    kmws.fill_uniform_descs(descs, stride, L, 11)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    s = torch.cuda.current_stream()
    times = {v: [] for v in variants}
    for v in variants:  # warm every variant once
        kmws.unmask_batch(base, descs, ws, span, variant=v)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(rounds):
        for v in variants:
            if mode == "b2b":
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(reps):
                    kmws.unmask_batch(base, descs, ws, span, variant=v)
                e1.record(s)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) / reps)
                if os.environ.get("SWEEP_TRACE"):
                    print(json.dumps({"t": round(time.perf_counter() - t_start, 3), "variant": v,
                                      "ms": round(times[v][-1], 3)}), flush=True)
                continue
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                kmws.unmask_batch(base, descs, ws, span, variant=v)
                e1.record(s)
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1))
    assert ws.status() == 0
    alg = n * (2 * L + 16)
    print(json.dumps({"resident_blocks": kmws.unmask_resident_blocks(), "frames": n, "mode": mode,
                      "stride": stride, "len": L}), flush=True)
    for v in variants:
        med = statistics.median(times[v])
        print(json.dumps({"variant": v, "median_ms": round(med, 3), "min_ms": round(min(times[v]), 3),
                          "max_ms": round(max(times[v]), 3),
                          "frac": round(alg / (med * 1e-3) / 8.0e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
