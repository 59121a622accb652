"""Unmask schedule sweep on plain allocations: every placement kind with the
automatic, non-temporal and temporal store policy, on three layouts -- the
aligned 64 KiB arena (cfg2), the same frames as a packed wire (cfg2b: 14-byte
headers) and 4 KiB fragments behind 8-byte headers (cfg4 in place).  Median of
`reps` timed applies per schedule (even count: the payload ends unchanged);
prints one JSON line per layout.  Chooses kmws's default schedule.

usage: python tools/sched_sweep.py [reps] [gib]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kuma_amd import kmws
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    gib = float(sys.argv[2]) if len(sys.argv) > 2 else 64.0
    which = sys.argv[3].split(",") if len(sys.argv) > 3 else ["aligned_64k", "packed_wire_64k", "fragments_4k"]
    layouts = {"aligned_64k": (65536, 0), "packed_wire_64k": (65536, 14), "fragments_4k": (4096, 8),
               "zipf_wire": (None, None)}
    for name in which:
        L, H = layouts[name]
        if L is None:  # cfg3's Zipf sizes (128 B - 1 MiB) as a packed wire, 14-byte headers max
            import numpy as np
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
            import bench_configs as bc
            lens = bc.zipf_lens(np.random.default_rng(bc.SEED), 4_000_000)
            n = int(np.searchsorted(np.cumsum(lens + 14), gib * 2**30))
            lens = lens[:n]
            hl = np.where(lens <= 125, 6, np.where(lens <= 65535, 8, 14))
            offs = np.cumsum(hl + lens) - lens
            span = int(offs[-1] + lens[-1])
            descs = kmws.make_descs(offs, lens, bc.splitmix_keys(bc.SEED, n).astype(np.int64))
            L = int(lens.mean())
        else:
            n = int(gib * 2**30) // (L + H)
            span = n * (L + H)
            descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
            kmws.fill_uniform_descs(descs, L + H, L, 78)
            descs[:, 0] += H
        base = torch.empty(span, dtype=torch.uint8, device="cuda")
        kmws.fill_synthetic(base, 77)
        ws = kmws.Workspace(kmws.unmask_workspace_size(span))
        kmws.unmask_plan(descs, ws, span)
        span_payload = int((descs[:, 1] & 0xFFFFFFFF).sum())
        res = {}
        for kind in kmws.SCHED_KINDS:
            for store, tag in ((0, "auto"), (kmws.SCHED_NT_STORES, "nt"), (kmws.SCHED_TEMPORAL_STORES, "t")):
                kmws.unmask_set_schedule(ws, descs, span, kind | store)
                kmws.unmask_apply(base, descs, ws, span)  # warm
                kmws.unmask_apply(base, descs, ws, span)
                ts = []
                for _ in range(2 * (reps // 2)):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    kmws.unmask_apply(base, descs, ws, span)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e-3)
                ts.sort()
                t = ts[len(ts) // 2]
                res[f"{kind}{tag}"] = round((2 * span_payload + 16 * n) / t / 8e12, 4)
        assert ws.status() == 0
        best = max(res, key=res.get)
        print(json.dumps({"layout": name, "frames": n, "span": span, "frac_by_schedule": res, "best": best}),
              flush=True)
        del base, descs, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
