"""Does the unmask rate depend on where an allocation lands?  Allocates
`arenas` separate 64 GiB arenas in ONE process and times the same schedules
on each, interleaved (b2b launches).  usage: python tools/layout_probe.py [arenas] [variants] [torch|contig]
(torch: torch.empty arenas; contig: kmws_arena_alloc, physically contiguous)"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kuma_amd import kmws
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,21,23").split(",")]
    how = sys.argv[3] if len(sys.argv) > 3 else "torch"
    n, L = 1 << 20, 65536
    span = n * L
    s = torch.cuda.current_stream()
    arenas, keep = [], []
    for i in range(k):
        if how == "contig":
            a = kmws.Arena(span)
            keep.append(a)
            print(json.dumps({"arena": i, "contiguous": a.contiguous}), flush=True)
            base = a.tensor
        else:
            base = torch.empty(span, dtype=torch.uint8, device="cuda")
        descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
        kmws.fill_synthetic(base, 7 + i)
        kmws.fill_uniform_descs(descs, L, L, 11 + i)
        ws = kmws.Workspace(kmws.unmask_workspace_size(span))
        arenas.append((base, descs, ws))
    torch.cuda.synchronize()
    res = {}
    for rnd in range(3):
        for i, (base, descs, ws) in enumerate(arenas):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(4):
                    kmws.unmask_batch(base, descs, ws, span, variant=v)
                e1.record(s)
                e1.synchronize()
                res.setdefault((i, v), []).append(e0.elapsed_time(e1) / 4)
    alg = n * (2 * L + 16)
    for (i, v), t in sorted(res.items()):
        med = statistics.median(t)
        print(json.dumps({"arena": i, "ptr_GiB": round(arenas[i][0].data_ptr() / 2**30, 2), "variant": v,
                          "ms": round(med, 3), "frac": round(alg / (med * 1e-3) / 8e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
