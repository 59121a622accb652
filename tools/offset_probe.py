"""Split-schedule rate vs position in physical memory: one contiguous arena
(kmws_arena_alloc) of `total` GiB, the 64 GiB cfg2 batch placed at offsets
0, step, 2*step, ... GiB inside it, in-order vs split-8 timed at each.
usage: python tools/offset_probe.py [total_gib] [step_gib] [variants]"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kuma_amd import kmws
    total = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    step = float(sys.argv[2]) if len(sys.argv) > 2 else 4
    variants = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,23").split(",")]
    n, L = 1 << 20, 65536
    span = n * L
    a = kmws.Arena(total << 30)
    print(json.dumps({"contiguous": a.contiguous, "total_GiB": total, "va_GiB": a.tensor.data_ptr() / 2**30}), flush=True)
    kmws.fill_synthetic(a.tensor, 5)
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_uniform_descs(descs, L, L, 3)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    s = torch.cuda.current_stream()
    alg = n * (2 * L + 16)
    off = 0
    while off + span <= (total << 30):
        base = a.tensor[off:off + span]
        out = {"offset_GiB": off / 2**30}
        for v in variants:
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(2):
                    kmws.unmask_batch(base, descs, ws, span, variant=v)
                e1.record(s)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) / 2)
            out[str(v)] = round(alg / (statistics.median(ts) * 1e-3) / 8e12, 4)
        print(json.dumps(out), flush=True)
        off += int(step * 2**30)


if __name__ == "__main__":
    main()
