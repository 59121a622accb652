"""Placement probe for the cfg4 pack (kmws_encode_batch): does the position of
the payload arena and of the wire image inside one contiguous device arena move
the copy rate the way it moves the in-place unmask (bench.py placement)?

Prints one JSON line per (src_off, dst_off) pair in GiB, plus the torch.empty
baseline.  Every pack is verified once against the plain-allocation wire.
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_configs import SEED, timed  # noqa: E402

GIB = 1 << 30


def main():
    import torch
    from kuma_amd import kmws
    messages, reps = 262144, 9
    n, L = messages * 16, 4096
    P, H = n * L, n * 8
    dev = torch.device("cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device=dev)
    kmws.fill_uniform_descs(descs, L, L, SEED ^ 4)
    pos = np.arange(16)
    b0 = np.where(pos == 0, 1, 0) | np.where(pos == 15, 0x80, 0)
    fl16 = torch.from_numpy(np.tile((b0 | 0x100).astype(np.int16), messages)).to(dev)
    wire_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ws = kmws.Workspace(kmws.copy_workspace_size(n, P + H + 16))

    def frac(t):
        return (2 * P + H + 26 * n) / t / 8e12

    # baseline: separate torch allocations (what tools/bench_configs.py cfg4 does)
    src = torch.empty(P + 16, dtype=torch.uint8, device=dev)
    kmws.fill_synthetic(src, SEED)
    wire = torch.empty(P + H + 16, dtype=torch.uint8, device=dev)
    t = timed(torch, lambda: kmws.encode_batch(src, descs, fl16, wire, wire_off, ws), reps)
    assert ws.status() == 0
    ref_sum = int(wire[:P + H].view(torch.int64).sum())  # wrapping checksum of the plain result
    print(json.dumps({"layout": "torch.empty", "ms": round(t * 1e3, 4), "frac": round(frac(t), 4)}), flush=True)
    del src, wire
    torch.cuda.empty_cache()

    arena = kmws.Arena(128 * GIB, device=0)
    A = arena.tensor
    print(json.dumps({"arena_GiB": 128, "contiguous": arena.contiguous}), flush=True)
    pairs = [(s, d) for s in (0, 16, 32, 48, 64) for d in (s + 17, s + 33, s + 49) if d + 17 <= 128]
    pairs += [(d, s) for (s, d) in pairs[:4]]
    for so, do in pairs:
        src = A[so * GIB: so * GIB + P + 16]
        wire = A[do * GIB: do * GIB + P + H + 16]
        kmws.fill_synthetic(src, SEED)  # an earlier wire may have covered this range
        kmws.encode_batch(src, descs, fl16, wire, wire_off, ws)
        torch.cuda.synchronize()
        ok = ws.status() == 0 and int(wire[:P + H].view(torch.int64).sum()) == ref_sum
        t = timed(torch, lambda: kmws.encode_batch(src, descs, fl16, wire, wire_off, ws), reps)
        print(json.dumps({"src_GiB": so, "dst_GiB": do, "ms": round(t * 1e3, 4), "frac": round(frac(t), 4),
                          "verified": ok}), flush=True)


if __name__ == "__main__":
    main()
