"""Pinned host <-> device copy rates on one GPU: H2D alone, D2H alone, and both
at once on two streams (is the link full duplex for copy-engine traffic?), for
whole 1 GiB copies and for 64 MiB chunks issued back to back.  One JSON line.
usage: python tools/pcie_duplex.py"""
import json
import time

import torch


def main():
    n = 1 << 30
    h_src = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n, dtype=torch.uint8).pin_memory()
    d_a = torch.empty(n, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}

    def timed(fn, reps=3):
        best = 1e9
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    for chunk in (n, 64 << 20):
        k = n // chunk

        def h2d():
            with torch.cuda.stream(s1):
                for i in range(k):
                    d_a[i * chunk:(i + 1) * chunk].copy_(h_src[i * chunk:(i + 1) * chunk], non_blocking=True)

        def d2h():
            with torch.cuda.stream(s2):
                for i in range(k):
                    h_dst[i * chunk:(i + 1) * chunk].copy_(d_b[i * chunk:(i + 1) * chunk], non_blocking=True)

        def both():
            h2d()
            d2h()

        t1, t2, tb = timed(h2d), timed(d2h), timed(both)
        out[f"chunk_{chunk >> 20}MiB"] = {"h2d_GiB_s": round(n / t1 / 2**30, 2), "d2h_GiB_s": round(n / t2 / 2**30, 2),
                                          "both_at_once_each_GiB_s": round(n / tb / 2**30, 2),
                                          "both_total_GiB_s": round(2 * n / tb / 2**30, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
