"""Times kmws_pack_headers (with wire offsets) of ONE build of the library on
cfg4's 4 M x 4 KiB fragments; run once per build in the same gpurun call and
compare.  Usage: python tools/ab_pack_headers.py <lib.so> [reps]"""
import ctypes as C
import json
import sys

import numpy as np


def main():
    import torch
    L = C.CDLL(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    L.kmws_pack_headers_workspace_size.restype = C.c_size_t
    L.kmws_pack_headers_workspace_size.argtypes = [C.c_uint32]
    L.kmws_pack_headers.argtypes = [C.c_void_p] * 6 + [C.c_void_p, C.c_size_t, C.c_void_p]
    dev = torch.device("cuda")
    n = 4 << 20
    off = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    key = torch.randint(0, 2**31, (n,), dtype=torch.int64, device=dev)
    descs = torch.stack([off, 4096 | (key << 32)], dim=1).contiguous()
    fl = torch.full((n,), 0x100 | 0x82, dtype=torch.int16, device=dev)
    hdr = torch.empty(16 * n, dtype=torch.uint8, device=dev)
    hl = torch.empty(n, dtype=torch.uint8, device=dev)
    wo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ws = torch.empty(L.kmws_pack_headers_workspace_size(n), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def call():
        assert L.kmws_pack_headers(descs.data_ptr(), fl.data_ptr(), n, hdr.data_ptr(), hl.data_ptr(), wo.data_ptr(),
                                   ws.data_ptr(), ws.numel(), s) == 0
    call()
    torch.cuda.synchronize()
    ok = bool((wo[:n].cpu().numpy() == np.arange(n, dtype=np.int64) * 4104).all()) and int(wo[n]) == n * 4104
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    med = ts[len(ts) // 2]
    rec = {"lib": sys.argv[1], "frames": n, "us_median": med, "us_min": ts[0],
           "hbm_frac": 43 * n / (med * 1e-6) / 8e12, "offsets_ok": ok}
    if hasattr(L, "kmws_ab_trace_read"):  # tracing build: per-tile event times of one more call, us from the first start
        call()
        torch.cuda.synchronize()
        nt = (n + 2047) // 2048
        buf = np.zeros((1 << 16) * 6, dtype=np.uint64)
        L.kmws_ab_trace_read.argtypes = [C.c_void_p, C.c_size_t]
        assert L.kmws_ab_trace_read(buf.ctypes.data, buf.size) == 0
        ev = buf[:nt * 6].reshape(nt, 6).astype(np.float64)
        ev = (ev - ev[:, 0].min()) / 100.0  # s_memrealtime ticks at 100 MHz -> us
        names = ["start", "aggregate", "published", "pred_seen", "resolved", "end"]
        rec["trace_us"] = {nm: [round(float(np.percentile(ev[1:, k], q)), 2) for q in (0, 10, 50, 90, 100)]
                           for k, nm in enumerate(names)}
        rec["trace_note"] = "percentiles 0/10/50/90/100 over tiles 1.. of each event time"
        idx = np.argsort(ev[:, 1])[-5:]
        rec["last_aggregates"] = [[int(i), round(float(ev[i, 1]), 2)] for i in idx]
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
