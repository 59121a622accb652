"""Where the synchronous decoder's time per 64 KiB read goes (cfg1 shape):
feed of a chunk of 16 x 4 KiB UNMASKED frames (host parse only, no GPU) vs
MASKED frames (parse + staging + one GPU launch + wait + write-back), pageable
vs pinned chunk; plus memcpy into pinned memory and a bare torch launch+sync.
(The CPU decoder's time for the same read is bench.py --config cfg1's
cpu_baseline; profiles/r01i_cfg1_latency.txt has both.)"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from kuma_amd import kmws
    K = kmws.lib()
    n, L = 16, 4096
    rng = np.random.default_rng(1)
    payload = rng.integers(0, 256, size=n * L, dtype=np.uint8)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)

    def frames_wire(mask):
        """n x 4 KiB BINARY frames: 82 fe 10 00 [key] payload(^key)."""
        out = bytearray()
        for i in range(n):
            k = int(keys[i]).to_bytes(4, "little")
            p = payload[i * L:(i + 1) * L]
            out += bytes([0x82, (0x80 if mask else 0) | 126, L >> 8, L & 0xFF])
            if mask:
                out += k
                p = p ^ np.tile(np.frombuffer(k, dtype=np.uint8), L // 4)
            out += p.tobytes()
        return bytes(out)
    res = {}
    for name, mask in (("unmasked", 0), ("masked", 1)):
        wire = frames_wire(mask)
        for mem in ("pageable", "pinned"):
            mode = 1 if mask else 0  # SERVER needs masked frames, CLIENT unmasked
            d = K.kmws_decoder_create(mode, 0)
            if mem == "pinned":
                t = torch.empty(len(wire), dtype=torch.uint8).pin_memory()
                ptr = C.cast(t.data_ptr(), C.POINTER(C.c_uint8))
                src = torch.frombuffer(bytearray(wire), dtype=torch.uint8)
            else:
                b = bytearray(wire)
                ptr = (C.c_uint8 * len(b)).from_buffer(b)
            ts = []
            for i in range(300):
                if mem == "pinned":
                    t.copy_(src)
                else:
                    b[:] = wire
                t0 = time.perf_counter()
                r = K.kmws_decoder_feed(d, ptr, len(wire), C.cast(None, kmws.FRAME_CB), None)
                ts.append(time.perf_counter() - t0)
                assert r == 0, r
            K.kmws_decoder_destroy(d)
            res[f"{name}_{mem}_us"] = round(float(np.median(ts[50:])) * 1e6, 2)
    wire = frames_wire(1)
    # memcpy 64 KiB into pinned memory, bare launch + sync
    pin = torch.empty(1 << 16, dtype=torch.uint8).pin_memory()
    srcn = np.frombuffer(wire[:1 << 16], dtype=np.uint8)
    pn = pin.numpy()
    ts = []
    for i in range(300):
        t0 = time.perf_counter()
        np.copyto(pn, srcn)
        ts.append(time.perf_counter() - t0)
    res["memcpy_64k_to_pinned_us"] = round(float(np.median(ts[50:])) * 1e6, 2)
    x = torch.zeros(16, device="cuda")
    ts = []
    for i in range(300):
        t0 = time.perf_counter()
        x.add_(1)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["torch_launch_sync_us"] = round(float(np.median(ts[50:])) * 1e6, 2)
    print(res)


if __name__ == "__main__":
    main()
