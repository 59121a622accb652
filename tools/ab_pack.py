"""Times the copy kernels (encode / gather) of ONE build of the library, loaded
alone (two builds in one process interfere): run it once per build in the same
gpurun call and compare.  Usage: python tools/ab_pack.py <lib.so> [cfg3,cfg4,u64k,small]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def bind(path):
    L = C.CDLL(path)
    L.kmws_fill_synthetic.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p]
    L.kmws_copy_workspace_size.restype = C.c_size_t
    L.kmws_copy_workspace_size.argtypes = [C.c_uint32, C.c_uint64]
    L.kmws_encode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64,
                                    C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    L.kmws_gather_unmask.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p,
                                     C.c_void_p, C.c_size_t, C.c_void_p]
    return L


def main():
    import torch
    import bench_configs as bc
    libs = {"lib": bind(sys.argv[1])}
    L0 = libs["lib"]

    def make_descs(off, length, key):
        off = torch.as_tensor(off, dtype=torch.int64)
        lk = (torch.as_tensor(length, dtype=torch.int64) & 0xFFFFFFFF) | (torch.as_tensor(key, dtype=torch.int64) << 32)
        return torch.stack([off, lk], dim=1).contiguous().to(dev)
    dev = torch.device("cuda")
    s = torch.cuda.current_stream().cuda_stream
    out = {}
    for cfg in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("cfg3", "cfg4")):
        rng = np.random.default_rng(bc.SEED)
        if cfg == "cfg3":
            lens = bc.zipf_lens(rng, 4_000_000)
            n = int(np.searchsorted(np.cumsum(lens), 8 * 2**30)) + 1
            lens = lens[:n]
        elif cfg == "u64k":  # uniform 64 KiB frames, 8 GiB
            n = 1 << 17
            lens = np.full(n, 65536, np.int64)
        elif cfg == "small":  # 8 M frames of 1-300 bytes (chat-sized messages)
            n = 1 << 23
            lens = rng.integers(1, 301, n).astype(np.int64)
        else:
            n = 4 << 20
            lens = np.full(n, 4096, np.int64)
        P = int(lens.sum())
        src_off = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]]).astype(np.int64)
        src = torch.empty(int(src_off[-1] + lens[-1] + 32), dtype=torch.uint8, device=dev)
        assert libs["lib"].kmws_fill_synthetic(src.data_ptr(), src.numel(), bc.SEED, s) == 0
        descs = make_descs(src_off, lens, bc.splitmix_keys(bc.SEED ^ 3, n).astype(np.int64))
        fl = torch.from_numpy((0x80 | 2 | 0x100) * np.ones(n, np.int16)).to(dev)
        hl = np.where(lens <= 125, 2, np.where(lens <= 65535, 4, 10)) + 4
        H = int(hl.sum())
        wires = {}
        for name, L in libs.items():
            wire = torch.empty(P + H + 16, dtype=torch.uint8, device=dev)
            woff = torch.empty(n + 1, dtype=torch.int64, device=dev)
            wsz = L.kmws_copy_workspace_size(n, wire.numel())
            ws = torch.empty(wsz, dtype=torch.uint8, device=dev)
            dst = torch.empty(P + 16, dtype=torch.uint8, device=dev)
            doff = torch.empty(n + 1, dtype=torch.int64, device=dev)
            gd = torch.stack([woff[:n] + torch.from_numpy(hl).to(dev), descs[:, 1]], 1).contiguous()

            def enc():
                assert L.kmws_encode_batch(src.data_ptr(), descs.data_ptr(), fl.data_ptr(), n, wire.data_ptr(),
                                           wire.numel(), woff.data_ptr(), ws.data_ptr(), wsz, s) == 0

            def gat():
                assert L.kmws_gather_unmask(wire.data_ptr(), gd.data_ptr(), n, dst.data_ptr(), dst.numel(),
                                            doff.data_ptr(), ws.data_ptr(), wsz, s) == 0
            enc()
            torch.cuda.synchronize()
            gd.copy_(torch.stack([woff[:n] + torch.from_numpy(hl).to(dev), descs[:, 1]], 1))
            wires[name] = (enc, gat, wire)
        for name, (enc, gat, wire) in wires.items():
            enc()
        torch.cuda.synchronize()
        res = {"n": n, "payload": P}
        for rnd in range(3):  # interleave to cancel drift
            for name, (enc, gat, _) in wires.items():
                te = bc.timed(torch, enc, 5)
                tg = bc.timed(torch, gat, 5)
                res.setdefault(name, []).append({"enc_frac": (2 * P + H) / te / 8e12,
                                                 "gat_frac": (2 * P) / tg / 8e12})
        if hasattr(L0, "kmws_ab_trace_pro_read"):  # tracing build: prologue phases of one more encode / gather
            for name, (enc, gat, _) in wires.items():
                for label, fn in (("enc", enc), ("gat", gat)):
                    fn()
                    torch.cuda.synchronize()
                    buf = np.zeros((1 << 16) * 8, dtype=np.uint64)
                    L0.kmws_ab_trace_pro_read.argtypes = [C.c_void_p, C.c_size_t]
                    assert L0.kmws_ab_trace_pro_read(buf.ctypes.data, buf.size) == 0
                    nb = min((n + 255) // 256, 1 << 16)
                    ev = buf[:nb * 8].reshape(nb, 8)[:, :6].astype(np.float64)
                    ev = (ev - ev[:, 0].min()) / 100.0  # us from the first block's start
                    ph = ["start", "scan", "src_loaded", "composed", "edges_out", "end"]
                    res[f"trace_{label}"] = {p_: [round(float(np.percentile(ev[:, k], q)), 2) for q in (0, 10, 50, 90, 100)]
                                             for k, p_ in enumerate(ph)}
                    d = np.diff(ev, axis=1)
                    res[f"phase_us_{label}"] = {f"{ph[k]}->{ph[k+1]}": [round(float(np.percentile(d[:, k], q)), 2)
                                                                         for q in (50, 90, 100)] for k in range(5)}
        out[cfg] = res
        del wires, src, descs
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
