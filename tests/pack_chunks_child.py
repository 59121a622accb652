"""Child process of tests/test_gpu_pack.py::test_pack_chunks_knob: the library
reads KMWS_PACK_CHUNKS once per process, so the chunked pack pipeline (prologue
grids on a side stream under per-chunk copy grids) is checked here, with
the knob set by the parent.  Encode and gather-unmask of several layouts, each
compared byte for byte with the oracle; exit status 0 = all equal."""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle as orc  # noqa: E402
from test_gpu_pack import frames, gpu_encode, src_arena  # noqa: E402


def main():
    import torch as T
    from kuma_amd import kmws
    assert os.environ.get("KMWS_PACK_CHUNKS"), "run by test_pack_chunks_knob"
    for kind, n in (("frag4k", 16 * 640), ("tiny", 9000), ("mixed", 2600), ("zipf", 2100)):
        for aligned in (True, False):
            rng = np.random.default_rng(zlib.crc32(f"chunks-{kind}-{aligned}".encode()))
            lens, flags, keys = frames(rng, kind, n)
            src, offs = src_arena(rng, lens, aligned)
            want, want_off = orc.encode_batch(src, offs, lens, flags, keys)
            got, off, st, total = gpu_encode(T, src, offs, lens, flags, keys)
            assert st == 0 and total == len(want), (kind, aligned, st)
            assert np.array_equal(off[:n].astype(np.uint64), want_off), (kind, aligned)
            assert np.array_equal(got[:total], want), ("encode", kind, aligned)
            # gather-unmask of the GPU wire: the dense payloads equal the original source bytes
            m = (flags >> 8) & 1
            hl = np.where(lens <= 125, 2, np.where(lens <= 65535, 4, 10)) + 4 * m
            descs = kmws.make_descs(off[:n].astype(np.int64) + hl, lens,
                                    np.where(m, keys, 0).astype(np.uint32).astype(np.int64))
            P = int(lens.sum())
            dst = T.zeros(P + 32, dtype=T.uint8, device="cuda")
            dst_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
            ws = kmws.Workspace(kmws.copy_workspace_size(n, dst.numel()))
            d_wire = T.from_numpy(np.concatenate([want, np.zeros((-len(want)) % 16 + 16, np.uint8)])).cuda()
            kmws.gather_unmask(d_wire, descs, dst, dst_off, ws)
            T.cuda.synchronize()
            assert ws.status() == 0, ("gather", kind, aligned)
            orig = b"".join(bytes(src[int(o):int(o) + int(L)]) for o, L in zip(offs, lens))
            assert bytes(dst.cpu().numpy()[:P]) == orig, ("gather", kind, aligned)
    # dst too small: the wire exceeds dst_cap, so the unit bases run past the
    # records the workspace holds; the status word is set, nothing is written
    # and (the point) no copy wave reads a record slot past the workspace
    n = 16 * 640
    rng = np.random.default_rng(zlib.crc32(b"chunks-small-dst"))
    lens, flags, keys = frames(rng, "frag4k", n)
    src, offs = src_arena(rng, lens, True)
    want, _ = orc.encode_batch(src, offs, lens, flags, keys)
    for cap in (len(want) - 1, len(want) // 4):
        got, off, st, total = gpu_encode(T, src, offs, lens, flags, keys, cap=cap)
        assert st != 0, ("encode small dst", cap)
        assert (got == 0xEE).all(), ("encode small dst wrote", cap)
    descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64))
    d_src = T.from_numpy(np.concatenate([src, np.zeros((-len(src)) % 16 + 16, np.uint8)])).cuda()
    P = int(lens.sum())
    for cap in (P - 1, P // 4):
        dst = T.full((cap - cap % 16,), 0xEE, dtype=T.uint8, device="cuda")
        dst_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
        ws = kmws.Workspace(kmws.copy_workspace_size(n, dst.numel()))
        kmws.gather_unmask(d_src, descs, dst, dst_off, ws)
        T.cuda.synchronize()
        assert ws.status() != 0, ("gather small dst", cap)
        assert bool((dst == 0xEE).all()), ("gather small dst wrote", cap)
    print("pack chunks ok", os.environ["KMWS_PACK_CHUNKS"])


if __name__ == "__main__":
    main()
