"""The batch entry points are stream-ordered with no host synchronisation, so a
whole device pipeline can be captured once into a HIP graph and replayed: the
send side (kmws_encode_batch: scan + prologue + copy, header pack + mask) and
the receive side (kmws_unpack_headers -> kmws_gather_unmask, and the in-place
kmws_unmask_batch).  Each replay must give the oracle's bytes (encode:
WSHandler::encodeFrameHeader + handleDataMask per frame, WSHandler.cpp:46-106,
303-310), including replays on new inputs copied into the captured buffers.
(With hipMemsetAsync zeroing the status words, replays on this runtime left
pointer values in them: the calls zero them with a kernel instead.)"""
import zlib

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def T():
    import torch
    from kuma_amd import kmws
    if not torch.cuda.is_available() or kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    return torch


def batch(rng, n):
    lens = rng.choice([0, 1, 3, 125, 126, 1000, 4096, 65535, 65536, 70001], size=n).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16 + 16)[:-1]]).astype(np.uint64)
    src = rng.integers(0, 256, size=int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    fin = rng.integers(0, 2, size=n)
    op = rng.choice([0, 1, 2], size=n)
    flags = ((fin << 7) | op | (1 << 8)).astype(np.uint32)   # masked (client) frames
    keys = rng.integers(1, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    return src, offs, lens, flags, keys


@pytest.mark.parametrize("n", [1, 37, 600])
def test_graph_replay_encode_decode(T, n):
    from kuma_amd import kmws
    rng = np.random.default_rng(zlib.crc32(f"graph-{n}".encode()))
    src, offs, lens, flags, keys = batch(rng, n)
    want, want_off = orc.encode_batch(src, offs, lens, flags, keys)
    total = len(want)
    dev = "cuda"
    d_src = T.zeros(len(src) + 16, dtype=T.uint8, device=dev)
    descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64))
    fl = T.from_numpy(flags.astype(np.int16)).to(dev)
    wire = T.zeros(total + 16, dtype=T.uint8, device=dev)
    wire_off = T.zeros(n + 1, dtype=T.int64, device=dev)
    ws_e = kmws.Workspace(kmws.copy_workspace_size(n, total))
    out_desc = T.zeros((n, 2), dtype=T.int64, device=dev)
    out_err = T.zeros(n, dtype=T.uint8, device=dev)
    ws_u = kmws.Workspace(kmws.lib().kmws_unpack_workspace_size())
    P = int(lens.sum())
    dense = T.zeros(P + 16, dtype=T.uint8, device=dev)
    dense_off = T.zeros(n + 1, dtype=T.int64, device=dev)
    ws_g = kmws.Workspace(kmws.copy_workspace_size(n, P + 16))
    ws_m = kmws.Workspace(kmws.unmask_workspace_size(total))
    inplace = T.zeros(total + 16, dtype=T.uint8, device=dev)

    def pipeline():
        kmws.encode_batch(d_src, descs, fl, wire, wire_off, ws_e)
        kmws.unpack_headers(wire, wire_off[:n], kmws.SERVER, out_desc, None, out_err, ws_u, wire_len=total)
        kmws.gather_unmask(wire, out_desc, dense, dense_off, ws_g)
        inplace.copy_(wire)
        kmws.unmask_batch(inplace, out_desc, ws_m, total)

    d_src[:len(src)].copy_(T.from_numpy(src))
    s = T.cuda.Stream()
    s.wait_stream(T.cuda.current_stream())
    with T.cuda.stream(s):  # warm (and load every kernel) before capture
        pipeline()
    T.cuda.current_stream().wait_stream(s)
    T.cuda.synchronize()
    g = T.cuda.CUDAGraph()
    with T.cuda.graph(g):
        pipeline()
    T.cuda.synchronize()

    def check(src_now, want_now):
        wl = (("encode", ws_e), ("unpack", ws_u), ("gather", ws_g), ("unmask", ws_m))
        st = {k: w.status() for k, w in wl}
        assert all(v == 0 for v in st.values()), st
        assert bytes(wire.cpu().numpy()[:total]) == bytes(want_now)
        assert (out_err.cpu().numpy() == 0).all()
        plain = b"".join(bytes(src_now[int(o):int(o) + int(L)]) for o, L in zip(offs, lens))
        assert bytes(dense.cpu().numpy()[:P]) == plain
        ip = inplace.cpu().numpy()
        dd = out_desc.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
        assert b"".join(bytes(ip[int(o):int(o) + int(L)]) for o, L in zip(dd["off"], dd["len"])) == plain

    for rep in range(3):  # replays on fresh inputs written into the captured source buffer
        wire.fill_(0xEE)
        dense.fill_(0xEE)
        src2 = np.random.default_rng(rep).integers(0, 256, size=len(src), dtype=np.uint8)
        want2, _ = orc.encode_batch(src2, offs, lens, flags, keys)
        d_src[:len(src)].copy_(T.from_numpy(src2))
        g.replay()
        T.cuda.synchronize()
        check(src2, want2)


def test_graph_replay_pack_headers(T):
    """kmws_pack_headers with wire offsets (zero kernel + one-pass look-back
    kernel over 2048-frame tiles) captured once and replayed on new lengths,
    keys and flags written into the captured buffers: every replay's slots,
    lengths and offsets equal the vectorised encodeFrameHeader and the exclusive
    scan (the tile states are re-zeroed inside the graph)."""
    from kuma_amd import kmws
    from test_gpu_pack import np_header_slots
    n = 300_001  # 147 tiles
    dev = "cuda"
    descs = T.zeros((n, 2), dtype=T.int64, device=dev)
    fl = T.zeros(n, dtype=T.int16, device=dev)
    hdr = T.zeros(16 * n, dtype=T.uint8, device=dev)
    hl = T.zeros(n, dtype=T.uint8, device=dev)
    woff = T.zeros(n + 1, dtype=T.int64, device=dev)
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))

    def inputs(seed):
        rng = np.random.default_rng(seed)
        lens = rng.choice([0, 9, 125, 126, 4096, 65536, 200000], size=n).astype(np.int64)
        flags = (rng.integers(0, 256, size=n) | (rng.integers(0, 2, size=n) << 8)).astype(np.uint32)
        keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        descs.copy_(kmws.make_descs(np.zeros(n, np.int64), lens, keys.astype(np.int64)))
        fl.copy_(T.from_numpy(flags.astype(np.int16)))
        return lens, flags, keys

    inputs(99)
    s = T.cuda.Stream()
    s.wait_stream(T.cuda.current_stream())
    with T.cuda.stream(s):
        kmws.pack_headers(descs, fl, hdr, hl, woff, ws)
    T.cuda.current_stream().wait_stream(s)
    T.cuda.synchronize()
    g = T.cuda.CUDAGraph()
    with T.cuda.graph(g):
        kmws.pack_headers(descs, fl, hdr, hl, woff, ws)
    T.cuda.synchronize()
    for rep in range(3):
        lens, flags, keys = inputs(rep)
        woff.fill_(-1)
        g.replay()
        T.cuda.synchronize()
        S, H = np_header_slots(lens, flags, keys)
        assert ws.status() == 0, rep
        assert np.array_equal(hdr.cpu().numpy().reshape(n, 16), S), rep
        assert np.array_equal(hl.cpu().numpy(), H), rep
        assert np.array_equal(woff.cpu().numpy(), np.concatenate([[0], np.cumsum(lens + H.astype(np.int64))])), rep


def test_pack_headers_beside_a_streaming_kernel(T):
    """The one-pass header pack's blocks wait on lower-indexed blocks only, so it
    completes (and is exact) while another stream keeps the CUs busy: a 4 GiB
    in-place unmask runs on a second stream during three pack_headers calls of
    1 M frames (512 tiles, more than one block per CU)."""
    from kuma_amd import kmws
    from test_gpu_pack import np_header_slots
    n = 1 << 20
    rng = np.random.default_rng(5)
    lens = rng.choice([0, 5, 126, 4096, 70000], size=n).astype(np.int64)
    flags = (rng.integers(0, 256, size=n) | (1 << 8)).astype(np.uint32)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    descs = kmws.make_descs(np.zeros(n, np.int64), lens, keys.astype(np.int64))
    fl = T.from_numpy(flags.astype(np.int16)).cuda()
    hdr = T.zeros(16 * n, dtype=T.uint8, device="cuda")
    woff = T.zeros(n + 1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))
    L = 65536
    m = (4 << 30) // L
    big = T.empty(m * L, dtype=T.uint8, device="cuda")
    kmws.fill_synthetic(big, 11)
    bdesc = T.empty((m, 2), dtype=T.int64, device="cuda")
    kmws.fill_uniform_descs(bdesc, L, L, 12)
    wsb = kmws.Workspace(kmws.unmask_workspace_size(m * L))
    T.cuda.synchronize()
    side = T.cuda.Stream()
    with T.cuda.stream(side):
        for _ in range(6):  # even: the batch ends masked, as generated
            kmws.unmask_batch(big, bdesc, wsb, m * L)
    for _ in range(3):
        woff.fill_(-1)
        kmws.pack_headers(descs, fl, hdr, None, woff, ws)
    T.cuda.synchronize()
    S, H = np_header_slots(lens, flags, keys)
    assert ws.status() == 0 and wsb.status() == 0
    assert np.array_equal(hdr.cpu().numpy().reshape(n, 16), S)
    assert np.array_equal(woff.cpu().numpy(), np.concatenate([[0], np.cumsum(lens + H.astype(np.int64))]))
    kmws.unmask_batch(big, bdesc, wsb, m * L)
    T.cuda.synchronize()
    assert kmws.check_unmasked(big, 11, bdesc) == 0
