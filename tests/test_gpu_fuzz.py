"""Randomized GPU parity against the oracle, time-budgeted (KMWS_FUZZ_SECONDS,
default 8 s per path): every case draws a random layout and compares every
byte with the oracle's restatement of kuma's src/ws.

  unmask   random frame layouts (sizes 0 .. 300 KiB, gaps, misalignment,
           zero keys, > 256 frames per tile) through every unmask schedule
           (WSHandler.cpp:303-310 per frame);
  encode   random batches through kmws_encode_batch (encodeFrameHeader
           :46-106 + masked payload) and back through kmws_unpack_headers
           (:118-234) + kmws_gather_unmask;
  decoder  random client streams (any opcode, control frames, 0 .. 200 KiB
           payloads) fed to the GPU decoder in random chunkings: return codes,
           every callback field and the in-place bytes (:108-280);
  tx       random sends through kmws_tx_batch (WebSocketImpl.cpp:405-436).

Seeds are printed on failure; the run's case counts go to stdout."""
import os
import random
import time

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
BUDGET = float(os.environ.get("KMWS_FUZZ_SECONDS", "8"))
# product default + every placement kind with automatic, non-temporal and temporal stores
SCHEDULES = [None] + [k | s for k in range(6) for s in (0, 1 << 29, 1 << 30)]


@pytest.fixture(scope="module")
def T():
    import torch
    from kuma_amd import kmws
    if not torch.cuda.is_available() or kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    return torch


def rand_lens(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        return rng.integers(0, 40, size=n)
    if kind == 1:
        return rng.choice([0, 1, 2, 3, 4, 15, 16, 17, 124, 125, 126, 127, 4095, 4096, 4097, 65535, 65536, 65537],
                          size=n)
    if kind == 2:
        k = rng.integers(0, 12, size=n)
        return 128 * (2 ** k) - rng.integers(0, 64, size=n)
    return rng.integers(0, 300000, size=n)


def budget_loop(fn):
    t_end = time.time() + BUDGET
    cases = 0
    while cases < 3 or time.time() < t_end:
        seed = int.from_bytes(os.urandom(4), "little")
        try:
            fn(np.random.default_rng(seed))
        except AssertionError as e:
            raise AssertionError(f"seed {seed}: {e}") from e
        cases += 1
    return cases


def test_fuzz_unmask(T):
    from kuma_amd import kmws

    def case(rng):
        n = int(rng.integers(1, 400))
        lens = rand_lens(rng, n).astype(np.int64)
        gaps = rng.integers(0, 64, size=n) * int(rng.choice([1, 16]))
        starts = np.cumsum(np.concatenate([[0], gaps + lens]))
        offs = (starts[:-1] + gaps).astype(np.uint64) + np.uint64(rng.integers(0, 16))
        total = int(offs[-1] + lens[-1]) + int(rng.integers(0, 40))
        d = np.zeros(n, dtype=orc.DESC_DTYPE)
        d["off"], d["len"] = offs, lens
        d["key"] = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        d["key"][rng.random(n) < 0.05] = 0
        buf = rng.integers(0, 256, size=total, dtype=np.uint8)
        want = buf.copy()
        orc.unmask_batch(want, d)
        pad = (-total) % 16
        d_buf = T.from_numpy(np.concatenate([buf, np.zeros(pad, np.uint8)])).cuda()
        d_desc = T.from_numpy(d.view(np.int64).reshape(-1, 2).copy()).cuda()
        ws = kmws.Workspace(kmws.unmask_workspace_size(total))
        v = SCHEDULES[int(rng.integers(0, len(SCHEDULES)))]
        kmws.unmask_batch(d_buf, d_desc, ws, total, schedule=v)
        T.cuda.synchronize()
        assert ws.status() == 0, f"status (schedule {v})"
        got = d_buf.cpu().numpy()[:total]
        assert np.array_equal(got, want), f"bytes differ (schedule {v}, n {n})"

    print("unmask cases:", budget_loop(case))


def test_fuzz_encode_unpack_gather(T):
    from kuma_amd import kmws

    def case(rng):
        n = int(rng.integers(1, 300))
        lens = rand_lens(rng, n).astype(np.int64)
        op = rng.choice([0, 1, 2, 3, 9, 10], size=n)
        ctl = op >= 8
        lens = np.where(ctl, np.minimum(lens, 125), lens)
        fin = np.where(ctl, 1, rng.integers(0, 2, size=n))
        mask = np.ones(n, dtype=np.int64)  # SERVER-side decode needs masked frames
        flags = ((fin << 7) | op | (mask << 8)).astype(np.uint32)
        keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        gaps = rng.integers(0, 40, size=n)
        starts = np.cumsum(np.concatenate([[0], gaps + lens]))
        offs = (starts[:-1] + gaps).astype(np.uint64)
        src = rng.integers(0, 256, size=int(starts[-1]) + 64, dtype=np.uint8)
        want, want_off = orc.encode_batch(src, offs, lens, flags, keys)
        total = len(want)
        d_src = T.from_numpy(np.concatenate([src, np.zeros((-len(src)) % 16 + 16, np.uint8)])).cuda()
        descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64))
        fl = T.from_numpy(flags.astype(np.int16)).cuda()
        wire = T.zeros(total + 32, dtype=T.uint8, device="cuda")
        wire_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
        ws = kmws.Workspace(kmws.copy_workspace_size(n, wire.numel()))
        kmws.encode_batch(d_src, descs, fl, wire, wire_off, ws)
        T.cuda.synchronize()
        assert ws.status() == 0
        assert np.array_equal(wire.cpu().numpy()[:total], want), "wire image differs"
        assert np.array_equal(wire_off.cpu().numpy()[:n].astype(np.uint64), want_off)
        out_desc = T.zeros((n, 2), dtype=T.int64, device="cuda")
        out_err = T.full((n,), 99, dtype=T.uint8, device="cuda")
        ws_u = kmws.Workspace(16)
        kmws.unpack_headers(wire, wire_off[:n], kmws.SERVER, out_desc, None, out_err, ws_u, wire_len=total)
        dst = T.zeros(int(lens.sum()) + 32, dtype=T.uint8, device="cuda")
        dst_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
        ws_g = kmws.Workspace(kmws.copy_workspace_size(n, dst.numel()))
        kmws.gather_unmask(wire, out_desc, dst, dst_off, ws_g)
        T.cuda.synchronize()
        assert int(out_err.max()) == 0 and ws_u.status() == 0 and ws_g.status() == 0
        orig = b"".join(bytes(src[int(o):int(o) + int(L)]) for o, L in zip(offs, lens))
        assert bytes(dst.cpu().numpy()[:len(orig)]) == orig, "gathered payloads differ"
        # the fused forms: parse in the gather's scan; parse + plan, then unmask in place
        fd = T.zeros((n, 2), dtype=T.int64, device="cuda")
        fe = T.full((n,), 99, dtype=T.uint8, device="cuda")
        dst2 = T.zeros(dst.numel(), dtype=T.uint8, device="cuda")
        doff2 = T.zeros(n + 1, dtype=T.int64, device="cuda")
        kmws.unpack_gather(wire, wire_off[:n], kmws.SERVER, fd, None, fe, dst2, doff2, ws_g, wire_len=total)
        T.cuda.synchronize()
        assert ws_g.status() == 0 and T.equal(fd, out_desc) and T.equal(fe, out_err) and T.equal(doff2, dst_off)
        assert T.equal(dst2, dst), "fused gather differs"
        w2 = wire.clone()
        ws_m = kmws.Workspace(kmws.unmask_workspace_size(total))
        kmws.unpack_unmask(w2, wire_off[:n], kmws.SERVER, fd, None, fe, ws_m, wire_len=total)
        T.cuda.synchronize()
        assert ws_m.status() == 0 and T.equal(fd, out_desc)
        w2h = w2.cpu().numpy()
        dd = out_desc.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
        assert b"".join(bytes(w2h[int(o):int(o) + int(L)]) for o, L in zip(dd["off"], dd["len"])) == orig, \
            "fused in-place decode differs"
        # header-only pack: each 16-B slot is the wire image's header, zero-padded
        hdr = T.zeros(16 * n, dtype=T.uint8, device="cuda")
        hl = T.zeros(n, dtype=T.uint8, device="cuda")
        kmws.pack_headers(descs, fl, hdr, hl)
        # device header-chain walk of the wire cut into random streams at frame boundaries
        cuts = np.unique(np.concatenate([[0, n], rng.integers(0, n + 1, size=int(rng.integers(0, 8)))]))
        woff = np.concatenate([want_off, [total]]).astype(np.int64)
        soff = T.from_numpy(woff[cuts]).cuda()
        h_w, n_w, c_w = kmws.find_headers_streams(wire, soff, n, wire_len=total)
        T.cuda.synchronize()
        H, HL = hdr.cpu().numpy().reshape(n, 16), hl.cpu().numpy()
        for i in range(n):
            a = int(want_off[i])
            b = int(want_off[i + 1]) if i + 1 < n else total
            assert bytes(H[i, :int(HL[i])]) == bytes(want[a:a + int(HL[i])]) and not H[i, int(HL[i]):].any(), i
            assert int(HL[i]) + int(lens[i]) == b - a, i
        h_w, n_w, c_w = h_w.cpu().numpy(), n_w.cpu().numpy(), c_w.cpu().numpy()
        for j in range(len(cuts) - 1):
            lo, hi = int(cuts[j]), int(cuts[j + 1])
            assert int(n_w[j]) == hi - lo and int(c_w[j]) == int(woff[hi] - woff[lo]), j
            assert np.array_equal(h_w[j, :hi - lo], woff[lo:hi]), j

    print("encode/unpack/gather cases:", budget_loop(case))


def client_stream(rng):
    parts = []
    for _ in range(int(rng.integers(1, 40))):
        op = int(rng.choice([0, 1, 2, 3, 9, 10]))
        n = int(rng.choice([0, 1, 5, 125, 126, 127, 1000, 65535, 65536, 70000, 200000]))
        if op >= 8:
            n = min(n, 125)
        key = bytes(rng.integers(0, 256, size=4, dtype=np.uint8))
        payload = bytes(rng.integers(0, 256, size=n, dtype=np.uint8))
        h = orc.Hdr(fin=1 if op >= 8 else int(rng.integers(0, 2)), opcode=op, mask=1, maskey=key, length=n)
        parts.append(orc.encode_header(h) + orc.mask_bytes(key, payload))
    return b"".join(parts)


def test_fuzz_decoder(T):
    from kuma_amd import kmws

    def key(hd, p):
        return (hd.fin, hd.rsv1, hd.rsv2, hd.rsv3, hd.opcode, hd.mask, hd.plen, hd.xpl64, hd.maskey, hd.length, p)

    def case(rng):
        stream = client_stream(rng)
        if rng.random() < 0.2:  # a corrupted byte: error paths must agree too
            i = int(rng.integers(0, len(stream)))
            stream = stream[:i] + bytes([int(rng.integers(0, 256))]) + stream[i + 1:]
        chunk = int(rng.choice([0, 1, 7, 100, 4096, 65536, 1 << 20]))
        if chunk == 1 and len(stream) > 20000:
            chunk = 997
        step = chunk if chunk > 0 else max(1, len(stream))
        d = orc.Decoder(orc.SERVER)
        h = kmws.WSHandler(kmws.SERVER)
        got = []
        h.setFrameCallback(lambda hd, p: got.append(key(hd, p)))
        r_o, r_g, b_o, b_g = [], [], [], []
        for i in range(0, max(1, len(stream)), step):
            po, pg = bytearray(stream[i:i + step]), bytearray(stream[i:i + step])
            r_o.append(d.feed(po))
            r_g.append(h.handleData(pg))
            b_o.append(bytes(po))
            b_g.append(bytes(pg))
        assert r_g == r_o, "return codes"
        assert got == [f.key() for f in d.frames], "callbacks"
        assert b_g == b_o, "in-place bytes"

    print("decoder cases:", budget_loop(case))


def test_fuzz_tx_batch(T):
    from kuma_amd import kmws

    def case(rng):
        b = kmws.TxBatch()
        sends = []
        for i in range(int(rng.integers(1, 60))):
            segs = [bytearray(rng.integers(0, 256, size=int(rng.choice([0, 1, 3, 126, 4096, 70000])),
                                           dtype=np.uint8).tobytes()) for _ in range(int(rng.integers(0, 6)))]
            key = bytes(rng.integers(0, 256, size=4, dtype=np.uint8))
            hdr = kmws.Header(fin=int(rng.integers(0, 2)), opcode=int(rng.choice([0, 1, 2])),
                              mask=int(rng.random() < 0.9), maskey=key)
            plain = b"".join(bytes(x) for x in segs)
            h = orc.Hdr(fin=hdr.fin, opcode=hdr.opcode, mask=hdr.mask, maskey=key, length=len(plain))
            want_body = orc.mask_bytes(key, plain) if hdr.mask and plain else plain
            assert b.add(hdr, segs) == orc.encode_header(h)
            sends.append((segs, want_body))
        b.flush()
        for segs, want in sends:
            assert b"".join(bytes(x) for x in segs) == want

    print("tx cases:", budget_loop(case))


def test_fuzz_mask_chain_both_store_kinds(T):
    """Random kmws_mask_host_chain calls (1-3 segments, 0 .. 256 KiB, odd
    offsets) on the resident grid, some right after device batches were
    enqueued: small jobs and jobs under a running batch write through, large
    ones on an idle device release the L2 (kmws_resident.hip
    kResWriteThroughWords); every byte equals the oracle's, the batch's too."""
    from kuma_amd import kmws
    n, frame = 16384, 65536  # 1 GiB on the device
    base = T.empty(n * frame, dtype=T.uint8, device="cuda")
    descs = T.empty((n, 2), dtype=T.int64, device="cuda")
    kmws.fill_synthetic(base, 5)
    kmws.fill_uniform_descs(descs, frame, frame, 9)
    ws = kmws.Workspace(kmws.unmask_workspace_size(base.numel()))
    kmws.unmask_plan(descs, ws, base.numel())
    T.cuda.synchronize()
    applies = [0]
    s0 = kmws.resident_stores()

    def case(rng):
        if rng.random() < 0.3:
            for _ in range(4):
                kmws.unmask_apply(base, descs, ws)
            applies[0] += 4
        key = bytes(rng.integers(0, 256, size=4, dtype=np.uint8))
        sizes = [int(rng.choice([0, 1, 15, 4096, 16369, 16401, 65536, 100000])) for _ in range(int(rng.integers(1, 4)))]
        total = sum(sizes)
        if total > 262144:
            sizes = [262144 // len(sizes)] * len(sizes)
        data = [rng.integers(0, 256, size=s + 17, dtype=np.uint8).tobytes() for s in sizes]
        offs = [int(rng.integers(0, 17)) for _ in sizes]
        segs = [bytearray(d[o:o + s]) for d, o, s in zip(data, offs, sizes)]
        plain = b"".join(bytes(x) for x in segs)
        kmws.handle_data_mask(key, segs)
        assert b"".join(bytes(x) for x in segs) == orc.mask_bytes(key, plain)

    print("mask chain cases:", budget_loop(case))
    if applies[0] % 2 == 0:
        kmws.unmask_apply(base, descs, ws)
    T.cuda.synchronize()
    assert kmws.check_unmasked(base, 5, descs) == 0
    # the batches above were queued faster than they ran, so the device may
    # have been busy throughout (every job written through); once the estimate
    # runs out (it adds up per batch, so it can trail the real end by a second
    # after 8 s of them), large jobs release
    t_end = time.time() + 5
    while kmws.device_batch_busy() and time.time() < t_end:
        time.sleep(0.005)
    assert not kmws.device_batch_busy()
    rng = np.random.default_rng(1)
    for _ in range(3):
        seg = bytearray(rng.integers(0, 256, size=65536, dtype=np.uint8).tobytes())
        want = orc.mask_bytes(b"\x01\x02\x03\x04", bytes(seg))
        kmws.handle_data_mask(b"\x01\x02\x03\x04", [seg])
        assert bytes(seg) == want
    s1 = kmws.resident_stores()
    assert s1["write_through"] > s0["write_through"] and s1["released"] > s0["released"], (s0, s1)
