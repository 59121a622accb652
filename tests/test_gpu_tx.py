"""GPU parity of the batched send path (kmws_tx_batch) against
the oracle's restatement of WebSocket::Impl::sendWsFrame
(WebSocketImpl.cpp:405-436): per send, the header bytes (length = u32 of the
chain length, WSHandler::encodeFrameHeader) and, after ONE flush for all
sends, every segment masked in place with the key phase continuing across a
frame's segments (WSHandler.cpp:312-322); unmasked sends untouched; the
129-iovec limit (BUFFER_TOO_LONG, payload still masked as in kuma)."""
import random

import pytest

from kuma_amd import kmws
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")


def oracle_send(hdr, segments):
    """sendWsFrame: header for the chain length, payload masked across segments."""
    plen = sum(len(x) for x in segments)
    h = orc.Hdr(fin=hdr.fin, rsv1=hdr.rsv1, rsv2=hdr.rsv2, rsv3=hdr.rsv3, opcode=hdr.opcode, mask=hdr.mask,
                maskey=hdr.maskey, length=plen & 0xFFFFFFFF)
    wire_hdr = orc.encode_header(h)
    if hdr.mask and plen:
        masked = orc.mask_bytes(hdr.maskey, b"".join(bytes(x) for x in segments))
        out, pos = [], 0
        for x in segments:
            out.append(masked[pos:pos + len(x)])
            pos += len(x)
        return wire_hdr, out
    return wire_hdr, [bytes(x) for x in segments]


def random_send(rng, i):
    nseg = rng.choice([0, 1, 1, 2, 3, 7, 16])
    sizes = [rng.choice([0, 1, 3, 5, 100, 125, 126, 4096, 65535, 65536, 70001]) for _ in range(nseg)]
    segs = [bytearray(rng.getrandbits(8) for _ in range(n)) for n in sizes]
    hdr = kmws.Header(fin=rng.randrange(2), opcode=[0, 1, 2][i % 3], mask=1 if rng.random() < 0.8 else 0,
                      maskey=bytes(rng.getrandbits(8) for _ in range(4)))
    return hdr, segs


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_tx_batch_matches_send_ws_frame(seed):
    rng = random.Random(seed)
    b = kmws.TxBatch()
    sends = [random_send(rng, i) for i in range(60)]
    want = [oracle_send(h, segs) for h, segs in sends]
    got_hdrs = [b.add(h, segs) for h, segs in sends]
    assert got_hdrs == [w[0] for w in want]
    queued = sum(1 for h, segs in sends if h.mask and sum(map(len, segs)))
    assert b.pending() == queued
    assert b.flush() == queued and b.pending() == 0
    for (h, segs), (wh, wsegs) in zip(sends, want):
        assert [bytes(x) for x in segs] == wsegs
    assert b.flush() == 0  # empty batch


def test_tx_batch_iovec_limit_masks_like_kuma():
    b = kmws.TxBatch()
    key = bytes.fromhex("a1b2c3d4")
    hdr = kmws.Header(fin=1, opcode=2, mask=1, maskey=key)
    ok_segs = [bytearray([i & 0xFF]) for i in range(128)] + [bytearray()] * 5  # 128 non-empty + empties: fits
    long_segs = [bytearray([i & 0xFF]) for i in range(129)]
    want_ok = oracle_send(hdr, ok_segs)
    want_long = oracle_send(hdr, long_segs)
    assert b.add(hdr, ok_segs) == want_ok[0]
    with pytest.raises(kmws.KmwsError) as e:
        b.add(hdr, long_segs)
    assert e.value.status == kmws.ERR_BUFFER_TOO_LONG
    assert b.flush() == 2
    assert [bytes(x) for x in ok_segs] == want_ok[1]
    assert [bytes(x) for x in long_segs] == want_long[1]  # masked before the iovec count, as kuma


def test_tx_batch_then_decoder_roundtrip():
    """Client frames sent through the batch decode back (SERVER decoder on GPU)."""
    rng = random.Random(7)
    b = kmws.TxBatch()
    wire = bytearray()
    plain = []
    parts = []
    for i in range(40):
        n = rng.choice([0, 1, 125, 126, 4096, 65536, 100000])
        data = bytearray(rng.getrandbits(8) for _ in range(n))
        plain.append(bytes(data))
        cut = rng.randrange(n + 1)
        segs = [data[:cut], data[cut:]]
        hdr = kmws.Header(fin=1, opcode=2, mask=1, maskey=bytes(rng.getrandbits(8) for _ in range(4)))
        parts.append((b.add(hdr, segs), segs))
    b.flush()
    for h, segs in parts:
        wire += h + b"".join(bytes(x) for x in segs)
    d = kmws.WSHandler(kmws.SERVER)
    got = []
    d.setFrameCallback(lambda hd, p: got.append(p))
    assert d.handleData(bytes(wire)) == 0
    assert got == plain


def test_tx_batch_pinned_ring_zero_copy_and_mixed():
    """Segments inside an attached pinned send ring are masked in place there
    (zero-copy), others through staging -- also within one frame (phase runs
    across a ring segment and a pageable one); bytes around the segments in
    the ring are untouched."""
    import ctypes as C
    import numpy as np
    import torch
    rng = random.Random(11)
    ring = torch.from_numpy(np.frombuffer(bytes(rng.getrandbits(8) for _ in range(1 << 20)), dtype=np.uint8).copy())
    ring = ring.pin_memory()
    before = ring.numpy().copy()
    b = kmws.TxBatch()
    b.attach_ring(ring)
    base = ring.data_ptr()
    keep, expect_ring, expect_page = [], [], []
    pos = 3
    for i in range(50):
        key = bytes(rng.getrandbits(8) for _ in range(4))
        n1 = rng.choice([0, 1, 7, 125, 4096, 10000])
        n2 = rng.choice([0, 2, 126, 3000])
        o1 = pos
        pos += n1 + rng.randrange(0, 40)
        page = bytearray(rng.getrandbits(8) for _ in range(n2))
        pbuf = (C.c_uint8 * max(1, n2)).from_buffer(page) if n2 else None
        keep.append((page, pbuf))
        segs_plain = [bytes(before[o1:o1 + n1]), bytes(page)]
        hdr = kmws.Header(fin=1, opcode=2, mask=1, maskey=key)
        wh, wsegs = oracle_send(hdr, segs_plain)
        got = b.add_ptrs(hdr, [base + o1, C.cast(pbuf, C.c_void_p).value if pbuf else None], [n1, n2])
        assert got == wh
        expect_ring.append((o1, n1, wsegs[0]))
        expect_page.append((page, wsegs[1]))
    assert pos < ring.numel()
    b.flush()
    after = ring.numpy()
    want = before.copy()
    for o, n, w in expect_ring:
        want[o:o + n] = np.frombuffer(w, dtype=np.uint8)
    assert np.array_equal(after, want)
    for page, w in expect_page:
        assert bytes(page) == w
