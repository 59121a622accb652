"""GPU parity of the WSHandler-compatible streaming decoder (kmws_decoder_feed,
whose masked payloads are unmasked by the HIP kernel) against the oracle:
return codes, callback sequence (every FrameHeader field + payload) and the
in-place unmask of the caller's buffer."""
import json
import os
import random

import pytest

from kuma_amd import kmws
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")


def frame_key(hd, p):
    return (hd.fin, hd.rsv1, hd.rsv2, hd.rsv3, hd.opcode, hd.mask, hd.plen, hd.xpl64, hd.maskey,
            hd.length, p)


def run_kmws(stream, mode, chunk, inplace=False):
    h = kmws.WSHandler(mode)
    got = []
    h.setFrameCallback(lambda hd, p: got.append(frame_key(hd, p)))
    rets, bufs = [], []
    step = chunk if chunk > 0 else max(1, len(stream))
    for i in range(0, max(1, len(stream)), step):
        piece = bytearray(stream[i:i + step]) if inplace else stream[i:i + step]
        rets.append(h.handleData(piece))
        bufs.append(bytes(piece))
    return rets, got, b"".join(bufs)


def run_oracle(stream, mode, chunk, inplace=False):
    d = orc.Decoder(mode)
    rets, bufs = [], []
    step = chunk if chunk > 0 else max(1, len(stream))
    for i in range(0, max(1, len(stream)), step):
        piece = bytearray(stream[i:i + step]) if inplace else stream[i:i + step]
        rets.append(d.feed(piece))
        bufs.append(bytes(piece))
    return rets, [f.key() for f in d.frames], b"".join(bufs)


@pytest.mark.parametrize("c", GOLD["decode"], ids=lambda c: c["name"])
def test_golden_through_gpu_decoder(c):
    data = bytes.fromhex(c["input_hex"])
    if "tail_gen" in c:
        data += bytes(c["tail_len"]) if c["tail_gen"] == "zeros" else \
            bytes(i & 0xFF for i in range(c["tail_len"]))
    mode = kmws.SERVER if c["mode"] == "SERVER" else kmws.CLIENT
    h = kmws.WSHandler(mode)
    frames = []
    h.setFrameCallback(lambda hd, p: frames.append((hd, p)))
    step = c["chunk"] or len(data) or 1
    rets = [h.handleData(data[i:i + step]) for i in range(0, max(1, len(data)), step)]
    assert rets == c["expect_rets"]
    assert len(frames) == len(c["expect_frames"])
    for (hd, p), e in zip(frames, c["expect_frames"]):
        assert (hd.fin, hd.rsv1, hd.rsv2, hd.rsv3, hd.opcode, hd.mask, hd.length) == \
            (e["fin"], e["rsv1"], e["rsv2"], e["rsv3"], e["opcode"], e["mask"], e["length"])
        assert hd.maskey.hex() == e["maskey"]
        want = bytes.fromhex(e["payload_hex"]) if "payload_hex" in e else (
            bytes(e["length"]) if e["payload_gen"] == "zeros" else bytes(i & 0xFF for i in range(e["length"])))
        assert p == want
    for s in c.get("then", []):
        assert h.handleData(bytes.fromhex(s["input_hex"])) == s["expect_rets"][0]


def masked_stream(seed, nframes, sizes=(0, 1, 3, 4, 5, 125, 126, 127, 1000, 4096, 65535, 65536, 100000)):
    rng = random.Random(seed)
    out = b""
    for _ in range(nframes):
        op = rng.choice([0, 1, 2, 2, 9, 10])
        n = rng.choice(sizes)
        if op >= 8:
            n = min(n, 125)
        key = bytes(rng.randrange(256) for _ in range(4))
        h = orc.Hdr(fin=1 if op >= 8 else rng.randrange(2), rsv1=rng.randrange(2) if op < 8 else 0,
                    opcode=op, mask=1, maskey=key, length=n)
        payload = bytes(rng.randrange(256) for _ in range(n))
        out += orc.encode_header(h) + orc.mask_bytes(key, payload)
    return out


@pytest.mark.parametrize("chunk", [0, 1, 7, 1000, 4096, 65536])
def test_masked_streams_match_oracle(chunk):
    stream = masked_stream(chunk + 1, 8 if chunk == 1 else 80)
    assert run_kmws(stream, kmws.SERVER, chunk, inplace=True) == \
        run_oracle(stream, orc.SERVER, chunk, inplace=True)


def test_close_then_trailing_and_error_sequences():
    key = b"\x01\x02\x03\x04"
    close = orc.encode_header(orc.Hdr(opcode=8, mask=1, maskey=key, length=2)) + orc.mask_bytes(key, b"\x03\xe8")
    data = orc.encode_header(orc.Hdr(opcode=1, mask=1, maskey=key, length=5)) + orc.mask_bytes(key, b"Hello")
    for stream in (data + close + data, data + b"\x09\x00" + data, data + b"\x81\x05Hello"):
        for chunk in (0, 3):
            assert run_kmws(stream, kmws.SERVER, chunk, True) == run_oracle(stream, orc.SERVER, chunk, True)


def test_callback_destroy_stops_delivery():
    stream = masked_stream(99, 10, sizes=(5, 100, 3000))
    d = orc.Decoder(orc.SERVER)
    d.destroy_on = 3
    r_o = d.feed(stream)
    h = kmws.WSHandler(kmws.SERVER)
    got = []

    def cb(hd, p):
        got.append(frame_key(hd, p))
        return len(got) - 1 == 3

    h.setFrameCallback(cb)
    assert h.handleData(stream) == r_o == kmws.WS_DESTROYED
    assert got == [f.key() for f in d.frames]


@pytest.mark.parametrize("chunk", [0, 4096, 65536])
def test_pinned_chunk_unmasked_in_place(chunk):
    """Caller's receive buffer in pinned memory: the kernel unmasks it in place
    (zero-copy); callbacks and the buffer's bytes match the oracle."""
    import torch
    stream = masked_stream(1000 + chunk, 60)
    want_rets, want_frames, want_buf = run_oracle(stream, orc.SERVER, chunk, inplace=True)
    h = kmws.WSHandler(kmws.SERVER)
    got = []
    h.setFrameCallback(lambda hd, p: got.append(frame_key(hd, p)))
    step = chunk if chunk > 0 else len(stream)
    rets, bufs = [], []
    for i in range(0, len(stream), step):
        piece = torch.frombuffer(bytearray(stream[i:i + step]), dtype=torch.uint8).pin_memory()
        rets.append(h.handleDataPtr(piece.data_ptr(), piece.numel()))
        bufs.append(bytes(piece.numpy()))
    assert rets == want_rets
    assert got == want_frames
    assert b"".join(bufs) == want_buf


def test_deferred_batch_many_connections():
    """Interleaved reads of several connections fed deferred, one flush per
    'loop iteration': per-connection callbacks and return codes == oracle."""
    nconn, chunk = 5, 3000
    streams = [masked_stream(500 + c, 25) for c in range(nconn)]
    want = [run_oracle(s, orc.SERVER, chunk) for s in streams]
    batch = kmws.RxBatch(0)
    hs, got, rets = [], [[] for _ in range(nconn)], [[] for _ in range(nconn)]
    for c in range(nconn):
        h = kmws.WSHandler(kmws.SERVER)
        h.setFrameCallback(lambda hd, p, c=c: got[c].append(frame_key(hd, p)))
        hs.append(h)
    pos = [0] * nconn
    it = 0
    while any(pos[c] < len(streams[c]) for c in range(nconn)):
        for c in range(nconn):
            if pos[c] < len(streams[c]):
                rets[c].append(hs[c].handleDataDeferred(batch, streams[c][pos[c]:pos[c] + chunk]))
                pos[c] += chunk
        it += 1
        if it % 3 == 0:  # several reads per loop iteration
            batch.flush()
    batch.flush()
    assert batch.pending() == 0
    for c in range(nconn):
        assert rets[c] == want[c][0]
        assert got[c] == want[c][1]


def test_deferred_destroy_drops_only_that_connection():
    a_stream, b_stream = masked_stream(71, 10, sizes=(5, 300)), masked_stream(72, 10, sizes=(7, 200))
    batch = kmws.RxBatch(0)
    ha, hb = kmws.WSHandler(kmws.SERVER), kmws.WSHandler(kmws.SERVER)
    ga, gb = [], []

    def cba(hd, p):
        ga.append(p)
        return len(ga) == 2  # "destroyed" after its 2nd frame

    ha.setFrameCallback(cba)
    hb.setFrameCallback(lambda hd, p: gb.append(p))
    ha.handleDataDeferred(batch, a_stream)
    hb.handleDataDeferred(batch, b_stream)
    n = batch.flush()
    _, fb, _ = run_oracle(b_stream, orc.SERVER, 0)
    _, fa, _ = run_oracle(a_stream, orc.SERVER, 0)
    assert ga == [f[-1] for f in fa[:2]]
    assert gb == [f[-1] for f in fb]
    assert n == 2 + len(fb)


def test_deferred_destroy_covers_every_generation_in_flight():
    """a callback that reports "destroyed" must stop delivery of
    that decoder's frames in every generation the batch still holds -- later
    generations already submitted and the one still being fed -- while the
    other connection's frames are all delivered."""
    streams_a = [masked_stream(81 + g, 4, sizes=(5, 300)) for g in range(3)]
    streams_b = [masked_stream(91 + g, 4, sizes=(7, 200)) for g in range(3)]
    batch = kmws.RxBatch(0)
    ha, hb = kmws.WSHandler(kmws.SERVER), kmws.WSHandler(kmws.SERVER)
    ga, gb = [], []

    def cba(hd, p):
        ga.append(p)
        return len(ga) == 2  # "destroyed" after its 2nd frame (generation 1)

    ha.setFrameCallback(cba)
    hb.setFrameCallback(lambda hd, p: gb.append(p))
    for g in range(2):  # two generations submitted, in flight together
        ha.handleDataDeferred(batch, streams_a[g])
        hb.handleDataDeferred(batch, streams_b[g])
        assert batch.submit() == 8
    ha.handleDataDeferred(batch, streams_a[2])  # the generation being fed
    hb.handleDataDeferred(batch, streams_b[2])
    assert batch.inflight() == 2 and batch.pending() == 8
    n = batch.poll(wait=True)
    n += batch.flush()
    fa = run_oracle(streams_a[0], orc.SERVER, 0)[1]
    fb = [f[-1] for s in streams_b for f in run_oracle(s, orc.SERVER, 0)[1]]
    assert ga == [f[-1] for f in fa[:2]]
    assert gb == fb
    assert n == 2 + len(fb)


def test_mask_host_chain_golden_and_random():
    """handleDataMask(key, KMBuffer&) over host segments: phase continues across
    segments (SURVEY a-2 vector) and equals the oracle's chain mask."""
    import json as _json
    gold = _json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
    for c in gold["mask"]:
        segs = [bytearray.fromhex(s) for s in c["segments_hex"]]
        kmws.handle_data_mask(bytes.fromhex(c["key"]), segs)
        assert [s.hex() for s in segs] == c["expect_hex"], c["name"]
    rng = random.Random(5)
    for _ in range(20):
        segs = [bytearray(rng.randrange(256) for _ in range(rng.choice([0, 1, 3, 5, 17, 1000, 70000])))
                for _ in range(rng.randrange(1, 6))]
        key = bytes(rng.randrange(256) for _ in range(4))
        want = orc.mask_chain(key, [bytes(s) for s in segs])
        kmws.handle_data_mask(key, segs)
        assert [bytes(s) for s in segs] == want


def test_deferred_ring_zero_copy():
    """Reads placed in an attached pinned ring are unmasked in place at flush;
    callbacks == oracle, frames reassembled across reads still correct."""
    import torch
    nconn, chunk = 3, 5000
    streams = [masked_stream(900 + c, 20) for c in range(nconn)]
    want = [run_oracle(s, orc.SERVER, chunk) for s in streams]
    ring = torch.zeros(1 << 20, dtype=torch.uint8).pin_memory()
    batch = kmws.RxBatch(0)
    batch.attach_ring(ring)
    hs, got, rets = [], [[] for _ in range(nconn)], [[] for _ in range(nconn)]
    for c in range(nconn):
        h = kmws.WSHandler(kmws.SERVER)
        h.setFrameCallback(lambda hd, p, c=c: got[c].append(frame_key(hd, p)))
        hs.append(h)
    pos, wr = [0] * nconn, 0
    base = ring.data_ptr()
    while any(pos[c] < len(streams[c]) for c in range(nconn)):
        for c in range(nconn):
            piece = streams[c][pos[c]:pos[c] + chunk]
            if not piece:
                continue
            if wr + len(piece) > ring.numel():  # ring full: flush, then wrap
                batch.flush()
                wr = 0
            ring[wr:wr + len(piece)] = torch.frombuffer(bytearray(piece), dtype=torch.uint8)
            rets[c].append(hs[c].handleDataDeferredPtr(batch, base + wr, len(piece)))
            wr += len(piece) + 7  # leave gaps like unaligned socket reads
            pos[c] += chunk
    batch.flush()
    for c in range(nconn):
        assert rets[c] == want[c][0]
        assert got[c] == want[c][1]


@pytest.mark.parametrize("length,chunk", [(10485760, 65536), (10485760, 0), (10485761, 65536), (10485759, 1 << 20)])
def test_max_frame_length_through_gpu_decoder(length, chunk):
    """The decoder's cap WS_MAX_FRAME_DATA_LENGTH = 10 MiB (WSHandler.cpp:110,
    :192-196): a masked 10 MiB frame (127-class header) is unmasked on the GPU
    and delivered as the reference delivers it, whole or fed in 64 KiB / 1 MiB
    reads (reassembled across reads); 10 MiB + 1 is INVALID_LENGTH (6) on both."""
    rng = random.Random(length ^ chunk)
    key = bytes(rng.randrange(256) for _ in range(4))
    payload = bytes(rng.randrange(256) for _ in range(997)) * (length // 997) + bytes(length % 997)
    hdr = orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=1, maskey=key, length=length))
    stream = hdr + orc.mask_bytes(key, payload) + orc.encode_header(orc.Hdr(fin=1, opcode=9, mask=1, maskey=key,
                                                                             length=3)) + orc.mask_bytes(key, b"end")
    want = run_oracle(stream, kmws.SERVER, chunk, inplace=True)
    got = run_kmws(stream, kmws.SERVER, chunk, inplace=True)
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]
    if length <= 10485760:
        assert want[0][-1] == 0 and len(want[1]) == 2 and want[1][0][-1] == payload
    else:
        assert 6 in want[0] and want[1] == []


# ---- the resident worker behind the synchronous entries (kmws_resident.hip) ----

def test_sync_feed_runs_on_the_resident_worker():
    """kmws_decoder_feed's GPU step goes to the device's resident worker (no
    launch per call): jobs are counted, every frame equals the oracle's, and
    the same stream with the worker switched off (a launch per call) gives the
    same bytes."""
    stream = masked_stream(101, 200, sizes=(0, 1, 5, 125, 126, 1000, 4096))
    reads = (len(stream) + 16383) // 16384
    before = kmws.resident_info()
    want = run_oracle(stream, orc.SERVER, 16384, inplace=True)
    got = run_kmws(stream, kmws.SERVER, 16384, inplace=True)  # 16 KiB reads: every job fits the worker
    assert got == want
    after = kmws.resident_info()
    assert after["jobs"] - before["jobs"] >= reads // 2, (reads, before, after)
    kmws.resident_enable(False)
    try:
        assert run_kmws(stream, kmws.SERVER, 16384, inplace=True) == want
        assert kmws.resident_info()["jobs"] == after["jobs"]
    finally:
        kmws.resident_enable(True)


def test_resident_worker_idles_out_and_relaunches():
    """With no job for 200 us the worker kernel exits by itself (the grid drains);
    the next synchronous call relaunches it and is still exact."""
    import time
    key = bytes.fromhex("a1b2c3d4")
    seg = bytearray(range(256)) * 16
    kmws.handle_data_mask(key, [seg])
    t0 = time.time()
    while kmws.resident_info()["running"] and time.time() - t0 < 2.0:
        time.sleep(0.01)
    info = kmws.resident_info()
    assert not info["running"]  # left by itself
    kmws.handle_data_mask(key, [seg])  # back to the original bytes
    assert seg == bytearray(range(256)) * 16
    after = kmws.resident_info()
    assert after["launches"] == info["launches"] + 1 and after["jobs"] == info["jobs"] + 1


@pytest.mark.parametrize("which", ["default", "side"])
def test_resident_worker_does_not_block_other_streams(which):
    """While another thread keeps its worker busy with back-to-back jobs,
    kernels on torch's default (legacy null) stream or on side streams -- four
    of them, so that every hardware queue the runtime hands out in turn is
    covered -- complete (stream synchronize) in well under a millisecond at
    the median and within a few milliseconds at worst.  The worker runs on a
    non-blocking stream of the greatest priority (a hardware queue of its own)
    and leaves after a 1 ms lease however busy it is, so even a kernel that
    shares its queue waits at most that long."""
    import threading
    import time
    import torch
    x = torch.ones(1 << 20, device="cuda")
    if which == "default":
        streams = [torch.cuda.current_stream()]
    else:
        streams = [torch.cuda.Stream() for _ in range(4)]
    for s in streams:
        with torch.cuda.stream(s):
            y = x * 2  # the elementwise kernel's code object is loaded here, not in the timed loop
    torch.cuda.synchronize()
    stop = threading.Event()
    busy = {"jobs": 0, "resident": False, "launches": []}

    def feeder():
        buf = bytearray(4096)
        while not stop.is_set():
            kmws.handle_data_mask(b"\x01\x02\x03\x04", [buf])
            busy["jobs"] += 1
            info = kmws.resident_info()
            busy["resident"] = busy["resident"] or info["running"]
            busy["launches"].append(info["launches"])

    th = threading.Thread(target=feeder)
    th.start()
    try:
        while busy["jobs"] < 100:
            time.sleep(0.001)
        lat = []
        for _ in range(20):
            for s in streams:
                t0 = time.perf_counter()
                with torch.cuda.stream(s):
                    y = x * 2
                s.synchronize()
                lat.append(time.perf_counter() - t0)
    finally:
        stop.set()
        th.join()
    assert busy["resident"] and busy["jobs"] > 100
    print(f"\n[{which}] kernel+sync latency ms: median {1e3 * sorted(lat)[len(lat) // 2]:.3f} "
          f"max {1e3 * max(lat):.3f}; worker jobs {busy['jobs']} "
          f"launches {busy['launches'][-1] - busy['launches'][0] + 1}")
    assert sorted(lat)[len(lat) // 2] < 0.002, lat
    assert max(lat) < 0.05, lat
    assert float(y.sum()) == 2 * (1 << 20)


def test_resident_lease_relaunches_a_busy_worker():
    """A worker fed back to back for ~50 ms leaves at every 1 ms lease and is
    relaunched for the next job: many incarnations, every job exact."""
    import time
    rng = random.Random(11)
    data = bytes(rng.randrange(256) for _ in range(2048))
    key = b"\x9a\x01\xfe\x33"
    want = orc.mask_bytes(key, data)
    before = kmws.resident_info()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < 0.05:
        a = bytearray(data)
        kmws.handle_data_mask(key, [a])
        assert bytes(a) == want
        n += 1
    after = kmws.resident_info()
    assert after["jobs"] - before["jobs"] == n
    assert after["launches"] - before["launches"] >= 10, (n, before, after)


def test_decoders_per_connection_borrow_pooled_staging():
    """kuma creates a WSHandler per connection.  300 short-lived decoders, each
    fed one masked frame, borrow the process's pooled pinned stages (no stream
    or pinned allocation per connection): every payload exact and the mean
    connection well under a stream creation's milliseconds.  A callback that
    feeds a second decoder (a relay) borrows a second stage: both exact."""
    import time
    rng = random.Random(41)
    payload = bytes(rng.randrange(256) for _ in range(1024))
    key = b"\x11\x22\x33\x44"
    wire = orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=1, maskey=key, length=len(payload))) + \
        orc.mask_bytes(key, payload)
    got = []

    def one():
        h = kmws.WSHandler(kmws.SERVER)
        h.setFrameCallback(lambda hdr, data: got.append(data))
        assert h.handleData(bytearray(wire)) == 0
        del h

    one()
    got.clear()
    t0 = time.perf_counter()
    for _ in range(300):
        one()
    dt = (time.perf_counter() - t0) / 300
    print(f"\nper connection (create, one masked 1 KiB frame, destroy): {dt * 1e6:.1f} us")
    assert got == [payload] * 300
    assert dt < 2e-3, dt  # (a stream and a pinned area per connection cost milliseconds; measured ~10 us)
    # nested: decoder A's callback feeds decoder B while A's staged payload is delivered
    key_b = b"\xa0\xb1\xc2\xd3"
    inner = orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=1, maskey=key_b, length=len(payload))) + \
        orc.mask_bytes(key_b, payload[::-1])
    outer = orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=1, maskey=key, length=len(inner))) + \
        orc.mask_bytes(key, inner)
    b = kmws.WSHandler(kmws.SERVER)
    seen = []
    b.setFrameCallback(lambda hdr, data: seen.append(("b", data)))
    a = kmws.WSHandler(kmws.SERVER)

    def relay(hdr, data):
        seen.append(("a", data))
        assert b.handleData(bytearray(data)) == 0
    a.setFrameCallback(relay)
    assert a.handleData(bytearray(outer + outer)) == 0
    assert seen == [("a", inner), ("b", payload[::-1])] * 2


def test_resident_worker_slot_per_thread():
    """Four threads masking concurrently each hold their own mailbox slot of
    the device's resident grid (no lock between them): distinct slots, every
    result exact, the jobs on the worker (but the few of a slot claimed while
    the running incarnation did not cover it: that incarnation is asked to
    leave at once, and its jobs launch until the relaunch serves it), and the
    median call stays in the tens of microseconds."""
    import threading
    import time
    rng = random.Random(23)
    data = bytes(rng.randrange(256) for _ in range(2048))
    res = {}
    start = threading.Barrier(4)

    def run(tid):
        key = bytes([tid, 0x5a, 0xa5, tid ^ 0xff])
        want = orc.mask_bytes(key, data)
        lat, bad = [], 0
        start.wait()
        for _ in range(400):
            a = bytearray(data)
            t0 = time.perf_counter()
            kmws.handle_data_mask(key, [a])
            lat.append(time.perf_counter() - t0)
            bad += bytes(a) != want
        res[tid] = (sorted(lat)[len(lat) // 2], bad, kmws.resident_info()["thread_slot"])
        finish.wait()  # holds the slot until every thread has reported (a thread that
        # exited early would free its slot for a late starter: the GIL can run one
        # thread's 400 calls before another's first)

    finish = threading.Barrier(4)
    before = kmws.resident_info()
    ths = [threading.Thread(target=run, args=(i,)) for i in (1, 2, 3, 4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    after = kmws.resident_info()
    print(f"\nper-thread median us / slot: {[(round(m * 1e6, 1), s) for m, _, s in res.values()]}")
    assert all(b == 0 for _, b, _ in res.values()), res
    slots = [s for _, _, s in res.values()]
    assert all(s >= 0 for s in slots) and len(set(slots)) == 4, slots
    assert 1560 <= after["jobs"] - before["jobs"] <= 1600, (before, after)
    assert max(m for m, _, _ in res.values()) < 1e-3, res  # loose: a shared box; measured ~6 us (C++ rows)
    # the threads have exited: their slots are free again
    assert kmws.resident_info()["slots_claimed"] <= before["slots_claimed"], (before, kmws.resident_info())


def test_rx_batch_pending_bytes_counts_masked_payloads():
    """kmws_rx_batch_pending_bytes (what RxLoop keeps within the resident job
    limits): the masked payload bytes fed since the last submit -- unmasked
    frames and control payloads of length 0 not counted -- and 0 after a
    submit; the frames then deliver exact."""
    rng = random.Random(43)
    b = kmws.RxBatch()
    h = kmws.WSHandler(kmws.SERVER)
    got = []
    h.setFrameCallback(lambda hdr, data: got.append((hdr.opcode, data)))
    wire, want, masked_bytes = b"", [], 0
    for i, n in enumerate((100, 0, 5000, 70000, 7)):
        payload = bytes(rng.randrange(256) for _ in range(n))
        key = bytes(rng.randrange(256) for _ in range(4))
        mask = i != 4  # the last one unmasked (a client-bound frame)
        wire += orc.encode_header(orc.Hdr(fin=1, opcode=2, mask=int(mask), maskey=key if mask else b"\0" * 4,
                                          length=n)) + (orc.mask_bytes(key, payload) if mask else payload)
        want.append((2, payload))
        masked_bytes += n if mask else 0
    assert b.pending_bytes() == 0
    assert h.handleDataDeferred(b, wire[:-(7 + 2)]) in (0, 1)  # all but the unmasked frame
    assert b.pending_bytes() == masked_bytes, (b.pending_bytes(), masked_bytes)
    assert b.pending() == 4
    assert b.submit() == 4
    assert b.pending_bytes() == 0 and b.pending() == 0
    b.poll(wait=True)
    assert got == want[:4]


def test_resident_large_jobs_write_through_while_a_device_batch_runs():
    """A job above 16 KiB of hull words releases the L2 once on an idle device
    and writes through while this library's device batches run (kmws_resident.hip
    kResWriteThroughWords, kmws::note_device_batch); a 4 KiB one always writes
    through.  Every byte exact, the batch's too."""
    import time
    import torch
    n, frame = 131072, 65536  # 8 GiB: three applies keep the device busy ~8 ms
    base = torch.empty(n * frame, dtype=torch.uint8, device="cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(base, 7)
    kmws.fill_uniform_descs(descs, frame, frame, 11)
    ws = kmws.Workspace(kmws.unmask_workspace_size(base.numel()))
    kmws.unmask_plan(descs, ws, base.numel())
    torch.cuda.synchronize()
    rng = random.Random(77)
    key = bytes(rng.randrange(256) for _ in range(4))

    def mask(nbytes):
        data = rng.randbytes(nbytes)
        buf = bytearray(data)
        kmws.handle_data_mask(key, [buf])
        assert bytes(buf) == orc.mask_bytes(key, data)

    t0 = time.monotonic()
    while kmws.device_batch_busy() and time.monotonic() - t0 < 2:
        time.sleep(0.001)
    mask(4096)  # the thread's slot claimed (and the grid sized for it)
    mask(4096)
    s0 = kmws.resident_stores()
    mask(65536)
    mask(4096)
    s1 = kmws.resident_stores()
    assert (s1["released"] - s0["released"], s1["write_through"] - s0["write_through"]) == (1, 1), (s0, s1)
    # the boundary: 16 KiB of hull words writes through, one word more releases
    # (a bytearray's buffer is 16-byte aligned or not; 16 KiB - 15 B fits 1,024
    # words wherever it lies, 16 KiB + 17 B never does)
    mask(16384 - 15)
    mask(16384 + 17)
    s1b = kmws.resident_stores()
    assert (s1b["released"] - s1["released"], s1b["write_through"] - s1["write_through"]) == (1, 1), (s1, s1b)
    s1 = s1b
    for _ in range(3):
        kmws.unmask_apply(base, descs, ws)
    assert kmws.device_batch_busy()
    mask(65536)
    mask(262144 - 64)  # four parts, written through
    s2 = kmws.resident_stores()
    assert (s2["released"] - s1["released"], s2["write_through"] - s1["write_through"]) == (0, 2), (s1, s2)
    torch.cuda.synchronize()
    assert kmws.check_unmasked(base, 7, descs) == 0
    t0 = time.monotonic()
    while kmws.device_batch_busy() and time.monotonic() - t0 < 2:
        time.sleep(0.001)
    assert not kmws.device_batch_busy()
    mask(65536)
    s3 = kmws.resident_stores()
    assert s3["released"] - s2["released"] == 1, (s2, s3)


def test_resident_busy_grid_leaves_only_at_its_lease():
    """Four threads masking 4 KiB back to back: over ~30 ms of that (read while
    they still run), every workgroup exit is a lease exit -- none decides the
    grid idle and none leaves on another's idle decision (the first idle test
    compared workgroups' clocks and closed busy grids every ~0.3 ms, DESIGN.md
    sec.4)."""
    import threading
    import time
    rng = random.Random(31)
    data = bytes(rng.randrange(256) for _ in range(4096))
    ready = threading.Barrier(5)
    stop = threading.Event()
    bad = []

    def run(tid):
        key = bytes([tid, 7, 9, 11])
        want = orc.mask_bytes(key, data)
        a = bytearray(data)
        kmws.handle_data_mask(key, [a])  # claims the slot
        ready.wait()
        while not stop.is_set():
            a = bytearray(data)
            kmws.handle_data_mask(key, [a])
            if bytes(a) != want:
                bad.append(tid)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    ready.wait()  # every thread holds its slot and masks from now on
    time.sleep(0.005)
    before = kmws.resident_exit_reasons()
    time.sleep(0.03)
    after = kmws.resident_exit_reasons()
    stop.set()
    for t in ths:
        t.join()
    d = {k: after[k] - before[k] for k in after}
    print(f"\nexits while busy: {d}")
    assert not bad
    # a grid of 4 slots x 4 parts leaves as idle with up to 16 exits (one idle,
    # the rest closing); four GIL-bound threads can all pause past the 200 us
    # idle time now and then (r06aq: one such close in 30 ms), while the
    # round-5 defect closed busy grids 650-1,199 times in 25 ms
    assert d["idle"] + d["closing"] <= 4 * 16, d
    assert d["lease"] >= 4 * 4 * 10, d  # ~30 incarnations of >= 4 slots x 4 parts


def test_resident_slot_claimed_outside_the_grid_resizes_it():
    """A thread keeps the grid busy; a second claims a slot the running
    incarnation does not serve: the grid is asked to leave (a resize exit --
    or, if that incarnation reached its lease first, the relaunch serves the
    slot anyway), and every one of the late thread's 300 masks is exact.  (How
    many of its calls launched shows in the C++ mask_threads rows, not here:
    Python's timing includes the GIL the busy thread holds.)"""
    import threading
    import time
    rng = random.Random(37)
    data = bytes(rng.randrange(256) for _ in range(2048))
    stop = threading.Event()
    busy_started = threading.Event()

    def busy():
        key = b"\x01\x02\x03\x04"
        want = orc.mask_bytes(key, data)
        while not stop.is_set():
            a = bytearray(data)
            kmws.handle_data_mask(key, [a])
            assert bytes(a) == want
            busy_started.set()

    tb = threading.Thread(target=busy)
    tb.start()
    busy_started.wait(5)
    time.sleep(0.002)
    res = {}

    def late():
        key = b"\x0a\x0b\x0c\x0d"
        want = orc.mask_bytes(key, data)
        before = kmws.resident_exit_reasons()
        jobs0 = kmws.resident_info()["jobs"]
        lat = []
        for _ in range(300):
            a = bytearray(data)
            t0 = time.perf_counter()
            kmws.handle_data_mask(key, [a])
            lat.append(time.perf_counter() - t0)
            assert bytes(a) == want
        res["exits"] = {k: v - before[k] for k, v in kmws.resident_exit_reasons().items()}
        res["slot"] = kmws.resident_info()["thread_slot"]
        res["median_us"] = sorted(lat)[len(lat) // 2] * 1e6

    tl = threading.Thread(target=late)
    tl.start()
    tl.join()
    stop.set()
    tb.join()
    print(f"\nlate thread: {res}")
    assert res["slot"] >= 0
    assert res["exits"]["resize"] + res["exits"]["lease"] >= 1, res
    assert res["median_us"] < 1000, res  # loose: Python + GIL on a shared box


def test_resident_more_threads_than_slots_launch_instead():
    """Twenty threads at once (the grid has 16 slots): the threads that find no
    free slot launch on their own streams instead of waiting; every result is
    exact, and the slots are all given back when the threads exit."""
    import threading
    rng = random.Random(29)
    data = bytes(rng.randrange(256) for _ in range(3000))
    res = {}
    start = threading.Barrier(20)
    hold = threading.Barrier(20)

    def run(tid):
        key = bytes([tid, 1, 2, 3])
        want = orc.mask_bytes(key, data)
        start.wait()
        bad = 0
        for _ in range(50):
            a = bytearray(data)
            kmws.handle_data_mask(key, [a])
            bad += bytes(a) != want
        res[tid] = (bad, kmws.resident_info()["thread_slot"])
        hold.wait()  # every thread still holds its slot here

    base = kmws.resident_info()["slots_claimed"]
    ths = [threading.Thread(target=run, args=(i,)) for i in range(20)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    slots = [s for _, s in res.values()]
    assert all(b == 0 for b, _ in res.values()), res
    held = [s for s in slots if s >= 0]
    assert len(held) == len(set(held)) <= 16 - base, slots
    assert slots.count(-1) >= 20 - (16 - base), slots
    assert kmws.resident_info()["slots_claimed"] == base


def test_resident_and_launch_paths_interleaved_on_many_threads():
    """Four threads at once, 40 jobs each of 1 B to 512 KiB at odd offsets,
    chains of up to three segments: jobs of up to 256 KiB run on each thread's
    slot of the resident grid, larger ones are launched on the thread's own
    stream, interleaved on every thread.  Every byte equals the oracle's, and
    the jobs that fit the worker ran on it (but a new slot's first ones, until
    the grid's next incarnation covers it)."""
    import threading
    res = {}

    def run(tid):
        rng = random.Random(1000 + tid)
        bad = small = 0
        for i in range(40):
            n = rng.choice([rng.randrange(1, 4096), rng.randrange(32768, 70000), rng.randrange(70000, 524288)])
            key = bytes(rng.randrange(256) for _ in range(4))
            data = rng.randbytes(n + 17)
            off = rng.randrange(0, 17)
            cuts = sorted(rng.randrange(0, n + 1) for _ in range(rng.randrange(0, 3)))
            segs = [bytearray(data[off + a:off + b]) for a, b in zip([0] + cuts, cuts + [n])]
            want = orc.mask_bytes(key, data[off:off + n])
            kmws.handle_data_mask(key, segs)
            bad += b"".join(segs) != want
            small += n <= 262144
        res[tid] = (bad, small)

    before = kmws.resident_info()
    ths = [threading.Thread(target=run, args=(i,)) for i in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    after = kmws.resident_info()
    assert all(b == 0 for b, _ in res.values()), res
    small = sum(s for _, s in res.values())
    assert small - 12 <= after["jobs"] - before["jobs"] <= small, (before, after, res)


def _testhooks_lib():
    """The test-only build (kuma_amd/build.py TEST_DEFINES): job timeout 50 ms,
    drain 150 ms, a job keyed 0xDEAD5Exx stalls its workgroup xx * 10 ms."""
    import ctypes as C
    import os
    from kuma_amd import build as kb
    assert os.path.exists(kb.TEST_LIB), "run __graft_entry__.build()"
    return kmws.bind(C.CDLL(kb.TEST_LIB))


def test_resident_timeout_withdraws_job_and_other_threads_run_on():
    """VERDICT r04 #3.  A job whose workgroup stalls past the 50 ms timeout
    (test build, 80 ms stall) is withdrawn: the quit bit makes the workgroup
    drop it and leave, the call waits until it has (so nothing writes the
    buffer after the call returns), then launches the job itself and returns
    exact bytes.  Meanwhile another thread masking on its own slot keeps
    completing calls in well under the stall (no lock between slots: once its
    own workgroup left, its job is withdrawn and launched too)."""
    import threading
    import time
    from kuma_amd import build as kb
    TL = _testhooks_lib()
    data = bytes(range(256)) * 16
    stall_key = (kb.RESIDENT_STALL_KEY | 8).to_bytes(4, "little")  # 80 ms
    key_b = b"\x10\x20\x30\x40"
    kmws.handle_data_mask(key_b, [bytearray(data)], L=TL)  # the grid is up
    before = kmws.resident_info(L=TL)
    stop = threading.Event()
    other = {"n": 0, "bad": 0, "lat": []}

    def feeder():
        want = orc.mask_bytes(key_b, data)
        while not stop.is_set():
            a = bytearray(data)
            t0 = time.perf_counter()
            kmws.handle_data_mask(key_b, [a], L=TL)
            other["lat"].append(time.perf_counter() - t0)
            other["bad"] += bytes(a) != want
            other["n"] += 1

    th = threading.Thread(target=feeder)
    th.start()
    try:
        time.sleep(0.01)
        n0 = other["n"]
        a = bytearray(data)
        t0 = time.perf_counter()
        kmws.handle_data_mask(stall_key, [a], L=TL)
        took = time.perf_counter() - t0
        n1 = other["n"]
    finally:
        stop.set()
        th.join()
    info = kmws.resident_info(L=TL)
    assert bytes(a) == orc.mask_bytes(stall_key, data)
    assert took >= 0.05, took
    assert info["timeouts"] - before["timeouts"] == 1 and info["withdrawn"] > before["withdrawn"], info
    assert other["bad"] == 0 and n1 - n0 >= 20, (n0, n1)
    assert max(other["lat"]) < 0.03, max(other["lat"])
    print(f"\nstalled call {took * 1e3:.1f} ms; other thread {n1 - n0} calls meanwhile, "
          f"max {max(other['lat']) * 1e3:.2f} ms; {info}")
    # the worker is still in service after a stall it recovered from
    b = bytearray(data)
    kmws.handle_data_mask(key_b, [b], L=TL)
    assert bytes(b) == orc.mask_bytes(key_b, data)


def test_resident_timeout_past_drain_returns_timeout_status():
    """A workgroup that neither finishes nor leaves within timeout + drain
    (test build: a 400 ms stall against 50 + 150 ms) makes the call return
    KMWS_ERR_TIMEOUT (KMError::TIMEOUT, -6): the device may still write the
    job's staging memory, which is abandoned, never reused.  The caller's
    buffer is untouched, and the worker is no longer used (later calls launch,
    exact); the stalled workgroup drops the job and the grid drains."""
    import time
    from kuma_amd import build as kb
    TL = _testhooks_lib()
    data = bytes(range(256)) * 8
    stall_key = (kb.RESIDENT_STALL_KEY | 40).to_bytes(4, "little")  # 400 ms
    a = bytearray(data)
    t0 = time.perf_counter()
    with pytest.raises(kmws.KmwsError) as e:
        kmws.handle_data_mask(stall_key, [a], L=TL)
    took = time.perf_counter() - t0
    assert e.value.status == kmws.ERR_TIMEOUT
    assert 0.15 <= took < 0.39, took
    assert bytes(a) == data
    jobs = kmws.resident_info(L=TL)["jobs"]
    b = bytearray(data)
    kmws.handle_data_mask(b"\x01\x02\x03\x04", [b], L=TL)
    assert bytes(b) == orc.mask_bytes(b"\x01\x02\x03\x04", data)
    assert kmws.resident_info(L=TL)["jobs"] == jobs  # launched, not posted
    t0 = time.time()
    while kmws.resident_info(L=TL)["running"] and time.time() - t0 < 2.0:
        time.sleep(0.02)
    assert not kmws.resident_info(L=TL)["running"]
    assert bytes(a) == data


@pytest.mark.parametrize("n", [1, 3, 15, 16, 17, 1024, 4096, 16384, 16385, 65536, 65537, 262144, 262145, 300000,
                               (1 << 20) + 5])
def test_mask_host_chain_sizes_resident_and_launch(n):
    """handleDataMask(key, data, len) at every size class through the resident
    grid (<= 256 KiB: one to four parts) and beyond it (the launch path), against the oracle's
    byte loop, at odd alignments inside a larger buffer."""
    rng = random.Random(n)
    key = bytes(rng.randrange(256) for _ in range(4))
    buf = bytearray(rng.randrange(256) for _ in range(n + 37))
    for off in (0, 3, 17):
        seg = memoryview(buf)[off:off + n]
        want = orc.mask_bytes(key, bytes(seg))
        arr = bytearray(seg)
        kmws.handle_data_mask(key, [arr])
        assert bytes(arr) == want


def test_resident_many_small_jobs_stay_exact():
    """Thousands of back-to-back jobs (the steady state of a loop thread): each
    1-64 byte payload masked twice returns to its original bytes, checked
    against the oracle after the first pass."""
    rng = random.Random(7)
    for i in range(3000):
        n = rng.randrange(1, 65)
        key = bytes(rng.randrange(256) for _ in range(4))
        data = bytes(rng.randrange(256) for _ in range(n))
        a = bytearray(data)
        kmws.handle_data_mask(key, [a])
        assert bytes(a) == orc.mask_bytes(key, data), i
        kmws.handle_data_mask(key, [a])
        assert bytes(a) == data, i


def test_sync_feed_views_mode_leaves_chunk_masked():
    """kmws_decoder_set_in_place(0): every frame (header fields and payload)
    equals the oracle's, and the caller's pageable chunk keeps its masked
    bytes (the payload views point at the unmasked staging copy)."""
    stream = masked_stream(202, 60, sizes=(0, 1, 3, 125, 126, 4096, 20000, 65535, 70000))
    want = run_oracle(stream, orc.SERVER, 65536)[:2]
    h = kmws.WSHandler(kmws.SERVER)
    h.setInPlace(False)
    got = []
    h.setFrameCallback(lambda hd, p: got.append(frame_key(hd, p)))
    rets, chunks = [], []
    for i in range(0, len(stream), 65536):
        piece = bytearray(stream[i:i + 65536])
        rets.append(h.handleData(piece))
        chunks.append(bytes(piece))
    assert (rets, got) == want
    assert b"".join(chunks) == stream
