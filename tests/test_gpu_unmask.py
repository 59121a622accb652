"""GPU parity: kmws_unmask_batch (HIP, gfx950) vs the CPU oracle, bit-exact.

Every case builds a host buffer + descriptors, unmasks a copy with the oracle
(WSHandler.cpp:303-310 byte loop, restated in oracle/kmws_oracle.c) and the
other copy on the GPU through the C ABI, and compares every byte of the
buffer (payload, headers, gaps)."""
import zlib

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    from kuma_amd import kmws
    if not torch.cuda.is_available() or kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    return torch


def run_gpu(torch, buf: np.ndarray, descs: np.ndarray, span=None, schedule=None, stream=None):
    from kuma_amd import kmws
    span = len(buf) if span is None else span
    pad = (-len(buf)) % 16
    d_buf = torch.from_numpy(np.concatenate([buf, np.zeros(pad, np.uint8)])).cuda()
    d_desc = torch.from_numpy(descs.view(np.int64).reshape(-1, 2).copy()).cuda() if len(descs) else \
        torch.zeros((0, 2), dtype=torch.int64, device="cuda")
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    kmws.unmask_batch(d_buf, d_desc, ws, span, schedule=schedule, stream=stream)
    torch.cuda.synchronize()
    return d_buf.cpu().numpy()[:len(buf)], ws.status()


KINDS_X_STORES = [k | s for k in range(6) for s in (0, 1 << 29, 1 << 30)]  # placement kind x auto / NT / temporal


def make_descs(offs, lens, keys):
    d = np.zeros(len(offs), dtype=orc.DESC_DTYPE)
    d["off"], d["len"], d["key"] = offs, lens, keys
    return d


def layout(kind, rng):
    """Returns (buffer, descs) for a named layout."""
    if kind == "aligned64k":
        n, L = 96, 65536
        offs = np.arange(n, dtype=np.uint64) * L
        lens = np.full(n, L)
        total = n * L
    elif kind == "packed_wire":  # payloads behind 2..14-byte headers: misaligned starts
        n = 400
        lens = rng.choice([0, 1, 7, 125, 126, 1000, 4096, 65535, 65536, 70001], size=n)
        hdr = np.where(lens <= 125, 2, np.where(lens <= 65535, 4, 10)) + 4
        wire = np.cumsum(np.concatenate([[0], hdr + lens]))
        offs = (wire[:-1] + hdr).astype(np.uint64)
        total = int(wire[-1])
    elif kind == "zipf_mixed":  # SURVEY 8d cfg3 size classes 128*2^k, k<=13, tails not multiples of 4
        n = 300
        k = rng.choice(14, size=n, p=(np.arange(1, 15) ** -1.2) / np.sum(np.arange(1, 15) ** -1.2))
        lens = 128 * (2 ** k) - rng.integers(0, 64, size=n)
        gaps = rng.integers(0, 24, size=n)
        starts = np.cumsum(np.concatenate([[0], gaps + lens]))
        offs = (starts[:-1] + gaps).astype(np.uint64)
        total = int(starts[-1]) + 5
    elif kind == "tiny_many":  # > 256 frames per 16 KiB tile: several LDS rounds
        n = 20000
        lens = rng.integers(0, 21, size=n)
        gaps = rng.integers(0, 15, size=n)
        starts = np.cumsum(np.concatenate([[0], gaps + lens]))
        offs = (starts[:-1] + gaps).astype(np.uint64)
        total = int(starts[-1])
    elif kind == "zero_len_runs":  # empty frames at equal offsets, adjacent frames, no gaps
        n = 3000
        lens = rng.choice([0, 0, 0, 1, 2, 3, 17, 300], size=n)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        total = int(np.sum(lens)) + 3
    elif kind == "sparse_gaps":  # big holes between frames (untouched bytes)
        n = 40
        lens = rng.integers(1, 5000, size=n)
        gaps = rng.integers(0, 200000, size=n)
        starts = np.cumsum(np.concatenate([[0], gaps + lens]))
        offs = (starts[:-1] + gaps).astype(np.uint64)
        total = int(starts[-1]) + 11
    elif kind == "long_gaps":  # regions >= one tile (capped grids, two-frame path): every header-gap size
        n = 80                   # around a boundary, some frames ending exactly on a tile edge
        gaps = rng.choice([0, 1, 2, 4, 8, 10, 14, 15, 16, 17, 31, 1024], size=n)
        lens = rng.integers(16384, 70000, size=n)
        offs = np.zeros(n, dtype=np.uint64)
        pos = 0
        for i in range(n):
            pos += int(gaps[i])
            offs[i] = pos
            if i % 5 == 4:  # end on the next tile edge at least 16 KiB away
                lens[i] = (pos + 16384 + 16383) // 16384 * 16384 - pos
            pos += int(lens[i])
        total = pos + 9
    else:
        raise ValueError(kind)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    keys[::17] = 0
    buf = rng.integers(0, 256, size=total, dtype=np.uint8)
    return buf, make_descs(offs, lens, keys)


KINDS = ["aligned64k", "packed_wire", "zipf_mixed", "tiny_many", "zero_len_runs", "sparse_gaps", "long_gaps"]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("schedule", [None] + KINDS_X_STORES)
def test_unmask_parity(torch_dev, kind, schedule):
    rng = np.random.default_rng(zlib.crc32(f"{kind}-{schedule}".encode()))
    buf, descs = layout(kind, rng)
    want = buf.copy()
    orc.unmask_batch(want, descs)
    got, st = run_gpu(torch_dev, buf, descs, schedule=schedule)
    assert st == 0
    assert np.array_equal(got, want)


def test_unmask_empty_batch(torch_dev):
    buf = np.arange(100, dtype=np.uint8)
    got, st = run_gpu(torch_dev, buf, make_descs([], [], []))
    assert st == 0 and np.array_equal(got, buf)


@pytest.mark.parametrize("bad", ["unsorted", "overlap", "past_span"])
def test_unmask_rejects_bad_descriptors(torch_dev, bad):
    rng = np.random.default_rng(3)
    buf = rng.integers(0, 256, size=50000, dtype=np.uint8)
    offs, lens = [0, 1000, 2000, 3000], [100, 100, 100, 100]
    if bad == "unsorted":
        offs = [0, 2000, 1000, 3000]
    elif bad == "overlap":
        lens = [100, 1500, 100, 100]
    else:
        offs[-1], lens[-1] = 49990, 100
    got, st = run_gpu(torch_dev, buf, make_descs(offs, lens, [1, 2, 3, 4]))
    assert st == 1
    assert np.array_equal(got, buf)  # untouched


def test_unmask_single_frame_every_alignment(torch_dev):
    rng = np.random.default_rng(11)
    for off in range(0, 20):
        for L in (1, 2, 3, 4, 5, 15, 16, 17, 31, 33):
            buf = rng.integers(0, 256, size=64, dtype=np.uint8)
            d = make_descs([off], [L], [0xA1B2C3D4])
            want = buf.copy()
            orc.unmask_batch(want, d)
            got, st = run_gpu(torch_dev, buf, d)
            assert st == 0 and np.array_equal(got, want), (off, L)


def test_unmask_large_device_resident(torch_dev):
    """4 GiB arena, 64 KiB frames (cfg2 shape at 1/16 scale): device checker over
    every byte + sampled frames against the oracle + double-unmask identity."""
    torch = torch_dev
    from kuma_amd import kmws
    n, L, seed = 65536, 65536, 1234567
    span = n * L
    base = torch.empty(span, dtype=torch.uint8, device="cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(base, seed)
    kmws.fill_uniform_descs(descs, L, L, 99)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    kmws.unmask_batch(base, descs, ws, span)
    assert ws.status() == 0
    assert kmws.check_unmasked(base, seed, descs) == 0
    hd = descs.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
    rng = np.random.default_rng(5)
    for i in rng.choice(n, size=24, replace=False).tolist() + [0, n - 1]:
        want = orc.synthetic(seed, i * L, L)
        orc.unmask_batch(want, make_descs([0], [L], [int(hd["key"][i])]))
        got = base[i * L:(i + 1) * L].cpu().numpy()
        assert np.array_equal(got, want), i
    kmws.unmask_batch(base, descs, ws, span)  # XOR twice == identity
    head = base[:1 << 20].cpu().numpy()
    assert np.array_equal(head, orc.synthetic(seed, 0, 1 << 20))


def test_synthetic_fill_matches_host(torch_dev):
    torch = torch_dev
    from kuma_amd import kmws
    for nbytes in (16, 17, 1000, 123457):
        t = torch.empty(nbytes + 16, dtype=torch.uint8, device="cuda")
        kmws.fill_synthetic(t, 77, nbytes)
        assert np.array_equal(t[:nbytes].cpu().numpy(), orc.synthetic(77, 0, nbytes))


def test_unmask_on_side_stream(torch_dev):
    torch = torch_dev
    rng = np.random.default_rng(8)
    buf, descs = layout("packed_wire", rng)
    want = buf.copy()
    orc.unmask_batch(want, descs)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        got, st = run_gpu(torch, buf, descs, stream=s)
    assert st == 0 and np.array_equal(got, want)


def _to_dev(torch, buf, descs):
    d_buf = torch.from_numpy(np.concatenate([buf, np.zeros((-len(buf)) % 16, np.uint8)])).cuda()
    d_desc = torch.from_numpy(descs.view(np.int64).reshape(-1, 2).copy()).cuda()
    return d_buf, d_desc


def _valid_schedule(code):
    store = code & (3 << 29)
    return (code & 0xFF) in range(6) and store != 3 << 29 and code & ~(0xFF | 3 << 29) == 0


def test_autotune_keeps_payload_and_picks_valid_schedule(torch_dev):
    """kmws_unmask_autotune runs every schedule twice (XOR twice = identity):
    the payload is unchanged, the pick is returned (and kept on THIS
    Workspace, the caller's plan), and unmask parity holds under it."""
    torch = torch_dev
    from kuma_amd import kmws
    rng = np.random.default_rng(31)
    buf, descs = layout("packed_wire", rng)
    d_buf, d_desc = _to_dev(torch, buf, descs)
    ws = kmws.Workspace(kmws.unmask_workspace_size(len(buf)))
    choice = kmws.unmask_autotune(d_buf, d_desc, ws, len(buf))
    assert _valid_schedule(choice) and choice & (3 << 29)  # the autotune times forced store policies
    assert kmws.unmask_get_schedule(ws, d_desc, len(buf)) == choice
    ws2 = kmws.Workspace(kmws.unmask_workspace_size(len(buf)))
    dflt = kmws.sched_default(len(buf), len(descs))
    assert kmws.unmask_get_schedule(ws2, d_desc, len(buf)) == dflt  # other plans: default
    assert np.array_equal(d_buf.cpu().numpy()[:len(buf)], buf)
    want = buf.copy()
    orc.unmask_batch(want, descs)
    kmws.unmask_batch(d_buf, d_desc, ws, len(buf))
    torch.cuda.synchronize()
    assert ws.status() == 0 and np.array_equal(d_buf.cpu().numpy()[:len(buf)], want)
    kmws.unmask_set_schedule(ws, None)  # forget: back to the default
    assert kmws.unmask_get_schedule(ws, d_desc, len(buf)) == dflt


def test_default_schedule_matches_rule(torch_dev):
    from kuma_amd import kmws
    assert kmws.sched_default(1 << 30, 1 << 14) == kmws.SCHED_SPLIT4       # 64 KiB regions
    assert kmws.sched_default(1 << 30, 1 << 16) == kmws.SCHED_SPLIT4       # exactly one tile
    assert kmws.sched_default(1 << 30, (1 << 16) + 1) == kmws.SCHED_GROUPED_RUNS
    assert kmws.sched_default(1 << 20, 0) == kmws.SCHED_GROUPED_RUNS


def test_tuned_workspace_freed_new_one_at_same_address_gets_default(torch_dev):
    """the library holds no pointer-keyed schedule table.  A
    tuned Workspace is freed; torch's caching allocator hands its block to a
    new Workspace serving another batch at the same descriptor address; that
    batch runs the default schedule, and both stay bit-exact.  The C entries
    take the schedule as an argument: a plain kmws_unmask_apply on the old
    pointers after the tune is the default schedule too."""
    torch = torch_dev
    from kuma_amd import kmws
    n, L = 4096, 65536
    span = n * L
    base = torch.empty(span, dtype=torch.uint8, device="cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(base, 5)
    kmws.fill_uniform_descs(descs, L, L, 6)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    kmws.unmask_set_schedule(ws, kmws.SCHED_SPLIT2 | kmws.SCHED_TEMPORAL_STORES)  # as a tune may pick
    picked = kmws.unmask_autotune(base, descs, ws, span)
    assert ws.schedule == picked
    kmws.unmask_batch(base, descs, ws, span)  # the aligned batch under its tuned schedule
    assert ws.status() == 0 and kmws.check_unmasked(base, 5, descs) == 0
    old_ws, old_desc = ws.ptr, descs.data_ptr()
    ws_bytes = ws.nbytes
    del ws
    torch.cuda.synchronize()
    ws2 = kmws.Workspace(ws_bytes)
    assert ws2.ptr == old_ws  # torch recycled the block
    # another batch through it: a packed wire image
    rng = np.random.default_rng(77)
    buf, wd = layout("packed_wire", rng)
    d_buf, _ = _to_dev(torch, buf, wd)
    assert ws2.schedule is None
    got = kmws.unmask_get_schedule(ws2, descs, len(buf))
    assert got == kmws.sched_default(len(buf), n) and not got & kmws.SCHED_TEMPORAL_STORES
    wdesc = torch.from_numpy(wd.view(np.int64).reshape(-1, 2).copy()).cuda()
    want = buf.copy()
    orc.unmask_batch(want, wd)
    kmws.unmask_batch(d_buf, wdesc, ws2, len(buf))
    torch.cuda.synchronize()
    assert ws2.status() == 0 and np.array_equal(d_buf.cpu().numpy()[:len(buf)], want)
    # the raw C apply on the tuned batch's own pointers: default schedule, still exact
    kmws.fill_synthetic(base, 9)
    lib = kmws.lib()
    assert lib.kmws_unmask_plan(span, old_desc, n, ws2.ptr, ws2.nbytes, kmws._stream_handle()) == 0
    assert lib.kmws_unmask_apply(base.data_ptr(), span, old_desc, n, ws2.ptr, ws2.nbytes,
                                 kmws._stream_handle()) == 0
    torch.cuda.synchronize()
    assert ws2.status() == 0 and kmws.check_unmasked(base, 9, descs) == 0


def test_apply_sched_rejects_bad_codes(torch_dev):
    from kuma_amd import kmws
    ws = kmws.Workspace(1024)
    d = torch_dev.zeros((1, 2), dtype=torch_dev.int64, device="cuda")
    b = torch_dev.zeros(64, dtype=torch_dev.uint8, device="cuda")
    h = kmws._stream_handle()
    for bad in (6, 64, 0xFF, (1 << 29) | (1 << 30), 1 << 28, 65537):
        assert kmws.lib().kmws_unmask_apply_sched(b.data_ptr(), 64, d.data_ptr(), 1, ws.ptr, ws.nbytes, bad,
                                                  h) == kmws.ERR_INVALID_PARAM
    assert kmws.lib().kmws_unmask_apply_sched(b.data_ptr(), 64, d.data_ptr(), 1, None, 0, 0, h) == \
        kmws.ERR_INVALID_PARAM
    ws.schedule = 6  # an invalid pinned code fails at the apply, loudly
    with pytest.raises(RuntimeError):
        kmws.unmask_apply(b, d, ws, 64)


@pytest.mark.parametrize("frame_len,tail", [(65536, 0), (65531, 0), (3000, 0), (65531, 7 * 16384 + 100)])
@pytest.mark.parametrize("schedule", [None] + KINDS_X_STORES)
def test_unmask_schedules_many_tiles_per_block(torch_dev, schedule, frame_len, tail):
    """512 MiB arena (32 K tiles: whole runs and parts of the XCD-run and split
    mappings), plus a
    tail that is not a whole number of runs / parts (and a partial last tile):
    payload generated on the device, every byte checked on the device against
    the generator (payload ^ key inside frames, untouched gaps).  Applied three
    times (odd), so a schedule that skipped or doubled a tile shows up."""
    torch = torch_dev
    from kuma_amd import kmws
    stride = 65536 if frame_len > 4096 else 4096
    span = (512 << 20) + tail
    n = span // stride
    base = torch.empty(span, dtype=torch.uint8, device="cuda")
    descs = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(base, 1234)
    kmws.fill_uniform_descs(descs, stride, frame_len, 99)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    for _ in range(3):
        kmws.unmask_batch(base, descs, ws, span, schedule=schedule)
    torch.cuda.synchronize()
    assert ws.status() == 0
    assert kmws.check_unmasked(base, 1234, descs) == 0


def test_arena_alloc_unmask_roundtrip(torch_dev):
    """kmws_arena_alloc: a (physically contiguous where possible) arena usable
    as a torch view; unmask on it, checked on the device; freed without error."""
    torch = torch_dev
    from kuma_amd import kmws
    span, L = 256 << 20, 65536
    a = kmws.Arena(span)
    assert a.tensor.data_ptr() == a._p and a.tensor.numel() == span
    descs = torch.empty((span // L, 2), dtype=torch.int64, device="cuda")
    kmws.fill_synthetic(a.tensor, 77)
    kmws.fill_uniform_descs(descs, L, L - 5, 5)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    kmws.unmask_batch(a.tensor, descs, ws, span)
    torch.cuda.synchronize()
    assert ws.status() == 0 and kmws.check_unmasked(a.tensor, 77, descs) == 0
    del a
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("span_mib,step_mib,arena_mib", [(64, 32, 160), (1, 1, 3), (96, 48, 96)])
def test_arena_place_picks_an_offset_and_leaves_bytes(torch_dev, span_mib, step_mib, arena_mib):
    """kmws_arena_place: returns one of the probed offsets (multiples of step,
    offset + span inside the arena), one rate per offset, and the arena's bytes
    unchanged (the probe XORs every region twice); the batch placed there
    unmasks bit-exactly.  A span that is not a whole number of 64 KiB probe
    frames is covered too (96 MiB / 48 MiB steps: 1 offset)."""
    torch = torch_dev
    from kuma_amd import kmws
    span, step = span_mib << 20, step_mib << 20
    a = kmws.Arena(arena_mib << 20)
    kmws.fill_synthetic(a.tensor, 4242)
    torch.cuda.synchronize()
    off, probe = kmws.arena_place(a, span, step)
    assert sorted(probe) == list(range(0, (arena_mib << 20) - span + 1, step))
    assert off in probe and off % step == 0 and off + span <= a.nbytes
    assert all(v > 0 for v in probe.values())
    n = a.nbytes // 65536  # nothing changed anywhere in the arena
    d_all = torch.zeros((n, 2), dtype=torch.int64, device="cuda")
    assert kmws.check_unmasked(a.tensor, 4242, d_all) == 0
    L = 65536 - 7
    descs = torch.empty((span // 65536, 2), dtype=torch.int64, device="cuda")
    kmws.fill_uniform_descs(descs, 65536, L, 17)
    ws = kmws.Workspace(kmws.unmask_workspace_size(span))
    view = a.tensor[off:off + span]
    kmws.unmask_batch(view, descs, ws, span)
    torch.cuda.synchronize()
    assert ws.status() == 0 and kmws.check_unmasked(view, 4242 + (off >> 3), descs) == 0


@pytest.mark.gpu
def test_arena_place_rejects_bad_arguments(torch_dev):
    import ctypes as C
    from kuma_amd import kmws
    a = kmws.Arena(4 << 20)
    lib = kmws.lib()
    assert lib.kmws_arena_place(a._p, a.nbytes, 8 << 20, 1 << 20, None, None, 0) == kmws.ERR_INVALID_PARAM  # span > arena
    assert lib.kmws_arena_place(a._p, a.nbytes, 1 << 20, 0, None, None, 0) == kmws.ERR_INVALID_PARAM        # step 0
    assert lib.kmws_arena_place(a._p, a.nbytes, 1 << 20, 24, None, None, 0) == kmws.ERR_INVALID_PARAM       # step % 16
    assert lib.kmws_arena_place(None, a.nbytes, 1 << 20, 1 << 20, None, None, 0) == kmws.ERR_INVALID_PARAM
    assert lib.kmws_arena_place(a._p, a.nbytes, 0, 1 << 20, None, None, 0) == kmws.ERR_INVALID_PARAM
