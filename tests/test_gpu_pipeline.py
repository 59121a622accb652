"""Host-resident batches through kmws_pipeline (pinned H2D -> unmask -> D2H),
bit-exact vs the oracle; small chunks force many frame-boundary cuts."""
import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kmws():
    from kuma_amd import kmws as k
    if k.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    return k


def wire_like(rng, n, maxlen):
    lens = rng.integers(0, maxlen, size=n)
    hdr = rng.integers(2, 15, size=n)
    starts = np.cumsum(np.concatenate([[0], hdr + lens]))
    offs = (starts[:-1] + hdr).astype(np.uint64)
    buf = rng.integers(0, 256, size=int(starts[-1]) + 7, dtype=np.uint8)
    d = np.zeros(n, dtype=orc.DESC_DTYPE)
    d["off"], d["len"] = offs, lens
    d["key"] = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    return buf, d


@pytest.mark.parametrize("chunk,max_frames,depth", [(65536, 1 << 16, 2), (70000, 7, 3), (1 << 20, 100, 1)])
def test_pipeline_pageable(kmws, chunk, max_frames, depth):
    rng = np.random.default_rng(chunk + max_frames)
    buf, d = wire_like(rng, 700, 60000)
    want = buf.copy()
    orc.unmask_batch(want, d)
    p = kmws.Pipeline(0, chunk, max_frames, depth)
    p.unmask(buf, d)
    assert np.array_equal(buf, want)


@pytest.mark.parametrize("transfer,chunk,depth", [(0, 8 << 20, 3), (0, 256 << 20, 3), (1, 8 << 20, 8), (2, 8 << 20, 3)])
def test_pipeline_pinned(kmws, transfer, chunk, depth):
    """ZEROCOPY (and AUTO under two chunks): the kernel works on pinned host
    memory over PCIe; COPY (and AUTO from two chunks): the 3-stream SDMA ring,
    at most 3 slots in flight whatever the depth."""
    import torch
    rng = np.random.default_rng(9 + transfer + depth + (chunk >> 20))
    buf, d = wire_like(rng, 3000, 70000)
    want = buf.copy()
    orc.unmask_batch(want, d)
    t = torch.from_numpy(buf).pin_memory()
    kmws.Pipeline(0, chunk, 4096, depth, transfer=transfer).unmask(t, d)
    assert np.array_equal(t.numpy(), want)


def test_pipeline_zerocopy_needs_pinned(kmws):
    rng = np.random.default_rng(2)
    buf, d = wire_like(rng, 10, 1000)
    with pytest.raises(RuntimeError):
        kmws.Pipeline(0, 1 << 20, 64, 2, transfer=2).unmask(buf, d)


def test_pipeline_rejects_oversized_frame(kmws):
    rng = np.random.default_rng(1)
    buf, d = wire_like(rng, 3, 100)
    d["len"][1] = 200000
    buf = np.zeros(int(d["off"][-1]) + 300000, np.uint8)
    d["off"][2] = d["off"][1] + 200010
    with pytest.raises(RuntimeError):
        kmws.Pipeline(0, 65536, 16, 2).unmask(buf, d)


@pytest.mark.parametrize("defect,code", [("unsorted", -8), ("out_of_span", -8), ("oversized", -17)])
@pytest.mark.parametrize("pinned", [False, True])
def test_pipeline_late_bad_descriptor_leaves_buffer_untouched(kmws, defect, code, pinned):
    """A defect in the LAST descriptor (after many chunks' worth of good frames)
    is reported before any chunk is queued: the call fails with the reference's
    error value and not one byte of the host buffer has been rewritten."""
    import torch
    rng = np.random.default_rng(77 + len(defect))
    buf, d = wire_like(rng, 400, 60000)
    if defect == "unsorted":
        d["off"][-1] = d["off"][-3]
    elif defect == "out_of_span":
        d["len"][-1] = buf.nbytes  # runs past the span
    else:  # a frame larger than one chunk, placed after the others
        big = np.zeros(buf.nbytes + 300000, np.uint8)
        big[:buf.nbytes] = buf
        buf = big
        d["off"][-1] = d["off"][-2] + d["len"][-2] + 16
        d["len"][-1] = 200000
    orig = buf.copy()
    host = torch.from_numpy(buf).pin_memory() if pinned else buf
    # COPY transfer: the chunked ring (the path that used to queue earlier chunks)
    p = kmws.Pipeline(0, 1 << 17, 1 << 16, 3, transfer=1)
    with pytest.raises(RuntimeError, match=f"kmws_status {code}"):
        p.unmask(host, d)
    got = host.numpy() if pinned else host
    assert np.array_equal(got, orig)
    # the pipeline stays usable: a good batch afterwards is exact
    good, gd = wire_like(rng, 300, 60000)
    want = good.copy()
    orc.unmask_batch(want, gd)
    p.unmask(good, gd)
    assert np.array_equal(good, want)
