"""GPU round trips of BASELINE.json configs 3 and 4 and of the host-memory
pipeline at reduced sizes, through tools/bench_configs.py (the same code that
produces the measured numbers), verified on the device:

  cfg2b 64 KiB frames as a packed wire (14-byte headers, misaligned
        payloads) unmasked in place: every byte checked on the device;
  cfg3  Zipf 128 B - 1 MiB frames: encode (header pack + mask) -> unpack
        headers -> gather + unmask; every payload byte equals the source
        (index-gather check independent of the kernels);
  cfg4  16 x 4 KiB fragment chains (a-12): pack -> unpack (flags == the
        packed ones, no WSError) -> in-place unmask == the source payloads;
  cfg3_e2e  pinned host Zipf payloads -> H2D -> encode -> unpack ->
        gather-unmask -> D2H == the input, every byte (chunks of whole frames
        on three slots, frames straddling no chunk);
  e2e   pinned host wire image unmasked an even number of times (zero-copy
        and SDMA ring) == its initial bytes, every byte.

Round trip = identity is size-independent, so the same checks hold at the
full bench sizes, where bench_configs.py runs them too."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def bc():
    import torch
    from kuma_amd import kmws
    if not torch.cuda.is_available() or kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    import bench_configs
    return bench_configs


def test_cfg3_roundtrip(bc):
    r = bc.cfg3(1, 0.5)
    assert r["verified"] and r["frames"] > 10000


def test_cfg4_roundtrip(bc):
    r = bc.cfg4(1, 4096)
    assert r["verified"] and r["frames"] == 4096 * 16


def test_e2e_pipeline_roundtrip(bc):
    r = bc.e2e(0.25, 16, 3)
    assert r["verified"]


def test_cfg3_e2e_roundtrip(bc):
    r = bc.cfg3_e2e(0.25, 8, 1)  # 8 MiB chunks: ~32 chunks, every slot reused many times
    assert r["verified"] and r["chunks"] > 6


def test_cfg2b_packed_wire(bc):
    r = bc.cfg2b(2, 8192)  # 512 MiB: beyond the MALL, boundary tiles on the general path
    assert r["verified"]
