"""C-ABI checks that need no GPU: the library loads and exports every symbol
include/kmws_gpu.h and include/kmws_bench.h declare; host codec entries match
the oracle."""
import os
import random
import re

import pytest

from kuma_amd import kmws
from oracle import oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_decls(name="kmws_gpu.h"):
    txt = open(os.path.join(ROOT, "include", name)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = set(re.findall(r"\b(kmws_[a-z0-9_]+)\s*\(", txt))
    return sorted(n for n in names if n != "kmws_make_flags")  # static inline helper


def test_exports_every_declared_symbol():
    L = kmws.lib()
    decl = header_decls()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(kmws.EXPORTS) == decl
    bench = header_decls("kmws_bench.h")
    for name in bench:
        assert hasattr(L, name), name
    assert sorted(kmws.BENCH_EXPORTS) == bench


def test_public_header_has_no_tuning_entries():
    """The drop-in header carries only boundary entries: no tuning variants,
    no device-global schedule query, no persistent-grid probes."""
    decl = header_decls()
    for gone in ("kmws_unmask_batch_variant", "kmws_unmask_schedule", "kmws_unmask_resident_blocks",
                 "kmws_arena_alloc", "kmws_fill_synthetic"):
        assert gone not in decl
    L = kmws.lib()
    assert not hasattr(L, "kmws_unmask_batch_variant") and not hasattr(L, "kmws_unmask_resident_blocks")


def test_encode_header_matches_oracle():
    rng = random.Random(7)
    lens = [0, 1, 2, 124, 125, 126, 127, 65534, 65535, 65536, 65537, 10485760, 2**31, 2**32 - 1]
    lens += [rng.randrange(2**32) for _ in range(200)]
    for L in lens:
        for mask in (0, 1):
            h = dict(fin=rng.randrange(2), rsv1=rng.randrange(2), rsv2=rng.randrange(2),
                     rsv3=rng.randrange(2), opcode=rng.randrange(16), mask=mask,
                     maskey=bytes(rng.randrange(256) for _ in range(4)), length=L)
            got = kmws.encode_frame_header(kmws.Header(**h))
            assert got == orc.encode_header(orc.Hdr(**h))
            assert len(got) == kmws.header_size(L, mask)


def _client_stream(rng, nframes):
    out = b""
    for _ in range(nframes):
        n = rng.choice([0, 1, 3, 125, 126, 200, 65535, 65536, 70001])
        op = rng.choice([0, 1, 2, 3, 9, 10])
        h = orc.Hdr(fin=1 if op >= 8 else rng.randrange(2), opcode=op, mask=0,
                    length=min(n, 125) if op >= 8 else n)
        out += orc.encode_header(h) + bytes(rng.randrange(256) for _ in range(h.length))
    return out


@pytest.mark.parametrize("chunk", [0, 1, 5, 64, 1000, 65536])
def test_decoder_unmasked_matches_oracle(chunk):
    """CLIENT-mode streams carry no masked payload, so no device work is needed."""
    rng = random.Random(100 + chunk)
    stream = _client_stream(rng, 12 if chunk == 1 else 60)
    rets_o, frames_o = orc.decode_chunks(stream, orc.CLIENT, chunk)
    h = kmws.WSHandler(kmws.CLIENT)
    got = []
    h.setFrameCallback(lambda hd, p: got.append((hd.fin, hd.rsv1, hd.rsv2, hd.rsv3, hd.opcode, hd.mask,
                                                 hd.plen, hd.xpl64, hd.maskey, hd.length, p)))
    rets = []
    if chunk <= 0:
        rets.append(h.handleData(stream))
    else:
        for i in range(0, len(stream), chunk):
            rets.append(h.handleData(stream[i:i + chunk]))
    assert rets == rets_o
    assert got == [f.key() for f in frames_o]


def test_decoder_golden_client_cases():
    import json
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
    ran = 0
    for c in gold["decode"]:
        if c["mode"] != "CLIENT":
            continue
        data = bytes.fromhex(c["input_hex"])
        if "tail_gen" in c:
            data += bytes(c["tail_len"]) if c["tail_gen"] == "zeros" else \
                bytes(i & 0xFF for i in range(c["tail_len"]))
        h = kmws.WSHandler(kmws.CLIENT)
        frames = []
        h.setFrameCallback(lambda hd, p: frames.append((hd, p)))
        step = c["chunk"] or len(data) or 1
        rets = [h.handleData(data[i:i + step]) for i in range(0, max(1, len(data)), step)]
        assert rets == c["expect_rets"], c["name"]
        assert len(frames) == len(c["expect_frames"]), c["name"]
        for (hd, p), e in zip(frames, c["expect_frames"]):
            assert (hd.fin, hd.opcode, hd.mask, hd.length) == (e["fin"], e["opcode"], e["mask"], e["length"])
        for s in c.get("then", []):
            assert h.handleData(bytes.fromhex(s["input_hex"])) == s["expect_rets"][0]
        ran += 1
    assert ran >= 15


def test_masked_frame_without_gpu_fails_loudly():
    if kmws.device_count() > 0:
        pytest.skip("GPU present")
    h = kmws.WSHandler(kmws.SERVER)
    assert h.handleData(bytes.fromhex("818537fa213d7f9f4d5158")) == kmws.ERR_NOT_SUPPORTED


def test_synthetic_host_generator():
    a = orc.synthetic(5, 0, 64)
    b = orc.synthetic(5, 13, 40)
    assert (a[13:53] == b).all()
    w = orc.splitmix64(5 + 1).to_bytes(8, "little")
    assert bytes(a[8:16]) == w


def test_find_headers_matches_oracle_walk():
    rng = random.Random(21)
    stream, offs = b"", []
    for _ in range(200):
        n = rng.choice([0, 1, 125, 126, 65535, 65536, 70000])
        h = orc.encode_header(orc.Hdr(opcode=rng.choice([0, 1, 2]), mask=rng.randrange(2),
                                      maskey=b"abcd", length=n))
        offs.append(len(stream))
        stream += h + bytes(n)
    got, used = kmws.find_headers(stream)
    assert got == offs and used == len(stream)
    # truncated tail: last frame recorded, consumed stops before it
    got, used = kmws.find_headers(stream[:-1])
    assert got == offs and used == offs[-1]
    # CLOSE stops the walk (WSHandler.cpp:265-268)
    close = orc.encode_header(orc.Hdr(opcode=8, length=0))
    got, used = kmws.find_headers(close + stream)
    assert got == [0] and used == 2
    # invalid 127-class length is recorded and ends the walk
    got, _ = kmws.find_headers(bytes.fromhex("827f4000000000000000") + stream)
    assert got == [0]


def test_arena_alloc_without_device_returns_null():
    """No gfx950 device here: kmws_arena_alloc reports failure (NULL), no crash."""
    import ctypes as C
    from kuma_amd import kmws
    if kmws.lib().kmws_device_count() > 0:
        pytest.skip("a device is present")
    flag = C.c_int(7)
    assert not kmws.lib().kmws_arena_alloc(1 << 20, 0, C.byref(flag))
    assert flag.value == 0
    kmws.lib().kmws_arena_free(None, 0)


def test_tx_batch_without_device_is_null():
    """No gfx950 device here: kmws_tx_batch_create returns NULL (no CPU fallback)."""
    from kuma_amd import kmws
    if kmws.lib().kmws_device_count() > 0:
        pytest.skip("a device is present")
    assert not kmws.lib().kmws_tx_batch_create(0)
    with pytest.raises(RuntimeError):
        kmws.TxBatch()


def test_batch_entries_reject_bad_arguments_before_any_device_work():
    """Argument checks of the device batch entries return kuma's INVALID_PARAM /
    BUFFER_TOO_SMALL without launching anything (so they hold with no GPU)."""
    import ctypes as C
    L = kmws.lib()
    fake = C.c_void_p(16)      # never dereferenced: every call below fails its checks first
    odd = C.c_void_p(16 + 8)   # not 16-byte aligned
    assert L.kmws_pack_headers(None, None, 5, fake, None, None, None, 0, None) == kmws.ERR_INVALID_PARAM
    assert L.kmws_pack_headers(fake, fake, 5, odd, None, None, None, 0, None) == kmws.ERR_INVALID_PARAM
    assert L.kmws_pack_headers(fake, fake, 5, fake, None, fake, None, 0, None) == kmws.ERR_INVALID_PARAM
    need = L.kmws_pack_headers_workspace_size(5)
    assert need >= 16
    assert L.kmws_pack_headers(fake, fake, 5, fake, None, fake, fake, need - 1, None) == kmws.ERR_BUFFER_TOO_SMALL
    assert L.kmws_find_headers_streams(fake, 64, None, 3, fake, 4, fake, None, None) == kmws.ERR_INVALID_PARAM
    assert L.kmws_find_headers_streams(fake, 64, fake, 3, None, 4, fake, None, None) == kmws.ERR_INVALID_PARAM
    assert L.kmws_find_headers_streams(None, 0, None, 0, None, 0, None, None, None) == 0  # nothing to do


def test_copy_workspace_size_follows_the_copy_form():
    """kmws_copy_workspace_size (no device needed): below a 16 KiB mean region
    bound (dst_cap / n) the chunk form's 8 B per 4 KiB output chunk, from it the
    unit form's edge words (80 B per frame) and 32-byte unit records -- so the
    same (n, dst_cap) the call passes must size the workspace."""
    n = 1000
    small = kmws.copy_workspace_size(n, n * 4104)        # cfg4-like: chunk form
    large = kmws.copy_workspace_size(n, n * 65550)       # 64 KiB frames: unit form
    chunks = -(-n * 4104 // 4096)
    assert small >= 8 * chunks and small < 8 * chunks + 64 * 1024
    assert large >= 80 * n + 32 * (n * 65550 // 4096)
    # the threshold: dst_cap / n crosses 16 KiB
    below = kmws.copy_workspace_size(n, n * 16383)
    above = kmws.copy_workspace_size(n, n * 16384)
    assert above > below + 80 * n // 2
    assert kmws.copy_workspace_size(0, 0) > 0


def test_device_batch_busy_without_batches():
    """kmws_device_batch_busy (no device needed): 0 before any device batch was
    enqueued, and for devices out of range."""
    L = kmws.lib()
    assert [L.kmws_device_batch_busy(d) for d in (0, 1, -1, 64, 1 << 20)] == [0, 0, 0, 0, 0]
    assert kmws.device_batch_busy(0) is False
