"""GPU parity of the batched pack/unpack path vs the oracle, bit-exact:
kmws_encode_batch (header pack + masked payload), kmws_unpack_headers
(descriptor-indexed header decode/validation), kmws_gather_unmask, and the
encode -> find headers -> unpack -> unmask round trip."""
import json
import zlib
import os

import numpy as np
import pytest

from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def T():
    import torch
    from kuma_amd import kmws
    if not torch.cuda.is_available() or kmws.device_count() < 1:
        pytest.fail("gpu test needs a gfx950 device")
    return torch


def frames(rng, kind, n):
    if kind == "mixed":
        lens = rng.choice([0, 1, 2, 3, 5, 124, 125, 126, 127, 1000, 4096, 65535, 65536, 65537, 100003], size=n)
    elif kind == "zipf":
        k = rng.choice(14, size=n, p=(np.arange(1, 15) ** -1.2) / np.sum(np.arange(1, 15) ** -1.2))
        lens = 128 * (2 ** k) - rng.integers(0, 64, size=n)
    elif kind == "large":
        lens = rng.integers(65536, 300000, size=n)
    elif kind == "tiny":
        lens = rng.integers(0, 9, size=n)
    elif kind == "frag4k":  # cfg4: 16 x 4 KiB per message
        lens = np.full(n, 4096)
    elif kind == "max":  # the decoder's cap WS_MAX_FRAME_DATA_LENGTH (WSHandler.cpp:110) and neighbours
        lens = np.resize(np.array([10485760, 3, 10485759, 0, 10485760 - 13, 10485760]), n)
    elif kind == "chat":  # a small mean (the chunk form) with large frames (interior chunks) and a
        # run of tiny ones (chunks of more than 64 frames: the dense kernel)
        cat = rng.choice(3, size=n, p=[0.6, 0.25, 0.15])
        lens = np.where(cat == 0, rng.integers(0, 301, size=n),
                        np.where(cat == 1, rng.integers(0, 9, size=n), rng.integers(4096, 150000, size=n)))
        run = rng.integers(0, max(1, n - 200))
        lens[run:run + 200] = rng.integers(0, 6, size=min(200, n - run))
    else:
        raise ValueError(kind)
    fin = rng.integers(0, 2, size=n)
    op = rng.choice([0, 1, 2, 3, 9, 10], size=n)
    if kind == "frag4k":
        pos = np.arange(n) % 16
        fin = (pos == 15).astype(int)
        op = np.where(pos == 0, 1 + (np.arange(n) // 16) % 2, 0)
    rsv = rng.integers(0, 8, size=n)
    mask = rng.integers(0, 2, size=n) if kind != "frag4k" else np.ones(n, int)
    flags = (fin << 7) | (rsv << 4) | op | (mask << 8)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    return lens.astype(np.int64), flags.astype(np.uint32), keys


def src_arena(rng, lens, aligned):
    gaps = rng.integers(0, 40, size=len(lens)) * (16 if aligned else 1)
    if aligned:
        lens16 = (lens + 15) // 16 * 16
        starts = np.concatenate([[0], np.cumsum(gaps + lens16)])
    else:
        starts = np.concatenate([[0], np.cumsum(gaps + lens)])
    offs = (starts[:-1] + gaps).astype(np.uint64)
    total = int(starts[-1]) + 64
    return rng.integers(0, 256, size=total, dtype=np.uint8), offs


def to_dev(T, a):
    pad = (-len(a)) % 16
    return T.from_numpy(np.concatenate([a, np.zeros(pad + 16, a.dtype)])).cuda()


def gpu_encode(T, src, offs, lens, flags, keys, cap=None):
    from kuma_amd import kmws
    n = len(lens)
    descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64))
    fl = T.from_numpy(flags.astype(np.int16)).cuda()
    total = int(np.sum(lens) + sum(kmws.header_size(int(L), bool(f >> 8 & 1)) for L, f in zip(lens, flags)))
    cap = total if cap is None else cap
    dst = T.full((cap + 16 - cap % 16,), 0xEE, dtype=T.uint8, device="cuda")
    wire_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.copy_workspace_size(n, cap))
    from kuma_amd.kmws import lib
    st = lib().kmws_encode_batch(to_dev(T, src).data_ptr(), descs.data_ptr(), fl.data_ptr(), n, dst.data_ptr(),
                                 cap, wire_off.data_ptr(), ws.ptr, ws.nbytes, 0)
    assert st == 0
    T.cuda.synchronize()
    return dst.cpu().numpy(), wire_off.cpu().numpy(), ws.status(), total


@pytest.mark.parametrize("kind", ["mixed", "zipf", "large", "tiny", "frag4k", "max", "chat"])
@pytest.mark.parametrize("aligned", [True, False])
@pytest.mark.parametrize("room", [0, 20000])
def test_encode_parity(T, kind, aligned, room):
    """room = spare output capacity per frame (an output buffer larger than
    the wire: nothing past the wire may be written)."""
    rng = np.random.default_rng(zlib.crc32(f"{kind}-{aligned}".encode()))
    n = {"mixed": 300, "zipf": 200, "large": 40, "tiny": 6000, "frag4k": 320, "max": 6, "chat": 900}[kind]
    lens, flags, keys = frames(rng, kind, n)
    src, offs = src_arena(rng, lens, aligned)
    want, want_off = orc.encode_batch(src, offs, lens, flags, keys)
    got, off, st, total = gpu_encode(T, src, offs, lens, flags, keys,
                                     cap=len(want) + room * n if room else None)
    assert st == 0 and total == len(want)
    assert np.array_equal(off[:n].astype(np.uint64), want_off) and off[n] == len(want)
    assert np.array_equal(got[:total], want)
    assert (got[total:total + 16] == 0xEE).all()  # nothing written past the wire


def test_encode_rejects_small_dst(T):
    rng = np.random.default_rng(4)
    lens, flags, keys = frames(rng, "mixed", 50)
    src, offs = src_arena(rng, lens, True)
    want, _ = orc.encode_batch(src, offs, lens, flags, keys)
    got, off, st, total = gpu_encode(T, src, offs, lens, flags, keys, cap=len(want) - 1)
    assert st != 0
    assert (got == 0xEE).all()


def wire_and_offsets(rng, kind, n, mode_mask=1):
    lens, flags, keys = frames(rng, kind, n)
    flags = (flags & 0xFF) | (mode_mask << 8)
    # control frames must be fin and <=125 to be valid for the decoder
    ctl = (flags & 0x0F) >= 8
    flags = np.where(ctl, flags | 0x80, flags)
    lens = np.where(ctl, np.minimum(lens, 125), lens)
    flags = flags & ~np.uint32(0x70)  # rsv bits off (decoder does not check them, keep streams plain)
    src, offs = src_arena(rng, lens, True)
    wire, wire_off = orc.encode_batch(src, offs, lens, flags, keys)
    return wire, wire_off, src, offs, lens, flags, keys


@pytest.mark.parametrize("kind", ["mixed", "zipf", "frag4k", "tiny", "max", "chat"])
@pytest.mark.parametrize("room", [0, 20000])
def test_unpack_gather_roundtrip(T, kind, room):
    """room = spare arena capacity per frame: 20000 puts the mean region bound
    past 16 KiB, so the gather takes the unit form; 0 the chunk form for every
    kind with a smaller mean (kmws_pack.hip, use_chunks)."""
    from kuma_amd import kmws
    rng = np.random.default_rng(zlib.crc32(str(kind).encode()))
    wire, wire_off, src, offs, lens, flags, keys = wire_and_offsets(rng, kind, 250 if kind != "max" else 6)
    hdr, used = kmws.find_headers(bytes(wire))
    # CLOSE frames stop the reference parser: cut the batch there like it does
    assert hdr == [int(x) for x in wire_off[:len(hdr)]]
    n = len(hdr)
    d_wire = to_dev(T, wire)
    d_hdr = T.tensor(hdr, dtype=T.int64, device="cuda")
    out_desc = T.zeros((n, 2), dtype=T.int64, device="cuda")
    out_flags = T.zeros(n, dtype=T.int16, device="cuda")
    out_err = T.full((n,), 99, dtype=T.uint8, device="cuda")
    ws = kmws.Workspace(kmws.lib().kmws_unpack_workspace_size())
    kmws.unpack_headers(d_wire, d_hdr, kmws.SERVER, out_desc, out_flags, out_err, ws, wire_len=len(wire))
    T.cuda.synchronize()
    assert ws.status() == 0 and (out_err.cpu().numpy() == 0).all()
    for shift in (1, 7, 15):  # the same wire at unaligned addresses: identical descriptors (offsets relative)
        u = T.zeros(len(wire) + 64, dtype=T.uint8, device="cuda")
        u[shift:shift + len(wire)] = d_wire[:len(wire)]
        od2 = T.zeros((n, 2), dtype=T.int64, device="cuda")
        oe2 = T.full((n,), 99, dtype=T.uint8, device="cuda")
        kmws.unpack_headers(u[shift:shift + len(wire)], d_hdr, kmws.SERVER, od2, None, oe2, ws, wire_len=len(wire))
        T.cuda.synchronize()
        assert T.equal(od2, out_desc) and T.equal(oe2, out_err), shift
    dd = out_desc.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
    # oracle decode of the same stream (SERVER) gives the frames
    rets, ofr = orc.decode_chunks(bytes(wire[:used]), orc.SERVER, 0)
    assert len(ofr) == n
    assert [int(x) for x in dd["len"]] == [f.length for f in ofr]
    assert [int(x) for x in dd["key"]] == [int.from_bytes(f.maskey, "little") if f.mask else 0 for f in ofr]
    fl = out_flags.cpu().numpy().astype(np.uint16)
    assert [int(x) for x in fl] == [(f.fin << 7 | f.rsv1 << 6 | f.rsv2 << 5 | f.rsv3 << 4 | f.opcode) |
                                    (f.mask << 8) for f in ofr]
    # gather + unmask into a dense arena == the oracle's payloads == the original source bytes
    total = int(dd["len"].sum())
    dst = T.zeros(total + 32 + room * n, dtype=T.uint8, device="cuda")
    dst_off = T.zeros(n + 1, dtype=T.int64, device="cuda")
    ws2 = kmws.Workspace(kmws.copy_workspace_size(n, dst.numel()))
    kmws.gather_unmask(d_wire, out_desc, dst, dst_off, ws2)
    T.cuda.synchronize()
    assert ws2.status() == 0
    assert bytes(dst.cpu().numpy()[:total]) == b"".join(f.payload for f in ofr)
    assert int(dst[total:].count_nonzero()) == 0  # nothing written past the arena's payloads
    orig = b"".join(bytes(src[int(o):int(o) + int(L)]) for o, L in zip(offs[:n], lens[:n]))
    assert bytes(dst.cpu().numpy()[:total]) == orig
    # in-place alternative: unmask the wire itself with the unpacked descriptors
    ws3 = kmws.Workspace(kmws.unmask_workspace_size(len(wire)))
    kmws.unmask_batch(d_wire, out_desc, ws3, len(wire))
    T.cuda.synchronize()
    w2 = d_wire.cpu().numpy()
    assert b"".join(bytes(w2[int(o):int(o) + int(L)]) for o, L in zip(dd["off"], dd["len"])) == orig


@pytest.mark.parametrize("kind", ["mixed", "zipf", "frag4k", "tiny", "max", "large", "chat"])
def test_fused_unpack_unmask_and_gather_equal_the_two_step_forms(T, kind):
    """kmws_unpack_unmask (header parse writing the unmask plan
    in one kernel, then the in-place unmask) and kmws_unpack_gather (header
    parse inside the gather's scan) produce exactly what kmws_unpack_headers +
    kmws_unmask_batch / kmws_gather_unmask produce -- descriptors, flags,
    errors, the unmasked wire, the dense payloads and offsets -- and the
    payloads equal the oracle decoder's, at an aligned and a shifted wire."""
    from kuma_amd import kmws
    rng = np.random.default_rng(zlib.crc32(f"fused-{kind}".encode()))
    wire, wire_off, src, offs, lens, flags, keys = wire_and_offsets(rng, kind, 300 if kind != "max" else 6)
    hdr, used = kmws.find_headers(bytes(wire))
    n = len(hdr)
    rets, ofr = orc.decode_chunks(bytes(wire[:used]), orc.SERVER, 0)
    want_pay = b"".join(f.payload for f in ofr)
    d_hdr = T.tensor(hdr, dtype=T.int64, device="cuda")
    W = len(wire)
    for shift in (0, 16 * 3):
        base = T.zeros(W + shift + 64, dtype=T.uint8, device="cuda")
        base[shift:shift + W] = T.from_numpy(wire.copy()).cuda()
        d_wire = base[shift:]
        # two-step reference forms
        od, of, oe = (T.zeros((n, 2), dtype=T.int64, device="cuda"), T.zeros(n, dtype=T.int16, device="cuda"),
                      T.full((n,), 99, dtype=T.uint8, device="cuda"))
        kmws.unpack_headers(d_wire, d_hdr, kmws.SERVER, od, of, oe, kmws.Workspace(16), wire_len=W)
        total = int(od[:, 1].bitwise_and(0xFFFFFFFF).sum())
        dst0 = T.zeros(total + 32, dtype=T.uint8, device="cuda")
        doff0 = T.zeros(n + 1, dtype=T.int64, device="cuda")
        kmws.gather_unmask(d_wire, od, dst0, doff0, kmws.Workspace(kmws.copy_workspace_size(n, dst0.numel())))
        # fused gather
        fd, ff, fe = (T.zeros((n, 2), dtype=T.int64, device="cuda"), T.zeros(n, dtype=T.int16, device="cuda"),
                      T.full((n,), 99, dtype=T.uint8, device="cuda"))
        dst1 = T.full((total + 32,), 0xEE, dtype=T.uint8, device="cuda")
        dst1[total:] = 0
        doff1 = T.zeros(n + 1, dtype=T.int64, device="cuda")
        wsg = kmws.Workspace(kmws.copy_workspace_size(n, dst1.numel()))
        kmws.unpack_gather(d_wire, d_hdr, kmws.SERVER, fd, ff, fe, dst1, doff1, wsg, wire_len=W)
        T.cuda.synchronize()
        assert wsg.status() == 0
        assert T.equal(fd, od) and T.equal(ff, of) and T.equal(fe, oe) and int(oe.max()) == 0
        assert T.equal(doff1, doff0) and T.equal(dst1, dst0)
        assert bytes(dst1.cpu().numpy()[:total]) == want_pay
        # fused in place
        wire2 = base.clone()
        fd2 = T.zeros((n, 2), dtype=T.int64, device="cuda")
        fe2 = T.full((n,), 99, dtype=T.uint8, device="cuda")
        wsm = kmws.Workspace(kmws.unmask_workspace_size(W))
        kmws.unpack_unmask(wire2[shift:], d_hdr, kmws.SERVER, fd2, None, fe2, wsm, wire_len=W)
        wire3 = base.clone()
        kmws.unmask_batch(wire3[shift:], od, kmws.Workspace(kmws.unmask_workspace_size(W)), W)
        T.cuda.synchronize()
        assert wsm.status() == 0 and T.equal(fd2, od) and T.equal(fe2, oe)
        assert T.equal(wire2, wire3)
        w2 = wire2[shift:shift + W].cpu().numpy()
        dd = od.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
        assert b"".join(bytes(w2[int(o):int(o) + int(L)]) for o, L in zip(dd["off"], dd["len"])) == want_pay


def test_fused_decode_header_errors_and_bad_offsets(T):
    """A bad header inside the batch: both fused forms report it per frame
    (out_err, status bit 2), give it no payload, and still decode every other
    frame; offsets out of order make kmws_unpack_unmask store nothing (bit 1)."""
    from kuma_amd import kmws
    rng = np.random.default_rng(5)
    wire, wire_off, src, offs, lens, flags, keys = wire_and_offsets(rng, "mixed", 60)
    hdr, used = kmws.find_headers(bytes(wire))
    n = len(hdr)
    bad = n // 2
    wire = wire.copy()
    wire[hdr[bad] + 1] &= 0x7F  # clear the MASK bit: a SERVER must reject an unmasked non-empty frame
    expect_err = 7 if lens[bad] > 0 else 0
    d_hdr = T.tensor(hdr, dtype=T.int64, device="cuda")
    W = len(wire)
    d_wire = to_dev(T, wire)
    od = T.zeros((n, 2), dtype=T.int64, device="cuda")
    oe = T.full((n,), 99, dtype=T.uint8, device="cuda")
    kmws.unpack_headers(d_wire, d_hdr, kmws.SERVER, od, None, oe, kmws.Workspace(16), wire_len=W)
    T.cuda.synchronize()
    assert int(oe[bad]) == expect_err
    ref = d_wire.clone()
    kmws.unmask_batch(ref, od, kmws.Workspace(kmws.unmask_workspace_size(W)), W)
    w = d_wire.clone()
    fd = T.zeros((n, 2), dtype=T.int64, device="cuda")
    fe = T.full((n,), 99, dtype=T.uint8, device="cuda")
    wsm = kmws.Workspace(kmws.unmask_workspace_size(W))
    kmws.unpack_unmask(w, d_hdr, kmws.SERVER, fd, None, fe, wsm, wire_len=W)
    T.cuda.synchronize()
    assert T.equal(fd, od) and T.equal(fe, oe) and T.equal(w, ref)
    assert wsm.status() == (2 if expect_err else 0)
    total = int(od[:, 1].bitwise_and(0xFFFFFFFF).sum())
    dst = T.zeros(total + 32, dtype=T.uint8, device="cuda")
    doff = T.zeros(n + 1, dtype=T.int64, device="cuda")
    wsg = kmws.Workspace(kmws.copy_workspace_size(n, dst.numel()))
    kmws.unpack_gather(d_wire, d_hdr, kmws.SERVER, fd, None, fe, dst, doff, wsg, wire_len=W)
    dst0 = T.zeros(total + 32, dtype=T.uint8, device="cuda")
    doff0 = T.zeros(n + 1, dtype=T.int64, device="cuda")
    kmws.gather_unmask(d_wire, od, dst0, doff0, kmws.Workspace(kmws.copy_workspace_size(n, dst0.numel())))
    T.cuda.synchronize()
    assert T.equal(fd, od) and T.equal(fe, oe) and T.equal(dst, dst0) and T.equal(doff, doff0)
    assert wsg.status() == (2 if expect_err else 0)
    # offsets out of order: nothing unmasked, bit 1
    sw = d_hdr.clone()
    sw[3], sw[4] = d_hdr[4], d_hdr[3]
    w = d_wire.clone()
    kmws.unpack_unmask(w, sw, kmws.SERVER, fd, None, fe, wsm, wire_len=W)
    T.cuda.synchronize()
    assert wsm.status() & 1 and T.equal(w, d_wire)


def test_unpack_error_codes_match_reference(T):
    """Single-frame wires from the golden set: per-frame WSError == the
    reference decoder's return code for that frame."""
    from kuma_amd import kmws
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")))
    ran = 0
    for c in gold["decode"]:
        data = bytes.fromhex(c["input_hex"])
        if "tail_gen" in c or not data or c["chunk"]:
            continue
        mode = kmws.SERVER if c["mode"] == "SERVER" else kmws.CLIENT
        hdr, _ = kmws.find_headers(data, cap=1)
        want = c["expect_rets"][0]
        want = 0 if want == 8 else want  # CLOSE: the frame itself decodes fine
        d_wire = to_dev(T, np.frombuffer(data, np.uint8))
        out_desc = T.zeros((1, 2), dtype=T.int64, device="cuda")
        out_err = T.full((1,), 99, dtype=T.uint8, device="cuda")
        ws = kmws.Workspace(16)
        kmws.unpack_headers(d_wire, T.tensor(hdr, dtype=T.int64, device="cuda"), mode, out_desc, None, out_err,
                            ws, wire_len=len(data))
        T.cuda.synchronize()
        got = int(out_err.cpu()[0])
        if c["expect_frames"] and want == 0:
            assert got == 0, c["name"]
            assert int(out_desc.cpu().numpy()[0, 1] & 0xFFFFFFFF) == c["expect_frames"][0]["length"]
        else:
            assert got == want, c["name"]
        ran += 1
    assert ran >= 15


def test_unpack_quirk127_lengths(T):
    from kuma_amd import kmws
    cases = [("0000000100000005", 0, 5), ("0000010000000000", 0, 256), ("4000000000000000", 6, 0),
             ("0000000080000000", 6, 0), ("0000000000a00001", 6, 0)]
    for ext, err, L in cases:
        data = bytes.fromhex("827f" + ext) + bytes(L)
        d_wire = to_dev(T, np.frombuffer(data, np.uint8))
        out_desc = T.zeros((1, 2), dtype=T.int64, device="cuda")
        out_err = T.full((1,), 99, dtype=T.uint8, device="cuda")
        ws = kmws.Workspace(16)
        kmws.unpack_headers(d_wire, T.zeros(1, dtype=T.int64, device="cuda"), kmws.CLIENT, out_desc, None,
                            out_err, ws, wire_len=len(data))
        T.cuda.synchronize()
        assert int(out_err.cpu()[0]) == err, ext
        assert int(out_desc.cpu().numpy()[0, 1] & 0xFFFFFFFF) == L


@pytest.mark.parametrize("kind", ["mixed", "zipf", "frag4k", "max", "tiny"])
def test_pack_headers_parity(T, kind):
    """kmws_pack_headers: every 16-B slot == the oracle's encodeFrameHeader bytes
    (zero-padded), lengths and wire offsets == the oracle's encode_batch; the
    payloads masked in place by kmws_unmask_batch on the same descriptors then
    equal the oracle wire image's payload bytes (kuma's iovec {hdr, payload})."""
    from kuma_amd import kmws
    rng = np.random.default_rng(zlib.crc32(f"pack-headers-{kind}".encode()))
    n = 300 if kind != "max" else 6
    lens, flags, keys = frames(rng, kind, n)
    src, offs = src_arena(rng, lens, True)
    want, want_off = orc.encode_batch(src, offs, lens, flags, keys)
    descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64))
    fl = T.from_numpy(flags.astype(np.int16)).cuda()
    hdr = T.full((16 * n,), 0xEE, dtype=T.uint8, device="cuda")
    hl = T.zeros(n, dtype=T.uint8, device="cuda")
    woff = T.zeros(n + 1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))
    kmws.pack_headers(descs, fl, hdr, hl, woff, ws)
    T.cuda.synchronize()
    assert ws.status() == 0
    H = hdr.cpu().numpy().reshape(n, 16)
    L = hl.cpu().numpy()
    wo = woff.cpu().numpy()
    for i in range(n):
        m = bool(flags[i] >> 8 & 1)
        want_h = orc.encode_header(orc.Hdr(fin=int(flags[i] >> 7 & 1), rsv1=int(flags[i] >> 6 & 1),
                                           rsv2=int(flags[i] >> 5 & 1), rsv3=int(flags[i] >> 4 & 1),
                                           opcode=int(flags[i] & 15), mask=int(m),
                                           maskey=int(keys[i]).to_bytes(4, "little"), length=int(lens[i])))
        assert int(L[i]) == len(want_h), i
        assert bytes(H[i]) == want_h + bytes(16 - len(want_h)), i
        assert int(wo[i]) == int(want_off[i]), i
        assert bytes(want[int(wo[i]):int(wo[i]) + len(want_h)]) == want_h
    assert int(wo[n]) == len(want)
    # payloads masked in place with the same descriptors (masked frames only carry a key)
    d_src = to_dev(T, src)
    mk = np.where((flags >> 8) & 1, keys, 0).astype(np.int64)
    d2 = kmws.make_descs(offs.astype(np.int64), lens, mk)
    wsm = kmws.Workspace(kmws.unmask_workspace_size(len(src)))
    kmws.unmask_batch(d_src, d2, wsm, len(src))
    T.cuda.synchronize()
    got = d_src.cpu().numpy()
    for i in range(n):
        p0 = int(wo[i]) + int(L[i])
        assert bytes(got[int(offs[i]):int(offs[i]) + int(lens[i])]) == bytes(want[p0:p0 + int(lens[i])]), i
    # headers only, no offsets (no workspace)
    hdr2 = T.zeros((16 * n,), dtype=T.uint8, device="cuda")
    kmws.pack_headers(descs, fl, hdr2)
    T.cuda.synchronize()
    assert T.equal(hdr2, hdr)


def np_header_slots(lens, flags, keys):
    """encodeFrameHeader (WSHandler.cpp:46-106) vectorised: (n, 16) zero-padded
    slots and lengths.  Checked against the oracle's encode_header on a sample in
    test_pack_headers_chain_many_tiles."""
    n = len(lens)
    L = lens.astype(np.int64)
    m = ((flags >> 8) & 1).astype(np.int64)
    cls = np.where(L <= 125, 0, np.where(L <= 0xFFFF, 1, 2))
    S = np.zeros((n, 16), dtype=np.uint8)
    S[:, 0] = flags & 0xFF
    S[:, 1] = (m << 7) | np.where(cls == 0, L, np.where(cls == 1, 126, 127))
    c1, c2 = cls == 1, cls == 2
    S[c1, 2], S[c1, 3] = (L[c1] >> 8) & 0xFF, L[c1] & 0xFF
    for k in range(4):  # 127 class: 4 zero bytes, then the 32-bit length big-endian
        S[c2, 6 + k] = (L[c2] >> (8 * (3 - k))) & 0xFF
    base = np.array([2, 4, 10])[cls]
    rows = np.nonzero(m)[0]
    for k in range(4):
        S[rows, base[rows] + k] = (keys[rows].astype(np.int64) >> (8 * k)) & 0xFF
    return S, (base + 4 * m).astype(np.uint8)


@pytest.mark.parametrize("n", [2047, 2048, 2049, 6145, 1_500_001])
def test_pack_headers_chain_many_tiles(T, n):
    """The one-pass header pack over many 2048-frame tiles: 1.5 M frames = 733
    tiles, more than one 512-tile look-back window.  Slots, lengths and wire
    offsets == the vectorised encodeFrameHeader and the exclusive scan of
    header + payload bytes (the oracle's encode_batch offsets), every frame;
    the vectorised headers == the oracle's on a sample.  Repeated on the same
    workspace (the tile states are re-zeroed per call)."""
    from kuma_amd import kmws
    rng = np.random.default_rng(n)
    lens = rng.choice([0, 7, 125, 126, 4096, 65535, 65536, 70000, 10485760], size=n).astype(np.int64)
    flags = (rng.integers(0, 256, size=n) | (rng.integers(0, 2, size=n) << 8)).astype(np.uint32)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    S, hl = np_header_slots(lens, flags, keys)
    for i in list(rng.integers(0, n, size=64)) + [0, n - 1]:
        want_h = orc.encode_header(orc.Hdr(fin=int(flags[i] >> 7 & 1), rsv1=int(flags[i] >> 6 & 1),
                                           rsv2=int(flags[i] >> 5 & 1), rsv3=int(flags[i] >> 4 & 1),
                                           opcode=int(flags[i] & 15), mask=int(flags[i] >> 8 & 1),
                                           maskey=int(keys[i]).to_bytes(4, "little"), length=int(lens[i])))
        assert bytes(S[i]) == want_h + bytes(16 - len(want_h)) and hl[i] == len(want_h), i
    woff_want = np.concatenate([[0], np.cumsum(lens + hl.astype(np.int64))])
    descs = kmws.make_descs(np.zeros(n, np.int64), lens, keys.astype(np.int64))
    fl = T.from_numpy(flags.astype(np.int16)).cuda()
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))
    for rep in range(2):
        hdr = T.full((16 * n,), 0xEE, dtype=T.uint8, device="cuda")
        hlo = T.zeros(n, dtype=T.uint8, device="cuda")
        woff = T.full((n + 1,), -1, dtype=T.int64, device="cuda")
        kmws.pack_headers(descs, fl, hdr, hlo, woff, ws)
        T.cuda.synchronize()
        assert ws.status() == 0, rep
        assert np.array_equal(hdr.cpu().numpy().reshape(n, 16), S), rep
        assert np.array_equal(hlo.cpu().numpy(), hl), rep
        assert np.array_equal(woff.cpu().numpy(), woff_want), rep


def test_pack_headers_lookback_timeout_sets_its_own_bit(T):
    """VERDICT r03 #7 / ADVICE r03: a look-back predecessor that never
    publishes must end the wait with kStatusLookbackTimeout (4), not the
    bad-descriptor bit, and the call must return.  Test-only library
    (kuma_amd/build.py TEST_DEFINES): tile 1 of the header pack never
    publishes, the spin bound is 4096 polls.  The product binding then refuses
    the offsets (KmwsError with the workspace status)."""
    import ctypes as C
    from kuma_amd import build as kb
    from kuma_amd import kmws
    assert os.path.exists(kb.TEST_LIB), "run __graft_entry__.build()"
    L = C.CDLL(kb.TEST_LIB)
    vp = C.c_void_p
    L.kmws_pack_headers.restype, L.kmws_pack_headers.argtypes = C.c_int, [vp, vp, C.c_uint32, vp, vp, vp, vp,
                                                                         C.c_size_t, vp]
    L.kmws_read_status.restype, L.kmws_read_status.argtypes = C.c_int, [vp, C.POINTER(C.c_uint32), vp]
    n = 4 * 2048 + 5
    rng = np.random.default_rng(44)
    lens = rng.integers(0, 70000, size=n)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.int64)
    descs = kmws.make_descs(np.zeros(n, np.int64), lens, keys)
    fl = T.full((n,), 0x182, dtype=T.int16, device="cuda")
    hdr = T.zeros(16 * n, dtype=T.uint8, device="cuda")
    woff = T.zeros(n + 1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))
    h = kmws._stream_handle()
    assert L.kmws_pack_headers(descs.data_ptr(), fl.data_ptr(), n, hdr.data_ptr(), None, woff.data_ptr(), ws.ptr,
                               ws.nbytes, h) == 0
    st = C.c_uint32(0)
    assert L.kmws_read_status(ws.ptr, C.byref(st), h) == 0
    assert st.value & 4 and not st.value & 1, st.value
    # the product library on the same batch: clean status, offsets exact
    kmws.pack_headers(descs, fl, hdr, None, woff, ws)
    hl = np.where(lens <= 125, 2, np.where(lens <= 65535, 4, 10)) + 4
    assert np.array_equal(woff.cpu().numpy(), np.concatenate([[0], np.cumsum(lens + hl)]))
    # a nonzero status after the call surfaces as an error in the binding
    ws.status = lambda stream=None: 4
    with pytest.raises(kmws.KmwsError) as e:
        kmws.pack_headers(descs, fl, hdr, None, woff, ws, check=True)
    assert e.value.ws_status == 4


def test_chunk_scan_lookback_timeout_stores_nothing(T):
    """the chunk form's one-pass front (chunk_scan_kernel, used when
    dst_cap / n < 16 KiB) waits on a decoupled look-back too.  In the test build
    tile 1 never publishes: encode_batch and gather_unmask then report status
    bit 4 (not the bad-input bit), store nothing into dst, and the binding's
    check=True raises; the product library on the same batch is exact."""
    import ctypes as C
    from kuma_amd import build as kb
    from kuma_amd import kmws
    assert os.path.exists(kb.TEST_LIB), "run __graft_entry__.build()"
    TL = kmws.bind(C.CDLL(kb.TEST_LIB))
    n = 3 * 2048 + 7
    rng = np.random.default_rng(45)
    lens = rng.integers(1, 120, size=n)
    keys = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.int64)
    offs = np.arange(n, dtype=np.int64) * 128
    src = T.from_numpy(rng.integers(0, 256, size=n * 128, dtype=np.uint8)).cuda()
    descs = kmws.make_descs(offs, lens, keys)
    fl = T.full((n,), 0x182, dtype=T.int16, device="cuda")
    h = kmws._stream_handle()
    for what in ("encode", "gather"):
        cap = int(lens.sum()) + (6 * n if what == "encode" else 0)
        assert cap // n < 16384  # the chunk form
        dst = T.full((cap,), 0xAB, dtype=T.uint8, device="cuda")
        off = T.zeros(n + 1, dtype=T.int64, device="cuda")
        ws = kmws.Workspace(kmws.copy_workspace_size(n, cap))
        if what == "encode":
            rc = TL.kmws_encode_batch(src.data_ptr(), descs.data_ptr(), fl.data_ptr(), n, dst.data_ptr(), cap,
                                      off.data_ptr(), ws.ptr, ws.nbytes, h)
        else:
            rc = TL.kmws_gather_unmask(src.data_ptr(), descs.data_ptr(), n, dst.data_ptr(), cap, off.data_ptr(),
                                       ws.ptr, ws.nbytes, h)
        assert rc == 0
        st = C.c_uint32(0)
        assert TL.kmws_read_status(ws.ptr, C.byref(st), h) == 0
        assert st.value & 4 and not st.value & 1, (what, st.value)
        assert int((dst != 0xAB).sum()) == 0, what  # nothing stored
        # the product library: clean status, the binding's check passes
        if what == "encode":
            kmws.encode_batch(src, descs, fl, dst, off, ws, check=True)
            hl = 6
        else:
            kmws.gather_unmask(src, descs, dst, off, ws, check=True)
            hl = 0
        assert np.array_equal(off.cpu().numpy(), np.concatenate([[0], np.cumsum(lens + hl)]))
        ws.status = lambda stream=None: 4  # a nonzero status surfaces as an error with check=True
        with pytest.raises(kmws.KmwsError) as e:
            if what == "encode":
                kmws.encode_batch(src, descs, fl, dst, off, ws, check=True)
            else:
                kmws.gather_unmask(src, descs, dst, off, ws, check=True)
        assert e.value.ws_status == 4


def test_find_headers_streams_matches_host_walk(T):
    """kmws_find_headers_streams (one lane per stream) == kmws_find_headers on
    each stream: complete streams, streams cut mid-frame, a corrupted length,
    a CLOSE in the middle, empty and 1-byte streams, a cap smaller than the
    frame count; then the complete streams' offsets feed kmws_unpack_headers."""
    from kuma_amd import kmws
    rng = np.random.default_rng(zlib.crc32(b"walk-streams"))
    streams = []
    for s in range(300):
        kind = ["mixed", "zipf", "frag4k", "tiny"][s % 4]
        wire, wire_off, *_ = wire_and_offsets(rng, kind, int(rng.integers(1, 40)))
        wire = bytearray(wire)
        cut = s % 7
        if cut == 1 and len(wire) > 3:    # truncated mid-frame
            wire = wire[:int(rng.integers(1, len(wire)))]
        elif cut == 2 and len(wire_off) > 2:  # a 127-class length with bit 63 set
            wire[int(wire_off[1]) + 1] = (wire[int(wire_off[1]) + 1] & 0x80) | 127
            wire[int(wire_off[1]) + 2:int(wire_off[1]) + 3] = b"\x80"
        elif cut == 3:
            wire = wire[:s % 2]           # empty or one byte
        elif cut == 4 and len(wire_off) > 2:  # a CLOSE in the middle: the walk stops after it
            wire[int(wire_off[1])] = (wire[int(wire_off[1])] & 0xF0) | 8
        streams.append(bytes(wire))
    cap = 25
    buf = b"".join(streams)
    offs = np.concatenate([[0], np.cumsum([len(x) for x in streams])]).astype(np.int64)
    d_wire = to_dev(T, np.frombuffer(buf, np.uint8).copy() if buf else np.zeros(1, np.uint8))
    d_off = T.from_numpy(offs).cuda()
    hdr, n_out, consumed = kmws.find_headers_streams(d_wire, d_off, cap, wire_len=len(buf))
    T.cuda.synchronize()
    hdr, n_out, consumed = hdr.cpu().numpy(), n_out.cpu().numpy(), consumed.cpu().numpy()
    for s, w in enumerate(streams):
        h, used = kmws.find_headers(w, cap)
        assert int(n_out[s]) == len(h), s
        assert [int(x) - int(offs[s]) for x in hdr[s, :len(h)]] == h, s
        assert int(consumed[s]) == used, s
    # offsets past the wire are cut at its end (no read beyond it)
    bad = offs.copy()
    bad[-1] = len(buf) + 4096
    hb, nb, cb = kmws.find_headers_streams(d_wire, T.from_numpy(bad).cuda(), cap, wire_len=len(buf))
    T.cuda.synchronize()
    assert T.equal(nb.cpu(), T.from_numpy(n_out)) and T.equal(cb.cpu(), T.from_numpy(consumed))
    # complete streams back to back: their offsets are one unpackable header list
    whole = [s for s, w in enumerate(streams) if int(consumed[s]) == len(w) and len(w) and int(n_out[s]) < cap]
    hl = np.concatenate([hdr[s, :int(n_out[s])] for s in whole])
    ends = {int(offs[s]) + len(streams[s]) for s in whole}
    d_hl = T.from_numpy(hl.astype(np.int64)).cuda()
    od = T.zeros((len(hl), 2), dtype=T.int64, device="cuda")
    oe = T.full((len(hl),), 99, dtype=T.uint8, device="cuda")
    ws = kmws.Workspace(kmws.lib().kmws_unpack_workspace_size())
    kmws.unpack_headers(d_wire, d_hl, kmws.SERVER, od, None, oe, ws, wire_len=len(buf))
    T.cuda.synchronize()
    dd = od.cpu().numpy().view(orc.DESC_DTYPE).reshape(-1)
    assert (oe.cpu().numpy() == 0).all()
    i = 0
    for s_ in whole:  # the oracle decoding each whole stream gives the same frames
        rets, fr = orc.decode_chunks(streams[s_], orc.SERVER, 0)
        assert rets == [0] and len(fr) == int(n_out[s_]), s_
        for f in fr:
            assert int(dd["len"][i]) == f.length and int(dd["key"][i]) == int.from_bytes(f.maskey, "little"), (s_, i)
            i += 1
    assert i == len(hl)
    assert ends  # some complete streams were checked


@pytest.mark.parametrize("n", [0, 1])
def test_batch_entries_empty_and_single(T, n):
    """0 and 1 frames through every device batch entry of the pack path:
    kmws_pack_headers (one-pass offsets), kmws_encode_batch, kmws_unpack_headers
    and kmws_gather_unmask.  Empty batches write wire_off[0] = 0 and a clear
    status; a single frame equals the oracle (WSHandler.cpp:46-106, 303-310)."""
    from kuma_amd import kmws
    rng = np.random.default_rng(77 + n)
    lens = np.array([70000], np.int64)[:n]
    flags = np.array([0x182], np.uint32)[:n]           # FIN | BINARY, masked
    keys = np.array([0x3D21FA37], np.uint32)[:n]
    src = rng.integers(0, 256, size=70016 + 64, dtype=np.uint8)
    offs = np.array([16], np.uint64)[:n]
    want, want_off = orc.encode_batch(src, offs, lens, flags, keys) if n else (np.zeros(0, np.uint8), np.zeros(0))
    total = len(want)
    descs = kmws.make_descs(offs.astype(np.int64), lens, keys.astype(np.int64)).reshape(n, 2)
    fl = T.from_numpy(flags.astype(np.int16)).cuda()
    # header-only pack with offsets
    hdr = T.zeros(16 * max(n, 1), dtype=T.uint8, device="cuda")
    woff = T.full((n + 1,), -1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.pack_headers_workspace_size(n))
    kmws.pack_headers(descs, fl, hdr, None, woff, ws)
    T.cuda.synchronize()
    assert ws.status() == 0 and int(woff[n]) == total
    if n:
        assert int(woff[0]) == 0 and bytes(hdr.cpu().numpy()[:len(want) - int(lens[0])]) == bytes(want[:len(want) - int(lens[0])])
    # encode
    wire = T.full((total + 16,), 0xEE, dtype=T.uint8, device="cuda")
    wire_off = T.full((n + 1,), -1, dtype=T.int64, device="cuda")
    ws_e = kmws.Workspace(kmws.copy_workspace_size(n, total + 16))
    kmws.encode_batch(to_dev(T, src), descs, fl, wire, wire_off, ws_e)
    T.cuda.synchronize()
    assert ws_e.status() == 0 and int(wire_off[n]) == total
    assert bytes(wire.cpu().numpy()[:total]) == bytes(want)
    # unpack + gather back
    out_desc = T.zeros((n, 2), dtype=T.int64, device="cuda")
    out_err = T.full((max(n, 1),), 99, dtype=T.uint8, device="cuda")
    ws_u = kmws.Workspace(kmws.lib().kmws_unpack_workspace_size())
    kmws.unpack_headers(wire, wire_off[:n], kmws.SERVER, out_desc, None, out_err[:n], ws_u, wire_len=total)
    dense = T.zeros(int(lens.sum()) + 16, dtype=T.uint8, device="cuda")
    doff = T.full((n + 1,), -1, dtype=T.int64, device="cuda")
    ws_g = kmws.Workspace(kmws.copy_workspace_size(n, dense.numel()))
    kmws.gather_unmask(wire, out_desc, dense, doff, ws_g)
    T.cuda.synchronize()
    assert ws_u.status() == 0 and ws_g.status() == 0 and int(doff[n]) == int(lens.sum())
    if n:
        assert int(out_err[0]) == 0
        assert bytes(dense.cpu().numpy()[:int(lens[0])]) == bytes(src[16:16 + int(lens[0])])


@pytest.mark.parametrize("room", [0, 20000])
def test_encode_4k_frames_past_4_gib(T, room):
    """cfg4's shape (masked 4 KiB frames, 8-byte headers) at 1.1 M frames: the
    output crosses 2 GiB and 4 GiB (an offset with bit 31 set was once
    sign-extended in a tuning build's fused row kernel), with an exact and a
    roomy output buffer.  Every byte and offset checked on the device against
    a torch restatement of encodeFrameHeader + mask."""
    from kuma_amd import kmws
    n, L, H = (1 << 20) + (1 << 16), 4096, 8
    src = T.empty(n * L + 16, dtype=T.uint8, device="cuda")
    kmws.fill_synthetic(src, 7)
    descs = T.empty((n, 2), dtype=T.int64, device="cuda")
    kmws.fill_uniform_descs(descs, L, L, 11)
    fl = T.full((n,), 0x182, dtype=T.int16, device="cuda")
    cap = n * (L + H) + room * n
    wire = T.full((cap + 16,), 0xEE, dtype=T.uint8, device="cuda")
    woff = T.empty(n + 1, dtype=T.int64, device="cuda")
    ws = kmws.Workspace(kmws.copy_workspace_size(n, cap))
    assert kmws.lib().kmws_encode_batch(src.data_ptr(), descs.data_ptr(), fl.data_ptr(), n, wire.data_ptr(), cap,
                                        woff.data_ptr(), ws.ptr, ws.nbytes, kmws._stream_handle()) == 0
    T.cuda.synchronize()
    assert ws.status() == 0
    assert T.equal(woff, T.arange(n + 1, device="cuda", dtype=T.int64) * (L + H))
    keys = (descs[:, 1] >> 32) & 0xFFFFFFFF
    kb = T.stack([(keys >> (8 * i)) & 0xFF for i in range(4)], 1).to(T.uint8)
    hdr = T.tensor([0x82, 0xFE, L >> 8, L & 0xFF], dtype=T.uint8, device="cuda")
    step = 1 << 16
    for a in range(0, n, step):
        b = min(n, a + step)
        w = wire[a * (L + H):b * (L + H)].view(b - a, L + H)
        assert bool((w[:, :4] == hdr).all()) and T.equal(w[:, 4:8], kb[a:b]), a
        assert T.equal(w[:, 8:], src[a * L:b * L].view(b - a, L) ^ kb[a:b].repeat(1, L // 4)), a
    assert bool((wire[n * (L + H):n * (L + H) + 16] == 0xEE).all())
