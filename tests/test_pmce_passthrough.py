"""permessage-deflate (RFC 7692) coexistence, SURVEY f-4: kuma inflates AFTER
the codec unmasks (WebSocketImpl.cpp:358-364, PMCE_Deflate.cpp:70-92), so the
codec must pass RSV1 and the compressed bytes through untouched.  A deflated
message (raw deflate, trailing 00 00 ff ff removed, RSV1 set, masked) is
decoded by the product decoder; the callback payload + 00 00 ff ff inflates
back to the message.  CPU part: the oracle; GPU part: kmws."""
import random
import zlib

import pytest

from kuma_amd import kmws
from oracle import oracle as orc


def deflate_msg(msg: bytes) -> bytes:
    c = zlib.compressobj(wbits=-15)
    out = c.compress(msg) + c.flush(zlib.Z_SYNC_FLUSH)
    assert out.endswith(b"\x00\x00\xff\xff")
    return out[:-4]


def inflate_msg(data: bytes) -> bytes:
    d = zlib.decompressobj(wbits=-15)
    return d.decompress(data + b"\x00\x00\xff\xff")


def stream(seed):
    rng = random.Random(seed)
    msgs, wire = [], b""
    for _ in range(12):
        msg = bytes(rng.choice(b"abcdefgh ") for _ in range(rng.choice([10, 500, 70000])))
        body = deflate_msg(msg)
        key = bytes(rng.randrange(256) for _ in range(4))
        wire += orc.encode_header(orc.Hdr(fin=1, rsv1=1, opcode=1, mask=1, maskey=key, length=len(body))) + \
            orc.mask_bytes(key, body)
        msgs.append(msg)
    return msgs, wire


def test_oracle_passes_rsv1_and_compressed_bytes():
    msgs, wire = stream(1)
    rets, frames = orc.decode_chunks(wire, orc.SERVER, 4096)
    assert all(f.rsv1 == 1 for f in frames)
    assert [inflate_msg(f.payload) for f in frames] == msgs


@pytest.mark.gpu
def test_gpu_decoder_passes_rsv1_and_compressed_bytes():
    msgs, wire = stream(2)
    h = kmws.WSHandler(kmws.SERVER)
    got = []
    h.setFrameCallback(lambda hd, p: got.append((hd.rsv1, p)))
    for i in range(0, len(wire), 4096):
        assert h.handleData(wire[i:i + 4096]) in (0, 1)
    assert all(r == 1 for r, _ in got)
    assert [inflate_msg(p) for _, p in got] == msgs
