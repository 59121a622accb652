"""Pins the CPU oracle (oracle/kmws_oracle.c) to the reference's recorded
outputs and the RFC 6455 known answers in tests/golden/reference_vectors.json.
No GPU needed."""
import json
import os

import pytest

from oracle import oracle as orc

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_vectors.json")))
MODES = {"CLIENT": orc.CLIENT, "SERVER": orc.SERVER}


def gen(name, n):
    if name == "zeros":
        return bytes(n)
    if name == "iota":
        return bytes(i & 0xFF for i in range(n))
    raise ValueError(name)


def case_input(c):
    data = bytes.fromhex(c["input_hex"])
    if "tail_gen" in c:
        data += gen(c["tail_gen"], c["tail_len"])
    return data


def expected_payload(f):
    if "payload_hex" in f:
        return bytes.fromhex(f["payload_hex"])
    return gen(f["payload_gen"], f["length"])


@pytest.mark.parametrize("c", GOLD["decode"], ids=lambda c: c["name"])
def test_decode_golden(c):
    d = orc.Decoder(MODES[c["mode"]])
    data = case_input(c)
    rets = []
    if c["chunk"] <= 0:
        rets.append(d.feed(data))
    else:
        for i in range(0, len(data), c["chunk"]):
            rets.append(d.feed(data[i:i + c["chunk"]]))
    assert rets == c["expect_rets"]
    assert len(d.frames) == len(c["expect_frames"])
    for got, exp in zip(d.frames, c["expect_frames"]):
        for k in ("fin", "rsv1", "rsv2", "rsv3", "opcode", "mask", "length"):
            assert getattr(got, k) == exp[k], k
        assert got.maskey.hex() == exp["maskey"]
        assert got.payload == expected_payload(exp)
    for step in c.get("then", []):
        assert d.feed(bytes.fromhex(step["input_hex"])) == step["expect_rets"][0]


@pytest.mark.parametrize("c", GOLD["encode"], ids=lambda c: c["name"])
def test_encode_golden(c):
    h = orc.Hdr(fin=c["fin"], rsv1=c["rsv1"], rsv2=c["rsv2"], rsv3=c["rsv3"], opcode=c["opcode"],
                mask=c["mask"], maskey=bytes.fromhex(c["maskey"]), length=c["length"])
    assert orc.encode_header(h).hex() == c["expect_hex"]


@pytest.mark.parametrize("c", GOLD["mask"], ids=lambda c: c["name"])
def test_mask_golden(c):
    key = bytes.fromhex(c["key"])
    segs = [bytes.fromhex(s) for s in c["segments_hex"]]
    assert [s.hex() for s in orc.mask_chain(key, segs)] == c["expect_hex"]


@pytest.mark.parametrize("chunk", [1, 2, 3, 7, 13, 4096])
def test_chunking_invariance(chunk):
    """any chunking yields identical callbacks."""
    import random
    rng = random.Random(1234 + chunk)
    stream = b""
    for i in range(40):
        n = rng.choice([0, 1, 5, 125, 126, 127, 300, 65535, 65536, 70000])
        key = bytes(rng.randrange(256) for _ in range(4))
        payload = bytes(rng.randrange(256) for _ in range(n))
        h = orc.Hdr(fin=rng.randrange(2), opcode=rng.choice([0, 1, 2]), mask=1, maskey=key, length=n)
        stream += orc.encode_header(h) + orc.mask_bytes(key, payload)
    _, whole = orc.decode_chunks(stream, orc.SERVER, 0)
    rets, parts = orc.decode_chunks(stream, orc.SERVER, chunk)
    assert [f.key() for f in parts] == [f.key() for f in whole]
    assert len(whole) == 40
    assert rets[-1] == 0 and all(r in (0, 1) for r in rets)
