"""Debug: test_pinned_chunk_unmasked_in_place's stream, every differing byte."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from kuma_amd import kmws  # noqa: E402
from oracle import oracle as orc  # noqa: E402
from test_gpu_decoder import masked_stream, run_oracle  # noqa: E402

for chunk in (4096, 65536, 0):
    stream = masked_stream(1000 + chunk, 60)
    _, _, want = run_oracle(stream, orc.SERVER, chunk, inplace=True)
    h = kmws.WSHandler(kmws.SERVER)
    h.setFrameCallback(lambda hd, p: None)
    step = chunk or len(stream)
    bufs = []
    for i in range(0, len(stream), step):
        piece = torch.frombuffer(bytearray(stream[i:i + step]), dtype=torch.uint8).pin_memory()
        h.handleDataPtr(piece.data_ptr(), piece.numel())
        bufs.append(bytes(piece.numpy()))
    got = b"".join(bufs)
    diff = [i for i in range(len(want)) if got[i] != want[i]]
    print(chunk, len(diff), [(i, hex(stream[i]), hex(want[i]), hex(got[i])) for i in diff[:40]], flush=True)
