"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper over oracle/kmws_oracle.c.

The CPU restatement of kuma's src/ws codec (see the header of kmws_oracle.c
for the reference lines each function restates and for how it is pinned).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the timed CPU baseline; the product
(kuma_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libkmws_oracle.so")

CLIENT, SERVER = 0, 1
WSERR = {0: "NOERR", 1: "NEED_MORE_DATA", 2: "HANDSHAKE", 3: "INVALID_PARAM",
         4: "INVALID_STATE", 5: "INVALID_FRAME", 6: "INVALID_LENGTH",
         7: "PROTOCOL_ERROR", 8: "CLOSED", 9: "DESTROYED"}


class OrcHdr(C.Structure):
    _fields_ = [("fin", C.c_uint8), ("rsv1", C.c_uint8), ("rsv2", C.c_uint8),
                ("rsv3", C.c_uint8), ("opcode", C.c_uint8), ("mask", C.c_uint8),
                ("plen", C.c_uint8), ("_pad", C.c_uint8), ("xpl64", C.c_uint64),
                ("maskey", C.c_uint8 * 4), ("length", C.c_uint32)]


FRAME_CB = C.CFUNCTYPE(C.c_int, C.POINTER(OrcHdr), C.POINTER(C.c_uint8), C.c_size_t, C.c_void_p)


def build() -> str:
    src = os.path.join(_HERE, "kmws_oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        L = _lib
        L.orc_mask.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t]
        L.orc_encode_header.argtypes = [C.POINTER(OrcHdr), C.c_void_p]
        L.orc_encode_header.restype = C.c_int
        L.orc_decoder_create.argtypes = [C.c_int]
        L.orc_decoder_create.restype = C.c_void_p
        L.orc_decoder_destroy.argtypes = [C.c_void_p]
        L.orc_decoder_reset.argtypes = [C.c_void_p]
        L.orc_decoder_set_mode.argtypes = [C.c_void_p, C.c_int]
        L.orc_decoder_feed.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, FRAME_CB, C.c_void_p]
        L.orc_decoder_feed.restype = C.c_int
        L.orc_decoder_state.argtypes = [C.c_void_p]
        L.orc_decoder_state.restype = C.c_int
        L.orc_unmask_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.orc_unmask_batch_mt.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        L.orc_unmask_batch_mt.restype = C.c_int
        L.orc_encode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p]
        L.orc_encode_batch.restype = C.c_uint64
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def mask(key: bytes, data: bytearray | np.ndarray, phase: int = 0) -> None:
    """In-place XOR, WSHandler.cpp:303-310 (phase: KMBuffer chain, :312-322)."""
    k = (C.c_uint8 * 4).from_buffer_copy(bytes(key))
    if isinstance(data, np.ndarray):
        lib().orc_mask(k, _ptr(data), data.nbytes, phase)
    else:
        buf = (C.c_uint8 * len(data)).from_buffer(data)
        lib().orc_mask(k, buf, len(data), phase)


def mask_bytes(key: bytes, data: bytes, phase: int = 0) -> bytes:
    b = bytearray(data)
    if b:
        mask(key, b, phase)
    return bytes(b)


def mask_chain(key: bytes, segments: Sequence[bytes]) -> List[bytes]:
    """KMBuffer-chain mask: phase continues across segments (WSHandler.cpp:312-322)."""
    out, phase = [], 0
    for s in segments:
        out.append(mask_bytes(key, s, phase))
        phase += len(s)
    return out


@dataclass
class Hdr:
    fin: int = 1
    rsv1: int = 0
    rsv2: int = 0
    rsv3: int = 0
    opcode: int = 2
    mask: int = 0
    maskey: bytes = b"\0\0\0\0"
    length: int = 0


def encode_header(h: Hdr) -> bytes:
    """WSHandler::encodeFrameHeader, WSHandler.cpp:46-106."""
    c = OrcHdr()
    c.fin, c.rsv1, c.rsv2, c.rsv3 = h.fin, h.rsv1, h.rsv2, h.rsv3
    c.opcode, c.mask, c.length = h.opcode, h.mask, h.length & 0xFFFFFFFF
    for i in range(4):
        c.maskey[i] = h.maskey[i]
    out = (C.c_uint8 * 14)()
    n = lib().orc_encode_header(C.byref(c), out)
    return bytes(out[:n])


@dataclass
class Frame:
    fin: int
    rsv1: int
    rsv2: int
    rsv3: int
    opcode: int
    mask: int
    plen: int
    xpl64: int
    maskey: bytes
    length: int
    payload: bytes

    def key(self) -> Tuple:
        return (self.fin, self.rsv1, self.rsv2, self.rsv3, self.opcode, self.mask,
                self.plen, self.xpl64, self.maskey, self.length, self.payload)


class Decoder:
    """WSHandler streaming decoder (WSHandler.cpp:108-280) over the C oracle."""

    def __init__(self, mode: int = SERVER):
        self._d = lib().orc_decoder_create(mode)
        self.frames: List[Frame] = []
        self.destroy_on: Optional[int] = None  # emulate callback destroying handler at frame k

        def _cb(hp, payload, n, user):
            h = hp.contents
            data = C.string_at(payload, n) if n else b""
            self.frames.append(Frame(h.fin, h.rsv1, h.rsv2, h.rsv3, h.opcode, h.mask, h.plen,
                                     h.xpl64, bytes(h.maskey), h.length, data))
            if self.destroy_on is not None and len(self.frames) - 1 == self.destroy_on:
                return 1
            return 0

        self._cb = FRAME_CB(_cb)

    def __del__(self):
        try:
            if self._d:
                lib().orc_decoder_destroy(self._d)
                self._d = None
        except Exception:
            pass

    def feed(self, data) -> int:
        """A bytearray is decoded in place (masked payloads unmasked in it, as
        WSHandler.cpp:247-250/:260 does with the caller's buffer)."""
        if isinstance(data, bytearray) and len(data):
            buf = (C.c_uint8 * len(data)).from_buffer(data)
        else:
            buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        return lib().orc_decoder_feed(self._d, buf, len(data), self._cb, None)

    def reset(self) -> None:
        lib().orc_decoder_reset(self._d)

    def set_mode(self, mode: int) -> None:
        lib().orc_decoder_set_mode(self._d, mode)

    @property
    def state(self) -> int:
        return lib().orc_decoder_state(self._d)


def decode_chunks(stream: bytes, mode: int, chunk: int) -> Tuple[List[int], List[Frame]]:
    """Feed `stream` in chunks of `chunk` bytes (0 = whole) and collect results."""
    d = Decoder(mode)
    rets = []
    if chunk <= 0:
        rets.append(d.feed(stream))
    else:
        for i in range(0, len(stream), chunk):
            rets.append(d.feed(stream[i:i + chunk]))
    return rets, d.frames


def synthetic(seed: int, start: int, nbytes: int) -> np.ndarray:
    """Host copy of kmws_fill_synthetic: byte i = byte (i & 7) of
    splitmix64(seed + (i >> 3)), for i in [start, start + nbytes)."""
    if nbytes <= 0:
        return np.zeros(0, dtype=np.uint8)
    w0, w1 = start >> 3, (start + nbytes + 7) >> 3
    with np.errstate(over="ignore"):
        z = np.arange(w0, w1, dtype=np.uint64) + np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    b = z.astype("<u8").view(np.uint8)
    s = start - (w0 << 3)
    return b[s:s + nbytes].copy()


def splitmix64(x: int) -> int:
    M = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    return z ^ (z >> 31)


DESC_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("key", "<u4")])


def unmask_batch(base: np.ndarray, descs: np.ndarray, threads: int = 1) -> None:
    """In-place unmask of every descriptor's span of `base` (uint8 array)."""
    assert base.dtype == np.uint8 and descs.dtype == DESC_DTYPE
    if threads <= 1:
        lib().orc_unmask_batch(_ptr(base), _ptr(descs), len(descs))
    else:
        lib().orc_unmask_batch_mt(_ptr(base), _ptr(descs), len(descs), threads)


def encode_batch(src: np.ndarray, src_off: np.ndarray, lens: np.ndarray, flags: np.ndarray,
                 keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Wire image of a frame batch (header pack + masked payload per frame)."""
    n = len(lens)
    src_off = np.ascontiguousarray(src_off, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    flags = np.ascontiguousarray(flags, dtype=np.uint32)
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    wire_off = np.zeros(n, dtype=np.uint64)
    total = lib().orc_encode_batch(_ptr(src), _ptr(src_off), _ptr(lens), _ptr(flags), _ptr(keys),
                                   n, None, _ptr(wire_off))
    dst = np.zeros(max(1, int(total)), dtype=np.uint8)
    lib().orc_encode_batch(_ptr(src), _ptr(src_off), _ptr(lens), _ptr(flags), _ptr(keys),
                           n, _ptr(dst), _ptr(wire_off))
    return dst[:int(total)], wire_off
