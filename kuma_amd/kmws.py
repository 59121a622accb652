"""ctypes binding of the kmws C ABI (include/kmws_gpu.h).

Mirrors the reference codec interface (kuma::ws::WSHandler, src/ws/WSHandler.h:
32-91) for Python callers and tests, and exposes the device batch entries over
torch tensors (torch is plumbing here: device memory and streams).  There is no
CPU fallback anywhere in this module: if libkmws_gpu.so is missing the import
fails, and device entries on a machine without a gfx950 GPU return
KMWS_ERR_NOT_SUPPORTED.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

from . import build as _build

# ---- constants (include/kmws_gpu.h) ----
OK, ERR_FAILED, ERR_TIMEOUT, ERR_INVALID_STATE, ERR_INVALID_PARAM = 0, -1, -6, -7, -8
ERR_BUFFER_TOO_SMALL, ERR_BUFFER_TOO_LONG, ERR_NOT_SUPPORTED = -17, -18, -19
CLIENT, SERVER = 0, 1
OP_CONTINUE, OP_TEXT, OP_BINARY, OP_CLOSE, OP_PING, OP_PONG = 0, 1, 2, 8, 9, 10
WS_NOERR, WS_NEED_MORE_DATA, WS_INVALID_FRAME, WS_INVALID_LENGTH = 0, 1, 5, 6
WS_PROTOCOL_ERROR, WS_CLOSED, WS_DESTROYED = 7, 8, 9
MAX_HEADER_SIZE = 14
FLAG_MASK = 0x100
DEVICE_AUTO = -1  # KMWS_DEVICE_AUTO: the calling thread's device
DEVICE_POLICY_NUMA, DEVICE_POLICY_ROUND_ROBIN, DEVICE_POLICY_FIRST = 0, 1, 2

#: every function include/kmws_gpu.h declares (tests check they are exported)
EXPORTS = [
    "kmws_encode_header", "kmws_header_size", "kmws_decoder_create", "kmws_decoder_destroy",
    "kmws_decoder_set_mode", "kmws_decoder_reset", "kmws_decoder_feed", "kmws_device_count",
    "kmws_decoder_set_in_place",
    "kmws_unmask_workspace_size", "kmws_unmask_batch", "kmws_unmask_plan", "kmws_unmask_apply",
    "kmws_unmask_autotune", "kmws_unmask_apply_sched", "kmws_unmask_default_schedule", "kmws_read_status",
    "kmws_copy_workspace_size", "kmws_encode_batch",
    "kmws_unpack_workspace_size", "kmws_unpack_headers", "kmws_gather_unmask", "kmws_find_headers",
    "kmws_pack_headers_workspace_size", "kmws_pack_headers", "kmws_find_headers_streams",
    "kmws_unpack_unmask", "kmws_unpack_gather",
    "kmws_pipeline_create", "kmws_pipeline_destroy", "kmws_pipeline_unmask", "kmws_pipeline_set_transfer",
    "kmws_rx_batch_create", "kmws_rx_batch_destroy", "kmws_decoder_feed_deferred", "kmws_rx_batch_flush",
    "kmws_rx_batch_pending", "kmws_rx_batch_pending_bytes", "kmws_rx_batch_discard", "kmws_mask_host_chain", "kmws_rx_batch_submit",
    "kmws_rx_batch_poll", "kmws_rx_batch_inflight", "kmws_tx_batch_submit", "kmws_tx_batch_poll",
    "kmws_rx_batch_attach_ring",
    "kmws_tx_batch_create", "kmws_tx_batch_destroy", "kmws_tx_batch_add", "kmws_tx_batch_flush",
    "kmws_tx_batch_pending", "kmws_tx_batch_attach_ring", "kmws_host_alloc", "kmws_host_free",
    "kmws_set_device_policy", "kmws_set_thread_device", "kmws_thread_device", "kmws_thread_attach",
]
#: every function include/kmws_bench.h declares (bench / test support, same library)
BENCH_EXPORTS = [
    "kmws_arena_alloc", "kmws_arena_free", "kmws_arena_place", "kmws_fill_synthetic", "kmws_fill_uniform_descs",
    "kmws_check_unmasked", "kmws_resident_enable", "kmws_resident_info", "kmws_resident_counters",
    "kmws_resident_exit_reasons", "kmws_resident_guard_counters", "kmws_device_policy_pick",
    "kmws_device_numa_node", "kmws_resident_store_counters", "kmws_device_batch_busy",
]

# unmask schedules (include/kmws_gpu.h KMWS_SCHED_*)
SCHED_GROUPED_RUNS, SCHED_IN_ORDER, SCHED_SPLIT2, SCHED_SPLIT8, SCHED_XCD_RUNS, SCHED_SPLIT4 = 0, 1, 2, 3, 4, 5
SCHED_KINDS = (0, 1, 2, 3, 4, 5)

SCHED_NT_STORES, SCHED_TEMPORAL_STORES = 1 << 29, 1 << 30


class FrameHdr(C.Structure):
    """kmws_frame_hdr == FrameHeader (src/ws/wsdefs.h:74-88), bitfields widened."""
    _fields_ = [("fin", C.c_uint8), ("rsv1", C.c_uint8), ("rsv2", C.c_uint8), ("rsv3", C.c_uint8),
                ("opcode", C.c_uint8), ("mask", C.c_uint8), ("plen", C.c_uint8),
                ("reserved", C.c_uint8), ("xpl64", C.c_uint64), ("maskey", C.c_uint8 * 4),
                ("length", C.c_uint32)]


FRAME_CB = C.CFUNCTYPE(C.c_int, C.POINTER(FrameHdr), C.POINTER(C.c_uint8), C.c_size_t, C.c_void_p)

_lib: Optional[C.CDLL] = None


def lib_path() -> str:
    """The product library, always: tuning and test variants of the same ABI
    (kuma_amd/build.py) are loaded by path by the tools and tests that need
    them, never through this binding."""
    return _build.LIB


def lib() -> C.CDLL:
    """Load libkmws_gpu.so (building it first when hipcc is available)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: torch ships its own libamdhip64 with the same
    # SONAME (libamdhip64.so.7) as /opt/rocm's.  Whichever loads first is used
    # by both, and torch only works on its own copy, so load torch first; our
    # library then binds to that runtime and shares its streams and memory.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    path = lib_path()
    if path == _build.LIB and not _build.up_to_date():
        try:
            _build.build()
        except (OSError, Exception) as e:  # no hipcc on this machine: use the shipped .so
            if not os.path.exists(path):
                raise RuntimeError(f"kmws: {path} missing and cannot be built: {e}") from e
    if not os.path.exists(path):
        raise RuntimeError(f"kmws: HIP library {path} not built (run __graft_entry__.build())")
    _lib = bind(C.CDLL(path))
    return _lib


def bind(L: C.CDLL) -> C.CDLL:
    """Sets the C signatures on a loaded libkmws_gpu.so (the product library, or
    a test variant a test loads by path)."""
    vp, u8p, sz, u32, u64, i32 = C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint64, C.c_int
    sig = {
        "kmws_encode_header": (i32, [C.POINTER(FrameHdr), u8p]),
        "kmws_header_size": (i32, [u32, i32]),
        "kmws_decoder_create": (vp, [i32, i32]),
        "kmws_decoder_destroy": (None, [vp]),
        "kmws_decoder_set_mode": (None, [vp, i32]),
        "kmws_decoder_reset": (None, [vp]),
        "kmws_decoder_set_in_place": (None, [vp, i32]),
        "kmws_decoder_feed": (i32, [vp, u8p, sz, FRAME_CB, vp]),
        "kmws_device_count": (i32, []),
        "kmws_unmask_workspace_size": (sz, [u64]),
        "kmws_unmask_batch": (i32, [u8p, u64, vp, u32, vp, sz, vp]),
        "kmws_unmask_plan": (i32, [u64, vp, u32, vp, sz, vp]),
        "kmws_unmask_apply": (i32, [u8p, u64, vp, u32, vp, sz, vp]),
        "kmws_unmask_autotune": (i32, [u8p, u64, vp, u32, vp, sz, vp]),
        "kmws_unmask_apply_sched": (i32, [u8p, u64, vp, u32, vp, sz, i32, vp]),
        "kmws_unmask_default_schedule": (i32, [u64, u32]),
        "kmws_read_status": (i32, [vp, C.POINTER(C.c_uint32), vp]),
        "kmws_fill_synthetic": (i32, [u8p, u64, u64, vp]),
        "kmws_arena_alloc": (vp, [u64, i32, C.POINTER(C.c_int)]),
        "kmws_arena_free": (None, [vp, i32]),
        "kmws_arena_place": (C.c_int64, [u8p, u64, u64, u64, vp, C.POINTER(C.c_float), u32]),
        "kmws_fill_uniform_descs": (i32, [vp, u32, u64, u32, u64, vp]),
        "kmws_check_unmasked": (i32, [u8p, u64, u64, vp, u32, vp, vp]),
        "kmws_resident_enable": (i32, [i32, i32]),
        "kmws_resident_info": (i32, [i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_int)]),
        "kmws_resident_exit_reasons": (i32, [i32, C.POINTER(C.c_uint64), i32]),
        "kmws_resident_store_counters": (i32, [i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "kmws_device_batch_busy": (i32, [i32]),
        "kmws_resident_counters": (i32, [i32, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint64)]),
        "kmws_copy_workspace_size": (sz, [u32, u64]),
        "kmws_encode_batch": (i32, [u8p, vp, vp, u32, u8p, u64, vp, vp, sz, vp]),
        "kmws_unpack_workspace_size": (sz, []),
        "kmws_pack_headers_workspace_size": (sz, [u32]),
        "kmws_pack_headers": (i32, [vp, vp, u32, u8p, vp, vp, vp, sz, vp]),
        "kmws_find_headers_streams": (i32, [u8p, u64, vp, u32, vp, u32, vp, vp, vp]),
        "kmws_unpack_headers": (i32, [u8p, u64, vp, u32, i32, vp, vp, vp, vp, sz, vp]),
        "kmws_gather_unmask": (i32, [u8p, vp, u32, u8p, u64, vp, vp, sz, vp]),
        "kmws_unpack_unmask": (i32, [u8p, u64, vp, u32, i32, vp, vp, vp, vp, sz, i32, vp]),
        "kmws_unpack_gather": (i32, [u8p, u64, vp, u32, i32, vp, vp, vp, u8p, u64, vp, vp, sz, vp]),
        "kmws_pipeline_create": (vp, [i32, u64, u32, i32]),
        "kmws_pipeline_destroy": (None, [vp]),
        "kmws_mask_host_chain": (i32, [vp, vp, vp, sz, i32]),
        "kmws_rx_batch_create": (vp, [i32]),
        "kmws_tx_batch_create": (vp, [i32]),
        "kmws_tx_batch_destroy": (None, [vp]),
        "kmws_tx_batch_add": (i32, [vp, C.POINTER(FrameHdr), vp, vp, sz, vp]),
        "kmws_tx_batch_flush": (C.c_int64, [vp]),
        "kmws_tx_batch_submit": (C.c_int64, [vp]),
        "kmws_tx_batch_poll": (i32, [vp, C.c_int64, i32]),
        "kmws_rx_batch_submit": (i32, [vp]),
        "kmws_rx_batch_poll": (i32, [vp, i32]),
        "kmws_rx_batch_inflight": (i32, [vp]),
        "kmws_tx_batch_pending": (i32, [vp]),
        "kmws_tx_batch_attach_ring": (i32, [vp, vp, sz]),
        "kmws_host_alloc": (vp, [sz, i32]),
        "kmws_host_free": (None, [vp]),
        "kmws_rx_batch_destroy": (None, [vp]),
        "kmws_decoder_feed_deferred": (i32, [vp, vp, u8p, sz, FRAME_CB, vp]),
        "kmws_rx_batch_flush": (i32, [vp]),
        "kmws_rx_batch_attach_ring": (i32, [vp, vp, sz]),
        "kmws_rx_batch_pending": (i32, [vp]),
        "kmws_rx_batch_pending_bytes": (C.c_uint64, [vp]),
        "kmws_rx_batch_discard": (None, [vp, vp]),
        "kmws_pipeline_set_transfer": (i32, [vp, i32]),
        "kmws_pipeline_unmask": (i32, [vp, u8p, u64, vp, u32]),
        "kmws_find_headers": (i32, [u8p, u64, vp, u32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
        "kmws_set_device_policy": (i32, [i32]),
        "kmws_set_thread_device": (i32, [i32]),
        "kmws_thread_device": (i32, []),
        "kmws_thread_attach": (i32, [i32]),
        "kmws_resident_guard_counters": (i32, [i32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                               C.POINTER(C.c_uint64)]),
        "kmws_device_policy_pick": (i32, [i32, i32, C.POINTER(C.c_int), i32, u32]),
        "kmws_device_numa_node": (i32, [i32, C.POINTER(C.c_int)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


class KmwsError(RuntimeError):
    """A negative kmws_status from the C ABI (.status)."""

    def __init__(self, status: int, what: str):
        super().__init__(f"{what} failed with kmws_status {status}")
        self.status = status
        self.ws_status = 0  # the workspace status word, when that is what failed


def _check_tensor(t, name: str, elem: int, device, min_numel: int = 0) -> None:
    """Raw data_ptr() goes to the kernels: element size, layout, device and
    size must match what the C ABI reads and writes, or a kernel would access
    memory past the tensor."""
    if t.element_size() != elem:
        raise TypeError(f"{name}: expected {elem}-byte elements, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.numel() < min_numel:
        raise ValueError(f"{name} has {t.numel()} elements, the call needs {min_numel}")


def _check_descs(descs) -> int:
    """kmws_desc array as an (n, 2) 8-byte tensor (make_descs); returns n."""
    if descs.dim() != 2 or descs.shape[1] != 2:
        raise ValueError(f"descs must have shape (n, 2) (kmws_desc), got {tuple(descs.shape)}")
    _check_tensor(descs, "descs", 8, descs.device)
    return descs.shape[0]


def _check(st: int, what: str) -> None:
    if st != OK:
        raise KmwsError(st, what)


# ====================== host codec (WSHandler mirror) ======================

@dataclass
class Header:
    fin: int = 1
    rsv1: int = 0
    rsv2: int = 0
    rsv3: int = 0
    opcode: int = OP_BINARY
    mask: int = 0
    maskey: bytes = b"\0\0\0\0"
    length: int = 0
    plen: int = 0
    xpl64: int = 0

    def to_c(self) -> FrameHdr:
        h = FrameHdr()
        h.fin, h.rsv1, h.rsv2, h.rsv3 = self.fin, self.rsv1, self.rsv2, self.rsv3
        h.opcode, h.mask, h.plen, h.xpl64 = self.opcode, self.mask, self.plen, self.xpl64
        h.length = self.length & 0xFFFFFFFF
        for i in range(4):
            h.maskey[i] = self.maskey[i]
        return h

    @staticmethod
    def from_c(h: FrameHdr) -> "Header":
        return Header(h.fin, h.rsv1, h.rsv2, h.rsv3, h.opcode, h.mask, bytes(h.maskey), h.length,
                      h.plen, h.xpl64)


def encode_frame_header(hdr: Header) -> bytes:
    """WSHandler::encodeFrameHeader (WSHandler.cpp:46-106)."""
    out = (C.c_uint8 * MAX_HEADER_SIZE)()
    n = lib().kmws_encode_header(C.byref(hdr.to_c()), out)
    if n < 0:
        raise RuntimeError(f"kmws_encode_header: {n}")
    return bytes(out[:n])


def header_size(length: int, mask: bool) -> int:
    return lib().kmws_header_size(length & 0xFFFFFFFF, int(bool(mask)))


class WSHandler:
    """kuma::ws::WSHandler over the C ABI (WSHandler.h:32-91).

    handleData(data) returns the WSError int and invokes the frame callback
    `cb(Header, payload: bytes)` for each frame, in order.  Masked payloads are
    unmasked on the GPU.  If `data` is a bytearray it is unmasked in place like
    the reference does with the caller's buffer.
    """

    def __init__(self, mode: int = CLIENT, device: int = 0):
        self._d = lib().kmws_decoder_create(mode, device)
        if not self._d:
            raise MemoryError("kmws_decoder_create")
        self._cb: Optional[Callable] = None
        self.destroyed_by_callback = False

        def tramp(hp, payload, n, user):
            if self._cb is None:
                return 0
            data = C.string_at(payload, n) if n else b""
            r = self._cb(Header.from_c(hp.contents), data)
            return 1 if r is True else 0

        self._tramp = FRAME_CB(tramp)

    def __del__(self):
        try:
            if getattr(self, "_d", None):
                lib().kmws_decoder_destroy(self._d)
                self._d = None
        except Exception:
            pass

    def setMode(self, mode: int) -> None:
        lib().kmws_decoder_set_mode(self._d, mode)

    def setFrameCallback(self, cb: Callable) -> None:
        """cb(Header, bytes) -> optional True to emulate 'callback destroyed the handler'."""
        self._cb = cb

    def reset(self) -> None:
        lib().kmws_decoder_reset(self._d)

    def setInPlace(self, on: bool) -> None:
        """kmws_decoder_set_in_place (default True)."""
        lib().kmws_decoder_set_in_place(self._d, int(bool(on)))

    def handleData(self, data) -> int:
        n = len(data)
        if isinstance(data, bytearray):
            buf = (C.c_uint8 * max(1, n)).from_buffer(data) if n else (C.c_uint8 * 1)()
        else:
            buf = (C.c_uint8 * max(1, n)).from_buffer_copy(bytes(data) if n else b"\0")
        return lib().kmws_decoder_feed(self._d, buf, n, self._tramp, None)

    def handleDataPtr(self, ptr: int, n: int) -> int:
        """Feed raw memory (e.g. a pinned torch CPU tensor's data_ptr()) in place."""
        return lib().kmws_decoder_feed(self._d, ptr, n, self._tramp, None)

    def handleDataDeferredPtr(self, batch: "RxBatch", ptr: int, n: int) -> int:
        """Deferred feed of raw memory (e.g. a slice of a ring attached to `batch`)."""
        return lib().kmws_decoder_feed_deferred(self._d, batch._b, ptr, n, self._tramp, None)

    def handleDataDeferred(self, batch: "RxBatch", data) -> int:
        """kmws_decoder_feed_deferred: parse now, deliver at batch.flush()."""
        n = len(data)
        buf = (C.c_uint8 * max(1, n)).from_buffer_copy(bytes(data) if n else b"\0")
        return lib().kmws_decoder_feed_deferred(self._d, batch._b, buf, n, self._tramp, None)

    encodeFrameHeader = staticmethod(encode_frame_header)


def resident_info(device: int = 0, L: Optional[C.CDLL] = None) -> dict:
    """kmws_resident_info of the device's resident worker (one grid per device,
    a mailbox slot per loop thread), plus kmws_resident_counters: the calling
    thread's slot (-1: none), slots held, timed-out and withdrawn jobs.  `L`: a
    test variant of the library (bind()), else the product library."""
    L = L or lib()
    jobs, launches, running = C.c_uint64(0), C.c_uint64(0), C.c_int(0)
    _check(L.kmws_resident_info(device, C.byref(jobs), C.byref(launches), C.byref(running)), "kmws_resident_info")
    slot, claimed, tmo, wd = C.c_int(0), C.c_int(0), C.c_uint64(0), C.c_uint64(0)
    _check(L.kmws_resident_counters(device, C.byref(slot), C.byref(claimed), C.byref(tmo), C.byref(wd)),
           "kmws_resident_counters")
    return {"jobs": jobs.value, "launches": launches.value, "running": bool(running.value),
            "thread_slot": slot.value, "slots_claimed": claimed.value, "timeouts": tmo.value,
            "withdrawn": wd.value}


def resident_guard(device: int = 0, L: Optional[C.CDLL] = None) -> dict:
    """kmws_resident_guard_counters: posts refused on a slot the caller did not
    hold (never expected), jobs asked for after a thread's exit hook gave its
    slots back (launched), releases that first waited for the slot's last job."""
    L = L or lib()
    a, b, c = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    _check(L.kmws_resident_guard_counters(device, C.byref(a), C.byref(b), C.byref(c)), "kmws_resident_guard_counters")
    return {"unowned_posts": a.value, "late_posts": b.value, "drained_releases": c.value}


def resident_stores(device: int = 0, L: Optional[C.CDLL] = None) -> dict:
    """kmws_resident_store_counters: resident jobs posted that wrote through
    (small ones, and all while a device batch runs) and that released the L2."""
    L = L or lib()
    a, b = C.c_uint64(0), C.c_uint64(0)
    _check(L.kmws_resident_store_counters(device, C.byref(a), C.byref(b)), "kmws_resident_store_counters")
    return {"write_through": a.value, "released": b.value}


def device_batch_busy(device: int = 0) -> bool:
    """kmws_device_batch_busy: device batches of this library estimated running."""
    return lib().kmws_device_batch_busy(device) == 1


def device_policy_pick(policy: int, thread_node: int, gpu_nodes: Sequence[int], seq: int) -> int:
    """kmws_device_policy_pick: the device `policy` gives a thread on NUMA node
    `thread_node` (-1 unknown) for GPUs on `gpu_nodes`, after `seq` threads."""
    arr = (C.c_int * max(1, len(gpu_nodes)))(*gpu_nodes)
    return lib().kmws_device_policy_pick(policy, thread_node, arr, len(gpu_nodes), seq & 0xFFFFFFFF)


def set_device_policy(policy: int) -> None:
    _check(lib().kmws_set_device_policy(policy), "kmws_set_device_policy")


def set_thread_device(device: int) -> None:
    _check(lib().kmws_set_thread_device(device), "kmws_set_thread_device")


def thread_device() -> int:
    """kmws_thread_device: the calling thread's GPU (raises without one)."""
    d = lib().kmws_thread_device()
    if d < 0:
        raise KmwsError(d, "kmws_thread_device")
    return d


RESIDENT_EXIT_REASONS = ("lease", "closing", "resize", "idle", "quit")


def resident_exit_reasons(device: int = 0, L: Optional[C.CDLL] = None) -> dict:
    """kmws_resident_exit_reasons: the worker's workgroup exits so far by reason
    (lease, closing = another workgroup found the grid idle, resize, idle =
    this one completed the idle count, quit)."""
    L = L or lib()
    out = (C.c_uint64 * len(RESIDENT_EXIT_REASONS))()
    _check(L.kmws_resident_exit_reasons(device, out, len(RESIDENT_EXIT_REASONS)), "kmws_resident_exit_reasons")
    return dict(zip(RESIDENT_EXIT_REASONS, list(out)))


def resident_enable(on: bool, device: int = 0) -> None:
    """kmws_resident_enable for the calling thread (False: a launch per sync call)."""
    _check(lib().kmws_resident_enable(device, int(bool(on))), "kmws_resident_enable")


def handle_data_mask(key: bytes, segments, device: int = 0, L: Optional[C.CDLL] = None) -> None:
    """WSHandler::handleDataMask over a chain of bytearrays (in place, GPU).
    `L`: a test variant of the library (bind()), else the product library."""
    segs = list(segments)
    bufs = [(C.c_uint8 * max(1, len(s))).from_buffer(s) if len(s) else (C.c_uint8 * 1)() for s in segs]
    ptrs = (C.c_void_p * max(1, len(segs)))(*[C.addressof(b) for b in bufs])
    lens = (C.c_size_t * max(1, len(segs)))(*[len(s) for s in segs])
    k = (C.c_uint8 * 4).from_buffer_copy(bytes(key))
    _check((L or lib()).kmws_mask_host_chain(k, ptrs, lens, len(segs), device), "kmws_mask_host_chain")


class RxBatch:
    """kmws_rx_batch: one GPU unmask per flush for frames of many feeds/connections."""

    def __init__(self, device: int = 0):
        self._b = lib().kmws_rx_batch_create(device)
        if not self._b:
            raise RuntimeError("kmws_rx_batch_create failed (no gfx950 device)")

    def flush(self) -> int:
        r = lib().kmws_rx_batch_flush(self._b)
        if r < 0:
            raise RuntimeError(f"kmws_rx_batch_flush: {r}")
        return r

    def pending(self) -> int:
        return lib().kmws_rx_batch_pending(self._b)

    def pending_bytes(self) -> int:
        """Masked payload bytes of the pending frames (kmws_rx_batch_pending_bytes)."""
        return lib().kmws_rx_batch_pending_bytes(self._b)

    def submit(self) -> int:
        """kmws_rx_batch_submit: enqueue this generation's unmask, return at once."""
        r = lib().kmws_rx_batch_submit(self._b)
        if r < 0:
            raise KmwsError(r, "kmws_rx_batch_submit")
        return r

    def poll(self, wait: bool = False) -> int:
        """kmws_rx_batch_poll: deliver every finished generation (all with wait)."""
        r = lib().kmws_rx_batch_poll(self._b, int(bool(wait)))
        if r < 0:
            raise KmwsError(r, "kmws_rx_batch_poll")
        return r

    def inflight(self) -> int:
        return lib().kmws_rx_batch_inflight(self._b)

    def attach_ring(self, ring) -> None:
        """ring: pinned torch uint8 CPU tensor (kept alive by this object)."""
        self._ring = ring
        _check(lib().kmws_rx_batch_attach_ring(self._b, ring.data_ptr() if ring is not None else None,
                                               ring.numel() if ring is not None else 0),
               "kmws_rx_batch_attach_ring")

    def discard(self, handler: WSHandler) -> None:
        lib().kmws_rx_batch_discard(self._b, handler._d)

    def __del__(self):
        try:
            if getattr(self, "_b", None):
                lib().kmws_rx_batch_destroy(self._b)
                self._b = None
        except Exception:
            pass


class TxBatch:
    """kmws_tx_batch: the send path of many frames masked by one GPU launch per
    flush (WebSocket::Impl::sendWsFrame, WebSocketImpl.cpp:381-436, batched).

    add(hdr, segments) packs the header now (returned as bytes) and queues the
    segments -- bytearrays, masked in place at flush -- when hdr.mask is set."""

    def __init__(self, device: int = 0):
        self._b = lib().kmws_tx_batch_create(device)
        if not self._b:
            raise RuntimeError("kmws_tx_batch_create failed (no gfx950 device)")
        self._keep = []

    def add(self, hdr: "Header", segments) -> bytes:
        bufs = [(C.c_uint8 * len(x)).from_buffer(x) if len(x) else None for x in segments]
        ptrs = (C.c_void_p * max(1, len(bufs)))(*[C.cast(b, C.c_void_p) if b is not None else None for b in bufs])
        lens = (C.c_size_t * max(1, len(bufs)))(*[len(x) for x in segments])
        out = (C.c_uint8 * MAX_HEADER_SIZE)()
        h = hdr.to_c()
        r = lib().kmws_tx_batch_add(self._b, C.byref(h), ptrs, lens, len(bufs), out)
        self._keep.append((segments, bufs))
        if r < 0:
            raise KmwsError(r, "kmws_tx_batch_add")
        return bytes(out[:r])

    def flush(self) -> int:
        r = lib().kmws_tx_batch_flush(self._b)
        self._keep.clear()
        if r < 0:
            raise KmwsError(r, "kmws_tx_batch_flush")
        return r

    def pending(self) -> int:
        return lib().kmws_tx_batch_pending(self._b)

    def submit(self) -> int:
        """kmws_tx_batch_submit: enqueue the masks, return the generation's ticket."""
        self._inflight = getattr(self, "_inflight", [])
        t = lib().kmws_tx_batch_submit(self._b)
        if t < 0:
            raise KmwsError(t, "kmws_tx_batch_submit")
        if t:
            self._inflight.append((t, list(self._keep)))
        self._keep.clear()
        return t

    def poll(self, ticket: int, wait: bool = False) -> bool:
        """kmws_tx_batch_poll: True once every generation up to `ticket` is masked."""
        r = lib().kmws_tx_batch_poll(self._b, ticket, int(bool(wait)))
        if r < 0:
            raise KmwsError(r, "kmws_tx_batch_poll")
        if r:
            self._inflight = [x for x in getattr(self, "_inflight", []) if x[0] > ticket]
        return bool(r)

    def attach_ring(self, ring) -> None:
        """ring: pinned torch uint8 CPU tensor (kept alive by this object)."""
        self._ring = ring
        _check(lib().kmws_tx_batch_attach_ring(self._b, ring.data_ptr() if ring is not None else None,
                                               ring.numel() if ring is not None else 0),
               "kmws_tx_batch_attach_ring")

    def add_ptrs(self, hdr: "Header", ptrs, lens) -> bytes:
        """add() for raw segment addresses (e.g. slices of an attached pinned ring)."""
        n = len(ptrs)
        pa = (C.c_void_p * max(1, n))(*ptrs)
        la = (C.c_size_t * max(1, n))(*lens)
        out = (C.c_uint8 * MAX_HEADER_SIZE)()
        h = hdr.to_c()
        r = lib().kmws_tx_batch_add(self._b, C.byref(h), pa, la, n, out)
        if r < 0:
            raise KmwsError(r, "kmws_tx_batch_add")
        return bytes(out[:r])

    def __del__(self):
        try:
            if getattr(self, "_b", None):
                lib().kmws_tx_batch_destroy(self._b)
                self._b = None
        except Exception:
            pass


# ====================== device batch entries (torch tensors) ======================

def device_count() -> int:
    return lib().kmws_device_count()


def _stream_handle(stream=None) -> int:
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def make_descs(off, length, key, device="cuda"):
    """(n, 2) int64 tensor laid out as kmws_desc {u64 off; u32 len; u32 key}."""
    import torch
    off = torch.as_tensor(off, dtype=torch.int64)
    lk = (torch.as_tensor(length, dtype=torch.int64) & 0xFFFFFFFF) | \
        (torch.as_tensor(key, dtype=torch.int64) << 32)
    return torch.stack([off, lk], dim=1).contiguous().to(device)


class Workspace:
    """Caller-owned device workspace (no allocation inside the batch calls).

    It is also the host plan of the batch it serves: `schedule` (None = the
    library default) is the unmask schedule code its applies pass to
    kmws_unmask_apply_sched -- set by unmask_autotune or unmask_set_schedule.
    The library keeps no schedule state, so a new Workspace (wherever torch
    places it) starts on the default."""

    def __init__(self, nbytes: int, device="cuda"):
        import torch
        self.tensor = torch.empty(max(16, int(nbytes)), dtype=torch.uint8, device=device)
        self.schedule: Optional[int] = None

    @property
    def ptr(self) -> int:
        return self.tensor.data_ptr()

    @property
    def nbytes(self) -> int:
        return self.tensor.numel()

    def status(self, stream=None) -> int:
        out = C.c_uint32(0)
        _check(lib().kmws_read_status(self.ptr, C.byref(out), _stream_handle(stream)), "kmws_read_status")
        return out.value


class Arena:
    """kmws_arena_alloc: a device payload arena, physically contiguous when the
    device can provide it.  `.tensor` is a uint8 torch view of it (through
    __cuda_array_interface__); keep the Arena alive while the view is used."""

    def __init__(self, nbytes: int, device: int = 0):
        import torch
        flag = C.c_int(0)
        p = lib().kmws_arena_alloc(int(nbytes), device, C.byref(flag))
        if not p:
            raise RuntimeError(f"kmws_arena_alloc({nbytes}) failed")
        self._p, self._dev, self.nbytes, self.contiguous = p, device, int(nbytes), bool(flag.value)
        self.__cuda_array_interface__ = {"shape": (self.nbytes,), "typestr": "|u1", "data": (p, False),
                                         "version": 2, "strides": None}
        self.tensor = torch.as_tensor(self, device=torch.device("cuda", device))
        assert self.tensor.data_ptr() == p

    def __del__(self):
        try:
            if getattr(self, "_p", None):
                self.tensor = None
                lib().kmws_arena_free(self._p, self._dev)
                self._p = None
        except Exception:
            pass


def arena_place(arena: "Arena", span: int, step: int, stream=None):
    """kmws_arena_place: byte offset inside `arena` (multiples of `step`) where an
    in-place split-8 unmask of `span` bytes runs fastest, and the probed rates
    {offset: fraction of 8 TB/s}.  The arena's bytes are unchanged."""
    k = (arena.nbytes - span) // step + 1 if span <= arena.nbytes else 0
    fr = (C.c_float * max(k, 1))()
    r = lib().kmws_arena_place(arena._p, arena.nbytes, span, step, _stream_handle(stream), fr, k)
    if r < 0:
        raise RuntimeError(f"kmws_arena_place failed with kmws_status {r}")
    return int(r), {i * step: round(float(fr[i]), 4) for i in range(k)}


def unmask_workspace_size(span: int) -> int:
    return lib().kmws_unmask_workspace_size(span)


def _sched_arg(ws: "Workspace", schedule: Optional[int]) -> int:
    if schedule is not None:
        return int(schedule)
    return -1 if ws.schedule is None else int(ws.schedule)


def unmask_batch(base, descs, ws: Workspace, span: Optional[int] = None, stream=None,
                 schedule: Optional[int] = None) -> None:
    """In-place batched unmask (kmws_unmask_plan + kmws_unmask_apply_sched) of
    uint8 device tensor `base`, with `schedule`, else ws.schedule, else the default."""
    span = base.numel() if span is None else span
    unmask_plan(descs, ws, span, stream)
    unmask_apply(base, descs, ws, span, stream, schedule)


def unmask_autotune(base, descs, ws: Workspace, span: Optional[int] = None, stream=None) -> int:
    """kmws_unmask_autotune: the fastest schedule of THIS batch (payload
    unchanged); kept as ws.schedule, the plan of the batch ws serves."""
    span = base.numel() if span is None else span
    r = lib().kmws_unmask_autotune(base.data_ptr(), span, descs.data_ptr(), descs.shape[0], ws.ptr, ws.nbytes,
                                   _stream_handle(stream))
    if r < 0:
        raise RuntimeError(f"kmws_unmask_autotune failed with kmws_status {r}")
    ws.schedule = r
    return r


def unmask_set_schedule(ws: Workspace, schedule: Optional[int]) -> None:
    """Pin (a code) or forget (None / < 0) the schedule of the batch ws serves.
    Host-side only; an invalid code fails at the next apply."""
    ws.schedule = None if schedule is None or schedule < 0 else int(schedule)


def sched_default(span: int, n: int) -> int:
    """kmws_unmask_default_schedule: the schedule of a batch nobody tuned."""
    return lib().kmws_unmask_default_schedule(span, n)


def unmask_get_schedule(ws: Workspace, descs, span: int) -> int:
    """The schedule code an apply through `ws` uses for this batch."""
    return sched_default(span, descs.shape[0]) if ws.schedule is None else ws.schedule


def unmask_plan(descs, ws: Workspace, span: int, stream=None) -> None:
    _check(lib().kmws_unmask_plan(span, descs.data_ptr(), descs.shape[0], ws.ptr, ws.nbytes,
                                  _stream_handle(stream)), "kmws_unmask_plan")


def unmask_apply(base, descs, ws: Workspace, span: Optional[int] = None, stream=None,
                 schedule: Optional[int] = None) -> None:
    span = base.numel() if span is None else span
    _check(lib().kmws_unmask_apply_sched(base.data_ptr(), span, descs.data_ptr(), descs.shape[0], ws.ptr,
                                         ws.nbytes, _sched_arg(ws, schedule), _stream_handle(stream)),
           "kmws_unmask_apply_sched")


def fill_synthetic(base, seed: int, nbytes: Optional[int] = None, stream=None) -> None:
    nbytes = base.numel() if nbytes is None else nbytes
    _check(lib().kmws_fill_synthetic(base.data_ptr(), nbytes, seed, _stream_handle(stream)),
           "kmws_fill_synthetic")


def fill_uniform_descs(descs, stride: int, length: int, key_seed: int, stream=None) -> None:
    _check(lib().kmws_fill_uniform_descs(descs.data_ptr(), descs.shape[0], stride, length, key_seed,
                                         _stream_handle(stream)), "kmws_fill_uniform_descs")


def check_unmasked(base, seed: int, descs, nbytes: Optional[int] = None, stream=None) -> int:
    import torch
    nbytes = base.numel() if nbytes is None else nbytes
    cnt = torch.zeros(1, dtype=torch.int64, device=base.device)
    _check(lib().kmws_check_unmasked(base.data_ptr(), nbytes, seed, descs.data_ptr(), descs.shape[0],
                                     cnt.data_ptr(), _stream_handle(stream)), "kmws_check_unmasked")
    return int(cnt.item())


# ---- pack / unpack ----

def copy_workspace_size(n: int, dst_cap: int) -> int:
    return lib().kmws_copy_workspace_size(n, dst_cap)


def _raise_on_status(ws: "Workspace", stream, what: str, out: str) -> None:
    """The synchronizing check of check=True: reads the workspace status back
    (a stream synchronize) and raises KmwsError (.ws_status) when it is nonzero
    -- a bad descriptor or batch (1), a header error (2), or a scan look-back
    that timed out (4): `out` is then invalid.  Skipped inside a graph capture."""
    if _capturing():
        return
    st = ws.status(stream)
    if st:
        e = KmwsError(ERR_FAILED, f"{what} (workspace status {st}: {out} invalid)")
        e.ws_status = st
        raise e


def encode_batch(src, descs, flags, dst, wire_off, ws: Workspace, stream=None, check: bool = False) -> None:
    """kmws_encode_batch: descs (n,2) int64, flags int16 (n,), wire_off int64 (n+1,).
    Stream-ordered; check=True synchronizes and raises on a nonzero workspace
    status (wire_off and dst are valid only when it is 0)."""
    n = _check_descs(descs)
    dev = descs.device
    _check_tensor(src, "src", 1, dev)
    _check_tensor(flags, "flags", 2, dev, n)
    _check_tensor(dst, "dst", 1, dev)
    _check_tensor(wire_off, "wire_off", 8, dev, n + 1)
    _check_tensor(ws.tensor, "workspace", 1, dev)
    _check(lib().kmws_encode_batch(src.data_ptr(), descs.data_ptr(), flags.data_ptr(), n,
                                   dst.data_ptr(), dst.numel(), wire_off.data_ptr(), ws.ptr, ws.nbytes,
                                   _stream_handle(stream)), "kmws_encode_batch")
    if check and n:
        _raise_on_status(ws, stream, "kmws_encode_batch", "wire_off")


def pack_headers_workspace_size(n: int) -> int:
    return lib().kmws_pack_headers_workspace_size(n)


def _capturing() -> bool:
    import torch
    return torch.cuda.is_current_stream_capturing()


def pack_headers(descs, flags, hdr, hdr_len=None, wire_off=None, ws: Optional[Workspace] = None,
                 stream=None, check: bool = False) -> None:
    """kmws_pack_headers (stream-ordered; check=True synchronizes): headers
    only, frame i's into the 16-B slot hdr[16 i:] (uint8 device tensor of >=
    16 n bytes), lengths into hdr_len (uint8, n), wire offsets into wire_off
    (int64, n+1; needs ws; valid only when the workspace status is 0).  With
    wire_off and check=True (outside a graph capture) the status is read back
    and a nonzero one -- a bad descriptor, or the look-back timeout that leaves
    wire_off invalid -- raises KmwsError."""
    n = _check_descs(descs)
    dev = descs.device
    _check_tensor(flags, "flags", 2, dev, n)
    _check_tensor(hdr, "hdr", 1, dev, 16 * n)
    if hdr_len is not None:
        _check_tensor(hdr_len, "hdr_len", 1, dev, n)
    if wire_off is not None:
        _check_tensor(wire_off, "wire_off", 8, dev, n + 1)
    if ws is not None:
        _check_tensor(ws.tensor, "workspace", 1, dev)
    _check(lib().kmws_pack_headers(descs.data_ptr(), flags.data_ptr(), n, hdr.data_ptr(),
                                   hdr_len.data_ptr() if hdr_len is not None else None,
                                   wire_off.data_ptr() if wire_off is not None else None,
                                   ws.ptr if ws is not None else None, ws.nbytes if ws is not None else 0,
                                   _stream_handle(stream)), "kmws_pack_headers")
    if check and wire_off is not None and ws is not None and n:
        _raise_on_status(ws, stream, "kmws_pack_headers", "wire_off")


def find_headers_streams(wire, stream_off, cap: int, wire_len: Optional[int] = None, stream=None):
    """kmws_find_headers_streams: the header-chain walk of every stream
    wire[stream_off[s]:stream_off[s+1]] on the device, one lane per stream.
    Returns (hdr_off (n_streams, cap) int64 absolute offsets, n_out int32,
    consumed int64) device tensors."""
    import torch
    _check_tensor(stream_off, "stream_off", 8, wire.device)
    if stream_off.dtype != torch.int64:
        raise TypeError("stream_off must be int64")
    ns = stream_off.shape[0] - 1
    wire_len = wire.numel() if wire_len is None else wire_len
    hdr = torch.empty((ns, max(cap, 1)), dtype=torch.int64, device=wire.device)
    n_out = torch.empty(ns, dtype=torch.int32, device=wire.device)
    consumed = torch.empty(ns, dtype=torch.int64, device=wire.device)
    _check(lib().kmws_find_headers_streams(wire.data_ptr(), wire_len, stream_off.data_ptr(), ns, hdr.data_ptr(), cap,
                                           n_out.data_ptr(), consumed.data_ptr(), _stream_handle(stream)),
           "kmws_find_headers_streams")
    return hdr, n_out, consumed


def unpack_headers(wire, hdr_off, mode: int, out_desc, out_flags, out_err, ws: Workspace,
                   wire_len: Optional[int] = None, stream=None) -> None:
    wire_len = wire.numel() if wire_len is None else wire_len
    _check(lib().kmws_unpack_headers(wire.data_ptr(), wire_len, hdr_off.data_ptr(), hdr_off.shape[0], mode,
                                     out_desc.data_ptr(),
                                     out_flags.data_ptr() if out_flags is not None else None,
                                     out_err.data_ptr() if out_err is not None else None,
                                     ws.ptr, ws.nbytes, _stream_handle(stream)), "kmws_unpack_headers")


def gather_unmask(src, descs, dst, dst_off, ws: Workspace, stream=None, check: bool = False) -> None:
    """kmws_gather_unmask (stream-ordered): dst_off and dst are valid only when
    the workspace status is 0; check=True synchronizes and raises otherwise."""
    n = _check_descs(descs)
    dev = descs.device
    _check_tensor(src, "src", 1, dev)
    _check_tensor(dst, "dst", 1, dev)
    _check_tensor(dst_off, "dst_off", 8, dev, n + 1)
    _check_tensor(ws.tensor, "workspace", 1, dev)
    _check(lib().kmws_gather_unmask(src.data_ptr(), descs.data_ptr(), n, dst.data_ptr(),
                                    dst.numel(), dst_off.data_ptr(), ws.ptr, ws.nbytes,
                                    _stream_handle(stream)), "kmws_gather_unmask")
    if check and n:
        _raise_on_status(ws, stream, "kmws_gather_unmask", "dst_off")


def _opt(t):
    return t.data_ptr() if t is not None else None


def unpack_unmask(wire, hdr_off, mode: int, out_desc, out_flags, out_err, ws: Workspace,
                  wire_len: Optional[int] = None, schedule: Optional[int] = None, stream=None) -> None:
    """kmws_unpack_unmask: header parse + unmask plan in one kernel, then the
    in-place unmask of the wire (ws: unmask_workspace_size(wire_len))."""
    wire_len = wire.numel() if wire_len is None else wire_len
    n = hdr_off.shape[0]
    dev = wire.device
    _check_tensor(hdr_off, "hdr_off", 8, dev, n)
    _check_tensor(out_desc, "out_desc", 8, dev, 2 * n)
    if out_flags is not None:
        _check_tensor(out_flags, "out_flags", 2, dev, n)
    if out_err is not None:
        _check_tensor(out_err, "out_err", 1, dev, n)
    if wire.numel() < wire_len:
        raise ValueError("wire shorter than wire_len")
    _check(lib().kmws_unpack_unmask(wire.data_ptr(), wire_len, hdr_off.data_ptr(), n, mode, out_desc.data_ptr(),
                                    _opt(out_flags), _opt(out_err), ws.ptr, ws.nbytes, _sched_arg(ws, schedule),
                                    _stream_handle(stream)), "kmws_unpack_unmask")


def unpack_gather(wire, hdr_off, mode: int, out_desc, out_flags, out_err, dst, dst_off, ws: Workspace,
                  wire_len: Optional[int] = None, stream=None) -> None:
    """kmws_unpack_gather: header parse inside the gather's scan, then the
    payloads unmasked densely into dst (ws: copy_workspace_size(n, dst.numel()))."""
    wire_len = wire.numel() if wire_len is None else wire_len
    n = hdr_off.shape[0]
    dev = wire.device
    _check_tensor(hdr_off, "hdr_off", 8, dev, n)
    _check_tensor(out_desc, "out_desc", 8, dev, 2 * n)
    if out_flags is not None:
        _check_tensor(out_flags, "out_flags", 2, dev, n)
    if out_err is not None:
        _check_tensor(out_err, "out_err", 1, dev, n)
    _check_tensor(dst, "dst", 1, dev)
    _check_tensor(dst_off, "dst_off", 8, dev, n + 1)
    if wire.numel() < wire_len:
        raise ValueError("wire shorter than wire_len")
    _check(lib().kmws_unpack_gather(wire.data_ptr(), wire_len, hdr_off.data_ptr(), n, mode, out_desc.data_ptr(),
                                    _opt(out_flags), _opt(out_err), dst.data_ptr(), dst.numel(), dst_off.data_ptr(),
                                    ws.ptr, ws.nbytes, _stream_handle(stream)), "kmws_unpack_gather")


def find_headers_into(buf, out) -> tuple:
    """kmws_find_headers over a uint8 numpy array into a preallocated uint64
    numpy array (no copies): -> (headers found, consumed bytes)."""
    n, used = C.c_uint32(0), C.c_uint64(0)
    _check(lib().kmws_find_headers(buf.ctypes.data, buf.nbytes, out.ctypes.data, len(out), C.byref(n),
                                   C.byref(used)), "kmws_find_headers")
    return n.value, used.value


def find_headers(wire, cap: Optional[int] = None):
    """Host header-chain walk -> (list of header offsets, consumed bytes)."""
    import numpy as np
    if isinstance(wire, np.ndarray):
        buf = wire
    else:
        buf = np.frombuffer(bytes(wire), dtype=np.uint8) if len(wire) else np.zeros(0, np.uint8)
    cap = buf.nbytes // 2 + 1 if cap is None else cap
    out = np.zeros(max(1, cap), dtype=np.uint64)
    n, used = find_headers_into(buf, out[:cap] if cap else out[:1])
    return out[:n].tolist(), used


class Pipeline:
    """kmws_pipeline: host-resident in-place unmask through pinned H2D/D2H."""

    AUTO, COPY, ZEROCOPY = 0, 1, 2

    def __init__(self, device: int = 0, chunk_bytes: int = 64 << 20, max_frames: int = 1 << 16,
                 depth: int = 3, transfer: int = 0):
        self._p = lib().kmws_pipeline_create(device, chunk_bytes, max_frames, depth)
        if not self._p:
            raise RuntimeError("kmws_pipeline_create failed (no gfx950 device or bad arguments)")
        _check(lib().kmws_pipeline_set_transfer(self._p, transfer), "kmws_pipeline_set_transfer")

    def unmask(self, host_u8, descs_np) -> None:
        """host_u8: numpy uint8 array or pinned torch CPU tensor; descs_np: DESC-layout numpy array."""
        ptr = host_u8.data_ptr() if hasattr(host_u8, "data_ptr") else host_u8.ctypes.data
        span = host_u8.numel() if hasattr(host_u8, "numel") else host_u8.nbytes
        _check(lib().kmws_pipeline_unmask(self._p, ptr, span, descs_np.ctypes.data, len(descs_np)),
               "kmws_pipeline_unmask")

    def __del__(self):
        try:
            if getattr(self, "_p", None):
                lib().kmws_pipeline_destroy(self._p)
                self._p = None
        except Exception:
            pass
