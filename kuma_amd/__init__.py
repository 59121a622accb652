"""kuma_amd -- MI355X-native WebSocket (RFC 6455) frame codec for kuma.

The hot path (payload mask/unmask, frame-header pack/unpack) is hand-written
HIP for gfx950 in kuma_amd/csrc, exported through the C ABI declared in
include/kmws_gpu.h; kuma_amd.kmws is the Python binding used by tests/bench.
"""
from . import kmws  # noqa: F401
