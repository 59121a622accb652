"""The drop-in boundary compiled against kuma's real types.

tests/cpp/kuma_types_adapter.cpp instantiates include/kmws_wshandler.hpp as
INTEGRATION.md sec.3 aliases it -- BasicWSHandler<kuma::ws::FrameHeader,
kuma::KMBuffer, kuma::ws::WSError, kuma::ws::WSMode, kuma::KMError> -- with the
reference checkout's own headers: src/ws/wsdefs.h, include/kmdefs.h,
include/kmconf.h, include/kevdefs.h and include/kmbuffer.h.  The shipped
kmbuffer.h does not compile (`auto* createSharedData` used at
:528 before its definition at :676), so the test writes a copy with that one
token changed into its own temporary build directory; nothing is committed
and nothing of it reaches the GPU box.  Skipped where /root/reference is
absent (the GPU box)."""
import os
import subprocess

import pytest

from kuma_amd import build as kb

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
NEEDED = [os.path.join(REF, "include", h) for h in ("kmbuffer.h", "kmdefs.h", "kmconf.h", "kevdefs.h")] + \
    [os.path.join(REF, "src", "ws", "wsdefs.h")]

pytestmark = pytest.mark.skipif(not all(os.path.exists(p) for p in NEEDED),
                                reason="reference checkout not present (container-only test)")


def _patched_kmbuffer(build_dir) -> None:
    src = open(os.path.join(REF, "include", "kmbuffer.h")).read()
    bad = "auto* createSharedData("
    assert src.count(bad) == 1, "the known kmbuffer.h defect moved; re-check SURVEY 8 a-15"
    (build_dir / "kmbuffer.h").write_text(src.replace(bad, "_SharedBase* createSharedData("))


def test_shipped_kmbuffer_header_does_not_compile(tmp_path):
    """Why the copy exists: the reference header as shipped is rejected."""
    t = tmp_path / "t.cpp"
    t.write_text('#include "kmbuffer.h"\nint main() { kuma::KMBuffer b; return (int)b.chainLength(); }\n')
    r = subprocess.run(["g++", "-std=c++14", "-fsyntax-only", "-I", os.path.join(REF, "include"), str(t)],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "createSharedData" in r.stderr


@pytest.mark.parametrize("std", ["c++14", "c++17"])
def test_adapter_with_kuma_types(tmp_path, std):
    lib = kb.build()
    bdir = tmp_path / "kuma_hdrs"
    bdir.mkdir()
    _patched_kmbuffer(bdir)
    exe = tmp_path / "kuma_types_adapter"
    subprocess.check_call(["g++", f"-std={std}", "-O1", "-g", "-Wall", "-Wno-unused-variable",
                           "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                           "-I", str(bdir), "-I", os.path.join(REF, "include"), "-I", os.path.join(REF, "src", "ws"),
                           "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "kuma_types_adapter.cpp"),
                           "-L", os.path.dirname(lib), "-lkmws_gpu", "-Wl,-rpath," + os.path.dirname(lib),
                           "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=0"})
    assert r.returncode == 0 and "OK kuma types" in r.stdout, r.stdout + r.stderr
