"""Builds the in-tree HIP library kuma_amd/lib/libkmws_gpu.so for gfx950.

Explicit hipcc (no torch JIT cache): the .so lives in the repo tree so it
travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libkmws_gpu.so")
ARCH = "gfx950"
# Test-only variant (never loaded by kuma_amd.kmws; tests load it by path):
#  - one tile of every look-back scan never publishes and the spin bound is
#    small, so the timeout path (kStatusLookbackTimeout) runs in
#    tests/test_gpu_pack.py;
#  - a resident-worker job whose first key is 0xDEAD5Exx stalls its workgroup
#    for xx * 10 ms, and the job timeout / drain bounds are 50 / 150 ms, so the
#    withdraw and KMWS_ERR_TIMEOUT paths run in tests/test_gpu_decoder.py.
TEST_LIB = os.path.join(LIB_DIR, "libkmws_gpu_testhooks.so")
TEST_DEFINES = ("KMWS_TEST_SKIP_PUBLISH_TILE=1", "KMWS_LOOKBACK_SPIN_LIMIT=4096",
                "KMWS_TEST_RESIDENT_STALL_KEY=0xDEAD5E00u", "KMWS_RESIDENT_TIMEOUT_MS=50",
                "KMWS_RESIDENT_DRAIN_MS=150")
RESIDENT_STALL_KEY = 0xDEAD5E00


def sources(srcdir: str | None = None):
    d = srcdir or os.path.join(HERE, "csrc")
    return sorted(glob.glob(os.path.join(d, "*.hip")) + glob.glob(os.path.join(d, "*.cpp")))


def deps():
    return sources() + glob.glob(os.path.join(HERE, "csrc", "*.hpp")) + \
        glob.glob(os.path.join(ROOT, "include", "*.h"))


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in deps())


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=(),
          srcdir: str | None = None) -> str:
    """Compiles the library; `out` + `defines` (-D flags) make the test build,
    `out` + `srcdir` (a patched copy of csrc/, tools/build_variant.py) a tuning
    variant, without touching the product library."""
    if out is None and not force and up_to_date():
        return LIB
    lib = out or LIB
    obj_dir = os.path.dirname(os.path.abspath(lib))  # beside the output: variant builds never share objects
    os.makedirs(obj_dir, exist_ok=True)
    objs = []
    inc = ["-I", os.path.join(ROOT, "include"), "-I", srcdir or os.path.join(HERE, "csrc")]
    cmds = []
    for src in sources(srcdir):
        obj = os.path.join(obj_dir, os.path.basename(lib) + "." + os.path.basename(src) + ".o")
        cmds.append(["hipcc", "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                     "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines], *inc, "-c", src, "-o", obj])
        objs.append(obj)

    def compile_one(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)

    with ThreadPoolExecutor(max_workers=min(len(cmds), 4)) as ex:
        list(ex.map(compile_one, cmds))
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib]
    subprocess.check_call(cmd)
    for o in objs:
        os.remove(o)
    return lib


def build_test_variants(force: bool = False) -> list:
    """Test-only libraries (tests load them by path; the product binding never does)."""
    if force or not os.path.exists(TEST_LIB) or os.path.getmtime(TEST_LIB) < max(
            os.path.getmtime(p) for p in deps()):
        build(out=TEST_LIB, defines=TEST_DEFINES)
    return [TEST_LIB]


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
