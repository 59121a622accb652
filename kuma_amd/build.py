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
# Test-only variant (never loaded by kuma_amd.kmws): one tile of the header-pack
# look-back never publishes and the spin bound is small, so the timeout path
# (kStatusLookbackTimeout) runs in tests/test_gpu_pack.py.
LOOKBACK_TEST_LIB = os.path.join(LIB_DIR, "libkmws_gpu_lbtest.so")
LOOKBACK_TEST_DEFINES = ("KMWS_TEST_SKIP_PUBLISH_TILE=1", "KMWS_LOOKBACK_SPIN_LIMIT=4096")


def sources():
    return sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")) +
                  glob.glob(os.path.join(HERE, "csrc", "*.cpp")))


def deps():
    return sources() + glob.glob(os.path.join(HERE, "csrc", "*.hpp")) + \
        glob.glob(os.path.join(ROOT, "include", "*.h"))


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(p) <= t for p in deps())


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=()) -> str:
    """Compiles the library; `out` + `defines` (-D flags) make a tuning variant
    (tools/ab_pack.py) without touching the product library."""
    if out is None and not force and up_to_date():
        return LIB
    lib = out or LIB
    os.makedirs(LIB_DIR, exist_ok=True)
    objs = []
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc")]
    cmds = []
    for src in sources():
        obj = os.path.join(LIB_DIR, os.path.basename(lib) + "." + os.path.basename(src) + ".o")
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
    if force or not os.path.exists(LOOKBACK_TEST_LIB) or os.path.getmtime(LOOKBACK_TEST_LIB) < max(
            os.path.getmtime(p) for p in deps()):
        build(out=LOOKBACK_TEST_LIB, defines=LOOKBACK_TEST_DEFINES)
    return [LOOKBACK_TEST_LIB]


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
