"""Builds the in-tree HIP library kuma_amd/lib/libkmws_gpu.so for gfx950.

Explicit hipcc (no torch JIT cache): the .so lives in the repo tree so it
travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libkmws_gpu.so")
ARCH = "gfx950"


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
    for src in sources():
        obj = os.path.join(LIB_DIR, os.path.basename(lib) + "." + os.path.basename(src) + ".o")
        cmd = ["hipcc", "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
               "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in defines], *inc, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        objs.append(obj)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib]
    subprocess.check_call(cmd)
    for o in objs:
        os.remove(o)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
