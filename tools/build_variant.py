"""Builds a tuning variant of libkmws_gpu.so from a patched COPY of the product
sources: the product sources carry no tuning switches, so an
A/B build is the product plus a patch, never a define.

usage: python tools/build_variant.py <patch> <out.so>
  the patch applies with `patch -p1` at the repository root (git diff format);
  only its kuma_amd/csrc/ hunks matter.  Example: tools/patches/copy_form_units.patch
  forces the unit copy form (tools/gpu_ab_chunk.sh LIBS=...)."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    patch, out = os.path.abspath(sys.argv[1]), os.path.abspath(sys.argv[2])
    from kuma_amd import build as kb
    with tempfile.TemporaryDirectory() as td:
        shutil.copytree(os.path.join(ROOT, "kuma_amd", "csrc"), os.path.join(td, "kuma_amd", "csrc"))
        subprocess.check_call(["patch", "-p1", "-s", "-i", patch], cwd=td)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        print(kb.build(out=out, srcdir=os.path.join(td, "kuma_amd", "csrc")))


if __name__ == "__main__":
    main()
