"""Dump one kernel's gfx950 assembly from a .hip file (dev helper).
usage: python tools/isa_dump.py <file.hip> <kernel-substring> [grep-regex]"""
import os, re, subprocess, sys, tempfile
src, pat = sys.argv[1], sys.argv[2]
rx = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = tempfile.mkdtemp()
subprocess.check_call(["hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
                       "-I", os.path.join(root, "include"), "-I", os.path.join(root, "kuma_amd", "csrc"),
                       "-c", os.path.abspath(src), "-save-temps", "-o", os.path.join(d, "x.o")], cwd=d,
                      stderr=subprocess.DEVNULL)
s = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
lines = open(os.path.join(d, s)).read().split("\n")
out, on = [], False
for ln in lines:
    if re.match(r"^_Z\S*:", ln) and pat in ln:
        on = True
    if on:
        out.append(ln)
        if ln.strip().startswith(".size") and pat in ln:
            break
meta = [l for l in lines if re.search(r"\.(vgpr|sgpr)_count|group_segment_fixed_size", l)]
for i, ln in enumerate(out):
    if rx is None or rx.search(ln):
        print(f"{i:5d} {ln}")
