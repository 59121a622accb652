"""Per-kernel HBM traffic of one program from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, separate runs of the same command): for every
kmws kernel, the first dispatch's grid, VGPRs, LDS and the counted KiB as MB.
FETCH_SIZE is printed as counted; MI355X_MICROARCH.md's gfx950 correction
(x2 for wide coalesced streaming reads) is applied by the reader where it
holds (the copy and unmask streams; not scattered header or descriptor reads).

usage: python tools/pmc_kernels.py <fetch_dir> <write_dir> [substr ...]
"""
import csv
import glob
import os
import sys


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        out += list(csv.DictReader(open(f)))
    if not out:
        raise SystemExit(f"no counter_collection csv under {d}")
    return out


def per_dispatch(rs, counter):
    d = {}
    for r in rs:
        if r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        e = d.setdefault(key, {"name": r.get("Kernel_Name", ""), "grid": r.get("Grid_Size", ""),
                               "vgpr": r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")),
                               "lds": r.get("LDS_Block_Size", ""), "v": 0.0})
        e["v"] += float(r["Counter_Value"])
    return d


def short(name):
    name = name.split("(")[0].replace("void ", "").replace("kmws::", "")
    return name[:44]


def main():
    fdir, wdir = sys.argv[1:3]
    subs = sys.argv[3:] or ["kmws"]
    f, w = per_dispatch(rows(fdir), "FETCH_SIZE"), per_dispatch(rows(wdir), "WRITE_SIZE")
    firstf, firstw = {}, {}
    for k in sorted(f, key=lambda x: int(x)):
        firstf.setdefault(short(f[k]["name"]), f[k])
    for k in sorted(w, key=lambda x: int(x)):
        firstw.setdefault(short(w[k]["name"]), w[k])
    print(f"# {'kernel':44s} {'grid':>10s} {'vgpr':>4s} {'lds':>6s} {'fetch_MB':>10s} {'write_MB':>10s}")
    for name, e in firstf.items():
        if not any(s in e["name"] for s in subs):
            continue
        wv = firstw.get(name, {"v": float("nan")})["v"]
        print(f"{name:46s} {e['grid']:>10s} {e['vgpr']:>4s} {e['lds']:>6s} {e['v'] * 1024 / 1e6:10.1f} "
              f"{wv * 1024 / 1e6:10.1f}")


if __name__ == "__main__":
    main()
