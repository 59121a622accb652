"""Turns rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs) into
HBM bytes per launch of one kernel, with the gfx950 corrections of
MI355X_MICROARCH.md sec. HBM: FETCH_SIZE counts half the bytes of wide (16 B
per lane) coalesced streaming reads -> x2; WRITE_SIZE is exact for 16-B
stores; both are in KiB.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substr> <frames> <frame_len> <out.json>
"""
import csv
import datetime
import glob
import json
import os
import sys


def counter_rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    return rows


def per_dispatch(rows, counter, kern):
    vals = {}
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        if kern not in name or r.get("Counter_Name") != counter:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, kern, frames, flen, out = sys.argv[1:7]
    schedule = int(sys.argv[7]) if len(sys.argv) > 7 else None  # kmws_unmask_schedule() code of the pass
    frames, flen = int(frames), int(flen)
    f = per_dispatch(counter_rows(fdir), "FETCH_SIZE", kern)
    w = per_dispatch(counter_rows(wdir), "WRITE_SIZE", kern)
    if not f or not w:
        raise SystemExit("kernel not found in counter rows")
    fetch_kib, write_kib = sum(f) / len(f), sum(w) / len(w)
    read_bytes = 2 * fetch_kib * 1024      # gfx950: FETCH_SIZE is half of wide streaming reads
    write_bytes = write_kib * 1024
    alg = frames * (2 * flen + 16)
    res = {"kernel": kern, "frames": frames, "frame_len": flen, "dispatches": [len(f), len(w)],
           "FETCH_SIZE_KiB": fetch_kib, "WRITE_SIZE_KiB": write_kib,
           "read_bytes_corrected": read_bytes, "write_bytes": write_bytes,
           "hbm_bytes_per_launch": read_bytes + write_bytes, "algorithmic_bytes_per_launch": alg,
           "traffic_over_algorithmic": (read_bytes + write_bytes) / alg,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB->bytes x1024",
           "measured_at": datetime.datetime.now(datetime.timezone.utc).isoformat(timespec="seconds")}
    if schedule is not None:
        res["schedule"] = schedule
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
