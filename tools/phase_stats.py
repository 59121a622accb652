"""rocprofv3 kernel trace of tools/grid_interference -> per-phase duration of
the unmask kernel from the trace itself: its dispatches sorted by start time,
the first `warm` skipped, then `phases` groups of `steps` (even phases quiet,
odd phases busy: 16 threads masking on the resident grid), as the program ran
them.  usage: python tools/phase_stats.py <rocprofv3 -d dir> <kernel> <steps> <phases> [warm]"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d, kern, steps, phases = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    warm = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    found = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = [r for f in found for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[warm:warm + steps * phases]
    out = []
    for p in range(phases):
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[p * steps:(p + 1) * steps]]
        out.append({"phase": p, "busy": p % 2 == 1, "dispatches": len(dur), "mean_ms": round(statistics.mean(dur), 4),
                    "min_ms": round(min(dur), 4), "max_ms": round(max(dur), 4)})
    q = statistics.mean(x["mean_ms"] for x in out if not x["busy"])
    b = statistics.mean(x["mean_ms"] for x in out if x["busy"])
    res = [r for f in found for r in csv.DictReader(open(f)) if "resident_unmask_kernel" in r["Kernel_Name"]]
    print(json.dumps({"kernel": kern, "phases": out, "quiet_mean_ms": round(q, 4), "busy_mean_ms": round(b, 4),
                      "busy_over_quiet": round(b / q, 4), "resident_grid_dispatches": len(res)}))


if __name__ == "__main__":
    main()
