"""rocprofv3 kernel trace -> stats of the timed steps only: the last `steps`
dispatches of `kernel` before the bench's verification launch (bench.py runs
autotune and warmup launches of the same kernel first, and one more launch
after the timed loop when warmup + steps is even, to restore the payload).
usage: python tools/trace_stats.py <run_kernel_trace.csv | rocprofv3 -d dir> <kernel-substring> <steps> [skip_tail]"""
import csv
import glob
import os
import statistics
import sys


def main():
    path, kern, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    if os.path.isdir(path):
        found = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if len(found) != 1:
            raise SystemExit(f"expected one kernel_trace.csv under {path}, found {found}")
        path = found[0]
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    rows = [r for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = rows[len(rows) - skip - steps:len(rows) - skip]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in sel]
    print('"Name","Calls","TotalDurationNs","AverageNs","MinNs","MaxNs","StdDev","Note"')
    print(f'"{sel[0]["Kernel_Name"]}",{len(d)},{sum(d)},{statistics.mean(d):.1f},{min(d)},{max(d)},'
          f'{statistics.pstdev(d):.1f},"timed steps: dispatches {len(rows) - skip - steps + 1}..{len(rows) - skip} '
          f'of {len(rows)}"')


if __name__ == "__main__":
    main()
