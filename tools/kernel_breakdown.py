"""rocprofv3 kernel trace -> per-kernel call count, mean and median duration (us),
kmws kernels only, sorted by total time.
usage: python tools/kernel_breakdown.py <run_kernel_trace.csv>"""
import collections
import csv
import statistics
import sys


def short(name: str) -> str:
    name = name.split("(")[0]
    return name.replace("void ", "").replace("kmws::", "")


def main():
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        if "kmws" not in r["Kernel_Name"]:
            continue
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'kernel':48s} {'calls':>5s} {'mean_us':>9s} {'median_us':>9s}")
    for k, v in rows:
        print(f"{k[:48]:48s} {len(v):5d} {statistics.mean(v):9.1f} {statistics.median(v):9.1f}")


if __name__ == "__main__":
    main()
