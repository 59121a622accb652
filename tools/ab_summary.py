"""Summarise a tools/r06_store_ab.sh run: python tools/ab_summary.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

d = sys.argv[1]
if os.path.exists(f"{d}/loopback_ab.jsonl"):
    for line in open(f"{d}/loopback_ab.jsonl"):
        r = json.loads(line)
        print("loopback", r["lib"], r.get("mode"), r.get("connections"), r.get("GiB_s"), r.get("verified"))
if os.path.exists(f"{d}/resident_ab.jsonl"):
    for line in open(f"{d}/resident_ab.jsonl"):
        r = json.loads(line)
        print("latency", r["lib"], r["threads"], r["masking"], r["len"], r["us_median"], r["calls_per_s"])
for f in sorted(glob.glob(f"{d}/**/interference_ab.jsonl", recursive=True)):
    for line in open(f):
        r = json.loads(line)
        ph = r["phases"]
        q = [p["mean_ms"] for p in ph if not p["busy"]]
        b = [p["mean_ms"] for p in ph if p["busy"]]
        print("interference", os.path.relpath(f, d), r["lib"], round(sum(b) / len(b) / (sum(q) / len(q)), 3),
              [p.get("mask_calls_per_s") for p in ph if p["busy"]])
