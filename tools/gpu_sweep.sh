#!/bin/bash
# Schedule sweep on one box, twice (two processes): tools/sweep_unmask.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sweep
mkdir -p "$OUT"
export TMPDIR=/tmp
V=${1:-0,8192,16384,24576,32768,65536,131072,2049,4097,8193,16385,32769,65537,131073,262145}
M=${2:-sync}
for k in 1 2; do
  timeout -k 10 240 python tools/sweep_unmask.py "$V" 3 ${3:-3} ${4:-$((1 << 20))} $M ${5:-65536} ${6:-${5:-65536}} > "$OUT/sweep_$k.jsonl" 2> "$OUT/sweep_$k.err" || { tail -5 "$OUT/sweep_$k.err"; exit 1; }
done
python - "$OUT" <<'PY'
import json, sys
a = [json.loads(l) for l in open(sys.argv[1] + "/sweep_1.jsonl")]
b = [json.loads(l) for l in open(sys.argv[1] + "/sweep_2.jsonl")]
print(a[0])
for x, y in zip(a[1:], b[1:]):
    v = x["variant"]
    kind = "tiles" if v == 0 else ("pipe %d" % (v - 1) if v & 1 else "persist %d" % v) if v >= 64 else "variant %d" % v
    print("%-16s %7.3f %7.3f ms  frac %.4f %.4f" % (kind, x["median_ms"], y["median_ms"], x["frac"], y["frac"]))
PY
