#!/bin/bash
# PMC traffic of the pack/gather copy kernels on cfg3 + cfg4 (FETCH_SIZE, WRITE_SIZE in separate passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}/pmc_copy
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$PWD/$OUT/$c" -o run -- \
    python3 tools/bench_configs.py cfg3 cfg4 --reps 1 > "$OUT/$c.jsonl" 2> "$OUT/$c.err" || exit 1
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(os.path.join(out, c, "**", "*counter_collection*.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    for r in rows:
        if r.get("Counter_Name") == c:
            per[(int(r["Dispatch_Id"]), r["Kernel_Name"][:60])] += float(r["Counter_Value"])
    for (d, k), v in sorted(per.items()):
        if "kmws::" in k:
            print(c, d, k, f"{v * 1024 / 1e9:.4f} GB (raw KiB x1024)")
PY
