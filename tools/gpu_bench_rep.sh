#!/bin/bash
# Three default bench runs (separate processes: each gets its own allocation / placement probe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/rep$i.json" 2>> "$OUT/rep.err" || exit 1
  python3 -c "import json;d=json.load(open('$OUT/rep$i.json'));print($i, d['value'], d['roofline']['frac'], d['config']['unmask_schedule'], d['config']['placement']['offset_GiB'], d['config']['placement']['probe_frac_by_offset_GiB'])"
done
