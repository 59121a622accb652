#!/bin/bash
# Placement A/B: bench with the placement probe (default) twice, then plain torch.empty, then a
# rocprofv3 kernel trace of the default command.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 10 > "$OUT/place_bench1.json" 2> "$OUT/place.err" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/place_bench2.json" 2>> "$OUT/place.err" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --placement plain > "$OUT/place_plain.json" 2>> "$OUT/place.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_place" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/place_prof_bench.json" 2>> "$OUT/place.err" &&
for f in place_bench1 place_bench2 place_plain place_prof_bench; do
  python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['value'], d['roofline']['frac'], d['config']['unmask_schedule'], json.dumps(d['config']['placement']))"
done
