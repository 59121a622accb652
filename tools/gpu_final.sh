#!/bin/bash
# Round-end style check on one box: smoke -> all GPU tests -> default bench (with cpu_baseline)
# -> rocprofv3 kernel trace + stats of the same bench command -> cfg1/3/4/e2e configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
tail -1 "$OUT/pytest_gpu.log" &&
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && cat "$OUT/bench.json" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
  python3 bench.py --cpu-seconds 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" &&
python3 tools/trace_stats.py "$OUT/prof/run_kernel_trace.csv" unmask_split_kernel 20 0 > "$OUT/prof_timed.csv" &&
cat "$OUT/prof_timed.csv" && python3 -c "import json;d=json.load(open('$OUT/prof_bench.json'));print('event kernel_ms', d['roofline']['kernel_ms'], d['config']['unmask_schedule'])" &&
timeout -k 10 500 python tools/bench_configs.py cfg1 cfg2b cfg3 cfg4 e2e cfg3_e2e > "$OUT/configs.jsonl" 2> "$OUT/configs.err" && echo configs ok
