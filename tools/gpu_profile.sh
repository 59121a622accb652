#!/bin/bash
# rocprofv3 evidence for the headline line (bench.py, N = 1), RUN_TAG=<tag>:
#  1. kernel trace + stats of the default bench command without the
#     plain-allocation leg (so the timed dispatches are the last `steps` of the
#     unmask kernel) -> kernel_stats.csv, kernel_stats_timed.csv, prof_bench.json;
#  2. PMC passes, FETCH_SIZE and WRITE_SIZE in separate runs (--kernel-trace only
#     beside --pmc), of the same command with the schedule run 1 picked pinned
#     -> traffic.json (HBM bytes per launch, MI355X_MICROARCH.md corrections).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/trace" -o run -- \
    python3 bench.py --no-plain --cpu-seconds 0 --cfg5-anchor 0 --e2e-gib 0 --steps $STEPS > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" &&
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv" &&
python3 tools/trace_stats.py "$OUT/trace" unmask_split_kernel $STEPS > "$OUT/kernel_stats_timed.csv" &&
SCHED=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['config']['unmask_schedule'])" "$OUT/prof_bench.json") &&
pass() {  # name counter
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$2" --kernel-trace --output-format csv -d "$PWD/$OUT/$1" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --cfg5-anchor 0 --e2e-gib 0 --no-verify --no-plain --placement plain --schedule "$SCHED" \
    > "$OUT/$1.json" 2> "$OUT/$1.err"
} &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" unmask_split_kernel 1048576 65536 "$OUT/traffic.json" "$SCHED"
