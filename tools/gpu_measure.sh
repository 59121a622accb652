#!/bin/bash
# Round-4 measurements on the current build, RUN_TAG=<tag> -> gpurun_out/<tag>/:
#  configs.jsonl  tools/bench_configs.py sync loopback cfg1 cfg3 cfg4 (plain allocations)
#  trace/ + breakdown_cfg4.txt  rocprofv3 kernel trace of cfg4 (per-kernel times)
#  fetch/, write/ + pmc_cfg4_kernels.txt  FETCH_SIZE and WRITE_SIZE passes of cfg4
#    (separate runs, --kernel-trace only beside --pmc)
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/bench_configs.py ${CONFIGS:-sync loopback cfg1 cfg3 cfg4} --placement plain \
    > "$OUT/configs.jsonl" 2> "$OUT/configs.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/trace" -o run -- \
    python3 tools/bench_configs.py cfg4 --reps 3 --placement plain > "$OUT/trace_cfg4.jsonl" 2> "$OUT/trace.err" &&
python3 tools/kernel_breakdown.py "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)" > "$OUT/breakdown_cfg4.txt" &&
timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/fetch" -o run -- \
    python3 tools/bench_configs.py cfg4 --reps 1 --placement plain > "$OUT/fetch.jsonl" 2> "$OUT/fetch.err" &&
timeout -k 10 -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/write" -o run -- \
    python3 tools/bench_configs.py cfg4 --reps 1 --placement plain > "$OUT/write.jsonl" 2> "$OUT/write.err" &&
python3 tools/pmc_kernels.py "$OUT/fetch" "$OUT/write" > "$OUT/pmc_cfg4_kernels.txt"
