#!/bin/bash
# Pack-path evidence, RUN_TAG=<tag>: the pack/unpack GPU tests, then a rocprofv3
# kernel trace of tools/bench_configs.py <configs> (default cfg4) on plain
# allocations -> gpurun_out/<tag>/{pytest_pack.log, configs.jsonl, breakdown.txt}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_pack.py -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_pack.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/trace" -o run -- \
    python3 tools/bench_configs.py ${CONFIGS:-cfg4} --reps 5 --placement plain > "$OUT/configs.jsonl" 2> "$OUT/configs.err" &&
python3 tools/kernel_breakdown.py "$(find "$OUT/trace" -name '*kernel_trace.csv')" > "$OUT/breakdown.txt"
