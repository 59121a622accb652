#!/bin/bash
# Round evidence on the current build, RUN_TAG=<tag>: the -m gpu suite, smoke,
# the default bench line, and tools/bench_configs.py <CONFIGS> (default: cfg1
# cfg2b cfg3 cfg4 e2e) on plain allocations -> gpurun_out/<tag>/.  Every GPU step
# has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 &&
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 500 python3 tools/bench_configs.py ${CONFIGS:-cfg1 cfg2b cfg3 cfg4 e2e} --placement plain \
    > "$OUT/configs.jsonl" 2> "$OUT/configs.err"
