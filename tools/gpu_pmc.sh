#!/bin/bash
# PMC passes for the headline kernel: FETCH_SIZE and WRITE_SIZE in separate runs
# (--kernel-trace only beside --pmc), then bytes per launch -> profiles/<tag>_traffic.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:-r01}
OUT=gpurun_out/$TAG/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
B="bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.json" 2> "$OUT/fetch.err" &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/write" -o run -- python3 $B > "$OUT/write.json" 2> "$OUT/write.err" &&
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" unmask_tiles_kernel 1048576 65536 "$OUT/traffic.json"
