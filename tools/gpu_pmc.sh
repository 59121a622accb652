#!/bin/bash
# PMC passes for the headline kernels: FETCH_SIZE and WRITE_SIZE in separate runs
# (--kernel-trace only beside --pmc), for the one-block-per-tile schedule and for
# the persistent schedule (bench --variant 4), -> bytes per launch per kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:-r01}
OUT=gpurun_out/$TAG/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counter bench-args
  timeout -k 10 300 rocprofv3 --pmc "$2" --kernel-trace --output-format csv -d "$PWD/$OUT/$1" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-verify $3 > "$OUT/$1.json" 2> "$OUT/$1.err"
}
pass split_fetch FETCH_SIZE "--no-autotune" &&
pass split_write WRITE_SIZE "--no-autotune" &&
python3 tools/pmc_traffic.py "$OUT/split_fetch" "$OUT/split_write" unmask_split_kernel 1048576 65536 "$OUT/traffic_split.json" 0 &&
pass split8_fetch FETCH_SIZE "--variant 23" &&
pass split8_write WRITE_SIZE "--variant 23" &&
python3 tools/pmc_traffic.py "$OUT/split8_fetch" "$OUT/split8_write" unmask_split_kernel 1048576 65536 "$OUT/traffic_split8.json" 3 &&
pass split4_fetch FETCH_SIZE "--variant 22" &&
pass split4_write WRITE_SIZE "--variant 22" &&
python3 tools/pmc_traffic.py "$OUT/split4_fetch" "$OUT/split4_write" unmask_split_kernel 1048576 65536 "$OUT/traffic_split4.json" 5 &&
pass runs_fetch FETCH_SIZE "--variant 27" &&
pass runs_write WRITE_SIZE "--variant 27" &&
python3 tools/pmc_traffic.py "$OUT/runs_fetch" "$OUT/runs_write" unmask_split_kernel 1048576 65536 "$OUT/traffic_runs.json" 4 &&
pass tiles_fetch FETCH_SIZE "--variant 0" &&
pass tiles_write WRITE_SIZE "--variant 0" &&
python3 tools/pmc_traffic.py "$OUT/tiles_fetch" "$OUT/tiles_write" unmask_tiles_kernel 1048576 65536 "$OUT/traffic.json" &&
pass persist_fetch FETCH_SIZE "--variant 4" &&
pass persist_write WRITE_SIZE "--variant 4" &&
python3 tools/pmc_traffic.py "$OUT/persist_fetch" "$OUT/persist_write" unmask_persist_kernel 1048576 65536 "$OUT/traffic_persist.json" &&
[ -n "$PMC_PIPE" ] || exit 0
pass pipe_fetch FETCH_SIZE "--variant 10" &&
pass pipe_write WRITE_SIZE "--variant 10" &&
python3 tools/pmc_traffic.py "$OUT/pipe_fetch" "$OUT/pipe_write" unmask_pipe_kernel 1048576 65536 "$OUT/traffic_pipe.json"
