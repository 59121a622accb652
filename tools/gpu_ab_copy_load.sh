#!/bin/bash
# A/B of the copy waves' source-load policy on cfg4, RUN_TAG=<tag>:
# the product build (non-temporal source loads) against tools/ab/libkmws_tload.so
# (KMWS_COPY_NT_LOAD=0: ordinary loads, so an edge line two wave instructions
# share can stay in the L2).  Timing with tools/ab_pack.py, then FETCH_SIZE and
# WRITE_SIZE passes (separate runs) of each build -> gpurun_out/<tag>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so cfg4 > "$OUT/ab_nt.json" 2> "$OUT/ab_nt.err" &&
timeout -k 10 200 python3 tools/ab_pack.py tools/ab/libkmws_tload.so cfg4 > "$OUT/ab_tload.json" 2> "$OUT/ab_tload.err" &&
pass() {  # dir counter lib
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$2" --kernel-trace --output-format csv -d "$PWD/$OUT/$1" -o run -- \
    python3 tools/ab_pack.py "$3" cfg4 > "$OUT/$1.json" 2> "$OUT/$1.err"
} &&
pass nt_fetch FETCH_SIZE kuma_amd/lib/libkmws_gpu.so &&
pass nt_write WRITE_SIZE kuma_amd/lib/libkmws_gpu.so &&
pass tl_fetch FETCH_SIZE tools/ab/libkmws_tload.so &&
pass tl_write WRITE_SIZE tools/ab/libkmws_tload.so &&
python3 tools/pmc_kernels.py "$OUT/nt_fetch" "$OUT/nt_write" > "$OUT/pmc_nt.txt" &&
python3 tools/pmc_kernels.py "$OUT/tl_fetch" "$OUT/tl_write" > "$OUT/pmc_tload.txt"
