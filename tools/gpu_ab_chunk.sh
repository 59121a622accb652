#!/bin/bash
# The copy path's chunk form (product: chunk_map + chunk_copy) checked and
# timed against the round-3 unit form, RUN_TAG=<tag>:
#  1. the pack / configs / fuzz GPU tests on the product build;
#  2. tools/ab_pack.py (cfg4, cfg3, small frames) per build, each loaded alone:
#     product (chunk, non-temporal source loads), tools/ab/libkmws_chunk_tl.so
#     (chunk, ordinary loads), tools/ab/libkmws_units.so (KMWS_PACK_UNITS=1),
#     tools/ab/libkmws_tload.so (units, ordinary loads).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_pack.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > "$OUT/pytest_pack.log" 2>&1 &&
for v in product:kuma_amd/lib/libkmws_gpu.so chunk_tl:tools/ab/libkmws_chunk_tl.so units:tools/ab/libkmws_units.so \
         tload:tools/ab/libkmws_tload.so; do
  timeout -k 10 240 python3 tools/ab_pack.py "${v#*:}" cfg4,cfg3,small > "$OUT/ab_${v%%:*}.json" 2> "$OUT/ab_${v%%:*}.err" || exit 1
done
