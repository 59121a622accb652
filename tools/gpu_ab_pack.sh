#!/bin/bash
# A/B of the pack path's kernel forms, RUN_TAG=<tag> -> gpurun_out/<tag>/ab_*.json:
# the product build (fused row kernel, two units in flight per wave), the
# prologue + copy-grid form (KMWS_PACK_ROWS_MAX_MEAN=0) and the row kernel with
# one unit in flight (KMWS_PACK_ROWS_PIPE=0), each loaded alone by
# tools/ab_pack.py (cfg4 encode/gather; interleaved rounds inside each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so cfg4 > "$OUT/ab_product.json" 2> "$OUT/ab_product.err" &&
timeout -k 10 200 python3 tools/ab_pack.py tools/ab/libkmws_rows0.so cfg4 > "$OUT/ab_rows0.json" 2> "$OUT/ab_rows0.err" &&
timeout -k 10 200 python3 tools/ab_pack.py tools/ab/libkmws_rows_nopipe.so cfg4 > "$OUT/ab_rows_nopipe.json" 2> "$OUT/ab_rows_nopipe.err"
