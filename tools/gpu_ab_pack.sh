#!/bin/bash
# A/B of the pack path's kernel forms, RUN_TAG=<tag> -> gpurun_out/<tag>/ab_*.json:
# the product build (prologue + copy grid) and the fused row kernel
# (tools/ab/libkmws_rows.so, KMWS_PACK_ROWS_MAX_MEAN=16384), each loaded alone
# by tools/ab_pack.py (cfg4 encode/gather; interleaved rounds inside each).
# (profiles/r04i_pack_rows_ab.txt: the round-4 run, when the fused kernel was
# the product's form.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so cfg4 > "$OUT/ab_product.json" 2> "$OUT/ab_product.err" &&
timeout -k 10 200 python3 tools/ab_pack.py tools/ab/libkmws_rows.so cfg4 > "$OUT/ab_rows.json" 2> "$OUT/ab_rows.err"
