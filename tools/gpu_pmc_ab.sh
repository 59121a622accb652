#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) of tools/ab_pack.py cfg4 for
# each build in LIBS="name:path ...", then their timing, RUN_TAG=<tag>:
# gpurun_out/<tag>/pmc_<name>.txt, ab_<name>.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in $LIBS; do
  name=${v%%:*}; lib=${v#*:}
  timeout -k 10 -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/f_$name" -o run -- \
    python3 tools/ab_pack.py "$lib" cfg4 > "$OUT/f_$name.json" 2> "$OUT/f_$name.err" || exit 1
  timeout -k 10 -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$PWD/$OUT/w_$name" -o run -- \
    python3 tools/ab_pack.py "$lib" cfg4 > "$OUT/w_$name.json" 2> "$OUT/w_$name.err" || exit 1
  python3 tools/pmc_kernels.py "$OUT/f_$name" "$OUT/w_$name" > "$OUT/pmc_$name.txt" || exit 1
done
for v in $LIBS; do
  timeout -k 10 240 python3 tools/ab_pack.py "${v#*:}" cfg4 > "$OUT/ab_${v%%:*}.json" 2> "$OUT/ab_${v%%:*}.err" || exit 1
done
