#!/bin/bash
# A/B of several library builds on the copy path (tools/ab_pack.py, one process per build,
# interleaved reps), after the pack tests pass on each candidate.  usage: tools/gpu_ab_libs.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abl
mkdir -p "$OUT"
export TMPDIR=/tmp
cp kuma_amd/lib/libkmws_gpu.so "$OUT/product.so"
for L in "$@"; do
  cp "$L" kuma_amd/lib/libkmws_gpu.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so; tail -30 "$OUT/pytest.log"; exit 1; }
  echo "$L: $(tail -1 "$OUT/pytest.log")"
done
cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so
for rep in 1 2 3; do
  for L in "$@"; do
    b=$(basename "$L" .so)
    timeout -k 10 300 python tools/ab_pack.py "$L" cfg3,cfg4 > "$OUT/$b.json" 2> "$OUT/$b.err" || exit 1
    python -c "
import json
d=json.load(open('$OUT/$b.json'))
print('rep $rep $b', ' '.join('%s enc %.4f gat %.4f'%(c, max(r['enc_frac'] for r in d[c]['lib']), max(r['gat_frac'] for r in d[c]['lib'])) for c in d))
"
  done
done
