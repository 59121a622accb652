#!/bin/bash
# Per-kernel breakdown of the pack/gather path: one rocprofv3 kernel trace per
# config (tools/ab_pack.py on the product library), summarised per kernel.
# usage: RUN_TAG=r02c tools/gpu_pack_prof.sh [lib.so ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-packprof}
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS=("$@")
[ ${#LIBS[@]} -eq 0 ] && LIBS=(kuma_amd/lib/libkmws_gpu.so)
for L in "${LIBS[@]}"; do
  b=$(basename "$L" .so)
  for cfg in cfg4 cfg3; do
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/prof_${b}_$cfg" -o run -- \
      python3 tools/ab_pack.py "$L" $cfg > "$OUT/${b}_$cfg.json" 2> "$OUT/${b}_$cfg.err" || exit 1
    python3 tools/kernel_breakdown.py "$OUT/prof_${b}_$cfg/run_kernel_trace.csv" > "$OUT/${b}_${cfg}_breakdown.txt" || exit 1
    echo "== $b $cfg"; cat "$OUT/${b}_${cfg}_breakdown.txt"
    python3 -c "
import json
d=json.load(open('$OUT/${b}_$cfg.json'))
print(' '.join('%s enc %.4f gat %.4f'%(c, max(r['enc_frac'] for r in d[c]['lib']), max(r['gat_frac'] for r in d[c]['lib'])) for c in d))
"
  done
done
