#!/bin/bash
# cfg2b / cfg4 (in-place unmask of packed wire images) at forced blocks-per-CU caps
# (KMWS_UNMASK_BLOCKS_PER_CU; 0 = no cap), REPS rounds interleaved.
# usage: BPC="0 3 4" REPS=2 TAG=bpc bash tools/gpu_unmask_cfg_bpc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bpc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in $(seq 1 "${REPS:-2}"); do
  for b in ${BPC:-0 3 4}; do
    KMWS_UNMASK_BLOCKS_PER_CU=$b timeout -k 10 300 python tools/bench_configs.py cfg2b cfg4 > "$OUT/b${b}_$rep.jsonl" \
      2>> "$OUT/err.log" || { tail -20 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
c=[json.loads(l) for l in open('$OUT/b${b}_$rep.jsonl')]
print('rep $rep blocks/CU $b', 'cfg2b %.4f (sched %s)' % (c[0]['hbm_frac'], c[0]['schedule']),
      'cfg4 unmask %.4f (sched %s)' % (c[1]['unmask_in_place']['hbm_frac'], c[1]['unmask_in_place'].get('schedule')))
"
  done
done
