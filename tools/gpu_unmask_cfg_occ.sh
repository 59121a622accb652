#!/bin/bash
# Packed-wire (cfg2b) and 4 KiB-fragment (cfg4) in-place unmask at forced blocks per
# CU (KMWS_UNMASK_BLOCKS_PER_CU; unset = product rule), tools/bench_configs.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cfgocc}
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-2}"); do
  for b in ${BLOCKS:-product 6 5 4 3}; do
    if [ "$b" = product ]; then env_b=""; else env_b="KMWS_UNMASK_BLOCKS_PER_CU=$b"; fi
    env $env_b timeout -k 10 300 python tools/bench_configs.py cfg2b cfg4 > "$OUT/b${b}_$rep.jsonl" 2>> "$OUT/err.log" ||
      { tail -5 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
c=[json.loads(l) for l in open('$OUT/b${b}_$rep.jsonl')]
print('rep $rep blocks/CU $b', 'cfg2b %.4f (sched %s)' % (c[0]['hbm_frac'], c[0]['schedule']),
      'cfg4 unmask %.4f (sched %s)' % (c[1]['unmask_in_place']['hbm_frac'], c[1]['unmask_in_place']['schedule']))
"
  done
done
