#!/bin/bash
# Headline bench over (blocks per CU, schedule) pairs: KMWS_UNMASK_BLOCKS_PER_CU caps
# the resident unmask blocks per CU (0 = no cap: 6, the registers' limit; product: 2),
# --variant pins the schedule (21 split 2, 23 split 8, 27 XCD runs of 16, 34/35 = 32 KiB
# tiles split 2/8; -1 = autotuned default).  usage: COMBOS="2:23 3:27" REPS=2 TAG=x bash ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-occ}
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-2}"); do
  for cv in ${COMBOS}; do
    pad=${cv%%:*}; var=${cv##*:}
    KMWS_UNMASK_BLOCKS_PER_CU=$pad timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --variant "$var" \
      > "$OUT/p${pad}_v${var}_$rep.json" 2>> "$OUT/err.log" || { tail -5 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
d=json.load(open('$OUT/p${pad}_v${var}_$rep.json'))
print('rep $rep blocks/CU $pad variant $var', d['roofline']['frac'], d['config']['unmask_schedule'][:50], d['config']['placement'].get('offset_GiB'))
"
  done
done
