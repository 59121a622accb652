#!/bin/bash
# Headline bench at smaller frame lengths (64 GiB batches), product occupancy rule
# vs the cap forced (KMWS_UNMASK_BLOCKS_PER_CU=2) or lifted (=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-flen}
mkdir -p "$OUT"
for L in ${LENS:-32768 16384 8192}; do
  F=$(( (64 << 30) / L ))
  for b in ${MODES:-product 2 0}; do
    if [ "$b" = product ]; then e=""; else e="KMWS_UNMASK_BLOCKS_PER_CU=$b"; fi
    env $e timeout -k 10 300 python bench.py --frame-len $L --frames $F --max-batch-frames $F --steps 10 --warmup 2 \
      --cpu-seconds 0 > "$OUT/L${L}_b${b}.json" 2>> "$OUT/err.log" || { tail -5 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
d=json.load(open('$OUT/L${L}_b${b}.json'))
print('frame_len $L blocks/CU $b', d['roofline']['frac'], d['config']['unmask_schedule'][:60])
"
  done
done
