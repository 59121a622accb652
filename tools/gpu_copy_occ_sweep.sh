#!/bin/bash
# Pack/gather copy kernel with its resident blocks per CU set by KMWS_COPY_LDS_PAD
# (dynamic LDS per block: 0 = 8 blocks, 32768 = 5, 40000 = 4, 50000 = 3, 60000 = 2;
# "default" = the product rule) and its block deal by KMWS_COPY_SPLIT (SPLITS; parts
# of the unit slots, or 1000 + c for XCD runs of c blocks), tools/ab_pack.py on the
# product library, REPS interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-copyocc}
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-2}"); do
  for pad in ${PADS:-0 32768 40000 50000 60000}; do
  for split in ${SPLITS:-8}; do
    envs="KMWS_COPY_SPLIT=$split"; [ "$pad" = default ] || envs="$envs KMWS_COPY_LDS_PAD=$pad"
    env $envs timeout -k 10 300 python tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so ${CFGS:-cfg3,cfg4,u64k} \
      > "$OUT/pad${pad}_s${split}_$rep.json" 2>> "$OUT/err.log" || { tail -5 "$OUT/err.log"; exit 1; }
    python3 -c "
import json
d=json.load(open('$OUT/pad${pad}_s${split}_$rep.json'))
print('rep $rep pad $pad split $split', ' '.join('%s enc %.4f gat %.4f'%(c, max(r['enc_frac'] for r in d[c]['lib']), max(r['gat_frac'] for r in d[c]['lib'])) for c in d))
"
  done
  done
done
