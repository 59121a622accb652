#!/bin/bash
# Small aligned frames (LENS), in-place unmask: the product (16 KiB tiles, LDS path uncapped) vs
# 8 KiB tiles (variants 40: split 8, 41: XCD runs of 32) at a forced occupancy cap of BPC blocks per CU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-smalltiles}
mkdir -p "$OUT"
for L in ${LENS:-4096}; do
  F=$(( (64 << 30) / L ))
  for cfg in "product:-1:" "v40_b4:40:4" "v41_b4:41:4" "v40_b3:40:3" "v41_b6:41:6"; do
    IFS=: read -r name var bpc <<< "$cfg"
    if [ -n "$bpc" ]; then e="KMWS_UNMASK_BLOCKS_PER_CU=$bpc"; else e=""; fi
    env $e timeout -k 10 300 python bench.py --frame-len $L --frames $F --max-batch-frames $F --steps 10 --warmup 2 \
      --cpu-seconds 0 --variant $var > "$OUT/L${L}_$name.json" 2>> "$OUT/err.log" || { tail -5 "$OUT/err.log"; exit 1; }
    echo "frame_len $L $name $(python3 -c "import json;d=json.load(open('$OUT/L${L}_$name.json'));print(d['roofline']['frac'], d['verify'])")"
  done
done
