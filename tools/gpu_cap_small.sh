#!/bin/bash
# Small frames with the occupancy cap forced (KMWS_UNMASK_BLOCKS_PER_CU=2) vs the product rule, per library build:
# cfg4 in place and bench.py at LENS aligned frame lengths.  usage: TAG=x bash tools/gpu_cap_small.sh lib.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-capsmall}
mkdir -p "$OUT"
cp kuma_amd/lib/libkmws_gpu.so "$OUT/product.so"
for L in "$@"; do
  b=$(basename "$L" .so)
  cp "$L" kuma_amd/lib/libkmws_gpu.so
  KMWS_UNMASK_BLOCKS_PER_CU=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py tests/test_gpu_fuzz.py -x -q \
    --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so; tail -20 "$OUT/pytest.log"; exit 1; }
  line="$b tests(cap 2): $(tail -1 "$OUT/pytest.log")"
  for cap in product 2; do
    if [ "$cap" = product ]; then e=""; else e="KMWS_UNMASK_BLOCKS_PER_CU=$cap"; fi
    env $e timeout -k 10 300 python tools/bench_configs.py cfg4 --placement plain > "$OUT/${b}_cfg4_$cap.json" 2>> "$OUT/err.log" || exit 1
    line="$line | cfg4/$cap $(python3 -c "import json;print(round(json.load(open('$OUT/${b}_cfg4_$cap.json'))['unmask_in_place']['hbm_frac'],4))")"
    for FL in ${LENS:-4096 1024}; do
      F=$(( (64 << 30) / FL ))
      env $e timeout -k 10 300 python bench.py --frame-len $FL --frames $F --max-batch-frames $F --steps 10 --warmup 2 \
        --cpu-seconds 0 > "$OUT/${b}_L${FL}_$cap.json" 2>> "$OUT/err.log" || exit 1
      line="$line L$FL/$cap $(python3 -c "import json;print(json.load(open('$OUT/${b}_L${FL}_$cap.json'))['roofline']['frac'])")"
    done
  done
  echo "$line"
done
cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so
