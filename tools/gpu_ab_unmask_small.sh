#!/bin/bash
# A/B of library builds on small-frame in-place unmask: each build passes the unmask,
# config and fuzz GPU tests (also with the occupancy cap forced on every batch), then,
# interleaved over REPS rounds, cfg4's in-place unmask (plain and placed) and the headline
# bench at LENS frame lengths, product occupancy rule and cap forced (2 blocks per CU).
# usage: REPS=2 TAG=abs LENS="4096 8192" bash tools/gpu_ab_unmask_small.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abs}
mkdir -p "$OUT"
export TMPDIR=/tmp
cp kuma_amd/lib/libkmws_gpu.so "$OUT/product.so"
restore() { cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so; }
for L in "$@"; do
  cp "$L" kuma_amd/lib/libkmws_gpu.so
  for cap in "" 2; do
    KMWS_UNMASK_BLOCKS_PER_CU=$cap timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py tests/test_gpu_configs.py \
      tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 ||
      { restore; tail -30 "$OUT/pytest.log"; exit 1; }
    echo "$L cap=${cap:-product}: $(tail -1 "$OUT/pytest.log")"
  done
done
for rep in $(seq 1 "${REPS:-2}"); do
  for L in "$@"; do
    b=$(basename "$L" .so)
    cp "$L" kuma_amd/lib/libkmws_gpu.so
    timeout -k 10 300 python tools/bench_configs.py cfg4 > "$OUT/${b}_cfg4_$rep.json" 2>> "$OUT/err.log" || { restore; tail -20 "$OUT/err.log"; exit 1; }
    line="rep $rep $b $(python3 -c "
import json
u=json.load(open('$OUT/${b}_cfg4_$rep.json'))['unmask_in_place']
print('cfg4 in place %.4f placed %.4f' % (u['hbm_frac'], (u.get('placed') or {}).get('hbm_frac', 0)))")"
    for FL in ${LENS:-4096 8192}; do
      F=$(( (64 << 30) / FL ))
      for cap in product 2; do
        if [ "$cap" = product ]; then e=""; else e="KMWS_UNMASK_BLOCKS_PER_CU=$cap"; fi
        env $e timeout -k 10 300 python bench.py --frame-len $FL --frames $F --max-batch-frames $F --steps 10 --warmup 2 \
          --cpu-seconds 0 > "$OUT/${b}_L${FL}_${cap}_$rep.json" 2>> "$OUT/err.log" || { restore; tail -5 "$OUT/err.log"; exit 1; }
        line="$line L$FL/$cap $(python3 -c "import json;print(json.load(open('$OUT/${b}_L${FL}_${cap}_$rep.json'))['roofline']['frac'])")"
      done
    done
    echo "$line"
  done
done
restore
