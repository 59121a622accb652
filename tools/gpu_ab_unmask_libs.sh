#!/bin/bash
# A/B of library builds on the in-place unmask path: each build runs the unmask
# parity tests, then (interleaved, REPS rounds) the headline bench and the packed
# wire (cfg2b) / 4 KiB-fragment (cfg4) configs.  The product library is restored.
# usage: REPS=2 TAG=abu bash tools/gpu_ab_unmask_libs.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abu}
mkdir -p "$OUT"
export TMPDIR=/tmp
cp kuma_amd/lib/libkmws_gpu.so "$OUT/product.so"
restore() { cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so; }
for L in "$@"; do
  cp "$L" kuma_amd/lib/libkmws_gpu.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py tests/test_gpu_configs.py -x -q --timeout 200 \
    --timeout-method thread > "$OUT/pytest.log" 2>&1 || { restore; tail -30 "$OUT/pytest.log"; exit 1; }
  echo "$L: $(tail -1 "$OUT/pytest.log")"
done
for rep in $(seq 1 "${REPS:-2}"); do
  for L in "$@"; do
    b=$(basename "$L" .so)
    cp "$L" kuma_amd/lib/libkmws_gpu.so
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/${b}_bench_$rep.json" 2>> "$OUT/err.log" &&
    timeout -k 10 300 python tools/bench_configs.py cfg2b cfg4 > "$OUT/${b}_cfg_$rep.jsonl" 2>> "$OUT/err.log" ||
      { restore; tail -20 "$OUT/err.log"; exit 1; }
    python -c "
import json
b=json.load(open('$OUT/${b}_bench_$rep.json'))
c=[json.loads(l) for l in open('$OUT/${b}_cfg_$rep.jsonl')]
print('rep $rep $b', 'cfg2 %.4f (%s)' % (b['roofline']['frac'], b['config']['unmask_schedule'][:40]),
      'cfg2b %.4f (sched %s)' % (c[0]['hbm_frac'], c[0]['schedule']),
      'placed %.4f (sched %s)' % (c[0].get('placed', {}).get('hbm_frac', 0), c[0].get('placed', {}).get('schedule')),
      'cfg4 unmask %.4f (sched %s)' % (c[1]['unmask_in_place']['hbm_frac'], c[1]['unmask_in_place'].get('schedule')),
      'placed %.4f' % ((c[1]['unmask_in_place'].get('placed') or {}).get('hbm_frac', 0)))
"
  done
done
restore
