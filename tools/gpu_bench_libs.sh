#!/bin/bash
# Default bench.py runs per library build, interleaved over REPS rounds (each run its own process,
# allocation and placement probe).  usage: REPS=3 TAG=x bash tools/gpu_bench_libs.sh lib1.so lib2.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-benchlibs}
mkdir -p "$OUT"
cp kuma_amd/lib/libkmws_gpu.so "$OUT/product.so"
for rep in $(seq 1 "${REPS:-3}"); do
  for L in "$@"; do
    b=$(basename "$L" .so)
    cp "$L" kuma_amd/lib/libkmws_gpu.so
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/${b}_$rep.json" 2>> "$OUT/err.log" ||
      { cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so; tail -5 "$OUT/err.log"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${b}_$rep.json'));p=d['config']['placement'];print('rep $rep $b', d['roofline']['frac'], d['config']['unmask_schedule'][-30:], p.get('offset_GiB'), p.get('probe_frac_by_offset_GiB'))"
  done
done
cp "$OUT/product.so" kuma_amd/lib/libkmws_gpu.so
