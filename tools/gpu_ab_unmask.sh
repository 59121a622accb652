#!/bin/bash
# A/B of unmask schedules on one box: parity for every variant, then interleaved
# bench passes (1 M x 64 KiB, device-resident).  Usage: tools/gpu_ab_unmask.sh "0 4 5 10 11 12"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abu
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_unmask.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python -c "import torch; from kuma_amd import kmws; p=torch.cuda.get_device_properties(0); print(\"cus\", p.multi_processor_count, \"resident\", kmws.unmask_resident_blocks())" || exit 1
for rep in 1 2; do
  for v in ${1:-0 4 5 10 11 12}; do
    timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-verify --variant $v > "$OUT/v${v}_$rep.json" 2>> "$OUT/bench.err" || exit 1
    python -c "import json;d=json.load(open('$OUT/v${v}_$rep.json'));print('rep $rep variant $v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
