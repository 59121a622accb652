#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> short bench (+ tile variants) -> rocprof kernel trace.
# Every GPU step has its own timeout and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "== host: $(nproc) cpus; $(grep -m1 'model name' /proc/cpuinfo)" | tee "$OUT/host.txt"
timeout -k 10 420 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
echo "smoke ok" &&
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1 &&
echo "gpu tests ok" && tail -2 "$OUT/pytest_gpu.log" &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 10 > "$OUT/bench.json" 2> "$OUT/bench.err" &&
cat "$OUT/bench.json" &&
for v in 0 23 27; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-verify --variant $v > "$OUT/bench_v$v.json" 2>> "$OUT/bench.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_v$v.json'));print('variant $v', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- \
  python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" &&
echo "rocprof ok" && find "$OUT/prof" -name "*stats*" | head
