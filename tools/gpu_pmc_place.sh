#!/bin/bash
# PMC traffic of the headline kernel as bench.py runs it (placement probe on, default schedule),
# FETCH_SIZE and WRITE_SIZE in separate passes; then a 2-rank gloo rehearsal of bench --gpus 2 on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:-r01}
OUT=gpurun_out/$TAG/pmc_place
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counter bench-args
  timeout -k 10 300 rocprofv3 --pmc "$2" --kernel-trace --output-format csv -d "$PWD/$OUT/$1" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-verify $3 > "$OUT/$1.json" 2> "$OUT/$1.err"
}
pass d_fetch FETCH_SIZE "--no-autotune" &&
pass d_write WRITE_SIZE "--no-autotune" &&
python3 tools/pmc_traffic.py "$OUT/d_fetch" "$OUT/d_write" unmask_split_kernel 1048576 65536 "$OUT/traffic_placed.json" 0 &&
cat "$OUT/traffic_placed.json" &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --frames 262144 --cpu-seconds 0 --dist-backend gloo > "$OUT/gloo2.json" 2> "$OUT/gloo2.err" &&
cat "$OUT/gloo2.json"
