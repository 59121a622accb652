#!/bin/bash
# bench.py after the sub-batch restructure: default (cfg2), cfg5 at N=1 (10 M frames as 8 resident
# sub-batches), and a 2-rank gloo rehearsal of the strong-scaling path on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > "$OUT/cfg2.json" 2> "$OUT/cfg5.err" &&
cat "$OUT/cfg2.json" &&
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --cpu-seconds 0 --job-frames 10485760 > "$OUT/cfg5_n1.json" 2>> "$OUT/cfg5.err" &&
cat "$OUT/cfg5_n1.json" &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 \
  bench.py --gpus 2 --steps 3 --warmup 1 --job-frames 1048576 --max-batch-frames 262144 --cpu-seconds 0 --dist-backend gloo \
  > "$OUT/cfg5_gloo2.json" 2>> "$OUT/cfg5.err" &&
cat "$OUT/cfg5_gloo2.json"
