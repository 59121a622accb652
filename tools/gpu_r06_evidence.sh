#!/bin/bash
# Round 6 evidence on one box (RUN_TAG=<tag>): the thread-exit check, the
# resident grid's cost to the cfg2 batch (plain run + rocprofv3 kernel trace),
# the host-resident e2e bench at N = 1 and N = 2 (gloo, one GPU), and the
# default bench line.  Every GPU step under its own time limit, chained.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
INC="-I include"
LIB="-L kuma_amd/lib -lkmws_gpu -Wl,-rpath,$PWD/kuma_amd/lib"
g++ -std=c++17 -O2 $INC tests/cpp/thread_exit_check.cpp $LIB -L oracle -lkmws_oracle -Wl,-rpath,$PWD/oracle -lpthread -o /tmp/tec &&
hipcc -std=c++17 -O2 $INC tools/grid_interference.cpp $LIB -lpthread -o /tmp/grid_interference &&
echo "== thread exit" && timeout -k 10 120 /tmp/tec 20 8 8 > "$OUT/thread_exit.json" &&
echo "== interference" && timeout -k 10 180 /tmp/grid_interference 1048576 20 6 16 > "$OUT/interference.json" &&
echo "== interference trace" && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/interf_trace" -o run -- \
    /tmp/grid_interference 1048576 20 6 16 > "$OUT/interference_prof.json" 2> "$OUT/interference_prof.err" &&
python3 tools/phase_stats.py "$OUT/interf_trace" unmask_split_kernel 20 6 3 > "$OUT/interference_trace_phases.json" &&
echo "== e2e N=1" && timeout -k 10 300 python3 bench.py --config e2e --gpus 1 --e2e-gib 8 --steps 10 --warmup 2 > "$OUT/e2e_n1.json" &&
echo "== e2e N=2 gloo" && timeout -k 10 300 python3 bench.py --config e2e --gpus 2 --dist-backend gloo --e2e-gib 4 --steps 10 --warmup 2 > "$OUT/e2e_n2_gloo.json" &&
echo "== bench" && timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo done
