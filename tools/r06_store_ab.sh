#!/bin/bash
# Round 6: the resident grid's payload stores A/B.  TESTS (pytest files) run
# first on the product; then per library in LIBS: loopback at 4 and 8
# connections, the grid's cost to a device batch (4 KiB and, GI_LENS, other
# mask sizes) and small-job latency.  RUN_TAG=<tag>; LB=0 skips the loopback,
# NO_GI=1 the interference and latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG; mkdir -p $OUT
LIBS=${LIBS:-kuma_amd/lib}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS > $OUT/pytest.log 2>&1 || exit 1
fi
g++ -std=c++17 -O2 -I include tests/cpp/loopback_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread \
    -Wl,-rpath,$PWD/oracle -o $OUT/lb || exit 1
for L in $LIBS; do
  [ "${LB:-1}" = 1 ] || break
  for c in 4 8; do
    for m in adapter replay_adapter; do
      LD_LIBRARY_PATH=$PWD/$L timeout -k 10 120 $OUT/lb $m 10 16 0 0 $c > $OUT/t.json || exit 1
      sed "s|^{|{\"lib\": \"$L\", |" $OUT/t.json >> $OUT/loopback_ab.jsonl
    done
  done
done
rm -f $OUT/t.json
[ -n "$NO_GI" ] && exit 0
RUN_TAG=$TAG LIBS="$LIBS" bash tools/gpu_ab_interference.sh || exit 1
for len in $GI_LENS; do
  GI_LEN=$len RUN_TAG=$TAG/len$len LIBS="$LIBS" LAT=0 bash tools/gpu_ab_interference.sh || exit 1
done
