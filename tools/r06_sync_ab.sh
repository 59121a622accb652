#!/bin/bash
# tests/cpp/sync_cfg1.cpp (every case: decode_sync, decode_sync_threads,
# mask_sync, mask_threads) per library in LIBS, the libraries interleaved,
# ROUNDS times, the order rotating each round.  RUN_TAG=<tag> -> gpurun_out/<tag>/sync_ab.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:?set RUN_TAG}; mkdir -p $OUT
g++ -std=c++17 -O2 -I include tests/cpp/sync_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread \
    -Wl,-rpath,$PWD/oracle -o $OUT/sync_cfg1 || exit 1
read -r -a LA <<< "$LIBS"
for r in $(seq 1 ${ROUNDS:-2}); do
  for k in $(seq 0 $((${#LA[@]} - 1))); do  # the order rotates each round
    L=${LA[$(( (k + r) % ${#LA[@]} ))]}
    LD_LIBRARY_PATH=$PWD/$L timeout -k 10 180 $OUT/sync_cfg1 10 > $OUT/t.jsonl 2>> $OUT/sync_ab.err || exit 1
    sed "s|^{|{\"lib\": \"$L\", \"round\": $r, |" $OUT/t.jsonl >> $OUT/sync_ab.jsonl
  done
done
rm -f $OUT/t.jsonl
