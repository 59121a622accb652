#!/bin/bash
# Loopback at 8 connections with small generations (1 / 2 / 4 frames of 4 KiB
# per loop iteration) per library in LIBS.  RUN_TAG=<tag>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:?set RUN_TAG}; mkdir -p $OUT
g++ -std=c++17 -O2 -I include tests/cpp/loopback_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread \
    -Wl,-rpath,$PWD/oracle -o $OUT/lb || exit 1
for L in $LIBS; do
  for g in 1 2 4; do
    for m in adapter replay_adapter; do
      LD_LIBRARY_PATH=$PWD/$L timeout -k 10 120 $OUT/lb $m 10 $g 0 0 8 > $OUT/t.json || exit 1
      sed "s|^{|{\"lib\": \"$L\", |" $OUT/t.json >> $OUT/loopback_ab.jsonl
    done
  done
done
rm -f $OUT/t.json
