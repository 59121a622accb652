#!/bin/bash
# A/B of the resident grid's cost to a device batch (tools/grid_interference)
# and of its small-job latency (tests/cpp/sync_cfg1.cpp mask_threads) per
# library build in LIBS (directories holding a libkmws_gpu.so; default: the
# product), RUN_TAG=<tag> -> gpurun_out/<tag>/interference_ab.jsonl, resident_ab.jsonl.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
LIBS=${LIBS:-kuma_amd/lib}
hipcc -std=c++17 -O2 -I include tools/grid_interference.cpp -L kuma_amd/lib -lkmws_gpu -lpthread -o "$OUT/gi" || exit 1
g++ -std=c++17 -O2 -I include tests/cpp/sync_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread \
    -Wl,-rpath,"$PWD/oracle" -o "$OUT/sync_cfg1" || exit 1
MODES=${MODES:-resident}
LAT=${LAT:-1}
for L in $LIBS; do
    for M in $MODES; do
        # (exit status 1 = wrong bytes, expected from measurement-only variants; a time limit or a crash ends the run)
        LD_LIBRARY_PATH="$PWD/$L" timeout -k 10 120 "$OUT/gi" 1048576 20 4 16 $M > "$OUT/gi.tmp" 2>> "$OUT/ab.err"
        rc=$?; [ $rc -le 1 ] && [ -s "$OUT/gi.tmp" ] || exit 1
        sed "s|^{|{\"lib\": \"$L\", |" "$OUT/gi.tmp" >> "$OUT/interference_ab.jsonl"
    done
    [ "$LAT" = 1 ] || continue
    LD_LIBRARY_PATH="$PWD/$L" timeout -k 10 120 "$OUT/sync_cfg1" 3 mask_threads > "$OUT/ab.tmp" 2>> "$OUT/ab.err" || exit 1
    sed "s|^{|{\"lib\": \"$L\", |" "$OUT/ab.tmp" >> "$OUT/resident_ab.jsonl"
done
rm -f "$OUT/ab.tmp" "$OUT/gi.tmp"
