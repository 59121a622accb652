#!/bin/bash
# A/B of the resident worker under concurrency: tests/cpp/sync_cfg1.cpp's
# mask_threads case (4 KiB / 64 KiB handleDataMask on 1-16 threads, and one
# masking thread beside idle slots) against each library in LIBS (directories
# holding a libkmws_gpu.so; default: the product), RUN_TAG=<tag> ->
# gpurun_out/<tag>/resident_ab.jsonl.  Variant builds: tools/build_variant.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
LIBS=${LIBS:-kuma_amd/lib}
g++ -std=c++17 -O2 -I include tests/cpp/sync_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread \
    -Wl,-rpath,"$PWD/oracle" -o "$OUT/sync_cfg1" || exit 1
for L in $LIBS; do
    for r in 1 2; do
        LD_LIBRARY_PATH="$PWD/$L" timeout -k 10 120 "$OUT/sync_cfg1" 3 mask_threads > "$OUT/ab.tmp" 2>> "$OUT/resident_ab.err" || exit 1
        sed "s|^{|{\"lib\": \"$L\", \"run\": $r, |" "$OUT/ab.tmp" >> "$OUT/resident_ab.jsonl"
    done
done
rm -f "$OUT/ab.tmp"
