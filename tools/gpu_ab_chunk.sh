#!/bin/bash
# The copy path's chunk form (product: chunk_map + chunk_copy) checked and
# timed, RUN_TAG=<tag>:
#  1. the pack / configs / fuzz GPU tests on the product build;
#  2. tools/ab_pack.py (cfg4, cfg3, small frames) per build, each loaded alone:
#     the product (chunk form below a 16 KiB mean region, unit form above) and
#     any other build named in LIBS -- the product sources carry no tuning
#     switches (round 5): a variant is built from a patched copy of
#     kuma_amd/csrc (tools/build_variant.py <patch> <out.so>);
#  3. FETCH_SIZE and WRITE_SIZE passes (separate runs) of the product on cfg4.
# LIBS="name:path ..." / CFGS / QUICK=1 (step 2 only) select another A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${RUN_TAG:?set RUN_TAG}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS=${LIBS:-"product:kuma_amd/lib/libkmws_gpu.so"}
CFGS=${CFGS:-cfg4,cfg3,small}
if [ -z "$QUICK" ]; then
  timeout -k 10 500 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread \
      tests/test_gpu_pack.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > "$OUT/pytest_pack.log" 2>&1 || exit 1
fi
for v in $LIBS; do
  timeout -k 10 240 python3 tools/ab_pack.py "${v#*:}" "$CFGS" > "$OUT/ab_${v%%:*}.json" 2> "$OUT/ab_${v%%:*}.err" || exit 1
done
[ -n "$QUICK" ] && exit 0
pass() {  # dir counter
  timeout -k 10 -s KILL 150 rocprofv3 --pmc "$2" --kernel-trace --output-format csv -d "$PWD/$OUT/$1" -o run -- \
    python3 tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so cfg4 > "$OUT/$1.json" 2> "$OUT/$1.err"
} &&
pass pmc_fetch FETCH_SIZE &&
pass pmc_write WRITE_SIZE &&
python3 tools/pmc_kernels.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_cfg4_pack_kernels.txt"
