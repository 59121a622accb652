#!/bin/bash
# Pack parity tests on the product library, then per-kernel profiles of library builds.
# usage: TAG=r02e LIBS="tools/ab/lib_A.so tools/ab/lib_C.so" bash tools/gpu_pack_ab.sh
set -o pipefail
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py tests/test_gpu_tx.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/$TAG/pytest.log | head -80; exit 1; }
RUN_TAG=$TAG bash tools/gpu_pack_prof.sh $LIBS
