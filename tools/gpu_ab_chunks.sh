#!/bin/bash
# Pack pipeline A/B: frame chunks K (KMWS_PACK_CHUNKS) for kmws_encode_batch / kmws_gather_unmask.
# Parity first (pack, fuzz, configs tests with K=4), then cfg3/cfg4 at K = 1, 2, 4, 8, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN_TAG:-r01}
mkdir -p "$OUT"
export TMPDIR=/tmp
KMWS_PACK_CHUNKS=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py \
  -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/chunks_pytest.log" 2>&1 && tail -1 "$OUT/chunks_pytest.log" || exit 1
for rep in 1 2; do
  for k in 1 2 4 8; do
    KMWS_PACK_CHUNKS=$k timeout -k 10 200 python tools/bench_configs.py cfg3 cfg4 --reps 9 > "$OUT/chunks_k${k}_r${rep}.jsonl" 2>> "$OUT/chunks.err" || exit 1
    python3 -c "
import json
r=[json.loads(l) for l in open('$OUT/chunks_k${k}_r${rep}.jsonl')]
c3=r[0]; c4=r[1]
print('rep $rep K=$k', 'cfg3 enc %.4f dec %.4f' % (c3['encode']['hbm_frac'], c3['decode_unpack_gather']['hbm_frac']), 'cfg4 pack %.4f verified %s %s' % (c4['pack']['hbm_frac'], c3.get('verified'), c4.get('verified')))
"
  done
done
