#!/bin/bash
# Pack/gather copy kernel: blocks dealt over KMWS_COPY_SPLIT parts, A/B per value
# (one process each; tools/ab_pack.py with the product library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abs
mkdir -p "$OUT"
export TMPDIR=/tmp
KMWS_COPY_SPLIT=1016 timeout -k 10 300 python -u -m pytest tests/test_gpu_pack.py tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
for k in ${1:-1 2 8 16}; do
  KMWS_COPY_SPLIT=$k timeout -k 10 300 python tools/ab_pack.py kuma_amd/lib/libkmws_gpu.so cfg3,cfg4,u64k > "$OUT/s$k.json" 2> "$OUT/s$k.err" || exit 1
  python -c "
import json
d=json.load(open('$OUT/s$k.json'))
print('split=$k', ' '.join('%s enc %.4f gat %.4f'%(c, max(r['enc_frac'] for r in d[c]['lib']), max(r['gat_frac'] for r in d[c]['lib'])) for c in d))
"
done
done
