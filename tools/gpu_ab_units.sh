set -o pipefail
mkdir -p gpurun_out/abw
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_pack.py tests/test_gpu_decoder.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/abw/pytest.log 2>&1 || { tail -30 gpurun_out/abw/pytest.log; exit 1; }
tail -1 gpurun_out/abw/pytest.log
for w in 2 3 4 2 3 4; do
  timeout -k 10 300 python tools/ab_pack.py tools/ab/lib_w$w.so cfg3,cfg4,u64k > gpurun_out/abw/w$w.json 2> gpurun_out/abw/w$w.err || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/abw/w$w.json'))
print('w=$w', ' '.join('%s enc %.4f gat %.4f'%(c, max(r['enc_frac'] for r in d[c]['lib']), max(r['gat_frac'] for r in d[c]['lib'])) for c in d))
"
done
