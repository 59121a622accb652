cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06aj; mkdir -p $OUT
for g in 1 2 4 8 16; do
  timeout -k 10 300 python3 bench.py --config e2e --gpus 1 --e2e-gib $g --steps 5 --warmup 2 > $OUT/e2e_$g.json || exit 1
done
