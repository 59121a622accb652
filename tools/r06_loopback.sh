cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06an; mkdir -p $OUT
g++ -std=c++17 -O2 -I include tests/cpp/loopback_cfg1.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread -Wl,-rpath,$PWD/oracle -o $OUT/lb || exit 1
for L in kuma_amd/lib build_variants/resident_one_hp_stream build_variants/resident_writeback_release; do
  for c in 4 8; do
    for m in adapter replay_adapter; do
      LD_LIBRARY_PATH=$PWD/$L timeout -k 10 120 $OUT/lb $m 10 16 0 0 $c > $OUT/t.json || exit 1
      sed "s|^{|{\"lib\": \"$L\", |" $OUT/t.json >> $OUT/loopback_ab.jsonl
    done
  done
done
