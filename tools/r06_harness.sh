cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r06ag; mkdir -p $OUT
hipcc -std=c++17 -O2 -I include tools/grid_interference.cpp -L kuma_amd/lib -lkmws_gpu -lpthread -o $OUT/gi || exit 1
export LD_LIBRARY_PATH=$PWD/build_variants/resident_second_hp_stream
run() { tag=$1; m=$2; shift 2; env "$@" timeout -k 10 120 $OUT/gi 1048576 20 4 16 $m > $OUT/$tag.json; rc=$?; [ $rc -le 1 ] || exit 1; }
run one1 one X=1 && run one2 one X=1 && run one3 one X=1 && run res1 resident X=1
