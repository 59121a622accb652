set -e
cd $GRAFT_REPO_ROOT
B="g++ -std=c++17 -O1 -g -Wall -Wextra -Werror -I include tests/cpp/thread_exit_check.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread -Wl,-rpath,$PWD/kuma_amd/lib -Wl,-rpath,$PWD/oracle"
$B -fsanitize=address -fno-omit-frame-pointer -o /tmp/tec_asan
$B -o /tmp/tec
echo "== asan both"; ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0 timeout -k 10 120 /tmp/tec_asan 6 8 8 both > gpurun_out/r06b_asan.log 2>&1; echo rc=$? >> gpurun_out/r06b_asan.log
echo "== loop only"; timeout -k 10 120 /tmp/tec 10 8 0 loop > gpurun_out/r06b_loop.log 2>&1; echo rc=$? >> gpurun_out/r06b_loop.log
echo "== raw only"; timeout -k 10 120 /tmp/tec 10 8 0 raw > gpurun_out/r06b_raw.log 2>&1; echo rc=$? >> gpurun_out/r06b_raw.log
