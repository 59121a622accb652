cd $GRAFT_REPO_ROOT
B="g++ -std=c++17 -O1 -g -Wall -Wextra -Werror -I include tests/cpp/thread_exit_check.cpp -L kuma_amd/lib -lkmws_gpu -L oracle -lkmws_oracle -lpthread -Wl,-rpath,$PWD/kuma_amd/lib -Wl,-rpath,$PWD/oracle"
$B -o /tmp/tec || exit 1
g++ -std=c++17 -O1 -pthread tools/thread_churn.cpp -o /tmp/churn || exit 1
echo "== churn (no GPU)"; timeout -k 10 120 /tmp/churn 1000 > gpurun_out/r06c_churn.log 2>&1; echo rc=$? >> gpurun_out/r06c_churn.log
echo "== loop only"; timeout -k 10 120 /tmp/tec 10 8 0 loop > gpurun_out/r06c_loop.log 2>&1; rc=$?; echo rc=$rc >> gpurun_out/r06c_loop.log
[ $rc -eq 0 ] || exit 0
echo "== raw only"; timeout -k 10 120 /tmp/tec 10 8 0 raw > gpurun_out/r06c_raw.log 2>&1; rc=$?; echo rc=$rc >> gpurun_out/r06c_raw.log
[ $rc -eq 0 ] || exit 0
echo "== maskers only"; timeout -k 10 120 /tmp/tec 3 0 8 both > gpurun_out/r06c_maskers.log 2>&1; echo rc=$? >> gpurun_out/r06c_maskers.log
