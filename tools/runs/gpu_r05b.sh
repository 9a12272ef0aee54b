set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r05b"; mkdir -p "$O"; cd "$R"
MISORT_TEST_LOGDIR="$O" timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rccl_large.py -k "dead_user_stream" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
echo "rc $rc"; tail -3 "$O/pytest.log"; tail -30 "$O"/rccl_P2_dead_user_stream.err
