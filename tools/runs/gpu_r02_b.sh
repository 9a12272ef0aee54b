# 4-way merge passes: merge-level parity, full-size SHA configs, psort P>1, bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r02b"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_baseline_configs.py tests/test_gpu_psort_bin.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"
grep -E "FAILED|passed|failed" "$O/pytest.log" | tail -15; fatal $rc pytest
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$O/bench_n1.json" 2> "$O/bench_n1.err"; rc=$?; echo "bench rc $rc"
tail -c 1500 "$O/bench_n1.json"; fatal $rc bench
