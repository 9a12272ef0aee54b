# Round 3, call D: is the box slow before the failure tests (bench first),
# the failure tests with MISORT_TRACE, and the bench again after them.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03d}"; mkdir -p "$O"; cd "$R"
timeout 1150 bash -c 'while sleep 30; do date; done' >> "$O/heartbeat" 2>&1 &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
rocm-smi --showclocks --showpower --showuse > "$O/smi_before.txt" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_before.json" 2> "$O/bench_before.err" || { echo bench failed; tail -5 "$O/bench_before.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_before.json'));print('before', d['value'], d['kernels']['tile_sort']['avg_launch_us'], d['kernels']['run_mergek_kernel']['avg_launch_us'])"
MISORT_TEST_LOGDIR="$O" timeout -k 10 330 python -u -m pytest tests/test_gpu_rccl_large.py -k failed_peer -v --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -4 "$O/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ps -eo pid,stat,etime,cmd | grep -v grep | grep -E "python|torchrun" > "$O/ps_after.txt" || true
rocm-smi --showpids --showuse > "$O/smi_after.txt" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_after.json" 2> "$O/bench_after.err" || { echo bench failed; tail -5 "$O/bench_after.err"; exit 1; }
python -c "import json;d=json.load(open('$O/bench_after.json'));print('after', d['value'], d['kernels']['tile_sort']['avg_launch_us'], d['kernels']['run_mergek_kernel']['avg_launch_us'])"
