# Round 3, call A: the RCCL transport at BASELINE sizes and on its failure
# paths (tests/test_gpu_rccl_large.py), then the default bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03a}"; mkdir -p "$O"; cd "$R"
timeout 1100 bash -c 'while sleep 30; do date; done' >> "$O/heartbeat" 2>&1 &
HB=$!
timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_gpu_rccl_large.py} -v --timeout 400 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?
echo "pytest rc $rc"; tail -20 "$O/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then kill $HB; exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err"
rc=$?
kill $HB
cat "$O/bench.json"; tail -3 "$O/bench.err"
exit $rc
