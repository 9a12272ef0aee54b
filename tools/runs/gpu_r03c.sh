# Round 3, call C: failure-detection tests, the bench line, then the HEAD
# profile set (kernel stats + HBM traffic per pass) under gpurun_out/r03c.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03c}"; mkdir -p "$O"; cd "$R"
timeout 1150 bash -c 'while sleep 30; do date; done' >> "$O/heartbeat" 2>&1 &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -z "$SKIP_TESTS" ]; then
  MISORT_TEST_LOGDIR="$O" NCCL_DEBUG=WARN timeout -k 10 330 python -u -m pytest ${TESTS:-tests/test_gpu_rccl_large.py -k failed_peer} -v --timeout 200 --timeout-method thread > "$O/pytest.log" 2>&1
  rc=$?; echo "pytest rc $rc"; tail -8 "$O/pytest.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
[ -n "$SKIP_PROF" ] && exit 0
OUTDIR=${OUTDIR:-r03c}/prof bash tools/runs/gpu_r02_prof.sh > "$O/prof.txt" 2>&1 || { echo prof failed; tail -20 "$O/prof.txt"; exit 1; }
cat "$O/prof.txt" | head -120
