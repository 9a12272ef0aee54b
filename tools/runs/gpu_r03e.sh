# Round 3, call E: the whole GPU suite with durations, then the default bench line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03e}"; mkdir -p "$O"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --durations=40 --timeout 300 --timeout-method thread ${PYARGS} > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc"; tail -60 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS} > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
