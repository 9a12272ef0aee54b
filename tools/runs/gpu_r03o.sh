# Round 3, call O: merge-level tests, then MISORT_PLAN_FUSE A/B (0: k_bounds +
# k_chunk_desc, 1: bounds inside k_chunk_desc for small sorts, 2: always).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03o"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
for args in "--logn=24" "--logn=26" "--logn=24 --dtype=u64" "" ; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=100; [ -z "$args" ] && steps=10
  echo "== $args"
  STEPS=$steps OUTDIR=r03o/$tag BENCH_ARGS="$args" RUNS="f0||MISORT_PLAN_FUSE=0;f1||MISORT_PLAN_FUSE=1;f2||MISORT_PLAN_FUSE=2" bash tools/gpu_envab.sh || exit $?
done
