# Round 3, call P: merge-level tests, then MISORT_PLAN_SCAN A/B (0: k_scan_totals,
# 1: block totals scanned inside the fused descriptor kernel).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03p"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
for args in "--logn=24" "--logn=25" "--logn=22" "--logn=24 --dtype=u64" ; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=100; [ -z "$args" ] && steps=10
  echo "== $args"
  STEPS=$steps OUTDIR=r03p/$tag BENCH_ARGS="$args" RUNS="s0||MISORT_PLAN_SCAN=0;s1||MISORT_PLAN_SCAN=1" bash tools/gpu_envab.sh || exit $?
done
