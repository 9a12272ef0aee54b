# (second run, r04q2: the merge levels barrier on LDS only -- lds_barrier -- so the prefetch stays in flight)
# Round 4, call Q: persistent k_mergek with register prefetch of the next chunk
# (MISORT_MK_PERSIST=1) -- merge/parity tests under it, then A/B benches.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04q2"; mkdir -p "$O"; cd "$R"
MISORT_MK_PERSIST=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for a in "--logn 30" "--logn 28" "--dtype u64 --logn 29"; do
  n=$(echo $a | tr -d ' -')
  RUNS="p0_$n||MISORT_MK_PERSIST=0;p1_$n||MISORT_MK_PERSIST=1;p2_$n||MISORT_MK_PERSIST=2" BENCH_ARGS="$a" STEPS=20 OUTDIR=r04q2 bash tools/gpu_envab.sh || exit $?
done
