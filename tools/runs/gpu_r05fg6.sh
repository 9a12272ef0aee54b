# Round 5: 64-key fences for large sorts (runsk_fg6.hip) -- merge/parity/baseline-config tests, then A/B
# against 128-key fences everywhere (MISORT_FENCE_FG6_MIN=0) at 2^30 / 2^29 / 2^28 u32 and 2^29 / 2^28 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/fg6"; mkdir -p "$O"; cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
for a in "--logn 30" "--logn 29" "--logn 28" "--dtype u64 --logn 29" "--dtype u64 --logn 28"; do
  n=$(echo $a | tr -d ' -')
  RUNS="fg7_$n||MISORT_FENCE_FG6_MIN=0 MISORT_FENCE_FG6_MIN_U64=0;fg6_$n||MISORT_FENCE_FG6_MIN=20 MISORT_FENCE_FG6_MIN_U64=20" BENCH_ARGS="$a" STEPS=20 OUTDIR=fg6 bash tools/runs/gpu_envab.sh || exit $?
done
