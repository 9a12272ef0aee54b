# Round 5: tests and benches after the per-build 16-way chunk capacity (10880 with 128-key fences).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/cap2"; mkdir -p "$O"; cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
for a in "--logn 30" "--logn 28" "--logn 27"; do
  RUNS="head||" BENCH_ARGS="$a" STEPS=20 OUTDIR=cap2 bash tools/runs/gpu_envab.sh || exit $?
done
