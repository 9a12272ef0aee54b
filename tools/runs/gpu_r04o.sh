# Round 4, call O: per-size u32 SORT tile (2^14 merge-level tiles from 2^25
# where they add no pass, 2^15 network tiles otherwise) -- the merge/parity/
# baseline-config tests, then the tile knob A/B at 2^25, 2^26, 2^29, 2^30.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04o"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
for L in 25 26 29 30; do
  RUNS="t14_$L||MISORT_SORT_TILE_U32=14;t15_$L||MISORT_SORT_TILE_U32=15" BENCH_ARGS="--logn $L" STEPS=20 OUTDIR=r04o bash tools/gpu_envab.sh || exit $?
done
