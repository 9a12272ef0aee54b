# Round 4, call B: the ds_read2 merge chain as the u32 default -- merge and
# full-size parity tests, chain A/B (base = ch1 vs ch0; u64 ch1), and the
# 8- vs 16-way u32 plan at 2^26..2^31 (verdict r03 item 3).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04b"; mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base ch0" DTYPES=u32 LOGNS="30 27" ROUNDS=2 OUTDIR=r04b/chain bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base u64ch1" DTYPES=u64 LOGNS="29 26" ROUNDS=2 OUTDIR=r04b/chain bash tools/gpu_abv.sh || exit $?
for L in 26 27 28 29 30 31; do
  RUNS="w8||MISORT_MULTIWAY=3;w16||MISORT_MULTIWAY=4" BENCH_ARGS="--logn $L" STEPS=10 OUTDIR=r04b/mw$L bash tools/gpu_envab.sh || exit $?
done
