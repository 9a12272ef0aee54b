# Round 4, call B: the ds_read2 merge chain as the u32 default -- merge and
# full-size parity tests, chain A/B (base = ch1 vs ch0 vs ch3 aligned pairs;
# u64 ch1/ch3).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O="$R/gpurun_out/r04b"; mkdir -p "$O"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="ch3 ch3it17" ROUNDS=0 OUTDIR=r04b/chain bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base ch0 ch3 ch3it17" DTYPES=u32 LOGNS="30 27" ROUNDS=2 OUTDIR=r04b/chain bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base u64ch1 ch3" DTYPES=u64 LOGNS="29 26" ROUNDS=2 OUTDIR=r04b/chain bash tools/gpu_abv.sh || exit $?
