# Round 4, call K: zero words before every LDS sequence (the phased search drops
# its compare with lo) against zw0 --
# merge/parity tests, A/B (u32 and u64), SQ probe modes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04k"; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base zw0" DTYPES=u32 LOGNS="30 28 24" ROUNDS=2 OUTDIR=r04k bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base zw0" DTYPES=u64 LOGNS="29" ROUNDS=2 OUTDIR=r04k bash tools/gpu_abv.sh &&
MISORT_MK_PROBE=1 OUTDIR=r04k/sq_probe bash tools/gpu_sq2.sh > "$O/sq_probe.txt" && echo "sq ok"
