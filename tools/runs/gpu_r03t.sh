# Round 3, call T: per-(chunk, run) u32 fence counters (base) vs packed u64
# fields (fc64): merge tests on base, then the bench A/B (after an init-stride fix).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03t"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
SKIP_TESTS=1 VARIANTS="base fc64" DTYPES="u32 u64" LOGNS="30 26" ROUNDS=2 OUTDIR=r03t/ab bash tools/gpu_abv.sh
