# Round 4, call AB: k_mergek stages even-shift chunks with pair writes (the
# default build) vs one write per key (nops) -- merge/parity tests, then A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04ab"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base nops" DTYPES="u32 u64" LOGNS="30 28" ROUNDS=2 OUTDIR=r04ab bash tools/gpu_abv.sh
