# Round 4, call AC: the u32 merge-level SORT tile with an even output count per
# lane (34: aligned pair writes at every level; the default build) vs the odd
# layout (odd33 -> 35 outputs per lane) -- merge/parity tests, then A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04ac"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base odd33" DTYPES="u32" LOGNS="30 28 26" ROUNDS=2 OUTDIR=r04ac bash tools/gpu_abv.sh
