# Round 4, call Y: the HEAD measurement set (call X's script), then in-wave
# levels up to 9 / 10 (MISORT_WAVE_LEVELS variants) and lane-contiguous SORT
# loads (MISORT_SORT_DIRECT) against the defaults.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/runs/gpu_r04x.sh || exit $?
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="wl10 direct" ROUNDS=0 OUTDIR=r04y bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base wl9 wl10 direct" DTYPES=u32 LOGNS="30 28 24" ROUNDS=2 OUTDIR=r04y bash tools/gpu_abv.sh
