# Round 3, call AA: u32 SORT tile with its in-wave levels up to 7 / 8 (base) / 9.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
SKIP_TESTS=1 VARIANTS="base wl7 wl9" DTYPES="u32" LOGNS="30 24" ROUNDS=2 OUTDIR=r03aa bash tools/gpu_abv.sh
