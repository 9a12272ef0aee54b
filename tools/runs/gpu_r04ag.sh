# Round 4, call AG: u64 in-LDS level outputs as one 8-byte write per key
# (p64off) vs 16-byte pair writes (the default) -- tests, then u64 A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="p64off" ROUNDS=0 OUTDIR=r04ag bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base p64off" DTYPES="u64" LOGNS="29 26" ROUNDS=2 OUTDIR=r04ag bash tools/gpu_abv.sh
