# Round 4, call AA: the merge-level u32 SORT tile on the persistent grid with
# the next tile's loads in flight (mpers: 128 VGPRs + 16 spilled) vs one tile
# per workgroup (the default).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TESTS="tests/test_gpu_parity.py" VARIANTS="mpers" ROUNDS=0 OUTDIR=r04aa bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base mpers" DTYPES=u32 LOGNS="30 28" ROUNDS=2 OUTDIR=r04aa bash tools/gpu_abv.sh
