# Round 4, call W: u32 chunk capacities (c32a: 16-way CAP 10880, the largest
# the 512 x 22 layout fits; c32b: 8-way CAP 8960) -- tests, then A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04w"; mkdir -p "$O"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="c32a c32b" ROUNDS=0 OUTDIR=r04w bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base c32a c32b" DTYPES=u32 LOGNS="30 28 24" ROUNDS=2 OUTDIR=r04w bash tools/gpu_abv.sh
