# Round 4, call V: u64 chunk shapes (c64a: CAP 8832 at 18 outputs per lane;
# c64b: CAP 9216 at 20) -- tests of both, then u64 2^29 / 2^26 A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04v"; mkdir -p "$O"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="c64a c64b" ROUNDS=0 OUTDIR=r04v bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base c64a c64b" DTYPES=u64 LOGNS="29 26" ROUNDS=2 OUTDIR=r04v bash tools/gpu_abv.sh
