# Round 4, call F: larger merge chunks for the 16-way passes -- IT 22 / 24
# outputs per lane (CAP 10752 / 11776 keys, 3 workgroups per CU) against the
# default (IT 18, CAP 8192, 4 per CU); tests of both variants.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="it22 it24" ROUNDS=0 OUTDIR=r04f bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base it22 it24" DTYPES=u32 LOGNS="30 28 27 24" ROUNDS=2 OUTDIR=r04f bash tools/gpu_abv.sh
