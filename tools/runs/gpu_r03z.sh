# Round 3, call Z: k_mergek chunks in one contiguous range per XCD (xcd
# variant) vs chunk = block (base): merge tests on the variant, bench A/B.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
VARIANTS="base xcd" TESTS="tests/test_gpu_runs.py" DTYPES="u32 u64" LOGNS="30 28" ROUNDS=2 OUTDIR=r03z bash tools/gpu_abv.sh
