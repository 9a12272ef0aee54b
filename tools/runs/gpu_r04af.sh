# Round 4, call AF: u64 pass widths re-measured at HEAD (MISORT_MULTIWAY_U64 =
# 4, the default, vs 3) at 2^29, 2^26, 2^24.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
for L in 29 26 24; do
  RUNS="w4_$L||MISORT_MULTIWAY_U64=4;w3_$L||MISORT_MULTIWAY_U64=3" BENCH_ARGS="--dtype u64 --logn $L" STEPS=20 OUTDIR=r04af bash tools/gpu_envab.sh || exit $?
done
