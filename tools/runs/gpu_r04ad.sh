# Round 4, call AD: the u32 SORT tile choice re-measured at HEAD (2^14 merge-
# level tile vs 2^15 network tile, MISORT_SORT_TILE_U32) around the rule's
# threshold (2^22 .. 2^25) and at 2^27.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
for L in ${LS:-22 23 24 25 27}; do
  RUNS="t14_$L||MISORT_SORT_TILE_U32=14;t15_$L||MISORT_SORT_TILE_U32=15" BENCH_ARGS="--logn $L" STEPS=30 OUTDIR=r04ad bash tools/gpu_envab.sh || exit $?
done
