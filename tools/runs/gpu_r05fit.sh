# Round 5: LDS fence merge (k_fence_merge) outputs per lane 16 vs 8.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
for a in "--logn 30" "--logn 28" "--dtype u64 --logn 29"; do
  RUNS="base||;fit16|$V/libmisort_fit16.so|" BENCH_ARGS="$a" STEPS=20 OUTDIR=fit bash tools/runs/gpu_envab.sh || exit $?
done
