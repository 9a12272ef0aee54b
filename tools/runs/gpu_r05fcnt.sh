# Round 5: k_fence_counts lanes per block (MISORT_FC_NT) and fences in flight (MISORT_FC_BATCH), 2^30 / 2^28 u32, 2^29 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
for a in "--logn 30" "--logn 28" "--dtype u64 --logn 29"; do
  RUNS="base||;fc512|$V/libmisort_fc512.so|;fc1024|$V/libmisort_fc1024.so|;fc1024b4|$V/libmisort_fc1024b4.so|;fcb16|$V/libmisort_fcb16.so|" BENCH_ARGS="$a" STEPS=20 OUTDIR=fcnt bash tools/runs/gpu_envab.sh || exit $?
done
