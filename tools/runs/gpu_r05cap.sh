# Round 5: 16-way chunk capacity 10880 keys (the largest the 22-output level layout holds) vs 10752.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
for a in "--logn 30" "--logn 28" "--logn 26" "--dtype u64 --logn 29"; do
  RUNS="base||;cap10880|$V/libmisort_cap10880.so|" BENCH_ARGS="$a" STEPS=20 OUTDIR=cap bash tools/runs/gpu_envab.sh || exit $?
done
