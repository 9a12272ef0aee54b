# Round 5: k_bounds reading the whole fence window (MISORT_BOUNDS_WIN bytes) vs the interpolated line probe.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
for a in "--logn 30" "--logn 29" "--logn 26" "--dtype u64 --logn 29" "--dtype u64 --logn 28"; do
  RUNS="base||;win256|$V/libmisort_win256.so|;win512|$V/libmisort_win512.so|;win1024|$V/libmisort_win1024.so|" BENCH_ARGS="$a" STEPS=20 OUTDIR=win bash tools/runs/gpu_envab.sh || exit $?
done
