# Round 3, call W: u32 SORT tile of 2^14 keys (lt14 variant: 512 lanes, two
# workgroups per CU, 16 merge levels after it) vs 2^15 (base), with the
# planner's default pass widths and the alternatives; then timelines and the
# N = 2 / 4 shared-GPU bench lines (call V's script).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants/libmisort_lt14.so
for args in "" "--logn=28" "--logn=24"; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=10; [ "$args" = "--logn=28" ] && steps=30; [ "$args" = "--logn=24" ] && steps=100
  echo "== $args"
  STEPS=$steps OUTDIR=r03w/$tag BENCH_ARGS="$args" RUNS="b15||;b15m4||MISORT_MULTIWAY=4;l14|$V|;l14m3|$V|MISORT_MULTIWAY=3" bash tools/gpu_envab.sh || exit $?
done
bash tools/runs/gpu_r03v.sh
