# Round 5: cost of the bench's kernel-carried timing events inside the timed region: default (stop events,
# ticks), MISORT_PROF_BIND=1 (start + stop on the recorded launch), and no events (--no-kernel-events).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
for a in "--logn 24" "--logn 30"; do
  RUNS="bind2||;bind1||MISORT_PROF_BIND=1" BENCH_ARGS="$a" STEPS=20 OUTDIR=ev bash tools/runs/gpu_envab.sh || exit $?
  RUNS="noev||" BENCH_ARGS="$a --no-kernel-events" STEPS=20 OUTDIR=ev bash tools/runs/gpu_envab.sh || exit $?
done
