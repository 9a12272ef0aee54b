# Round 5: planning shape knobs re-checked under 64-key fences at 2^30 u32 (env A/B, one box).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
RUNS="base||;dc4||MISORT_DESC16_MIN=1073741824;slices||MISORT_FC_SLICES_MAX=1000000;fuse2||MISORT_PLAN_FUSE=2" BENCH_ARGS="--logn 30" STEPS=20 OUTDIR=penv bash tools/runs/gpu_envab.sh || exit $?
