# Re-measure the planner's cost table (u32 at 2^30 and 2^28, every shape incl. wide passes).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for ln in 30 28; do
  timeout -k 10 500 python -u tools/pass_costs.py --logn $ln --reps 4 > gpurun_out/pc_u32_$ln.json 2> gpurun_out/pc_u32_$ln.log; rc=$?; tail -1 gpurun_out/pc_u32_$ln.log; [ $rc -eq 0 ] || exit $rc
done
