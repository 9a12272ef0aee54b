# Re-measure the planner's u64 cost table (the 2^13-key u64 tiles) at 2^29 and 2^26 keys.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for ln in 29 26; do
  timeout -k 10 500 python -u tools/pass_costs.py --dtype u64 --logn $ln --reps 4 > gpurun_out/pc_u64_$ln.json 2> gpurun_out/pc_u64_$ln.log; rc=$?; tail -1 gpurun_out/pc_u64_$ln.log; [ $rc -eq 0 ] || exit $rc
done
