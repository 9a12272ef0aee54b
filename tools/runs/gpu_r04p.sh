# Round 4, call P: phase costs of the 2^14 merge-level SORT tile (variants
# stopping after the load / register+DPP levels / LDS levels / relayout).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04p"; mkdir -p "$O"; cd "$R"
for rep in 1 2; do
  for v in base stop1 stop2 stop3 stop4; do
    if [ $v = base ]; then unset MISORT_LIBRARY; else export MISORT_LIBRARY="$R/parallel-computing-mpi_amd/lib/variants/libmisort_$v.so"; fi
    timeout -k 10 120 python3 tools/sort_levels_probe.py >> "$O/probe.log" 2>> "$O/probe.err" || exit $?
  done
  unset MISORT_LIBRARY
  TILE=15 timeout -k 10 120 python3 tools/sort_levels_probe.py >> "$O/probe.log" 2>> "$O/probe.err" || exit $?
done
cat "$O/probe.log"
