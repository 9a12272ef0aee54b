# rocprofv3 kernel stats of a merge-level sort (partition vs merge kernel split).
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd /tmp && export TMPDIR=/tmp
export MISORT_MERGE_FROM=${MFROM:-15}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_runs" -o runs --output-format csv -- python3 "$R/bench.py" --logn ${LOGN:-30} --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof_runs.log" 2>&1 || { tail -5 "$R/gpurun_out/rocprof_runs.log"; exit 1; }
python3 - <<'PY'
import csv, os, re
R = os.environ["GRAFT_REPO_ROOT"]
for r in csv.DictReader(open(f"{R}/gpurun_out/prof_runs/runs_kernel_stats.csv")):
    n = re.sub(r"misort::\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
    print(f'{n[:70]:70s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
