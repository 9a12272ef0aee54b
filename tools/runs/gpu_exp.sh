# Engine experiments: grid shape + per-instantiation rocprof breakdown.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for GM in 1 2 0; do
  MISORT_GRID_MULT=$GM timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/exp_gm$GM.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/exp_gm$GM.log').read().strip().splitlines()[-1]);print('GM=$GM', round(d['value'],2), d['check_errors'], {k:(v['launches_per_step'], round(v['ms_per_step'],2), round(v['achieved_GBs'])) for k,v in d['kernels'].items()})"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof2" -o r2 --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof2.log" 2>&1 || exit 1
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
for r in csv.DictReader(open(f"{R}/gpurun_out/prof2/r2_kernel_stats.csv")):
    print(r["Name"][:100], r["Calls"], round(float(r["AverageNs"])/1e3, 1), "us", r["Percentage"])
PY
