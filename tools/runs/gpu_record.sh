# Record run: GPU tests, bench (with CPU baseline), rocprofv3 kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_rec.log 2>&1; rc=$?; tail -1 gpurun_out/bench_rec.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_rec" -o rec --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof_rec.log" 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv, os
R = os.environ["GRAFT_REPO_ROOT"]
for r in csv.DictReader(open(f"{R}/gpurun_out/prof_rec/rec_kernel_stats.csv")):
    print(r["Name"][:100], r["Calls"], round(float(r["AverageNs"])/1e3, 1), "us", r["Percentage"])
PY
