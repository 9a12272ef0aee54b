# rocprofv3 kernel stats of one bench config (env passed through), summary printed.
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd /tmp && export TMPDIR=/tmp
TAG=${TAG:-p}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$TAG" -o $TAG --output-format csv -- python3 "$R/bench.py" --logn ${LOGN:-30} --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof_$TAG.log" 2>&1 || { tail -5 "$R/gpurun_out/rocprof_$TAG.log"; exit 1; }
python3 - <<'PY'
import csv, os, re
R = os.environ["GRAFT_REPO_ROOT"]; tag = os.environ.get("TAG", "p")
for r in csv.DictReader(open(f"{R}/gpurun_out/prof_{tag}/{tag}_kernel_stats.csv")):
    n = re.sub(r"misort::\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
    print(f'{n[:70]:70s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
