# rocprofv3 kernel stats of bench.py under several knob settings (one call).
#   VARIANTS="NAME=ENV1=v1,ENV2=v2 ..." bash tools/gpu_profab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"; cd /tmp && export TMPDIR=/tmp
for v in $VARIANTS; do
  name=${v%%=*}; envs=${v#*=}
  export $(echo "$envs" | tr ',' ' ')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$name" -o $name --output-format csv -- python3 "$R/bench.py" --logn ${LOGN:-30} --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof_$name.log" 2>&1 || { tail -5 "$R/gpurun_out/rocprof_$name.log"; exit 1; }
  unset $(echo "$envs" | tr ',' ' ' | sed 's/=[^ ]*//g')
  echo "== $name: $(grep -o '"value": [0-9.]*' "$R/gpurun_out/rocprof_$name.log" | head -1)"
  NAME=$name python3 - <<'PY'
import csv, os, re
R = os.environ["GRAFT_REPO_ROOT"]; tag = os.environ["NAME"]
for r in csv.DictReader(open(f"{R}/gpurun_out/prof_{tag}/{tag}_kernel_stats.csv")):
    n = re.sub(r"misort::\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
    if "k_stream" not in n: continue
    print(f'{n[:70]:70s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
done
