# End-of-round record: smoke, the whole -m gpu suite, the default bench line (reference CPU baseline
# included) and the rocprofv3 kernel stats of the same bench command on the same box, the other configs'
# bench lines, and the per-GPU work of configs 4 and 5 at P = 8 (tools/rank_work_probe.py under rocprofv3).
#   PARTS="smoke suite bench prof configs rankwork"   the parts to run (default: all, in this order)
#   OUTDIR=name                                      results under gpurun_out/NAME
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R="$(cd "$(dirname "$0")/../.." && pwd)"
O="$R/gpurun_out/${OUTDIR:-final}"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
P=" ${PARTS:-smoke suite bench prof configs rankwork} "
fatal() { case "$1" in 0) ;; *) echo "rc $1 in $2: stopping"; exit "$1";; esac; }
line() {  # bench JSON file -> one summary line
  python3 - "$1" <<'PY'
import json, os, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline", {})
print(os.path.basename(sys.argv[1]), round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms err", d["check_errors"],
      "roof", r.get("kernel"), round(r.get("frac", 0), 3), round(r.get("avg_launch_us", 0), 1), "us",
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
}
if [[ $P == *" smoke "* ]]; then
  timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?
  echo "smoke rc $rc: $(tail -1 "$O/smoke.log")"; fatal $rc smoke
fi
if [[ $P == *" suite "* ]]; then
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/gpu_suite.log" 2>&1; rc=$?
  echo "pytest rc $rc: $(tail -1 "$O/gpu_suite.log")"; [ $rc -ne 0 ] && grep -E "FAILED|Error" "$O/gpu_suite.log" | head; fatal $rc pytest
fi
if [[ $P == *" bench "* ]]; then
  timeout -k 10 400 python3 -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"; rc=$?
  [ $rc -ne 0 ] && tail -5 "$O/bench_default.err"; fatal $rc bench; line "$O/bench_default.json"
fi
if [[ $P == *" prof "* ]]; then
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_u32_30" -o u32_30 --output-format csv -- \
    python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof_bench.err"); rc=$?
  [ $rc -ne 0 ] && tail -5 "$O/prof_bench.err"; fatal $rc rocprof
  find "$O/prof_u32_30" -name "*kernel_stats.csv" -exec cp {} "$O/u32_30_kernel_stats.csv" \;
  find "$O/prof_u32_30" -name "*.db" -delete
  python3 - "$O/u32_30_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print("rocprof", r["Name"].split("(")[0][-55:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
fi
if [[ $P == *" configs "* ]]; then
  for a in "--logn 28" "--logn 27" "--logn 24" "--dtype u64 --logn 29" "--dtype f64 --logn 29"; do
    n=$(echo $a | tr -d ' -')
    timeout -k 10 200 python3 -u bench.py $a --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$n.json" 2> "$O/bench_$n.err"; rc=$?
    [ $rc -ne 0 ] && tail -5 "$O/bench_$n.err"; fatal $rc "bench $a"; line "$O/bench_$n.json"
  done
fi
if [[ $P == *" rankwork "* ]]; then
  for c in "c4:--logn 30 --p 8 --dtype u32" "c5:--n 536870909 --p 8 --dtype u64"; do
    k=${c%%:*}; a=${c#*:}
    # timings from a run without the profiler (its kernel trace adds ~4 us per dispatch),
    # the kernel breakdown from a second run under rocprofv3
    timeout -k 10 300 python3 tools/rank_work_probe.py $a > "$O/rw_$k.json" 2> "$O/rw_$k.err"; rc=$?
    [ $rc -ne 0 ] && tail -5 "$O/rw_$k.err"; fatal $rc "rank work $k"
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_$k" -o rw --output-format csv -- \
      python3 "$R/tools/rank_work_probe.py" $a > "$O/rw_${k}_prof.json" 2> "$O/rw_${k}_prof.err"); rc=$?
    [ $rc -ne 0 ] && tail -5 "$O/rw_${k}_prof.err"; fatal $rc "rank work $k (rocprofv3)"
    find "$O/rw_$k" -name "*.db" -delete
    python3 tools/rank_work_summary.py "$O/rw_$k" "$O/rw_$k.json" > "$O/rank_work_config${k#c}_p8.txt"; fatal $? "summary $k"
    grep -E "device work|stage 0" "$O/rank_work_config${k#c}_p8.txt"
  done
fi
echo done
