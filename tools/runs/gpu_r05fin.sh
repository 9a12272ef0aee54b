# Round 5 end-of-round record, part 1: smoke, the whole GPU suite, the default bench (reference CPU
# baseline included) and the other configs' benches.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r05fin}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?; echo "smoke rc $rc: $(tail -1 $O/smoke.log)"; fatal $rc smoke; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/gpu_suite.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/gpu_suite.log)"; fatal $rc pytest; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/gpu_suite.log" | head; exit $rc; }
timeout -k 10 400 python3 -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"; rc=$?; echo "bench default rc $rc"; fatal $rc bench; [ $rc -ne 0 ] && exit $rc
for a in "--logn 28" "--logn 24" "--dtype u64 --logn 29" "--dtype f64 --logn 29" "--logn 27"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$n.json" 2> "$O/bench_$n.err"; rc=$?; fatal $rc bench; [ $rc -ne 0 ] && exit $rc
done
python3 - "$O" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(sys.argv[1] + "/bench_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(os.path.basename(f), round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms err", d["check_errors"],
          "roof", r.get("kernel"), round(r.get("frac", 0), 3), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
