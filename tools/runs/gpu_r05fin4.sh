# Round 5 end-of-round record, part 4: the default bench line and the rocprofv3 kernel stats of the same
# bench command on the same box, so the roofline kernel's average duration can be checked against both.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r05fin4}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 -u "$R/bench.py" > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -5 "$O/bench_default.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_u32_30" -o u32_30 --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/prof_bench.json" 2> "$O/prof_bench.err" || { tail -5 "$O/prof_bench.err"; exit 1; }
python3 - "$O" <<'PY'
import csv, json, sys
O = sys.argv[1]
d = json.loads(open(O + "/bench_default.json").read().strip().splitlines()[-1])
print("bench", round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms; k_mergek events avg", round(d["roofline"]["avg_launch_us"], 1), "us")
for r in csv.DictReader(open(O + "/prof_u32_30/u32_30_kernel_stats.csv")):
    if "k_mergek<unsigned int, 4" in r["Name"] or "k_sort_u32" in r["Name"]:
        print("rocprof", r["Name"].split("(")[0][-45:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
