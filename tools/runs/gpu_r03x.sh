# Round 3, final call: the whole GPU suite, smoke(), the default bench line,
# and the rocprofv3 kernel stats of the same bench command.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03x}"; mkdir -p "$O"; cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=20 --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value'],2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o bench --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo rocprof failed; tail -5 "$O/prof.log"; exit 1; }
echo done
