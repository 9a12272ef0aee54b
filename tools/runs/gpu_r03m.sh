# Round 3, call M: the whole GPU suite and the default bench line (HEAD), then
# small merge tiles A/B (base vs rst0) and kernel stats at 2^24 / 2^26 u32.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03m"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err" || { echo bench failed; tail -5 "$O/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('bench', round(d['value'],2), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],3), 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])"
SKIP_TESTS=1 VARIANTS="base rst0" DTYPES="u32 u64" LOGNS="24 26" ROUNDS=2 OUTDIR=r03m/ab bash tools/gpu_abv.sh || exit $?
OUTDIR=r03m/small TAGS="u32_24:--logn=24 u32_26:--logn=26" bash tools/gpu_prof2.sh
