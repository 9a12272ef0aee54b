# Session-2: coalesced fence counts -- merge-pass/parity tests, bench 2^30 u32 and 2^29 u64, rocprof stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2i}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 "$O/pytest.log"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
for spec in "30 u32" "29 u64"; do
  set -- $spec
  timeout -k 10 200 python3 -u bench.py --logn $1 --dtype $2 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_$2_$1.json" 2> "$O/bench_$2_$1.err"; rc=$?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), round(d['ms_per_step'],3))" "$O/bench_$2_$1.json"
  fatal $rc "bench $spec"; [ $rc -ne 0 ] && exit $rc
done
OUTDIR=${OUTDIR:-s2i}/stats TAGS="u32_30:--logn=30" bash tools/gpu_prof2.sh
