# Session-3: planning kernels (k_chunk_desc lane-per-entry, k_bounds line probe) -- merge/parity tests,
# kernel stats of the 2^30 u32 bench, benches 2^24..2^30 u32 and 2^29 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s3a}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 "$O/pytest.log"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats30" -o u32_30 --output-format csv -- \
  python3 "$R/bench.py" --steps 4 --warmup 1 --no-cpu-baseline > "$O/stats30.log" 2>&1); rc=$?; echo "stats rc $rc"; fatal $rc stats; [ $rc -ne 0 ] && exit $rc
for L in 24 26 28 30; do
  timeout -k 10 200 python3 -u bench.py --logn $L --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_u32_$L.json" 2> "$O/bench_u32_$L.err"; rc=$?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), round(d['ms_per_step'],4), d['check_errors'])" "$O/bench_u32_$L.json"
  fatal $rc "bench $L"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 200 python3 -u bench.py --dtype u64 --logn 29 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_u64_29.json" 2> "$O/bench_u64_29.err"; rc=$?
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), round(d['ms_per_step'],4), d['check_errors'])" "$O/bench_u64_29.json"
exit 0
