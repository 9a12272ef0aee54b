# Round 5 first check: GPU suite, u32 2^30 bench, f64 2^29 bench + rocprofv3 stats (no k_f64_ord in the P = 1 path).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r05a"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed|Error" "$O/pytest.log" | tail -8; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
for spec in "u32 30" "f64 29" "u64 29"; do set -- $spec
  timeout -k 10 300 python3 -u bench.py --dtype $1 --logn $2 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$1_$2.json" 2> "$O/bench_$1_$2.err"; rc=$?
  echo "bench $1 $2 rc $rc"; fatal $rc bench; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],3), 'ms', 'err', d['check_errors'], {k:(round(v['avg_launch_us']),v['launches_per_step']) for k,v in d.get('kernels',{}).items()})" "$O/bench_$1_$2.json"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_f64" -o f64 -- python3 -u "$R/bench.py" --dtype f64 --logn 29 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_f64.log" 2>&1; rc=$?
echo "rocprof rc $rc"; fatal $rc rocprof
find "$O/prof_f64" -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -20'
