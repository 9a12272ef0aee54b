# Iteration loop: selected GPU tests (TESTS), the bench, rocprofv3 kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-iter}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" "$O/pytest.log" | tail -8; fatal $rc pytest
  [ $rc -ne 0 ] && [ -z "$FORCE" ] && exit 1
fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline $BENCH_ARGS > "$O/bench.json" 2> "$O/bench.err"; rc=$?; echo "bench rc $rc"
python3 -c "
import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'errors', d['check_errors'])
for k,v in d.get('kernels',{}).items(): print(' ', k, round(v['ms_per_step'],3), 'ms/step', round(v['avg_launch_us'],1), 'us/launch', v['launches_per_step'])
"; fatal $rc bench
if [ -n "$PROF" ]; then
  OUTDIR=${OUTDIR:-iter}/prof TAGS="${PROF}" bash tools/gpu_prof2.sh
fi
