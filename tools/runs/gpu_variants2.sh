# A/B of library variants on the bench (VARIANTS="name=path ..."), after the default's tests.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-var}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" "$O/pytest.log" | tail -8; fatal $rc pytest
  [ $rc -ne 0 ] && exit 1
fi
for v in default $VARIANTS; do
  name=${v%%=*}; lib=${v#*=}
  if [ "$name" = default ]; then unset MISORT_LIBRARY; else export MISORT_LIBRARY="$R/$lib"; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${STEPS:-10} $BENCH_ARGS > "$O/bench_$name.json" 2> "$O/bench_$name.err"; rc=$?
  fatal $rc "bench $name"; [ $rc -ne 0 ] && { tail -3 "$O/bench_$name.err"; continue; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1])
print('$name', round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],2), 'ms err', d['check_errors'], ' '.join(f'{k}:{v[\"launches_per_step\"]:.0f}x{v[\"avg_launch_us\"]:.0f}us' for k,v in d.get('kernels',{}).items()))"
done
unset MISORT_LIBRARY
[ -n "$PROF" ] && OUTDIR=${OUTDIR:-var}/prof TAGS="$PROF" bash tools/gpu_prof2.sh
exit 0
