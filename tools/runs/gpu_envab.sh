# A/B of (library, env) combinations on the bench: RUNS="name|lib|ENV=V ENV2=V2" entries separated by ';'.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-envab}"; mkdir -p "$O"; cd "$R"
IFS=';' read -ra specs <<< "$RUNS"
for rep in 1 2; do
for spec in "${specs[@]}"; do
  IFS='|' read -r name lib envs <<< "$spec"
  if [ -n "$lib" ]; then export MISORT_LIBRARY="$R/$lib"; else unset MISORT_LIBRARY; fi
  env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps ${STEPS:-10} $BENCH_ARGS > "$O/bench_${name}_$rep.json" 2> "$O/bench_${name}_$rep.err"; rc=$?
  case $rc in 124|137|134|139) echo "fatal rc $rc in $name"; exit $rc;; esac
  [ $rc -ne 0 ] && { echo "$name rc $rc"; tail -3 "$O/bench_${name}_$rep.err"; continue; }
  python3 -c "
import json; d=json.loads(open('$O/bench_${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', $rep, round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],2), 'ms err', d['check_errors'], ' '.join(f'{k}:{v[\"launches_per_step\"]:.0f}x{v[\"avg_launch_us\"]:.0f}us' for k,v in d.get('kernels',{}).items()))"
done
done
unset MISORT_LIBRARY
exit 0
