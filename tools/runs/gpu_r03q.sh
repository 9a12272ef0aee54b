# Round 3, call Q: profiler events without the system-scope release (default)
# vs with it (MISORT_PROF_SYSFENCE=1) vs no kernel events at all, per size;
# then the one-step kernel timeline at 2^24 u32.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03q"; mkdir -p "$O"; cd "$R"
for args in "--logn=24" "--logn=22" "--logn=24 --dtype=u64" "--logn=28" "" ; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=100; [ -z "$args" ] && steps=10; [ "$args" = "--logn=28" ] && steps=30
  echo "== $args"
  for rep in 1 2; do
    for v in "sf1|MISORT_PROF_SYSFENCE=1|" "sf0|MISORT_PROF_SYSFENCE=0|" "noev|MISORT_PROF_SYSFENCE=0|--no-kernel-events"; do
      IFS='|' read -r name envs extra <<< "$v"
      env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $steps $args $extra > "$O/${tag}_${name}_$rep.json" 2> "$O/${tag}_${name}_$rep.err"; rc=$?
      [ $rc -ne 0 ] && { echo "$name rc $rc"; tail -3 "$O/${tag}_${name}_$rep.err"; exit $rc; }
      python3 -c "
import json; d=json.loads(open('$O/${tag}_${name}_$rep.json').read().strip().splitlines()[-1])
print('$name', $rep, round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],3), 'ms err', d['check_errors'], ' '.join(f'{k}:{v[\"launches_per_step\"]:.0f}x{v[\"avg_launch_us\"]:.0f}us' for k,v in d.get('kernels',{}).items()))"
    done
  done
done
OUTDIR=r03q/timeline TAGS="u32_24:--logn=24" bash tools/gpu_timeline.sh > /dev/null
