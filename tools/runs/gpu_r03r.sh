# Round 3, call R: kernel-bound pass timing (default) vs marker events
# (MISORT_PROF_MARKERS=1) vs no events; profiler tests; one-step timeline.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03r"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_profile.py tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 "$O/pytest.log"; exit $rc; }
for args in "--logn=24" "--logn=22" "--logn=24 --dtype=u64" "--logn=28" "" ; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=100; [ -z "$args" ] && steps=10; [ "$args" = "--logn=28" ] && steps=30
  echo "== $args"
  for rep in 1 2; do
    for v in "mk|MISORT_PROF_MARKERS=1|" "bound|MISORT_PROF_MARKERS=0|" "noev|MISORT_PROF_MARKERS=0|--no-kernel-events"; do
      IFS='|' read -r name envs extra <<< "$v"
      env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $steps $args $extra > "$O/${tag}_${name}_$rep.json" 2> "$O/${tag}_${name}_$rep.err"; rc=$?
      [ $rc -ne 0 ] && { echo "$name rc $rc"; tail -3 "$O/${tag}_${name}_$rep.err"; exit $rc; }
      python3 -c "
import json; d=json.loads(open('$O/${tag}_${name}_$rep.json').read().strip().splitlines()[-1])
ps=d.get('roofline',{}).get('passes') or []
print('$name', $rep, round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],3), 'ms err', d['check_errors'], ' '.join(f'{k}:{v[\"launches_per_step\"]:.0f}x{v[\"avg_launch_us\"]:.0f}us' for k,v in d.get('kernels',{}).items()), 'frac', d['roofline']['frac'] and round(d['roofline']['frac'],3), 'passes', [round(p.get('ms',0),3) for p in ps])"
    done
  done
done
OUTDIR=r03r/timeline TAGS="u32_24:--logn=24" bash tools/gpu_timeline.sh > /dev/null
