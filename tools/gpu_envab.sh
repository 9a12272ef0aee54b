# Env A/B of bench.py: each line of $CASES is "<label>|<env assignments>|<bench args>".
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/envab
echo "$CASES" | while IFS='|' read -r lab envs args; do
  [ -z "$lab" ] && continue
  env $envs timeout -k 10 200 python -u bench.py $args --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/envab/$lab.log 2>&1 || { echo "FAIL $lab"; tail -5 gpurun_out/envab/$lab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/envab/$lab.log').read().strip().splitlines()[-1]); print('$lab', round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],2), 'ms err', d['check_errors'], {k:(v['launches_per_step'], round(v['avg_launch_us'])) for k,v in d['kernels'].items()})" || exit 1
done
