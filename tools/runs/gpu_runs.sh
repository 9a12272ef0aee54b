# Merge-level (runs.hip) experiment: parity with merge levels on, then bench A/B
# over MISORT_MERGE_FROM (first level done by merge passes; 0 = network only).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/runs
MISORT_MERGE_FROM=${PFROM:-15} MISORT_MERGE_FROM_U64=${PFROM64:-13} timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_staging.py -x -q --timeout 120 --timeout-method thread > gpurun_out/runs/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/runs/pytest.log; [ $rc -eq 0 ] || exit $rc
for m in ${FROMS:-0 15 17 19 21 23}; do
  MISORT_MERGE_FROM=$m timeout -k 10 200 python -u bench.py --logn ${LOGN:-30} --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/runs/b_$m.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/runs/b_$m.log').read().strip().splitlines()[-1]); print('from', $m, round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],2), 'ms err', d['check_errors'], {k:(v['launches_per_step'], round(v['avg_launch_us'])) for k,v in d['kernels'].items()})"
done
