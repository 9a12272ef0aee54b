# Parity tests + R sweep of the pass planner (invoked via gpurun from the repo root).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for RM in ${RMAXES:-5 6 7 8 9}; do
  MISORT_RMAX=$RM timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/tune_$RM.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/tune_$RM.log').read().strip().splitlines()[-1]);print('RMAX=$RM', round(d['value'],2), d['check_errors'], {k:(v['launches_per_step'], round(v['ms_per_step'],2), round(v['achieved_GBs'])) for k,v in d['kernels'].items()})"
done
