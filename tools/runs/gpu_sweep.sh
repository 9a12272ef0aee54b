# Config sweep: GPU parity tests under each config, then the 2^30 bench.
#   CONFIGS="MISORT_MULTIWAY=4 MISORT_FC_SLICES_MAX=0,..." (space-separated, comma = several vars)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
i=0
# throwaway warm-up (first run on a fresh box reads slow)
timeout -k 10 120 python -u bench.py --logn 28 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw_warm.log 2>&1 || { tail -5 gpurun_out/sw_warm.log; exit 1; }
for C in ${CONFIGS:-base}; do
  i=$((i+1))
  ENVS=$(echo "$C" | tr ',' ' '); [ "$C" = base ] && ENVS=""
  if [ -n "$TESTS" ]; then
    env $ENVS timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $TESTS > gpurun_out/sw_test_$i.log 2>&1 || { echo "TESTS FAIL [$C]"; tail -30 gpurun_out/sw_test_$i.log; exit 1; }
    echo "tests ok [$C]: $(tail -1 gpurun_out/sw_test_$i.log)"
  fi
  for L in ${LOGNS:-30}; do
    env $ENVS timeout -k 10 120 python -u bench.py --logn $L --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/sw_${i}_${L}.log 2>&1 || { echo "BENCH FAIL [$C]"; tail -5 gpurun_out/sw_${i}_${L}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/sw_${i}_${L}.log').read().strip().splitlines()[-1]);print('[$C] 2^$L', round(d['value'],2), 'Gkeys/s err', d['check_errors'], {k:(v['launches_per_step'], round(v['ms_per_step'],2), round(v['achieved_GBs'])) for k,v in d.get('kernels',{}).items()})"
  done
done
