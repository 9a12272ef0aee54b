# A/B runs of bench.py under planner/engine knobs, one summary line each.
#   VARIANTS="NAME=ENV1=v1,ENV2=v2 NAME2=..." bash tools/gpu_ab.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
TESTS=${TESTS:-1}
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for v in $VARIANTS; do
  name=${v%%=*}; envs=${v#*=}
  (export $(echo "$envs" | tr ',' ' '); timeout -k 10 300 python -u bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-}) > gpurun_out/ab_$name.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$name.log; exit $rc; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_$name.log').read().strip().splitlines()[-1])
k=d.get('kernels',{})
print('$name', round(d['value'],3), 'Gkeys/s', round(d['ms_per_step'],2), 'ms', ' '.join(f'{n}:{v[\"launches_per_step\"]:.0f}x{v[\"avg_launch_us\"]:.0f}us' for n,v in k.items()))
"
done
