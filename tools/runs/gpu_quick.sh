# Quick perf check: bench at 2^30 and a few sizes; optional env passed through.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for L in ${LOGNS:-30 28 26 24}; do
  timeout -k 10 120 python -u bench.py --logn $L --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/q_$L.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q_$L.log').read().strip().splitlines()[-1]);print($L, round(d['value'],2), d['check_errors'], {k:(v['launches_per_step'], round(v['ms_per_step'],2), round(v['achieved_GBs'])) for k,v in d['kernels'].items()})"
done
