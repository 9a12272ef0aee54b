# Bench variants on one GPU: u64 2^29 (config 5 size), sample-sort algo, sizes 2^24/2^28.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
for V in "--dtype u64 --logn 29" "--algo sample" "--logn 24" "--logn 28" ${EXTRA}; do
  tag=$(echo "$V" | tr -d ' -')
  timeout -k 10 120 python -u bench.py $V --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/var_$tag.log 2>&1 || { echo "FAIL $V"; tail -5 gpurun_out/var_$tag.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/var_$tag.log').read().strip().splitlines()[-1]);print('[$V]', round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],2),'ms err', d['check_errors'], {k:(v['launches_per_step'], round(v['ms_per_step'],2), round(v['achieved_GBs'])) for k,v in d.get('kernels',{}).items()})"
done
