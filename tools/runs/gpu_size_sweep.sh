# Size sweep of the 1-GPU bench (u32 2^20..2^31, u64 2^20..2^30), one JSON line per size.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/size_sweep.jsonl; : > $OUT
timeout -k 10 120 python -u bench.py --logn 28 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sw_warm.log 2>&1 || { tail -5 gpurun_out/sw_warm.log; exit 1; }
for DT in u32 u64; do
  for L in ${LOGNS:-20 22 24 26 28 29 30 31}; do
    [ $DT = u64 ] && [ $L -gt 30 ] && continue
    timeout -k 10 180 python -u bench.py --dtype $DT --logn $L --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sw.log 2>&1 || { echo "BENCH FAIL $DT $L"; tail -5 gpurun_out/sw.log; exit 1; }
    tail -1 gpurun_out/sw.log >> $OUT
    python -c "import json;d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]);print('$DT 2^$L', round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],3), 'ms err', d['check_errors'], 'frac', round(d['roofline']['frac'],3))"
  done
done
