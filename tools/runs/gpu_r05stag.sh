# Round 5: first-round stagger of the 2^14 SORT tile's second workgroup per CU (MISORT_SORT_STAGGER sleeps)
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/stag"; mkdir -p "$O"; cd "$R"
for rep in 1 2; do for st in 0 1 2 3 4 6; do
  MISORT_SORT_STAGGER=$st timeout -k 10 120 python3 tools/sort_pass_probe.py --dtype u32 --logn 30 --hi 13 > "$O/p_${st}_$rep.json" || exit 1
  echo "stagger $st: $(cat $O/p_${st}_$rep.json)"
done; done
for rep in 1 2; do for st in 0 ${BEST:-3}; do
  MISORT_SORT_STAGGER=$st timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/b_${st}_$rep.json" 2> "$O/b_${st}_$rep.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$O/b_${st}_$rep.json').read().strip().splitlines()[-1]); print('bench stagger $st', round(d['value'],2), round(d['ms_per_step'],3), d['check_errors'], [(p['kind'], round(p['ms'],3)) for p in d['roofline']['passes']][:2])"
done; done
