# Session-2: PMC traffic of the 2^30 u32 and 2^29 u64 sorts (multi-way passes),
# and the u64 SORT tile 2^13 vs 2^14 with multi-way passes (2^29 and 2^26).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2c}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
for spec in "29 13" "29 14" "26 13" "26 14"; do
  set -- $spec
  MISORT_TILE_LOG2_U64=$2 MISORT_ROWS_TILE_LOG2_U64=$2 timeout -k 10 200 python3 -u bench.py --logn $1 --dtype u64 \
    --steps 5 --warmup 2 --no-cpu-baseline > "$O/u64_$1_lt$2.json" 2> "$O/u64_$1_lt$2.err"; rc=$?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],2), round(d['ms_per_step'],3), {k: round(v['ms_per_step'],3) for k,v in d['kernels'].items()})" "$O/u64_$1_lt$2.json"
  fatal $rc "u64 $spec"; [ $rc -ne 0 ] && exit $rc
done
OUTDIR=${OUTDIR:-s2c}/pmc_u32_30 WORKLOAD=u32_2e30_n1 BENCH_ARGS="--logn 30" bash tools/gpu_pmc30.sh > /dev/null || exit $?
OUTDIR=${OUTDIR:-s2c}/pmc_u64_29 WORKLOAD=u64_2e29_n1 BENCH_ARGS="--logn 29 --dtype u64" bash tools/gpu_pmc30.sh > /dev/null || exit $?
for w in u32_30 u64_29; do echo "== $w"; cat "$O/pmc_$w/traffic.json"; done
