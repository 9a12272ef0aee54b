# Round-2 profile set: rocprofv3 kernel stats and HBM traffic (FETCH_SIZE / WRITE_SIZE, one
# counter per pass) at 2^30 u32, 2^28 u32 and 2^29 u64, written under gpurun_out/$OUTDIR.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OD=${OUTDIR:-r02prof}
OUTDIR=$OD/stats TAGS="u32_30:--logn=30 u32_28:--logn=28 u64_29:--logn=29,--dtype=u64" bash "$R/tools/gpu_prof2.sh" || exit $?
OUTDIR=$OD/pmc_u32_30 WORKLOAD=u32_2e30_n1 BENCH_ARGS="--logn 30" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$OD/pmc_u32_28 WORKLOAD=u32_2e28_n1 BENCH_ARGS="--logn 28" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$OD/pmc_u64_29 WORKLOAD=u64_2e29_n1 BENCH_ARGS="--logn 29 --dtype u64" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
for w in u32_30 u32_28 u64_29; do echo "== $w"; cat "$R/gpurun_out/$OD/pmc_$w/traffic.json"; done
