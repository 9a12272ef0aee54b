# Session-2 final PMC traffic (FETCH_SIZE/WRITE_SIZE passes) for 2^30 u32, 2^28 u32, 2^29 u64, 2^24 u32.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=${OUTDIR:-s2o}
OUTDIR=$O/pmc_u32_30 WORKLOAD=u32_2e30_n1 BENCH_ARGS="--logn 30" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$O/pmc_u32_28 WORKLOAD=u32_2e28_n1 BENCH_ARGS="--logn 28" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$O/pmc_u64_29 WORKLOAD=u64_2e29_n1 BENCH_ARGS="--logn 29 --dtype u64" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$O/pmc_u32_24 WORKLOAD=u32_2e24_n1 BENCH_ARGS="--logn 24" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
for w in u32_30 u32_28 u64_29 u32_24; do echo "== $w"; python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k in ('tile_sort','run_mergek_kernel','run_mergek','global_pass','span_pass','wide_pass','tile_merge'):
    if k in d: print(k, d[k]['launches'], round(d[k]['bytes_per_launch']/1e9,3), 'GB/launch')" "$R/gpurun_out/$O/pmc_$w/traffic.json"; done
