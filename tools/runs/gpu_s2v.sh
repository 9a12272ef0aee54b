# Session-2 final: u64 2^29 PMC traffic and rocprof stats with the 16-way default, 2^26 u64 line.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O=${OUTDIR:-s2v}
OUTDIR=$O/pmc_u64_29 WORKLOAD=u64_2e29_n1 BENCH_ARGS="--logn 29 --dtype u64" bash "$R/tools/gpu_pmc30.sh" > /dev/null || exit $?
OUTDIR=$O/stats TAGS="u64_29:--logn=29,--dtype=u64 u64_26:--logn=26,--dtype=u64" bash "$R/tools/gpu_prof2.sh" || exit $?
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
for k in ('tile_sort','run_mergek_kernel','run_mergek'):
    print(k, d[k]['launches'], round(d[k]['bytes_per_launch']/1e9,3), 'GB/launch')" "$R/gpurun_out/$O/pmc_u64_29/traffic.json"
