# Round 5 end-of-round record, part 2: rocprofv3 kernel stats of the benches and the calibrated PMC
# traffic captures (u32 2^30, u64 2^29) the bench lines read.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r05fin2}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for spec in "u32_30:--logn 30" "u64_29:--dtype u64 --logn 29" "f64_29:--dtype f64 --logn 29"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$tag" -o $tag --output-format csv -- python3 "$R/bench.py" $args --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof_$tag.log" 2>&1 || { echo "prof $tag failed"; tail -3 "$O/prof_$tag.log"; exit 1; }
  echo "prof $tag ok"
done
cd "$R"
OUTDIR=r05fin2/pmc_u32_30 WORKLOAD=u32_2e30_n1 bash tools/gpu_pmc30.sh > "$O/pmc_u32_30.out" 2>&1 && echo "pmc u32 ok" || exit 1
OUTDIR=r05fin2/pmc_u64_29 WORKLOAD=u64_2e29_n1 BENCH_ARGS="--dtype u64 --logn 29" bash tools/gpu_pmc30.sh > "$O/pmc_u64_29.out" 2>&1 && echo "pmc u64 ok" || exit 1
