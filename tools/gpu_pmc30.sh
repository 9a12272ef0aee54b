# HBM traffic of the bench's sort kernels at 2^30 (rocprofv3 --pmc, one counter
# group per run as MI355X_MICROARCH.md prescribes), summarised into traffic.json.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/${OUTDIR:-pmc30}"; mkdir -p "$OUT"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_sort_u32|k_sort_tile|k_runs_|k_mergek|k_fence|k_scan_totals|k_bounds|k_chunk_desc|k_split_desc" -d "$OUT/$name" -o $name --output-format csv -- python3 "$R/bench.py" $BENCH_ARGS --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-events > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -3 "$OUT/$name.log"; return 1; }
  echo "pass $name ok"
}
run fetch FETCH_SIZE && run write WRITE_SIZE && WORKLOAD=${WORKLOAD:-u32_2e30_n1} python3 "$R/tools/traffic.py" "$OUT" > "$OUT/traffic.json" && cat "$OUT/traffic.json"
