# Session-3: kernel stats new vs old planning kernels at 2^24 and 2^30 u32 (rocprofv3 --kernel-trace --stats).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s3c}"; mkdir -p "$O"
NEW="$R/parallel-computing-mpi_amd/lib/libmisort.so"; OLD="$R/parallel-computing-mpi_amd/lib/variants/libmisort_old.so"
cd /tmp && export TMPDIR=/tmp
for L in 24 30; do
  for v in new old; do
    lib=$NEW; [ $v = old ] && lib=$OLD
    MISORT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/${v}_$L" -o s --output-format csv -- \
      python3 "$R/bench.py" --logn $L --steps 10 --warmup 2 --no-cpu-baseline > "$O/${v}_$L.log" 2>&1 || { echo "rocprof $v $L failed"; exit 1; }
  done
done
exit 0
