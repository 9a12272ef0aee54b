# Session-3: planning-kernel shape sweep (k_bounds line probe on/off, k_chunk_desc 4/16 chunks per wave)
# by kernel stats at 2^24, 2^26, 2^28 u32 and 2^26 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s3d}"; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for cfg in "u32 24" "u32 26" "u32 28" "u64 26"; do
  set -- $cfg
  for line in 0 999999999999; do
    for dc in 0 999999999999; do
      tag="$1_$2_l$([ $line = 0 ] && echo 1 || echo 0)_d$([ $dc = 0 ] && echo 16 || echo 4)"
      MISORT_BOUNDS_LINE_MIN=$line MISORT_DESC16_MIN=$dc timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/$tag" -o s --output-format csv -- \
        python3 "$R/bench.py" --dtype $1 --logn $2 --steps 10 --warmup 2 --no-cpu-baseline > "$O/$tag.log" 2>&1 || { echo "rocprof $tag failed"; exit 1; }
    done
  done
done
exit 0
