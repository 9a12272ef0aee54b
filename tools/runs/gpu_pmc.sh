# PMC passes (one counter group per run, per MI355X_MICROARCH.md) over a 2^28 u32
# sort and over the calibration shapes (known 4 GiB read + 4 GiB write per kernel).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/pmc"; mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "k_stream|k_merge|inplace" -d "$OUT/$name" -o $name --output-format csv -- python3 "$R/bench.py" --logn 28 --steps 2 --warmup 0 --no-cpu-baseline --no-kernel-events > "$OUT/$name.log" 2>&1 || { echo "pass $name failed"; tail -3 "$OUT/$name.log"; return 1; }
  echo "pass $name ok"
}
runcal() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o $name --output-format csv -- "$R/tools/bin/hbm_shapes" > "$OUT/$name.log" 2>&1 || { echo "cal $name failed"; return 1; }
  echo "cal $name ok"
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY && \
runcal calfetch FETCH_SIZE && runcal calwrite WRITE_SIZE
ls "$OUT"
