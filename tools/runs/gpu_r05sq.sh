# SQ counters of k_mergek<u32,4> and k_sort_u32 at 2^30 (one --pmc pass per counter set), for the
# VALU / SALU / LDS / wait balance of the HEAD build.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${OUTDIR:-r05sq}"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${REGEX:-k_mergek|k_sort_u32}" -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-events $BENCH_ARGS > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
  echo "pass $i ok"
done
