# Round 5: the 2^14 u32 SORT tile by phase (MISORT_SORT_STOP probe builds: 1 = load + store, 2 = + levels 1..8,
# 3 = + levels 9..10, base = + merge levels 11..14), then SQ counters of the full tile (dynamic instructions per wave).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/tile"; mkdir -p "$O"; cd "$R"
for rep in 1 2; do for v in stop1 stop2 stop3 base; do
  if [ $v = base ]; then unset MISORT_LIBRARY; else export MISORT_LIBRARY=$R/parallel-computing-mpi_amd/lib/variants/libmisort_$v.so; fi
  timeout -k 10 120 python3 tools/sort_pass_probe.py --dtype u32 --logn 30 --hi 13 || exit 1
done; done
unset MISORT_LIBRARY
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  for v in stop3 base; do
    if [ $v = base ]; then unset MISORT_LIBRARY; else export MISORT_LIBRARY=$R/parallel-computing-mpi_amd/lib/variants/libmisort_$v.so; fi
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex k_sort_u32 -d "$O/sq_${v}/p$i" -o p$i --output-format csv -- \
      python3 "$R/tools/sort_pass_probe.py" --dtype u32 --logn 30 --hi 13 --reps 2 > "$O/sq_${v}_p$i.log" 2>&1 || { echo "sq $v $i failed"; tail -3 "$O/sq_${v}_p$i.log"; exit 1; }
  done
done
unset MISORT_LIBRARY
cd "$R" && for v in stop3 base; do echo "== $v"; python3 tools/sq_summary.py "$O/sq_$v" || true; done
echo done
