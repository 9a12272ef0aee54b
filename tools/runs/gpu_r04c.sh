# Round 4, call C: per-GPU device work of an 8-GPU step (config 4 and 5 at
# P = 8, tools/rank_work_probe.py under a rocprofv3 kernel trace); FETCH_SIZE /
# WRITE_SIZE calibration (tools/fetch_cal.hip); SQ counters of k_mergek (ch1);
# a HEAD PMC traffic capture at 2^30 u32 with the calibrated factors; the
# 8- vs 16-way u32 plan at 2^26..2^31 (verdict r03 item 3).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04c"; mkdir -p "$O/cal"; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$O/cal/fetch" -o fetch --output-format csv -- "$R/tools/bin/fetch_cal" > "$O/cal/fetch_cal.log" 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$O/cal/write" -o write --output-format csv -- "$R/tools/bin/fetch_cal" > "$O/cal/write.log" 2>&1 &&
python3 "$R/tools/fetch_cal.py" "$O/cal" > "$O/cal/fetch_cal.json" && cat "$O/cal/fetch_cal.json" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err"; rc=$?
echo "rw_c4 rc $rc"; case $rc in 0) ;; *) tail -5 "$O/rw_c4.err"; exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c5" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --n 536870909 --p 8 --dtype u64 > "$O/rw_c5.json" 2> "$O/rw_c5.err"; rc=$?
echo "rw_c5 rc $rc"; case $rc in 0) ;; *) tail -5 "$O/rw_c5.err"; exit $rc;; esac
cd "$R" && OUTDIR=r04c/sq_ch1 bash tools/gpu_sq2.sh &&
MISORT_LIBRARY=$R/parallel-computing-mpi_amd/lib/variants/libmisort_ch3it17.so OUTDIR=r04c/sq_ch3it17 bash tools/gpu_sq2.sh &&
FETCH_CAL="$O/cal/fetch_cal.json" OUTDIR=r04c/pmc30 bash tools/gpu_pmc30.sh > /dev/null && echo "pmc30 ok" || exit $?
cd "$R" && for L in 26 27 28 29 30 31; do
  RUNS="w8||MISORT_MULTIWAY=3;w16||MISORT_MULTIWAY=4" BENCH_ARGS="--logn $L" STEPS=10 OUTDIR=r04c/mw$L bash tools/gpu_envab.sh || exit $?
done
