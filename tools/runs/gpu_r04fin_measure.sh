# Round 4, final call: HEAD measurement set at the end of the round -- the default bench line (with the
# reference CPU baseline), rocprofv3 kernel stats of it, a PMC traffic capture
# at 2^30 u32, benches at 2^28 / 2^24 u32 and 2^29 u64, the per-GPU device work
# of an 8-GPU step (config 4 / 5 at P = 8).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04fin"; mkdir -p "$O"; cd "$R"
timeout -k 10 300 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err"; rc=$?
echo "bench rc $rc"; tail -c 300 "$O/bench_default.json"; [ $rc -ne 0 ] && exit $rc
for a in "--logn 28" "--logn 24" "--dtype u64 --logn 29"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 200 python3 bench.py $a --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_$n.json" 2> "$O/bench_$n.err" || exit $?
done
OUTDIR=r04fin/pmc30 bash tools/gpu_pmc30.sh > /dev/null && echo "pmc30 ok" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err" || exit $?
echo "stats ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c5" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --n 536870909 --p 8 --dtype u64 > "$O/rw_c5.json" 2> "$O/rw_c5.err" && echo "rw ok"
