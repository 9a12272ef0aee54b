# Round 4, call H: SQ attribution of k_mergek's LDS time (probe launches:
# MODE 1 no merge, 3 co-rank searches only, 0 the pass); a HEAD PMC traffic
# capture at 2^30 u32; rocprofv3 kernel stats of the default bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04h"; mkdir -p "$O"; cd "$R"
MISORT_MK_PROBE=1 OUTDIR=r04h/sq_probe bash tools/gpu_sq2.sh > "$O/sq_probe.txt" && echo "sq ok" &&
OUTDIR=r04h/pmc30 bash tools/gpu_pmc30.sh > /dev/null && echo "pmc30 ok" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/stats" -o bench --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err"; rc=$?
echo "stats rc $rc"; tail -1 "$O/bench_prof.json"
