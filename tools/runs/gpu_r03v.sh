# Round 3, call V: one-step kernel timelines at 2^30 u32 / 2^29 u64 (kernel-
# carried profiler events), then the N = 2 / 4 bench lines on the shared GPU.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03v"; mkdir -p "$O"; cd "$R"
OUTDIR=r03v/timeline TAGS="u32_30:--logn=30 u64_29:--logn=29,--dtype=u64" bash tools/gpu_timeline.sh > /dev/null || exit $?
cd "$R"
for N in 2 4; do
  MISORT_SHARE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_n$N.json" 2> "$O/bench_n$N.err"; rc=$?
  [ $rc -ne 0 ] && { echo "N=$N rc $rc"; tail -5 "$O/bench_n$N.err"; exit $rc; }
  python3 -c "import json; d=json.loads(open('$O/bench_n$N.json').read().strip().splitlines()[-1]); print('N=$N', round(d['value'],2), d['ms_per_step'], 'err', d.get('check_errors'), 'stages', len(d.get('stages') or []))"
done
