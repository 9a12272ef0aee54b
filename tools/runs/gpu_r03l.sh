# Round 3, call L: fence-count loads (base vs fc0), 16-way u32 passes at 2^27
# and 2^31, and the N > 1 bench line end to end (ranks sharing the one GPU).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r03l"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base fc0" LOGNS="30 28 24" ROUNDS=2 OUTDIR=r03l/ab bash tools/gpu_abv.sh || exit $?
for L in 27 31; do
  RUNS="mw3||MISORT_MULTIWAY=-1;mw4||MISORT_MULTIWAY=4" BENCH_ARGS="--logn $L" OUTDIR=r03l/mw_$L bash tools/gpu_envab.sh | sed "s/^/2^$L /" || exit $?
done
for N in 2 4; do
  MISORT_SHARE_GPU=1 timeout -k 10 300 python3 -u bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_n$N.json" 2> "$O/bench_n$N.err"; rc=$?
  fatal $rc "bench n$N"; [ $rc -ne 0 ] && { tail -5 "$O/bench_n$N.err"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('N', d['n_gpus'], round(d['value'],2), d['unit'], round(d['ms_per_step'],2), 'ms err', d['check_errors'], 'scaling_eff', d.get('scaling_eff'))" "$O/bench_n$N.json"
done
