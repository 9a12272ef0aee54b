# Session-2: small/medium u32 sizes, network vs multi-way passes (MISORT_MERGE_MIN_LOG2),
# and the merge-pass tests after the packed fence counts.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2f}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; tail -3 "$O/pytest.log"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
for logn in 20 22 24 26 28 30; do
  for mm in 24 0; do
    MISORT_MERGE_MIN_LOG2=$mm timeout -k 10 120 python3 -u bench.py --logn $logn --steps 20 --warmup 5 --no-cpu-baseline \
      > "$O/u32_${logn}_mm$mm.json" 2> "$O/u32_${logn}_mm$mm.err"; rc=$?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), round(d['ms_per_step'],4))" "$O/u32_${logn}_mm$mm.json"
    fatal $rc "u32 $logn $mm"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
