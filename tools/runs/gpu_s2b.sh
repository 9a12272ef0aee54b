# Session-2 check of the u64 multi-way passes: VALU probe, merge-pass tests,
# u64/u32 bench lines, rocprof kernel stats at 2^29 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2b}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 120 ./tools/bin/valu_probe > "$O/valu.jsonl" 2>&1; rc=$?; cat "$O/valu.jsonl"; fatal $rc valu; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest_runs.log" 2>&1; rc=$?; echo "pytest runs rc $rc"; tail -4 "$O/pytest_runs.log"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --logn 29 --dtype u64 --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_u64_29.json" 2> "$O/bench_u64_29.err"; rc=$?
echo "bench u64 rc $rc"; tail -c 1500 "$O/bench_u64_29.json"; fatal $rc bench_u64; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$O/bench_u32_30.json" 2> "$O/bench_u32_30.err"; rc=$?
echo "bench u32 rc $rc"; tail -c 600 "$O/bench_u32_30.json"; fatal $rc bench_u32; [ $rc -ne 0 ] && exit $rc
OUTDIR=${OUTDIR:-s2b}/stats TAGS="u64_29:--logn=29,--dtype=u64 u32_30:--logn=30" bash tools/gpu_prof2.sh
