# Session-2 record: default bench (CPU baseline included), u64 2^29 and u32 2^28/2^24 lines,
# rocprofv3 kernel stats of the same workloads (k_mergek rows vs bench events).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2g}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 400 python3 -u bench.py > "$O/bench_n1.json" 2> "$O/bench_n1.err"; rc=$?; echo "bench rc $rc"
tail -c 2500 "$O/bench_n1.json"; fatal $rc bench; [ $rc -ne 0 ] && { tail -5 "$O/bench_n1.err"; exit $rc; }
for spec in "29 u64" "28 u32" "24 u32"; do
  set -- $spec
  timeout -k 10 200 python3 -u bench.py --logn $1 --dtype $2 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench_$2_$1.json" 2> "$O/bench_$2_$1.err"; rc=$?
  echo "$2 $1 rc $rc"; fatal $rc "bench $spec"; [ $rc -ne 0 ] && exit $rc
done
OUTDIR=${OUTDIR:-s2g}/stats TAGS="u32_30:--logn=30 u64_29:--logn=29,--dtype=u64 u32_28:--logn=28" bash tools/gpu_prof2.sh
