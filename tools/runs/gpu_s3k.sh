# Session-3: fence LDS merge ranks by galloping from the previous fence -- merge/parity tests, then new vs old (lib/variants/libmisort_old.so)
# alternating benches and kernel stats.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s3k}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; tail -2 "$O/pytest.log"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
NEW="$R/parallel-computing-mpi_amd/lib/libmisort.so"; OLD="$R/parallel-computing-mpi_amd/lib/variants/libmisort_old.so"
one() {  # tag lib dtype logn
  MISORT_LIBRARY=$2 timeout -k 10 200 python3 -u bench.py --dtype $3 --logn $4 --steps 20 --warmup 5 --no-cpu-baseline > "$O/$1_$3_$4.json" 2> "$O/$1_$3_$4.err"; rc=$?
  fatal $rc "bench $1 $3 $4"; [ $rc -ne 0 ] && exit $rc
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], round(d['value'],2), round(d['ms_per_step'],4), d['check_errors'])" "$O/$1_$3_$4.json"
}
for rep in 1 2; do
  for L in 24 26 28 30; do one new$rep $NEW u32 $L; one old$rep $OLD u32 $L; done
  one new$rep $NEW u64 26; one old$rep $OLD u64 26; one new$rep $NEW u64 29; one old$rep $OLD u64 29
done
cd /tmp && export TMPDIR=/tmp
for v in new old; do
  lib=$NEW; [ $v = old ] && lib=$OLD
  for L in 24 30; do
    MISORT_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/st_${v}_$L" -o s --output-format csv -- \
      python3 "$R/bench.py" --logn $L --steps 10 --warmup 2 --no-cpu-baseline > "$O/st_${v}_$L.log" 2>&1 || { echo "rocprof $v $L failed"; exit 1; }
  done
done
exit 0
