# Round 4, call U: compact chunk descriptors (16-bit row entries, k_mergek
# derives the rows) -- merge/parity tests, then A/B against the previous HEAD
# (lib/variants/libmisort_prev.so) at 2^30 / 2^28 / 2^24 u32 and 2^29 u64.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04u"; mkdir -p "$O"; cd "$R"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
V=parallel-computing-mpi_amd/lib/variants
for a in "--logn 30" "--logn 28" "--logn 24" "--dtype u64 --logn 29"; do
  n=$(echo $a | tr -d ' -')
  RUNS="prev_$n|$V/libmisort_prev.so|;new_$n||" BENCH_ARGS="$a" STEPS=20 OUTDIR=r04u bash tools/gpu_envab.sh || exit $?
done
