# Round 3, call Y: 1024-lane k_mergek chunks (CAP 16384; nt1024 variant) for
# 16-way u32 passes (MISORT_MULTIWAY=4) against the 512-lane default.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants/libmisort_nt1024.so
MISORT_LIBRARY=$R/$V timeout -k 10 600 python -u -m pytest tests/test_gpu_runs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03y_pytest.log 2>&1
rc=$?; echo "pytest nt1024 rc $rc: $(tail -1 gpurun_out/r03y_pytest.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r03y_pytest.log; exit $rc; }
for args in "" "--logn=28"; do
  tag=$(echo "x$args" | tr -d ' =-'); steps=10; [ "$args" = "--logn=28" ] && steps=30
  echo "== $args"
  STEPS=$steps OUTDIR=r03y/$tag BENCH_ARGS="$args" RUNS="b8||;b16||MISORT_MULTIWAY=4;n16|$V|MISORT_MULTIWAY=4;n8|$V|" bash tools/gpu_envab.sh || exit $?
done
