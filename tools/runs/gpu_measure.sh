# Measurement run on the GPU box (invoked via gpurun from the repo root).
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
echo "== big parity"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k baseline_size > gpurun_out/pytest_big.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_big.log; [ $rc -eq 0 ] || exit $rc
echo "== bench (with cpu baseline)"
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_full.log 2>&1; rc=$?; tail -2 gpurun_out/bench_full.log; [ $rc -eq 0 ] || exit $rc
echo "== sweep"
for L in 22 24 25 26 27 28 29; do
  timeout -k 10 120 python -u bench.py --logn $L --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$L.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sweep_$L.log').read().strip().splitlines()[-1]);print($L, round(d['value'],2), {k:(round(v['ms_per_step'],3), round(v['achieved_GBs'])) for k,v in d['kernels'].items()})"
done
echo "== rocprof"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o r1 --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/rocprof.log" 2>&1; rc=$?; tail -2 "$R/gpurun_out/rocprof.log"; [ $rc -eq 0 ] || exit $rc
cd "$R"
echo "== psort"
for P in 1; do timeout -k 10 120 /opt/conda/bin/mpirun -np $P parallel-computing-mpi_amd/bin/psort 16777216 > gpurun_out/psort_$P.log 2>&1 || exit 1; cat gpurun_out/psort_$P.log; done
timeout -k 10 120 /opt/conda/bin/mpirun -np 1 parallel-computing-mpi_amd/bin/psort 1031 2>&1 | tail -3
find gpurun_out/prof -name "*.csv" | head
