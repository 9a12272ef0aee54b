set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== box"; nproc; rocm-smi --showproductname 2>&1 | head -8; ls /opt/conda/bin/mpirun
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not baseline_size" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.log 2>&1; rc=$?; tail -5 gpurun_out/bench1.log; exit $rc
