# Round record: GPU tests, bench with CPU baseline, rocprofv3 kernel stats, PMC traffic.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_rec.log 2>&1; rc=$?; tail -1 gpurun_out/bench_rec.log; [ $rc -eq 0 ] || exit $rc
TAG=rec bash tools/gpu_prof.sh && bash tools/gpu_pmc30.sh
