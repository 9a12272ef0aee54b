# Wide ROWS pass bring-up: parity tests, the GPU suite with wide passes on,
# bench A/B (wide off / on), and the wide shapes' measured costs at 2^30.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_wide.log; [ $rc -eq 0 ] || exit $rc
MISORT_WIDE=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_wide1.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_wide1.log; [ $rc -eq 0 ] || exit $rc
TESTS=0 VARIANTS="${VARIANTS:-w0=MISORT_WIDE=0 w1=MISORT_WIDE=1 w0b=MISORT_WIDE=0 w1b=MISORT_WIDE=1}" bash tools/gpu_ab.sh || exit $?
timeout -k 10 400 python -u tools/pass_costs.py --logn 30 --kinds wide_pass --reps 4 > gpurun_out/pc_wide_30.json 2> gpurun_out/pc_wide_30.log; rc=$?; tail -2 gpurun_out/pc_wide_30.log; exit $rc
