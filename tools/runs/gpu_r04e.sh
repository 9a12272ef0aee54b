# Round 4, call E: the 16-way default plan and the skewed co-rank (lanes
# 16..31 of each LDS group search from d + 1) -- merge/parity tests, A/B
# against the unskewed build, larger chunks (IT 20 / 22 outputs per lane,
# 3 workgroups per CU); per-GPU device work of an 8-GPU step (config 4
# and 5 at P = 8) under a rocprofv3 kernel trace; a HEAD PMC traffic capture
# at 2^30 u32.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04e"; mkdir -p "$O"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="it20 it22" ROUNDS=0 OUTDIR=r04e/skew bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base noskew it20 it22" DTYPES=u32 LOGNS="30 28 27" ROUNDS=2 OUTDIR=r04e/skew bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base noskew" DTYPES=u64 LOGNS="29" ROUNDS=2 OUTDIR=r04e/skew bash tools/gpu_abv.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err"; rc=$?
echo "rw_c4 rc $rc"; case $rc in 0) ;; *) tail -5 "$O/rw_c4.err"; exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c5" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --n 536870909 --p 8 --dtype u64 > "$O/rw_c5.json" 2> "$O/rw_c5.err"; rc=$?
echo "rw_c5 rc $rc"; case $rc in 0) ;; *) tail -5 "$O/rw_c5.err"; exit $rc;; esac
cd "$R" && OUTDIR=r04e/pmc30 bash tools/gpu_pmc30.sh > /dev/null && echo "pmc30 ok"
