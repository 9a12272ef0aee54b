# Round 5, call C: tail merge-split + coalesced codec gaps -- parity/multirank/rccl tests,
# then the per-GPU work of configs 4 and 5 at P = 8 under rocprofv3 (rank_work_config{4,5}_p8).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r05c"; mkdir -p "$O"; cd "$R"
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_rccl_large.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest.log" | head -20; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err" && echo "rw c4 ok" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c5" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --n 536870909 --p 8 --dtype u64 > "$O/rw_c5.json" 2> "$O/rw_c5.err" && echo "rw c5 ok" || exit $?
cd "$R" && python3 tools/rank_work_summary.py "$O/rw_c4" "$O/rw_c4.json" > "$O/rank_work_config4_p8.txt" && python3 tools/rank_work_summary.py "$O/rw_c5" "$O/rw_c5.json" > "$O/rank_work_config5_p8.txt"; tail -12 "$O/rank_work_config4_p8.txt"
