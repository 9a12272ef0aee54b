# Round 5 end-of-round record, part 3: the per-GPU device work of configs 4 and 5 at P = 8
# (tools/rank_work_probe.py under rocprofv3 -> rank_work_config{4,5}_p8.txt).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r05fin3}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err" && echo "rw c4 ok" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c5" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --n 536870909 --p 8 --dtype u64 > "$O/rw_c5.json" 2> "$O/rw_c5.err" && echo "rw c5 ok" || exit $?
cd "$R" && python3 tools/rank_work_summary.py "$O/rw_c4" "$O/rw_c4.json" > "$O/rank_work_config4_p8.txt" && python3 tools/rank_work_summary.py "$O/rw_c5" "$O/rw_c5.json" > "$O/rank_work_config5_p8.txt"; tail -12 "$O/rank_work_config4_p8.txt"
