# Round 5: kernel trace of the 2^24 u32 sort (config 2) -- per-sort kernel time vs the sort's wall time
# (launch gaps), for the small-sort planning path.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/small"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof24" -o p24 --output-format csv -- python3 "$R/bench.py" --logn 24 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench24.json" 2> "$O/bench24.err" || { tail -5 "$O/bench24.err"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof26" -o p26 --output-format csv -- python3 "$R/bench.py" --logn 26 --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench26.json" 2> "$O/bench26.err" || { tail -5 "$O/bench26.err"; exit 1; }
echo ok
