# Round 5: kernel trace of the 2^24 u32 sort (config 2): planning launches and the gaps between them.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/p24"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o u32_24 --output-format csv -- python3 "$R/bench.py" --logn 24 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "prof failed"; tail -3 "$O/prof.log"; exit 1; }
echo prof ok
