# Round 5: planning under 64-key fences -- nested fence merge threshold A/B at 2^30 u32, and the
# per-kernel rocprofv3 stats of the default 2^30 u32 bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/fg6b"; mkdir -p "$O"; cd "$R"
RUNS="n23||;n22||MISORT_FENCE_NEST_MIN=22;n24||MISORT_FENCE_NEST_MIN=24;n25||MISORT_FENCE_NEST_MIN=25" BENCH_ARGS="--logn 30" STEPS=20 OUTDIR=fg6b bash tools/runs/gpu_envab.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o u32_30 --output-format csv -- python3 "$R/bench.py" --logn 30 --steps 5 --warmup 2 --no-cpu-baseline > "$O/prof.log" 2>&1 || { echo "prof failed"; tail -3 "$O/prof.log"; exit 1; }
echo prof ok
