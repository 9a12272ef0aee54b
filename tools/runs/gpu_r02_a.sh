# Round-2 GPU check: CPU share probe, the full -m gpu suite, the N=1 bench and
# the N=2 launcher path (ranks sharing the GPU: RCCL over sockets).
# Any timeout / abort / segfault ends the script (no further GPU step).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r02a"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; grep -m1 "model name" /proc/cpuinfo; free -g | head -2; } > "$O/host.txt" 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc" | tee -a "$O/pytest.log"
tail -5 "$O/pytest.log"; fatal $rc pytest
timeout -k 10 400 python3 bench.py > "$O/bench_n1.json" 2> "$O/bench_n1.err"; rc=$?; echo "bench n1 rc $rc"
tail -c 3000 "$O/bench_n1.json"; fatal $rc bench_n1
timeout -k 10 300 python3 bench.py --gpus 2 --logn 26 --steps 3 --warmup 1 --no-cpu-baseline \
  > "$O/bench_n2_shared.json" 2> "$O/bench_n2_shared.err"; rc=$?; echo "bench n2 rc $rc"
tail -c 2000 "$O/bench_n2_shared.json"
