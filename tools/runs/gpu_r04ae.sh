# Round 4, call AE: after the per-size tile rule -- the whole GPU suite and
# smoke(), the per-GPU work of config 4 at P = 8 (2^27 u32 blocks, now on
# 2^14 tiles) and the 2^27 / 2^23 benches.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04ae"; mkdir -p "$O"; cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || exit $?
tail -1 "$O/smoke.log"
for a in "--logn 27" "--logn 23"; do
  n=$(echo $a | tr -d ' -'); timeout -k 10 200 python3 bench.py $a --steps 30 --warmup 5 --no-cpu-baseline > "$O/bench_$n.json" 2> "$O/bench_$n.err" || exit $?
  python3 -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value'],2), round(d['ms_per_step'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/rw_c4" -o rw --output-format csv -- python3 "$R/tools/rank_work_probe.py" --logn 30 --p 8 --dtype u32 > "$O/rw_c4.json" 2> "$O/rw_c4.err" && echo "rw ok"
