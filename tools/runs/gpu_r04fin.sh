# Round 4, final call: the HEAD measurement set (bench line with the CPU
# baseline, rocprofv3 stats, PMC traffic, 2^28 / 2^24 / u64 benches, per-GPU
# work of the 8-GPU configs), then the whole GPU suite and smoke().
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/runs/gpu_r04fin_measure.sh || exit $?
O="$R/gpurun_out/r04fin"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1; rc=$?; tail -2 "$O/smoke.log"; exit $rc
