# Round 4, call Z: end-of-round HEAD (merge-level tiles, chunk capacities) -- the
# whole GPU suite and smoke().
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04z"; mkdir -p "$O"; cd "$R"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest_gpu.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest_gpu.log" | head -20; exit $rc; }
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1; rc=$?; tail -2 "$O/smoke.log"; exit $rc
