# Round 5: k_bounds with the scanned-count loads issued beside the fence load and 32-bit chunk divisions
# (MISORT_BOUNDS_EARLY=1) vs HEAD; tests of the merge passes under the variant first.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/bearly"; mkdir -p "$O"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
MISORT_LIBRARY="$R/$V/libmisort_bearly.so" timeout -k 10 500 python3 -u -m pytest tests/test_gpu_runs.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$O/pytest.log" | head; exit $rc; }
for a in "--logn 30" "--logn 28" "--dtype u64 --logn 29"; do
  RUNS="base||;bearly|$V/libmisort_bearly.so|" BENCH_ARGS="$a" STEPS=20 OUTDIR=bearly bash tools/runs/gpu_envab.sh || exit $?
done
