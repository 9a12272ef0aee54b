# Round 4, call L: 4-ary co-rank searches (three probes per step, half the
# dependent LDS round trips; cor4) against the binary search --
# merge/parity tests, A/B (u32 and u64), SQ probe modes.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04l"; mkdir -p "$O"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="cor4" ROUNDS=0 OUTDIR=r04l bash tools/gpu_abv.sh || exit $?
SKIP_TESTS=1 VARIANTS="base cor4" DTYPES=u32 LOGNS="30 28 24" ROUNDS=2 OUTDIR=r04l bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base cor4" DTYPES=u64 LOGNS="29" ROUNDS=2 OUTDIR=r04l bash tools/gpu_abv.sh &&
MISORT_LIBRARY=$R/parallel-computing-mpi_amd/lib/variants/libmisort_cor4.so MISORT_MK_PROBE=1 OUTDIR=r04l/sq_probe bash tools/gpu_sq2.sh > "$O/sq_probe.txt" && echo "sq ok"
