# Round 4, call A: k_mergek merge chains -- one key per LDS read (base) vs two
# (ch1: ds_read2, ch2: one wide unaligned read), and ch2 at 256 lanes x 36 keys;
# SQ counters of k_mergek for base and ch2.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="ch2 ch2n256 ch2it24" OUTDIR=r04a ROUNDS=0 bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base ch1 ch2 ch2n256 ch2it24" DTYPES="u32" LOGNS="30 28" ROUNDS=2 OUTDIR=r04a bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base ch2" DTYPES="u64" LOGNS="29" ROUNDS=2 OUTDIR=r04a bash tools/gpu_abv.sh &&
OUTDIR=r04a/sq_base bash tools/gpu_sq2.sh &&
MISORT_LIBRARY=$R/parallel-computing-mpi_amd/lib/variants/libmisort_ch2.so OUTDIR=r04a/sq_ch2 bash tools/gpu_sq2.sh
