# Round 4, call S: more merge levels in the SORT tiles -- u64 F = 10 / 9 / 8
# (one tile per workgroup) and u32 2^14 tiles F = 12 (default) / 11 / 10;
# tests of m64f9 and m32f10, then A/B benches.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04s"; mkdir -p "$O"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="m64f9 m32f10" ROUNDS=0 OUTDIR=r04s bash tools/gpu_abv.sh || exit $?
V=parallel-computing-mpi_amd/lib/variants
RUNS="f10|$V/libmisort_m64f10.so|MISORT_PERSIST_U64=0;f9|$V/libmisort_m64f9.so|MISORT_PERSIST_U64=0;f8|$V/libmisort_m64f8.so|MISORT_PERSIST_U64=0" \
  BENCH_ARGS="--dtype u64 --logn 29" STEPS=10 OUTDIR=r04s bash tools/gpu_envab.sh || exit $?
RUNS="f10_26|$V/libmisort_m64f10.so|MISORT_PERSIST_U64=0;f9_26|$V/libmisort_m64f9.so|MISORT_PERSIST_U64=0" \
  BENCH_ARGS="--dtype u64 --logn 26" STEPS=20 OUTDIR=r04s bash tools/gpu_envab.sh || exit $?
RUNS="u12_30||;u11_30|$V/libmisort_m32f11.so|;u10_30|$V/libmisort_m32f10.so|" BENCH_ARGS="--logn 30" STEPS=10 OUTDIR=r04s bash tools/gpu_envab.sh || exit $?
RUNS="u12_26||;u11_26|$V/libmisort_m32f11.so|;u10_26|$V/libmisort_m32f10.so|" BENCH_ARGS="--logn 26" STEPS=20 OUTDIR=r04s bash tools/gpu_envab.sh
