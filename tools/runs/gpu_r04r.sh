# Round 4, call R: the u64 SORT tile's top levels as in-LDS merge levels
# (variants m64fF: levels F..13 merged, F = 12 / 11 / 10) -- tests of each,
# then u64 2^29 and 2^26 benches against the default, persistent (default) and
# one-tile-per-workgroup (MISORT_PERSIST_U64=0) grids.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04r"; mkdir -p "$O"; cd "$R"
TESTS="tests/test_gpu_runs.py tests/test_gpu_parity.py" VARIANTS="m64f12 m64f10" ROUNDS=0 OUTDIR=r04r bash tools/gpu_abv.sh || exit $?
L="$R/parallel-computing-mpi_amd/lib/variants"
RUNS="base||;f12|parallel-computing-mpi_amd/lib/variants/libmisort_m64f12.so|;f11|parallel-computing-mpi_amd/lib/variants/libmisort_m64f11.so|;f10|parallel-computing-mpi_amd/lib/variants/libmisort_m64f10.so|;f12np|parallel-computing-mpi_amd/lib/variants/libmisort_m64f12.so|MISORT_PERSIST_U64=0;f10np|parallel-computing-mpi_amd/lib/variants/libmisort_m64f10.so|MISORT_PERSIST_U64=0" \
  BENCH_ARGS="--dtype u64 --logn 29" STEPS=10 OUTDIR=r04r bash tools/gpu_envab.sh || exit $?
RUNS="base26||;f12_26|parallel-computing-mpi_amd/lib/variants/libmisort_m64f12.so|;f10_26|parallel-computing-mpi_amd/lib/variants/libmisort_m64f10.so|;f10np_26|parallel-computing-mpi_amd/lib/variants/libmisort_m64f10.so|MISORT_PERSIST_U64=0" \
  BENCH_ARGS="--dtype u64 --logn 26" STEPS=20 OUTDIR=r04r bash tools/gpu_envab.sh
