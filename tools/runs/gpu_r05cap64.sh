# Round 5: u64 16-way chunk capacity 8896 keys (139 64-key fences) vs 8832 -- the 64-key build is the one
# that runs at 2^29 u64; the 128-key rows (2^28) need CAP a multiple of 128, so the variant there is not valid
# for comparison and is not run.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
RUNS="base||;c8896|$V/libmisort_c64_8896.so|" BENCH_ARGS="--dtype u64 --logn 29" STEPS=20 OUTDIR=cap64 bash tools/runs/gpu_envab.sh || exit $?
RUNS="base||;c8896|$V/libmisort_c64_8896.so|" BENCH_ARGS="--dtype f64 --logn 29" STEPS=20 OUTDIR=cap64 bash tools/runs/gpu_envab.sh || exit $?
