# Round 5: 16-way chunk shapes under 64-key fences: 18 outputs per lane / 8832 keys / four workgroups per CU
# (c18w4) and 20 / 9728 / three (c20w3) vs 22 / 10752 / three (base); 2^28 rows force 64-key fences.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
V=parallel-computing-mpi_amd/lib/variants
RUNS="base||;c18w4|$V/libmisort_c18w4.so|;c20w3|$V/libmisort_c20w3.so|" BENCH_ARGS="--logn 30" STEPS=20 OUTDIR=shape bash tools/runs/gpu_envab.sh || exit $?
RUNS="base6||MISORT_FENCE_FG6_MIN=20;c18w4_6|$V/libmisort_c18w4.so|MISORT_FENCE_FG6_MIN=20;c20w3_6|$V/libmisort_c20w3.so|MISORT_FENCE_FG6_MIN=20" BENCH_ARGS="--logn 28" STEPS=20 OUTDIR=shape bash tools/runs/gpu_envab.sh || exit $?
