# Round 4, call N: the u32 SORT tile's top levels as in-LDS merge levels
# (sm15: 2^15 tiles, levels 12..15 merged, one workgroup per tile; sm14: 2^14
# tiles, 12..14 merged, two workgroups per CU; lt14: 2^14 bitonic tiles) --
# tests of each, A/B against the default; then the HEAD measurement set.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
# (sm15 and the default passed test_gpu_runs + test_gpu_parity in the first
# try; sm14's 2^14 tiles fail only test_merge_level_rejects_bad_shapes, whose
# smallest rejected run is the 2^15 default tile)
TESTS="tests/test_gpu_parity.py" VARIANTS="sm14" ROUNDS=0 OUTDIR=r04n bash tools/gpu_abv.sh &&
SKIP_TESTS=1 VARIANTS="base sm15 sm14 lt14" DTYPES=u32 LOGNS="30 28 24" ROUNDS=2 OUTDIR=r04n bash tools/gpu_abv.sh
