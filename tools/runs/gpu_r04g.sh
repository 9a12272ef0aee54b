# Round 4, call G: 16-way u32 passes on 22-key lanes (CAP 10752, three
# workgroups per CU) as the default -- merge, parity and full-size config
# tests, A/B against the 8-way chunk shape for every pass (it16off).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/r04g"; mkdir -p "$O"; cd "$R"
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; [ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 VARIANTS="base it16off" DTYPES=u32 LOGNS="30 29 28 27 26" ROUNDS=2 OUTDIR=r04g bash tools/gpu_abv.sh
