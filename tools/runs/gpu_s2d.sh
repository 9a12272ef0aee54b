# Session-2: exchange with the device-side count (one host wait per stage) and the
# hand-written codec scan: multi-rank/RCCL/staging/baseline-config GPU tests, codec probe,
# a P=8 group bench at 2^30 u32.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-s2d}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl.py tests/test_gpu_staging.py \
  tests/test_gpu_baseline_configs.py tests/test_gpu_psort_bin.py tests/test_gpu_quick.py tests/test_gpu_sample.py \
  -x -q --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; tail -5 "$O/pytest.log"
fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -u tools/codec_probe.py > "$O/codec.jsonl" 2>&1; rc=$?; tail -6 "$O/codec.jsonl"; fatal $rc codec
timeout -k 10 300 python3 -u tools/group_bench.py --p 8 --logn 30 --steps 3 > "$O/bench_g8.json" 2> "$O/bench_g8.err"; rc=$?
echo "bench g8 rc $rc"; tail -c 2500 "$O/bench_g8.json"; tail -3 "$O/bench_g8.err"
