# Round 3, call F: k_sort_u64 (512 x 16-key u64 SORT tile) and glds k_mergek:
# the sort/parity/baseline-config tests, then env A/B benches (MISORT_SORT_U64).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03f}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py tests/test_gpu_staging.py} -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc: $(tail -1 $O/pytest.log)"; fatal $rc pytest; [ $rc -ne 0 ] && { tail -30 "$O/pytest.log"; exit $rc; }
one() {  # tag env dtype logn
  f="$O/$1_$3_$4.json"
  env $2 timeout -k 10 200 python3 -u bench.py --dtype $3 --logn $4 --steps 20 --warmup 5 --no-cpu-baseline > "$f" 2> "${f%.json}.err"; rc=$?
  fatal $rc "bench $1"; [ $rc -ne 0 ] && { tail -3 "${f%.json}.err"; exit $rc; }
  python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
print(sys.argv[1].split("/")[-1][:-5], round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms err", d["check_errors"], " ".join(f"{n}:{v['launches_per_step']:.0f}x{v['avg_launch_us']:.0f}" for n, v in k.items()))
PY
}
for rep in 1 2; do
  for L in ${U64_LOGNS:-29 26}; do one new$rep MISORT_SORT_U64=1 u64 $L; one old$rep MISORT_SORT_U64=0 u64 $L; done
done
one new MISORT_SORT_U64=1 u32 30
exit 0
