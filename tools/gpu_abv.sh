# A/B of library variants on one box: the merge/parity tests under each
# variant (MISORT_LIBRARY), then alternating benches.
#   VARIANTS="base glds csel" LOGNS="30 28" DTYPES="u32" ROUNDS=2 bash tools/gpu_abv.sh
# base = lib/libmisort.so; NAME = lib/variants/libmisort_NAME.so
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-abv}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
lib() { [ "$1" = base ] && echo "$R/parallel-computing-mpi_amd/lib/libmisort.so" || echo "$R/parallel-computing-mpi_amd/lib/variants/libmisort_$1.so"; }
if [ -z "$SKIP_TESTS" ]; then
  for v in $VARIANTS; do
    [ "$v" = base ] && continue
    MISORT_LIBRARY=$(lib $v) timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_gpu_runs.py tests/test_gpu_parity.py tests/test_gpu_baseline_configs.py} -x -q --timeout 120 --timeout-method thread \
      > "$O/pytest_$v.log" 2>&1; rc=$?; echo "pytest $v rc $rc: $(tail -1 $O/pytest_$v.log)"; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
  done
fi
for rep in $(seq 1 ${ROUNDS:-2}); do
  for dt in ${DTYPES:-u32}; do for L in ${LOGNS:-30}; do for v in $VARIANTS; do
    f="$O/${v}_${dt}_${L}_$rep.json"
    MISORT_LIBRARY=$(lib $v) timeout -k 10 200 python3 -u bench.py --dtype $dt --logn $L --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > "$f" 2> "${f%.json}.err"; rc=$?
    fatal $rc "bench $v"; [ $rc -ne 0 ] && { tail -3 "${f%.json}.err"; exit $rc; }
    python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
ks = " ".join(f"{n}:{v['launches_per_step']:.0f}x{v['avg_launch_us']:.0f}" for n, v in k.items())
print(sys.argv[1].split("/")[-1][:-5], round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms err", d["check_errors"], ks)
PY
  done; done; done
done
