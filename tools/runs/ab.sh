#!/bin/bash
# Round-6 parameterised GPU A/B runner (replaces the one-off gpu_r0*.sh scripts).
#   TESTS="tests/test_gpu_runs.py ..."   pytest files run against every library in TESTLIBS first
#   TESTLIBS="base bi48"                 libraries to test (base = lib/libmisort.so, NAME = lib/variants/libmisort_NAME.so)
#   VARIANTS="base nobi base@MISORT_X=1,MISORT_Y=2" LOGNS="30 28" DTYPES="u32" ROUNDS=2 STEPS=20
#                                        alternating bench lines (LIB@ENV=V,...: a library under environment settings)
#   PROF="30:u32"                        rocprofv3 --kernel-trace --stats of bench.py per logn:dtype (base library)
#   OUTDIR=name                          results under gpurun_out/NAME
# Every GPU step runs under its own timeout; the script stops at the first failure.
set -o pipefail
R="$GRAFT_REPO_ROOT"; [ -n "$R" ] || R="$(cd "$(dirname "$0")/../.." && pwd)"
O="$R/gpurun_out/${OUTDIR:-ab}"; mkdir -p "$O"; cd "$R"
export TMPDIR=/tmp
fatal() { case "$1" in 0) ;; *) echo "rc $1 in $2: stopping"; exit "$1";; esac; }
lib() { [ "$1" = base ] && echo "$R/parallel-computing-mpi_amd/lib/libmisort.so" || echo "$R/parallel-computing-mpi_amd/lib/variants/libmisort_$1.so"; }
if [ -n "$TESTS" ]; then
  for v in ${TESTLIBS:-base}; do
    MISORT_LIBRARY=$(lib $v) timeout -k 10 ${TEST_TIMEOUT:-500} python3 -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
      > "$O/pytest_$v.log" 2>&1; rc=$?; echo "pytest $v rc $rc: $(tail -1 $O/pytest_$v.log)"; fatal $rc "pytest $v"
  done
fi
for rep in $(seq 1 ${ROUNDS:-2}); do
  for dt in ${DTYPES:-u32}; do for L in ${LOGNS:-30}; do for v in $VARIANTS; do
    lv=${v%%@*}; ev=""; [ "$lv" != "$v" ] && ev=$(echo "${v#*@}" | tr ',' ' ')
    f="$O/$(echo "$v" | tr '@=,' '_-_')_${dt}_${L}_$rep.json"
    env $ev MISORT_LIBRARY=$(lib $lv) timeout -k 10 200 python3 -u bench.py --dtype $dt --logn $L --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS > "$f" 2> "${f%.json}.err"; rc=$?
    [ $rc -eq 0 ] || tail -3 "${f%.json}.err"; fatal $rc "bench $v"
    python3 - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernels", {})
ks = " ".join(f"{n}:{v['launches_per_step']:.0f}x{v['avg_launch_us']:.0f}" for n, v in k.items())
print(sys.argv[1].split("/")[-1][:-5], round(d["value"], 2), "Gkeys/s", round(d["ms_per_step"], 3), "ms err", d["check_errors"], ks)
PY
  done; done; done
done
for p in $PROF; do
  L=${p%%:*}; dt=${p##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_${dt}_$L" -o run --output-format csv -- python3 -u bench.py --dtype $dt --logn $L --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline \
    > "$O/prof_${dt}_$L.json" 2> "$O/prof_${dt}_$L.err"; fatal $? "rocprof $p"
  find "$O/prof_${dt}_$L" -name "*kernel_stats.csv" -exec cp {} "$O/prof_${dt}_${L}_kernel_stats.csv" \;
  find "$O/prof_${dt}_$L" -name "*.db" -delete
  python3 - "$O/prof_${dt}_${L}_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:8]:
    print("rocprof", r["Name"].split("(")[0][-50:], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
echo done
