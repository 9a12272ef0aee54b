# Full round-end style check: smoke, the whole -m gpu suite, the default bench (CPU baseline included).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-full}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?; echo "smoke rc $rc"; tail -3 "$O/smoke.log"; fatal $rc smoke
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$O/pytest.log" 2>&1; rc=$?; echo "pytest rc $rc"; grep -E "FAILED|passed|failed" "$O/pytest.log" | tail -12; fatal $rc pytest
timeout -k 10 400 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.err"; rc=$?; echo "bench rc $rc"; tail -c 3000 "$O/bench.json"; fatal $rc bench
