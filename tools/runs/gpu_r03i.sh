# Round 3, call I: the network engine vs the multi-way passes for small u32
# sorts (verdict r2 item 8): default (network up to 2^23) vs
# MISORT_MERGE_MIN_LOG2=0 (multi-way from 2^16), 2 rounds per size.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-r03i}"; mkdir -p "$O"; cd "$R"
fatal() { case "$1" in 124|137|134|139) echo "fatal rc $1 in $2: stopping"; exit "$1";; esac; }
for rep in 1 2; do
  for L in ${LOGNS:-16 17 18 19 20 21 22 23 24}; do
    for v in net mw; do
      e="MISORT_MERGE_MIN_LOG2=23"; [ $v = mw ] && e="MISORT_MERGE_MIN_LOG2=0"
      f="$O/${v}_$L_$rep.json"; f="$O/${v}_${L}_${rep}.json"
      env $e timeout -k 10 120 python3 -u bench.py --logn $L --steps 50 --warmup 10 --no-cpu-baseline > "$f" 2> "${f%.json}.err"; rc=$?
      fatal $rc "bench $v $L"; [ $rc -ne 0 ] && { tail -3 "${f%.json}.err"; exit $rc; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1][:-5], round(d['value'],2), 'Gkeys/s', round(d['ms_per_step'],4), 'ms err', d['check_errors'])" "$f"
    done
  done
done
