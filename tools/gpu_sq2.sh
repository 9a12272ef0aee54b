# SQ counters of chosen kernels (REGEX) in one rocprofv3 --pmc pass per counter set; bench args in BENCH_ARGS.
set -o pipefail
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/${OUTDIR:-sq}"; mkdir -p "$OUT"; cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${REGEX:-k_mergek}" -d "$OUT/p$i" -o p$i --output-format csv -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-events $BENCH_ARGS > "$OUT/p$i.log" 2>&1 \
    || { echo "pass $i failed"; tail -3 "$OUT/p$i.log"; exit 1; }
done
python3 - <<'PY'
import csv, collections, os, re, glob
O = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out", os.environ.get("OUTDIR", "sq"))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        key = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void misort::(anonymous namespace)::", "")
        acc[key][r["Counter_Name"]] += float(r["Counter_Value"]); n[(key, r["Counter_Name"])] += 1
for k, c in sorted(acc.items()):
    d = {x: v / max(1, n[(k, x)]) for x, v in c.items()}
    wv = max(1, d.get("SQ_WAVES", 1)); w = max(1, d.get("SQ_WAVE_CYCLES", 1))
    print(k, " ".join(f"{x}={d[x]:.4g}" for x in sorted(d)))
    print("   per wave: valu %.0f lds %.0f salu %.0f | frac of wave-cycles: waitLDS %.3f waitany %.3f waitinst %.3f activeVALU %.3f activeLDS %.3f | bankconf/ldsinst %.3f" % (
        d.get("SQ_INSTS_VALU", 0) / wv, d.get("SQ_INSTS_LDS", 0) / wv, d.get("SQ_INSTS_SALU", 0) / wv,
        d.get("SQ_WAIT_INST_LDS", 0) / w, d.get("SQ_WAIT_ANY", 0) / w, d.get("SQ_WAIT_INST_ANY", 0) / w,
        d.get("SQ_ACTIVE_INST_VALU", 0) / w, d.get("SQ_ACTIVE_INST_LDS", 0) / w,
        d.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, d.get("SQ_INSTS_LDS", 1))))
PY
