# SQ counters (LDS/VALU/wait) of the sort kernels at 2^30 u32, one rocprofv3 --pmc pass.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
OUT="$R/gpurun_out/sq30"; mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --kernel-include-regex "k_stream" -d "$OUT/sq" -o sq --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-events > "$OUT/sq.log" 2>&1 || { tail -3 "$OUT/sq.log"; exit 1; }
python3 - <<'PY'
import csv, collections, os, re
R = os.environ["GRAFT_REPO_ROOT"]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f"{R}/gpurun_out/sq30/sq/sq_counter_collection.csv")):
    m = re.search(r"k_stream<unsigned int, (\d+), (\d), (\d+), (\w+), \w+, (\w+)>", r["Kernel_Name"])
    if not m: continue
    key = ("SORT", "MERGE", "ROWS", "SPAN")[int(m.group(2))] + " R=" + m.group(3)
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(key, r["Counter_Name"])] += 1
for k, c in sorted(acc.items()):
    d = {x: v / max(1, n[(k, x)]) for x, v in c.items()}
    w = d.get("SQ_WAVE_CYCLES", 1)
    print(f"{k:12s} waves {d.get('SQ_WAVES',0):9.0f} valu/wave {d.get('SQ_INSTS_VALU',0)/max(1,d.get('SQ_WAVES',1)):8.0f} "
          f"lds/wave {d.get('SQ_INSTS_LDS',0)/max(1,d.get('SQ_WAVES',1)):7.0f} waitLDS/wavecyc {d.get('SQ_WAIT_INST_LDS',0)/w:5.3f} "
          f"waitany/wavecyc {d.get('SQ_WAIT_ANY',0)/w:5.3f} bankconf/ldsinst {d.get('SQ_LDS_BANK_CONFLICT',0)/max(1,d.get('SQ_INSTS_LDS',1)):6.3f}")
PY
