# One sort's kernel timeline (rocprofv3 kernel trace of bench.py): every kernel
# of the step between the last two SORT-tile launches, with its start offset,
# duration and the idle gap before it.  TAGS: name:args (args ',' separated).
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-timeline}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for spec in ${TAGS:-u32_24:--logn=24}; do
  tag=${spec%%:*}; args=${spec#*:}; args=${args//=/ }; args=${args//,/ }
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/$tag" -o $tag --output-format csv -- \
    python3 "$R/bench.py" $args --steps 4 --warmup 1 --no-cpu-baseline > "$O/$tag.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$tag failed rc $rc"; tail -5 "$O/$tag.log"; exit $rc; }
  TAG=$tag O=$O python3 - <<'PY' | tee "$O/${TAG:-x}_timeline.txt"
import csv, os, re, glob
O, tag = os.environ["O"], os.environ["TAG"]
f = glob.glob(f"{O}/{tag}/**/{tag}_kernel_trace.csv", recursive=True)
rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: re.sub(r"misort::\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
sorts = [i for i, r in enumerate(rows) if "k_sort_" in name(r)]
a, b = sorts[-2], sorts[-1]
t0 = int(rows[a]["Start_Timestamp"]); prev = t0; busy = 0
print("==", tag, "one step:", b - a, "kernels")
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f'{(s - t0) / 1e3:8.1f} us  +{(s - prev) / 1e3:5.1f} gap  {(e - s) / 1e3:7.1f} us  {name(r)[:70]}')
    prev = e
span = int(rows[b]["Start_Timestamp"]) - t0
print(f"span {span / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, gaps {(span - busy) / 1e3:.1f} us")
PY
done
