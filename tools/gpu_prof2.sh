# rocprofv3 kernel stats for the bench configs (TAGS: name:args), summarised per kernel.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/${OUTDIR:-prof}"; mkdir -p "$O"; cd /tmp && export TMPDIR=/tmp
for spec in ${TAGS:-u32_30:--logn=30}; do
  tag=${spec%%:*}; args=${spec#*:}; args=${args//=/ }; args=${args//,/ }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/$tag" -o $tag --output-format csv -- \
    python3 "$R/bench.py" $args --steps 3 --warmup 1 --no-cpu-baseline > "$O/$tag.log" 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$tag failed rc $rc"; tail -5 "$O/$tag.log"; exit $rc; }
  TAG=$tag O=$O python3 - <<'PY'
import csv, os, re, glob
O, tag = os.environ["O"], os.environ["TAG"]
f = glob.glob(f"{O}/{tag}/**/{tag}_kernel_stats.csv", recursive=True) or glob.glob(f"{O}/{tag}/{tag}_kernel_stats.csv")
print("==", tag)
for r in csv.DictReader(open(f[0])):
    n = re.sub(r"misort::\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
    print(f'{n[:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f}%')
PY
done
