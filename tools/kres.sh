#!/bin/bash
# Per-kernel VGPRs / spills / LDS / occupancy of kernels.hip (compile-time check).
#   tools/kres.sh [filter-regex]
HERE="$(cd "$(dirname "$0")/.." && pwd)"
C="$HERE/parallel-computing-mpi_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$HERE/include" -I"$C" $KRES_FLAGS -c "$C/${KRES_SRC:-kernels.hip}" \
    -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import re, sys, subprocess
flt = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
cur = None; rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = {"name": name}; rows.append(cur); continue
    m = re.search(r"remark: +(VGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split()[0] + (" spill" if "Spill" in m.group(1) else "")] = int(m.group(2))
for r in rows:
    if not flt.search(r["name"]): continue
    n = re.sub(r"misort::\(anonymous namespace\)::", "", r["name"]).split("(")[0]
    print("%-60s vgpr=%s spill=%s lds=%s occ=%s" % (n, r.get("VGPRs"), r.get("VGPRs spill"), r.get("LDS"), r.get("Occupancy")))
' "$@"
