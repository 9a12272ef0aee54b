#!/usr/bin/env python3
"""One line per bench JSON of a tools/runs/ab.sh output directory:
    python tools/ab_summary.py gpurun_out/r06e [header text ...]"""
import glob
import json
import os
import sys

d = sys.argv[1]
if len(sys.argv) > 2:
    print("# " + " ".join(sys.argv[2:]))
for f in sorted(glob.glob(os.path.join(d, "*.json")), key=lambda p: (p.rsplit("_", 1)[-1], os.path.getmtime(p))):
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except (ValueError, IndexError):
        continue
    k = j.get("kernels", {})
    ks = " ".join(f"{n}:{v['launches_per_step']:.0f}x{v['avg_launch_us']:.0f}" for n, v in k.items())
    print(os.path.basename(f)[:-5], round(j["value"], 2), "Gkeys/s", round(j["ms_per_step"], 3), "ms err",
          j["check_errors"], ks)
