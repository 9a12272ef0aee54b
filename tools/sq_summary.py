#!/usr/bin/env python3
"""Per-kernel SQ counter summary of tools/gpu_sq2.sh output dirs:
   tools/sq_summary.py gpurun_out/<dir> [...]"""
import collections
import csv
import glob
import re
import sys

for O in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            key = r["Kernel_Name"].replace("misort::(anonymous namespace)::", "").replace("void ", "")
            key = re.sub(r"\(.*", "", key)
            acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(key, r["Counter_Name"])] += 1
    for k, c in sorted(acc.items()):
        d = {x: v / max(1, n[(k, x)]) for x, v in c.items()}
        wv = max(1, d.get("SQ_WAVES", 1))
        w = max(1, d.get("SQ_WAVE_CYCLES", 1))
        print(O, k, "launches", n[(k, "SQ_WAVES")], "waves", int(wv))
        print("   per wave: valu %.0f lds %.0f salu %.0f vmrd %.0f vmwr %.0f | busy %.3g wavecyc/wave %.0f | "
              "waitLDS %.3f waitany %.3f waitinst %.3f activeVALU %.3f activeLDS %.3f | bankconf/ldsinst %.3f" % (
                  d.get("SQ_INSTS_VALU", 0) / wv, d.get("SQ_INSTS_LDS", 0) / wv, d.get("SQ_INSTS_SALU", 0) / wv,
                  d.get("SQ_INSTS_VMEM_RD", 0) / wv, d.get("SQ_INSTS_VMEM_WR", 0) / wv,
                  d.get("SQ_BUSY_CYCLES", 0), w / wv,
                  d.get("SQ_WAIT_INST_LDS", 0) / w, d.get("SQ_WAIT_ANY", 0) / w, d.get("SQ_WAIT_INST_ANY", 0) / w,
                  d.get("SQ_ACTIVE_INST_VALU", 0) / w, d.get("SQ_ACTIVE_INST_LDS", 0) / w,
                  d.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, d.get("SQ_INSTS_LDS", 1))))
