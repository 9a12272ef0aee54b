#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration factors from a tools/bin/fetch_cal run.

    tools/fetch_cal.py DIR  > profiles/fetch_cal.json

DIR holds the two rocprofv3 --pmc passes (subdirectories with
*counter_collection.csv: one with FETCH_SIZE, one with WRITE_SIZE) and
fetch_cal.log, the program's stdout (one JSON line per shape, in launch order,
with the bytes it reads and writes).  For each shape: the counter's bytes
(KiB x 1024) and the factor that turns them into the known byte count
(read_scale = read_bytes / FETCH bytes).  tools/traffic.py applies these
factors per kernel."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]
shapes = [json.loads(x) for x in open(os.path.join(root, "fetch_cal.log")) if x.startswith("{")]
vals = {}
for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if "cal_" not in name:
            continue
        did = int(r.get("Dispatch_Id") or r.get("Dispatch-Id"))
        vals.setdefault(r["Counter_Name"], {}).setdefault(did, 0.0)
        vals[r["Counter_Name"]][did] += float(r["Counter_Value"])
out = {"note": "per access shape: counter bytes (KiB x 1024) vs the known bytes; "
               "read_scale / write_scale turn counter bytes into true bytes",
       "shapes": {}}
for cn, key in (("FETCH_SIZE", "read"), ("WRITE_SIZE", "write")):
    seq = [v for _, v in sorted(vals.get(cn, {}).items())]
    if len(seq) != len(shapes):
        sys.exit(f"{cn}: {len(seq)} dispatches for {len(shapes)} shapes")
    for sh, v in zip(shapes, seq):
        e = out["shapes"].setdefault(sh["shape"], {"read_bytes": sh["read_bytes"], "write_bytes": sh["write_bytes"]})
        e[f"{cn.lower()}_bytes"] = v * 1024
        known = sh[f"{key}_bytes"]
        e[f"{key}_scale"] = known / (v * 1024) if known > 0 and v > 0 else None
# probe4 reads 4 B per distinct 128-B line: its counter bytes per probe show
# the granule one scattered dword costs (not a counter error); for traffic a
# probe's counter bytes are scaled like the line reads'
pr = out["shapes"].get("probe4")
if pr and pr.get("fetch_size_bytes"):
    nprobe = pr["read_bytes"] / 4
    pr["counter_bytes_per_probe"] = pr["fetch_size_bytes"] / nprobe
    pr["read_scale_algorithmic"] = pr["read_scale"]
    pr["read_scale"] = out["shapes"]["line128"]["read_scale"]
    pr["note"] = ("a scattered 4-B read is counted as one 64-B request (counter bytes per probe), a 128-B "
                  "line by the x2 rule of the streaming shapes; "
                  "read_scale = line128's, read_scale_algorithmic = 4 B / counter bytes")
json.dump(out, sys.stdout, indent=1)
print()
