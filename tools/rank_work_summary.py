#!/usr/bin/env python3
"""Per-kernel stats of the measured part of a rocprofv3 --kernel-trace run of
tools/rank_work_probe.py: the dispatches after the probe's marker kernel (the
last torch fill before the timed ops), misort kernels only.

    tools/rank_work_summary.py TRACE_DIR [probe.json] > summary.txt

With the probe's JSON line (its stdout) it adds the algorithmic bytes and the
roofline fraction of the merge-split and of the local sort per launch."""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1]
rows = []
for path in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
cut = max((i for i, x in enumerate(rows) if "FillFunctor" in x[2]), default=-1)
acc = collections.defaultdict(list)
for s, e, name in rows[cut + 1:]:
    if "misort" not in name:
        continue
    key = name.replace("misort::(anonymous namespace)::", "").replace("misort::", "").replace("void ", "")
    key = re.sub(r"\(.*", "", key)
    acc[key].append((e - s) / 1e3)
print(f"# {os.path.basename(os.path.normpath(root))}: {sum(len(v) for v in acc.values())} misort dispatches "
      f"after the marker (dispatch {cut})")
print(f"{'kernel':<90} {'calls':>6} {'total_us':>10} {'avg_us':>9}")
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[:90]:<90} {len(v):>6} {sum(v):>10.1f} {sum(v) / len(v):>9.1f}")
if len(sys.argv) > 2:
    pr = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
    print()
    print(f"# probe: {pr['dtype']} N = {pr['n_total']} over P = {pr['p']}, rank 0 holds {pr['n_rank']} keys")
    w = 4 if pr["dtype"] == "u32" else 8
    ls = pr["local_sort"]
    print(f"local sort: {ls['ms']:.3f} ms (HIP events), passes {ls['passes']}")
    for r in pr["stages"]:
        if r["k"] == 0:
            print(f"stage {r['stage']}: partner {r['partner']}, k = 0 (skipped)")
            continue
        if r.get("merge_split_path", "whole block") == "whole block":
            ms = (f"merge-split {r['merge_split_ms']:.3f} ms = {r['merge_split_TBs']:.2f} TB/s "
                  f"(frac {r['merge_split_frac']:.3f} of 8 TB/s)")
        else:
            ms = (f"merge-split in place at the block's end {r['merge_split_ms']:.3f} ms (window "
                  f"{r['tail_window']} keys, {r['merge_split_window_bytes'] / 1e6:.2f} MB moved)")
        print(f"stage {r['stage']}: partner {r['partner']} keep_max {r['keep_max']} k = {r['k']} "
              f"({r['k'] / r['n_partner']:.3f} of the block): encode {r['encode_ms']:.3f} + decode "
              f"{r['decode_ms']:.3f} ms (coded {r['coded_bytes'] / max(1, r['raw_bytes']):.3f} of raw), " + ms)
    print(f"device work per sort (rank 0): {pr['device_ms_per_sort']:.3f} ms")
