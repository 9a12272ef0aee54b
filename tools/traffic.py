#!/usr/bin/env python3
"""Per-launch HBM bytes of the sort kernel families from rocprofv3 --pmc CSVs.

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes
of a 16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM section; confirmed
on this access shape by profiles/r01/pmc/calfetch_*), so it is doubled.
Families follow the k_stream TileMode template argument (0 SORT, 1 MERGE, 2 ROWS, 3 SPAN);
k_rows_wide (2^16-key register-tile ROWS) is its own family.  The merge levels
(runs.hip) are two launches per level: run_merge = k_runs_merge + k_runs_partition
per level.  Their loads are 4 B per lane, not 16 B; FETCH_SIZE still reports half the bytes
there (k_runs_merge reads every key exactly once: raw 2.197e9 vs 4.295e9 read
at 2^30, profiles/r01/pmc30_v11/), so the same doubling applies.  The raw value
is kept as "read_bytes_raw" and the factor as "fetch_scale".
The multi-way merge pass (runsk.hip) is k_mergek plus its small planning
kernels (k_fence_gather on the first multi-way pass, k_fence_merge / k_fence_lds
or the u64 fence merge levels, k_fence_counts, k_scan_totals, k_bounds,
k_chunk_desc); "run_mergek" sums them per launch
of k_mergek.  k_mergek's loads are 4 B per lane too, so the same doubling applies.
    WORKLOAD=u32_2e30_n1 tools/traffic.py gpurun_out/pmc30 > profiles/traffic.json
("workload" must match bench.py's f"{dtype}_2e{logn}_n{ranks}" for bench to use it).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

FAMILY = {"0": "tile_sort", "1": "tile_merge", "2": "global_pass", "3": "span_pass"}
root = sys.argv[1]
# u32 sorts: k_runs_* on unsigned long are the multi-way passes' fence merges;
# u64 sorts: they are the sort's own 2-way merge levels, and k_runs_* on
# unsigned __int128 the fence merges
U32 = not (os.environ.get("WORKLOAD") or "").startswith("u64")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
seq = collections.defaultdict(list)  # counter -> [(dispatch id, family, value)]
for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        m = re.search(r"k_stream<unsigned (?:int|long), (\d+), (\d)", name)
        if m:
            fam = FAMILY[m.group(2)]
        elif "k_sort_u32" in name or "k_sort_tile" in name:
            fam = "tile_sort"
        elif "k_rows_wide" in name:
            fam = "wide_pass"
        elif (U32 and re.search(r"k_runs_\w+<unsigned long", name)) or re.search(r"k_runs_\w+<unsigned __int128", name):
            fam = "runk_plan"  # the fence merges of a multi-way pass (u64 fences: u32 sorts; u128: u64 sorts)
        elif "k_runs_merge" in name:
            fam = "run_merge_kernel"
        elif "k_runs_partition" in name:
            fam = "run_partition"
        elif "k_mergek" in name:
            fam = "run_mergek_kernel"
        elif re.search(r"k_fence_gather|k_fence_lds|k_fence_merge|k_fence_counts|k_scan_totals|k_bounds|k_chunk_desc",
                       name):
            fam = "runk_plan"
        else:
            continue
        acc[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
        did = r.get("Dispatch_Id") or r.get("Dispatch-Id")
        if did is not None:
            seq[r["Counter_Name"]].append((int(did), fam, float(r["Counter_Value"])))
out = {"source": os.path.basename(os.path.normpath(root)),
       "workload": os.environ.get("WORKLOAD"),
       "note": "bytes per launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE correction)"}
SCALE = float(os.environ.get("RUN_FETCH_SCALE", "2"))  # 4-B-per-lane loads: see the docstring
for fam, cs in acc.items():
    scale = SCALE if fam.startswith("run_") else 2.0
    f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * scale if cs.get("FETCH_SIZE") else None
    w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024 if cs.get("WRITE_SIZE") else None
    out[fam] = {"launches": max(len(v) for v in cs.values()), "read_bytes_per_launch": f,
                "write_bytes_per_launch": w,
                "bytes_per_launch": (f + w) if f is not None and w is not None else None,
                "fetch_scale": scale,
                "read_bytes_raw": f / scale if f is not None else None}
if "run_merge_kernel" in out and "run_partition" in out:
    a, b = out["run_merge_kernel"], out["run_partition"]
    out["run_merge"] = {k: a[k] + b[k] for k in ("read_bytes_per_launch", "write_bytes_per_launch",
                                                 "bytes_per_launch", "read_bytes_raw")}
    out["run_merge"].update(launches=a["launches"], fetch_scale=SCALE)
    out["run_merge"]["note"] = "per level: k_runs_merge + k_runs_partition"
if "run_mergek_kernel" in out:
    a = out["run_mergek_kernel"]
    b = out.get("runk_plan")
    m = dict(a)
    if b:  # the planning kernels' bytes, spread over the k_mergek launches
        for k in ("read_bytes_per_launch", "write_bytes_per_launch", "bytes_per_launch", "read_bytes_raw"):
            if a.get(k) is not None and b.get(k) is not None:
                m[k] = a[k] + b[k] * b["launches"] / a["launches"]
    m["note"] = "per multi-way pass: k_mergek + its planning kernels (fences, bounds, descriptors)"
    out["run_mergek"] = m

# Per pass, in dispatch order (one profiled step): FETCH_SIZE and WRITE_SIZE
# come from separate runs of the same program, matched by position.  A
# multi-way pass is its planning kernels + k_mergek (kernel_bytes: k_mergek
# alone); a 2-way merge level is k_runs_partition + k_runs_merge.
def pass_list():
    f = sorted(seq.get("FETCH_SIZE", []))
    w = sorted(seq.get("WRITE_SIZE", []))
    if not f or len(f) != len(w) or any(a[1] != b[1] for a, b in zip(f, w)):
        return None
    passes, plan, part = [], 0.0, 0.0
    for (_, fam, fv), (_, _, wv) in zip(f, w):
        b = fv * 1024 * (SCALE if fam.startswith("run_") else 2.0) + wv * 1024
        if fam == "runk_plan":
            plan += b
        elif fam == "run_partition":
            part += b
        elif fam == "run_mergek_kernel":
            passes.append({"kind": "run_mergek", "bytes": plan + b, "kernel_bytes": b})
            plan = 0.0
        elif fam == "run_merge_kernel":
            passes.append({"kind": "run_merge", "bytes": part + b, "kernel_bytes": b})
            part = 0.0
        else:
            passes.append({"kind": fam, "bytes": b})
    return passes


pl = pass_list()
if pl:
    out["passes"] = pl
json.dump(out, sys.stdout, indent=1)
print()
