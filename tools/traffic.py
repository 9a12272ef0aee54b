#!/usr/bin/env python3
"""Per-launch HBM bytes of the sort kernel families from rocprofv3 --pmc CSVs.

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reports half the
bytes of a 16-B-per-lane streaming read (MI355X_MICROARCH.md, HBM section);
other access widths are calibrated on known byte counts by tools/fetch_cal.hip
(profiles/fetch_cal.json), and each kernel's counter bytes are scaled by the
factor of its own access shape (KERNEL_SHAPE below):
  k_sort_u32 / k_sort_tile   16-B loads                  v16
  k_mergek<u32>              global_load_lds_dword       lds4
  k_mergek<u64>, u64 runs    8-B loads                   v8
  k_runs_merge<u32>          4-B loads                   v4
  fences (u64 / u128)        8-B / 16-B loads            v8 / v16
  k_bounds, fused descs      128-B line probes           line128
  k_runs_partition, gather   scattered 4-B probes        probe4
WRITE_SIZE is scaled by the 16-B streaming store's factor (st16) for every
kernel (the sort's outputs are 16-B non-temporal stores).  Without
profiles/fetch_cal.json (or with FETCH_CAL=none) every read is doubled, the
guide's 16-B rule, as before round 4.
The merge levels (runs.hip) are two launches per level: run_merge =
k_runs_merge + k_runs_partition per level.  The multi-way merge pass (runsk.hip)
is k_mergek plus its small planning kernels (k_fence_gather on the first
multi-way pass, k_fence_merge / k_fence_lds or the u64 fence merge levels or
the nested u64 multi-way pass over the fences, k_fence_counts, k_scan_totals,
k_bounds, k_chunk_desc); "run_mergek" sums them per launch of k_mergek.
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

root = sys.argv[1]
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAL_PATH = os.environ.get("FETCH_CAL") or os.path.join(HERE, "profiles", "fetch_cal.json")
CAL = json.load(open(CAL_PATH))["shapes"] if CAL_PATH != "none" and os.path.exists(CAL_PATH) else None


def kernel_shape(name):
    """The calibrated access shape of a kernel's reads (tools/fetch_cal.hip)."""
    wide = "__int128" in name
    u64 = "unsigned long" in name
    if "k_sort_u32" in name or "k_sort_tile" in name:
        return "v16"
    if "k_mergek" in name:
        return "v8" if u64 else "lds4"
    if "k_bounds" in name or "k_chunk_desc" in name or "k_split_desc" in name:
        return "line128"
    if "k_runs_partition" in name or "k_fence_gather" in name:
        return "probe4"
    if "k_scan" in name:
        return "v4"
    return "v16" if wide else "v8" if u64 else "v4"


def read_scale(name):
    if CAL is None:
        return 2.0
    return CAL[kernel_shape(name)]["read_scale"]


def write_scale(name):
    if CAL is None:
        return 1.0
    return CAL["st16"]["write_scale"]

# u32 sorts: k_runs_* on unsigned long are the multi-way passes' fence merges;
# u64 sorts: they are the sort's own 2-way merge levels, and k_runs_* on
# unsigned __int128 the fence merges
U32 = not (os.environ.get("WORKLOAD") or "").startswith("u64")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
raw = collections.defaultdict(lambda: collections.defaultdict(list))
seq = collections.defaultdict(list)  # counter -> [(dispatch id, family, value)]
for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if "k_sort_u32" in name or "k_sort_tile" in name:
            fam = "tile_sort"
        elif (U32 and re.search(r"k_runs_\w+<unsigned long", name)) or re.search(r"k_runs_\w+<unsigned __int128", name):
            fam = "runk_plan"  # the fence merges of a multi-way pass (u64 fences: u32 sorts; u128: u64 sorts)
        elif "k_runs_merge" in name:
            fam = "run_merge_kernel"
        elif "k_runs_partition" in name:
            fam = "run_partition"
        elif "k_mergek" in name:
            # u32 sorts: k_mergek on unsigned long is a pass's nested fence
            # merge (runsk.hip MISORT_FENCE_NEST), planning of that pass
            fam = "runk_plan" if U32 and "k_mergek<unsigned long" in name else "run_mergek_kernel"
        elif re.search(r"k_fence_gather|k_fence_lds|k_fence_merge|k_fence_counts|k_scan_totals|k_bounds|k_chunk_desc|k_split_desc",
                       name):
            fam = "runk_plan"
        else:
            continue
        cn = r["Counter_Name"]
        # bytes, corrected by the kernel's own access shape
        v = float(r["Counter_Value"]) * 1024 * (read_scale(name) if cn == "FETCH_SIZE" else write_scale(name))
        raw[fam][cn].append(float(r["Counter_Value"]) * 1024)
        acc[fam][cn].append(v)
        did = r.get("Dispatch_Id") or r.get("Dispatch-Id")
        if did is not None:
            seq[cn].append((int(did), fam, v))
out = {"source": os.path.basename(os.path.normpath(root)),
       "workload": os.environ.get("WORKLOAD"),
       "calibration": os.path.relpath(CAL_PATH, HERE) if CAL is not None else "none (FETCH_SIZE x 2)",
       "note": "bytes per launch = FETCH_SIZE*1024*read_scale(kernel) + WRITE_SIZE*1024*write_scale; "
               "read scales are calibrated per kernel access shape; the write scale is the 16-B "
               "streaming store's for every kernel (ASSUMED for the 8-B / 16-B fence, descriptor and "
               "bounds writers, whose store shapes are not calibrated)"}
for fam, cs in acc.items():
    f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) if cs.get("FETCH_SIZE") else None
    w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) if cs.get("WRITE_SIZE") else None
    fr = raw[fam].get("FETCH_SIZE")
    fraw = sum(fr) / len(fr) if fr else None
    out[fam] = {"launches": max(len(v) for v in cs.values()), "read_bytes_per_launch": f,
                "write_bytes_per_launch": w,
                "bytes_per_launch": (f + w) if f is not None and w is not None else None,
                "fetch_scale": f / fraw if f and fraw else None,
                "read_bytes_raw": fraw}
if "run_merge_kernel" in out and "run_partition" in out:
    a, b = out["run_merge_kernel"], out["run_partition"]
    out["run_merge"] = {k: a[k] + b[k] for k in ("read_bytes_per_launch", "write_bytes_per_launch",
                                                 "bytes_per_launch", "read_bytes_raw")}
    out["run_merge"].update(launches=a["launches"])
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
        b = fv + wv
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
