#!/usr/bin/env python3
"""Time the SORT tile pass alone (misort_pass_probe, kind tile_sort) for u32/u64 at 2^logn
-- measurement only; with a MISORT_LIBRARY variant built with MISORT_SORT_TOP_U64 it
prices the tile's top levels.  python3 tools/sort_pass_probe.py --dtype u64 --logn 29"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))
import torch  # noqa: E402

import misort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", choices=["u32", "u64"], default="u64")
ap.add_argument("--logn", type=int, default=29)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--hi", type=int, default=0, help="13: the u32 2^14 merge-level tile (default: the largest tile)")
a = ap.parse_args()
n = 1 << a.logn
T = (torch.uint32 if hasattr(torch, "uint32") else torch.int32) if a.dtype == "u32" else \
    (torch.uint64 if hasattr(torch, "uint64") else torch.int64)
ctx = misort.Context(0)
d = torch.empty(n, dtype=T, device="cuda")
ctx.fill_splitmix(d, 0x5EED0003)
o = torch.empty_like(d)
ms = ctx.pass_probe(d, o, "tile_sort", a.hi, 0, False, reps=a.reps)
print(json.dumps({"dtype": a.dtype, "logn": a.logn, "hi": a.hi, "sort_pass_ms": ms,
                  "library": os.path.basename(misort.library_path())}))
ctx.close()
