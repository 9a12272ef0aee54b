#!/usr/bin/env python3
"""Time of the u32 SORT pass (misort_pass_probe, 2^30 keys) for the library in
MISORT_LIBRARY: with variants built by tools/build_variant.sh NAME
"-DMISORT_SORT_TOP=L" the LDS phases stop after level L (2^15 tile), or
"-DMISORT_SORT_STOP=P" the 2^14 merge-level tile stops after phase P, so the
difference between variants prices the tile's top levels / phases.  TILE=14 or
15 picks the tile (default 14)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))


def main():
    import torch
    import misort
    ctx = misort.Context(0)
    n = 1 << int(os.environ.get("LOGN", "30"))
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    ctx.fill_splitmix(a, seed=0x5EED0003)
    b = torch.empty_like(a)
    lt = int(os.environ.get("TILE", "14"))
    ms = ctx.pass_probe(a, b, "tile_sort", lt - 1, 0, False, reps=10)
    print(json.dumps({"library": os.path.basename(misort.library_path()), "n": n, "tile": lt, "sort_ms": ms}))


if __name__ == "__main__":
    main()
