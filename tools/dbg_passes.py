"""Debug helper: run each multi-way pass shape of a plan alone (pass probe) and report errors."""
import sys
import numpy as np
import torch
sys.path.insert(0, "parallel-computing-mpi_amd")
import misort

ctx = misort.Context(0)
for n in map(int, sys.argv[1:]):
    d = torch.randint(0, 2**31, (n,), dtype=torch.int32, device="cuda")
    o = torch.empty_like(d)
    for hi, lk in [(15, 4), (19, 4), (23, 3), (23, 4), (19, 3), (21, 3), (22, 3), (23, 2), (24, 2)]:
        try:
            ctx.pass_probe(d, o, "run_mergek", hi, lk, False, reps=1)
            r = "ok"
        except Exception as e:  # noqa: BLE001
            r = repr(e)
        print(n, hi, lk, r, flush=True)
ctx.close()
