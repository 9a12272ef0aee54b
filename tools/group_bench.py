#!/usr/bin/env python3
"""P-rank bitonic sort on ONE GPU through the in-process rank group (measurement
only): P threads, one misort context each, exchange = device-to-device copies
instead of RCCL over xGMI.  All ranks share the GPU, so the times are NOT
multi-GPU numbers; they show the per-stage structure (exchange leg: samples,
device count, codec, copies; merge-split) and the host waits between them.

    python3 tools/group_bench.py --p 8 --logn 30 --steps 3
prints one JSON line: wall ms per sort (max over ranks) and per-stage
exchange / merge ms of rank 0 (HIP events)."""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))
import torch  # noqa: E402

import misort  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--logn", type=int, default=30)
    ap.add_argument("--dtype", choices=["u32", "u64"], default="u32")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    n, p = 1 << a.logn, a.p
    sizes = misort.block_sizes(n, p)
    tdt = (torch.uint32 if hasattr(torch, "uint32") else torch.int32) if a.dtype == "u32" else \
        (torch.uint64 if hasattr(torch, "uint64") else torch.int64)
    nst = len(misort.schedule(p, 0))
    bar = threading.Barrier(p)
    walls = [[] for _ in range(p)]

    def rank_fn(r, ctx):
        off = sum(sizes[:r])
        buf = torch.empty(sizes[r], dtype=tdt, device="cuda")
        out = torch.empty_like(buf)
        ctx.fill_splitmix(buf, 0x5EED0003, off, stream=ctx.native_stream)
        ctx.synchronize()
        for i in range(a.warmup + a.steps):
            if i == a.warmup:
                ctx.profile(True)
                ctx.profile_reset()
            bar.wait()
            t0 = time.perf_counter()
            ctx.parallel_bitonic_sort(buf, sizes[r], sizes[r], out=out, stream=ctx.native_stream)
            ctx.synchronize()
            t1 = time.perf_counter()
            bar.wait()
            if i >= a.warmup:
                walls[r].append((t1 - t0) * 1e3)
        errs = ctx.check_sort(out, sizes[r], stream=ctx.native_stream)
        stages = ctx.profile_stages(nst)
        kern = ctx.profile_read()
        return errs, stages, kern

    g = misort.Group(p)
    try:
        res = g.run(rank_fn)
    finally:
        g.close()
    ms = [max(walls[r][i] for r in range(p)) for i in range(a.steps)]
    st0 = res[0][1]
    print(json.dumps({
        "what": f"{p}-rank group on one GPU (device-to-device exchange, ranks share the GPU)",
        "keys": n, "dtype": a.dtype, "p": p, "errors": int(res[0][0]),
        "ms_per_sort": sum(ms) / len(ms), "ms_min": min(ms),
        "stages_rank0": [{"stage": i, "exchange_ms": round(x / max(c, 1), 4), "merge_ms": round(m / max(c, 1), 4),
                          "exchange_MB": round(b / max(c, 1) / 1e6, 2)} for i, (c, x, m, b) in enumerate(st0)],
        "kernels_rank0_ms": {k: round(v[1] / a.steps, 4) for k, v in res[0][2].items() if v[0]},
    }))


if __name__ == "__main__":
    main()
