#!/usr/bin/env python3
"""Device compare-split (merge-split, psort.cc:116-164) throughput on one GPU.

    python tools/merge_probe.py > gpurun_out/merge_probe.jsonl

Two sorted runs of n keys each; keep-min and keep-max.  "GBs" counts
(n + n + n) * key bytes (both whole runs read, n written); the merge path only
reads the n keys it keeps, so the HBM traffic is 2/3 of that."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))


def main():
    import torch
    import misort
    ctx = misort.Context(0)
    st = torch.cuda.Stream()  # explicit stream: a null stream handle means "the context's own stream"
    for dt, kb in (("u32", 4), ("u64", 8)):
        tdt = torch.int32 if kb == 4 else torch.int64
        for lg in (22, 24, 26, 27, 28):
            n = 1 << lg
            a = torch.empty(2 * n, dtype=tdt, device="cuda")
            ctx.fill_splitmix(a, seed=0x5EED0003 + lg)
            sa = torch.empty_like(a)
            ctx.local_sort(a[:n], sa[:n])
            ctx.local_sort(a[n:], sa[n:])
            A, B = sa[:n], sa[n:]
            out = torch.empty_like(A)
            for keep in (0, 1):
                ctx.compare_split(A, B, keep, out=out)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 10
                e0.record(st)
                for _ in range(reps):
                    ctx.compare_split(A, B, keep, out=out, stream=st.cuda_stream)
                e1.record(st)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                print(json.dumps({"dtype": dt, "n": n, "keep_max": keep, "ms": ms,
                                  "GBs": 3 * n * kb / ms / 1e6}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
