#!/usr/bin/env python3
"""Does a second local sort fill the planning gaps of the first?  A proxy for
pipelining the multi-way passes of two halves on two streams: two processes
on one GPU each sort 2^logn u32 keys K times, started at the same wall-clock
instant, against one process alone.  If two concurrent sorts take less than
twice one sort's time, the GPU was idle (latency-bound planning launches)
during part of a sort.

    python3 tools/overlap_probe.py --logn 29 --k 20
prints one JSON line: alone ms per sort, concurrent ms per sort pair, the
fraction saved."""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(logn, k, start_at):
    sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))
    import torch
    import misort
    ctx = misort.Context(0)
    x = torch.empty(1 << logn, dtype=torch.int32, device="cuda")
    ctx.fill_splitmix(x, 0x5EED0003, 0)
    out = torch.empty_like(x)
    for _ in range(3):
        ctx.local_sort(x, out)
    torch.cuda.synchronize()
    while time.time() < start_at:
        time.sleep(0.001)
    t0 = time.time()
    for _ in range(k):
        ctx.local_sort(x, out)
    torch.cuda.synchronize()
    t1 = time.time()
    print(json.dumps({"t0": t0, "t1": t1}), flush=True)


def run(n_proc, logn, k):
    start_at = time.time() + 60.0
    ps = [subprocess.Popen([sys.executable, __file__, "--worker", str(logn), str(k), repr(start_at)],
                           stdout=subprocess.PIPE, text=True) for _ in range(n_proc)]
    outs = [json.loads(p.communicate(timeout=300)[0].strip().splitlines()[-1]) for p in ps]
    if any(p.returncode for p in ps):
        raise SystemExit("worker failed")
    return (max(o["t1"] for o in outs) - min(o["t0"] for o in outs)) * 1e3


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--worker":
        worker(int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]))
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--logn", type=int, default=29)
    ap.add_argument("--k", type=int, default=20)
    a = ap.parse_args()
    alone = run(1, a.logn, a.k) / a.k
    pair = run(2, a.logn, a.k) / a.k
    print(json.dumps({"logn": a.logn, "k": a.k, "alone_ms_per_sort": alone, "pair_ms_per_two_sorts": pair,
                      "saved_frac": 1.0 - pair / (2 * alone)}))


if __name__ == "__main__":
    main()
