#!/usr/bin/env python3
"""The device work ONE GPU does in a P-GPU bitonic sort (psort.cc:167-201),
measured in isolation on one GPU: the local sort of its block (psort.cc:175),
then per hypercube stage (psort.cc:184-196) the exchange bracket's samples and
count, the codec's encode (the partner's side) and decode (this side) of the k
keys that cross, and the merge-split of the block with them (the merge half of
compare_split_{min,max}, psort.cc:128-137,153-162).  The xGMI legs are not
here: they are the driver's 8-GPU measurement.

The stage inputs are real: the P blocks are first run through the whole
schedule on this GPU, one rank after another with whole-block compare-splits
(the reference's semantics), keeping each stage's rank-0 block, partner block
and the bracket k (misort.exchange_count on the two blocks' samples, the count
the runtime sends).  Then rank 0's work is timed op by op with HIP events on
one stream, after a marker kernel, so a rocprofv3 kernel trace of this script
can be cut at the marker (tools/rank_work_summary.py).

    python3 tools/rank_work_probe.py --logn 30 --p 8 --dtype u32      # config 4, P = 8
    python3 tools/rank_work_probe.py --n 536870909 --p 8 --dtype u64  # config 5, P = 8

u64 keys follow BASELINE config 5's mix (40 % from a 1024-value alphabet, 30 %
ODD_DIST double patterns, 20 % uniform < 2^63, 5 % zero, 5 % all-ones,
shuffled), drawn with torch's generator: the same distribution as the golden
fixtures' generator, not the same keys.  Prints one JSON line."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import misort  # noqa: E402


def u64_mix(n, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    kind = torch.rand(n, generator=g, device="cuda")
    def bits(m, hi_bits):  # m random int64 of hi_bits + 32 bits
        hi = torch.randint(0, 1 << hi_bits, (m,), generator=g, device="cuda", dtype=torch.int64)
        return (hi << 32) | torch.randint(0, 1 << 32, (m,), generator=g, device="cuda", dtype=torch.int64)
    alpha = bits(1024, 32)  # full 64-bit patterns (int64 wraps: u64 keys)
    x = alpha[torch.randint(0, 1024, (n,), generator=g, device="cuda")]
    u = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    odd = (u * u).view(torch.int64)
    uni = bits(n, 31)  # uniform < 2^63
    x = torch.where(kind >= 0.4, odd, x)
    x = torch.where(kind >= 0.7, uni, x)
    x = torch.where(kind >= 0.9, torch.zeros_like(x), x)
    x = torch.where(kind >= 0.95, torch.full_like(x, -1), x)
    return x  # int64 storage = u64 keys (misort compares unsigned)


def samples(block, npdt):
    idx = torch.from_numpy(misort.sample_indices(block.numel())).cuda()
    return block[idx].cpu().numpy().view(npdt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--logn", type=int, default=30)
    ap.add_argument("--n", type=int, default=0, help="total keys (overrides --logn)")
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--dtype", choices=["u32", "u64"], default="u32")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tail-div", type=int, default=8, help="the runtime rule: k * tail_div <= block -> in-place tail merge")
    a = ap.parse_args()
    n = a.n or (1 << a.logn)
    p = a.p
    sizes = misort.block_sizes(n, p)
    ctx = misort.Context(0)
    # one non-default stream for torch and misort alike: misort takes the
    # current torch stream (stream=None), but maps the null stream to its own
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    kb = 4 if a.dtype == "u32" else 8
    npdt = np.uint32 if kb == 4 else np.uint64
    blocks = []
    if kb == 4:
        for r in range(p):
            b = torch.empty(sizes[r], dtype=torch.int32, device="cuda")  # int32 storage = u32 keys
            ctx.fill_splitmix(b, 0x5EED0003, sum(sizes[:r]))
            blocks.append(b)
    else:
        allk = u64_mix(n, 0x5EED0005)
        blocks = [allk[sum(sizes[:r]):sum(sizes[:r + 1])].clone() for r in range(p)]
        del allk
    first = blocks[0].clone()
    # emulate the schedule, one rank after another (whole-block compare-splits)
    for r in range(p):
        out = torch.empty_like(blocks[r])
        ctx.local_sort(blocks[r], out)
        blocks[r] = out
    sched = [misort.schedule(p, r) for r in range(p)]
    stages = []
    for st in range(len(sched[0])):
        q, keep0 = sched[0][st]
        mine, theirs = blocks[0], blocks[q]
        # the bracket, from the min side's and the max side's samples
        lo, hi = (mine, theirs) if keep0 == 0 else (theirs, mine)
        k = misort.exchange_count(samples(lo, npdt), lo.numel(), samples(hi, npdt), hi.numel())
        k = theirs.numel() if k < 0 else k
        # what rank 0 receives: the partner's bottom k (rank 0 keeps the
        # minimum) or top k (keeps the maximum)
        recv = (theirs[:k] if keep0 == 0 else theirs[theirs.numel() - k:]).clone()
        stages.append({"stage": st, "partner": q, "keep_max": keep0, "n_me": mine.numel(),
                       "n_partner": theirs.numel(), "k": int(k), "mine": mine.clone(), "recv": recv})
        new = []
        for r in range(p):
            pr, kp = sched[r][st]
            new.append(ctx.compare_split(blocks[r], blocks[pr], kp))
        blocks = new
    torch.cuda.synchronize()
    errs = sum(ctx.check_sort(b) for b in blocks)
    del blocks
    torch.cuda.empty_cache()

    # marker: a rocprofv3 trace of this script is cut here
    torch.full((1,), 7, device="cuda").add_(1)
    torch.cuda.synchronize()

    def timed(fn, setup=None):
        if setup is None:
            # back to back between one pair of events: device time, not the
            # host's launch latency of one op (a sort is ~40 launches)
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                fn()
            e1.record(s)
            e1.synchronize()
            return e0.elapsed_time(e1) / a.reps
        ms = []
        for _ in range(a.reps + 1):
            if setup:
                setup()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn()
            e1.record(s)
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        return sum(ms[1:]) / a.reps  # the first is a warm-up

    w = kb
    res = {"n_total": n, "p": p, "dtype": a.dtype, "rank": 0, "n_rank": sizes[0], "reps": a.reps,
           "check_errors": int(errs)}
    out0 = torch.empty_like(first)
    t = timed(lambda: ctx.local_sort(first, out0))
    res["local_sort"] = {"ms": t, "keys": sizes[0], "passes": [x[0] for x in misort.plan(sizes[0], kb)]}
    rows = []
    for x in stages:
        k = x["k"]
        row = {key: x[key] for key in ("stage", "partner", "keep_max", "n_me", "n_partner", "k")}
        if k > 0:
            dec = torch.empty_like(x["recv"])
            enc_ms, dec_ms, nbytes = ctx.codec_probe(x["recv"], dec, reps=a.reps)
            row.update(encode_ms=enc_ms, decode_ms=dec_ms, coded_bytes=nbytes, raw_bytes=k * w,
                       codec_ok=bool(torch.equal(dec, x["recv"])))
            mo = torch.empty_like(x["mine"])
            # merge-split bytes: read n_me + k, write n_me
            mb = (2 * x["n_me"] + k) * w
            if k * a.tail_div <= x["n_me"]:
                # the runtime's small-bracket path: in place at the block's end
                # (misort_merge_split_tail); the block is restored before each rep
                t = timed(lambda: ctx.compare_split(mo, x["recv"], x["keep_max"], out=mo, in_place_tail=True),
                          setup=lambda: mo.copy_(x["mine"]))
                mine, rv = x["mine"], x["recv"]
                if x["keep_max"]:
                    win = int(torch.searchsorted(mine, rv[-1:], right=True).item())
                else:
                    win = x["n_me"] - int(torch.searchsorted(mine, rv[:1], right=True).item())
                tb = (3 * win + k) * w  # stage the window, read it and the k keys, write it back
                row.update(merge_split_path="tail (in place)", tail_window=win, merge_split_ms=t,
                           merge_split_window_bytes=tb, merge_split_bytes=mb)
            else:
                t = timed(lambda: ctx.compare_split(x["mine"], x["recv"], x["keep_max"], out=mo))
                row.update(merge_split_path="whole block", merge_split_ms=t, merge_split_bytes=mb,
                           merge_split_TBs=mb / (t * 1e-3) / 1e12, merge_split_frac=mb / (t * 1e-3) / 8e12)
        rows.append(row)
    res["stages"] = rows
    dev = res["local_sort"]["ms"] + sum(r.get("encode_ms", 0) + r.get("decode_ms", 0) + r.get("merge_split_ms", 0)
                                        for r in rows)
    res["device_ms_per_sort"] = dev
    res["note"] = ("rank 0's device work per P-GPU sort, isolated on one GPU (no xGMI): local sort + per stage "
                   "encode + decode + merge-split; samples/count kernels are in the rocprofv3 trace")
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
