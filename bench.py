#!/usr/bin/env python3
"""Headline benchmark: bitonic sort of 2^30 uint32 keys (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N ... bench.py --gpus N   (one process per GPU)

A step = one full parallel_bitonic_sort (psort.cc:167) of the 2^30 keys that
are already resident in HBM: local sort of each rank's block (hand-written
gfx950 kernels) plus, for N > 1, the d(d+1)/2 RCCL compare-split rounds.
Total keys are fixed (strong scaling).  Keys: counter-based SplitMix64
(seed 0x5EED0003), top 32 bits, generated on the GPU outside the timed region;
the sort is out of place so every step sorts the same unsorted input.

Rank 0 prints ONE JSON line with the metric, the per-kernel roofline of the
dominant kernel (HIP events on the sort stream inside the timed region;
algorithmic bytes = 2 * keys * 4 B per pass) and the CPU baseline: the
reference's own parallel_bitonic_sort (oracle/_ref, compiled from the
unmodified psort.cc) under mpirun on this host's cores, on a bounded sample.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))

METRIC = "Gkeys/s + % HBM roofline, bitonic sort 2^30 uint32 keys at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED = 0x5EED0003
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "psort_ref")
MPIRUN = "/opt/conda/bin/mpirun"


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sample_logn, cores):
    """The reference sorter's parallel_bitonic_sort on host cores (mpirun)."""
    n = 1 << sample_logn
    sample = (f"2^{sample_logn} u32 keys (SplitMix64 seed {SEED:#x}, the bench workload's "
              f"generator), reference psort.cc parallel_bitonic_sort on doubles via "
              f"oracle/_ref harness, mpirun -np {cores}, CPU: {cpu_model()}")
    if os.path.exists(REF_BIN) and os.path.exists(MPIRUN):
        cmd = [MPIRUN, "-np", str(cores), REF_BIN, "--dtype", "u32", "--gen-splitmix", hex(SEED),
               "--n", str(n)]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
            m = re.search(r'"sort_s": ([0-9.eE+-]+)', r.stdout)
            errs = re.search(r"(\d+) errors in sorting", r.stdout)
            if r.returncode == 0 and m:
                t = float(m.group(1))
                return {"value": n / t / 1e9, "unit": "Gkeys/s", "cores": cores,
                        "kind": "reference", "sample": sample, "sort_s": t,
                        "errors": int(errs.group(1)) if errs else None}
            sys.stderr.write(f"cpu baseline failed ({r.returncode}): {r.stderr[-400:]}\n")
        except (subprocess.TimeoutExpired, OSError) as e:
            sys.stderr.write(f"cpu baseline failed: {e}\n")
    # Fallback: the C restatement (single thread) on a smaller sample.
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O
    n = 1 << min(sample_logn, 24)
    x = O.splitmix(SEED, n, np.uint32)
    t0 = time.perf_counter()
    O.parallel_bitonic_sort(x, 1)
    t = time.perf_counter() - t0
    return {"value": n / t / 1e9, "unit": "Gkeys/s", "cores": 1, "kind": "port",
            "sample": f"2^{min(sample_logn, 24)} u32 keys, oracle/oracle.c restatement, 1 thread",
            "sort_s": t}


def load_traffic():
    """Per-launch HBM bytes from committed rocprofv3 --pmc summaries (or None)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--logn", type=int, default=30, help="log2 of the total key count")
    ap.add_argument("--dtype", choices=["u32", "u64"], default="u32")
    ap.add_argument("--algo", choices=["bitonic", "sample"], default="bitonic",
                    help="bitonic = psort.cc:167 (the metric); sample = psort.cc:203-375 redesigned")
    ap.add_argument("--no-alt", action="store_true",
                    help="N>1: skip the extra sample-sort timing reported under 'alt'")
    ap.add_argument("--cpu-sample-logn", type=int, default=27)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time without per-launch HIP events (roofline omitted)")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the PCIe-inclusive path (host keys -> misort_sort_host -> host "
                         "keys), staged and overlapped vs one chunk; reported under 'host_io', "
                         "never as value")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    # The CPU baseline runs first, before this process touches the GPU.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cores = 1
        while cores * 2 <= min(os.cpu_count() or 1, 16):
            cores *= 2
        cpu = cpu_baseline(args.cpu_sample_logn, cores)

    import torch
    import torch.distributed as dist
    import misort

    if world > 1:
        dist.init_process_group("gloo")  # host plumbing only: ids, barriers, max
    torch.cuda.set_device(local_rank)
    ctx = misort.Context(local_rank)
    if world > 1:
        ctx.comm_init_torch()

    n_total = 1 << args.logn
    sizes = misort.block_sizes(n_total, world)
    loc, max_size = sizes[rank], n_total // world + 1
    g0 = sum(sizes[:rank])
    kdt = (torch.uint32 if hasattr(torch, "uint32") else torch.int32) if args.dtype == "u32" else \
          (torch.uint64 if hasattr(torch, "uint64") else torch.int64)
    key_bytes = 4 if args.dtype == "u32" else 8
    d_in = torch.empty(max(loc, 1), dtype=kdt, device="cuda")
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream()
    ctx.fill_splitmix(d_in[:loc], SEED, g0)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def run(algo):
        if algo == "sample":
            ctx.parallel_sample_sort(d_in, loc, max_size, out=d_out, stream=stream.cuda_stream)
        else:
            ctx.parallel_bitonic_sort(d_in, loc, max_size, out=d_out, stream=stream.cuda_stream)

    def step():
        run(args.algo)

    def timed(algo, steps):
        """warm, then barrier + sync around `steps` sorts; max over ranks (s)."""
        run(algo)
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            run(algo)
        torch.cuda.synchronize()
        barrier()
        tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.exchange_stats()  # reset
    events = not args.no_kernel_events
    if events:
        ctx.profile(True)
        ctx.profile_reset()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kern = ctx.profile_read() if events else {}
    ctx.profile(False)
    xst = ctx.exchange_stats()

    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    errors = ctx.check_sort(d_out, loc)  # psort.cc:497-520 over all ranks
    alt = None
    if world > 1 and args.algo == "bitonic" and not args.no_alt:
        # the redesigned sample sort (one RCCL all-to-all) on the same input, same contract
        ts = timed("sample", args.steps)
        alt = {"sample_sort": {"value": n_total * args.steps / ts / 1e9, "unit": "Gkeys/s",
                               "ms_per_step": ts / args.steps * 1e3,
                               "check_errors": ctx.check_sort(d_out, loc),
                               "note": "psort.cc:203-375 redesigned: samples, one all-to-all-v, "
                                       "merge tree, rebalance to the reference layout"}}

    host_io = None
    if args.host_io:
        # host keys of the same workload; sorted through the pinned staging pipeline
        h_in = d_in[:loc].cpu().numpy().view(np.uint32 if key_bytes == 4 else np.uint64)
        h_buf = np.zeros_like(h_in)  # the caller's output block, already paged in
        res = {}
        for name, chunk in (("staged_overlapped", 1 << 24), ("one_chunk", loc)):
            os.environ["MISORT_STAGE_CHUNK"] = str(chunk)
            h_out = ctx.sort_host(h_in, max_size, out=h_buf)  # warm (pins the ring)
            best = None
            for _ in range(2):
                barrier()
                t0 = time.perf_counter()
                h_out = ctx.sort_host(h_in, max_size, out=h_buf)
                barrier()
                tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
                if world > 1:
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                best = float(tt.item()) if best is None else min(best, float(tt.item()))
            res[name] = {"value": n_total / best / 1e9, "unit": "Gkeys/s", "ms": best * 1e3,
                         "chunk_keys": chunk}
            assert bool(np.all(h_out[1:] >= h_out[:-1])) if loc > 1 else True
        os.environ.pop("MISORT_STAGE_CHUNK", None)
        res["note"] = ("PCIe-inclusive: host numpy keys in, host keys out (pinned ring, H2D/D2H, "
                       "host copies); not the metric value")
        host_io = res

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        out = {
            "metric": METRIC,
            "value": n_total * args.steps / elapsed / 1e9,
            "unit": "Gkeys/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (SplitMix64 keys generated in HBM, seed 0x5EED0003)",
            "config": {"workload": f"bitonic sort 2^{args.logn} {args.dtype} keys "
                                   f"(BASELINE config {'3/4' if args.logn == 30 else 'custom'})",
                       "keys": n_total, "keys_per_gpu": loc,
                       "algo": args.algo,
                       "parallelism": (f"hypercube bitonic, {world} GPU(s), RCCL compare-split"
                                       if args.algo == "bitonic" else
                                       f"sample sort, {world} GPU(s), RCCL all-to-all")},
            "check_errors": errors,
        }
        if world > 1:
            out["exchange"] = {"stages_per_step": xst[0] / args.steps,
                               "rank0_bytes_per_step": xst[1] / args.steps,
                               "rank0_whole_block_bytes_per_step": xst[2] / args.steps}
        if kern:
            per = {}
            for name, (nl, tms, byt) in kern.items():
                if nl:
                    per[name] = {"launches_per_step": nl / args.steps, "ms_per_step": tms / args.steps,
                                 "avg_launch_us": tms / nl * 1e3,
                                 "achieved_GBs": byt / (tms * 1e-3) / 1e9 if tms > 0 else None}
            out["kernels"] = per
            dom = max(kern.items(), key=lambda kv: kv[1][1])
            name, (nl, tms, byt) = dom
            traffic = load_traffic()
            tr = None
            if traffic and name in traffic and traffic[name].get("bytes_per_launch"):
                tr = traffic[name]["bytes_per_launch"]
            achieved = byt / (tms * 1e-3) / 1e9
            out["roofline"] = {"kernel": name, "bound": "hbm", "achieved": achieved,
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                               "traffic": tr, "algorithmic_bytes_per_launch": byt / nl,
                               "avg_launch_us": tms / nl * 1e3}
            kt = sum(v[1] for v in kern.values()) / args.steps
            out["kernel_ms_per_step"] = kt
        if alt:
            out["alt"] = alt
        if host_io:
            out["host_io"] = host_io
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
