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

`--gpus N` without a torchrun environment (no WORLD_SIZE) relaunches this file
under `python -m torch.distributed.run --nproc-per-node N` as a child process
BEFORE anything touches the GPU, and exits with the child's status.

Rank 0 prints ONE JSON line with the metric, the per-kernel roofline of the
dominant kernel (HIP events on the sort stream inside the timed region;
algorithmic bytes = 2 * keys * 4 B per pass) and the CPU baseline: the
reference's own parallel_bitonic_sort (oracle/_ref, compiled from the
unmodified psort.cc) under mpirun on this host's cores, on the same workload.
At N > 1 it adds per-stage exchange / merge-split times, the xGMI bytes and
rate of every hypercube stage, and t1 / (P * tP) against a 1-GPU leg of the
same keys run in the same job.
"""
import argparse
import faulthandler
import json
import os
import re
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))

METRIC = "Gkeys/s + % HBM roofline, bitonic sort 2^30 uint32 keys at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED = 0x5EED0003
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "psort_ref")
MPIRUN = "/opt/conda/bin/mpirun"


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--logn", type=int, default=30, help="log2 of the total key count")
    ap.add_argument("--dtype", choices=["u32", "u64", "f64"], default="u32",
                    help="f64: the reference's own key type (psort.cc:565), SplitMix64 top 53 bits as "
                         "uniform doubles in [0, 1)")
    ap.add_argument("--algo", choices=["bitonic", "sample"], default="bitonic",
                    help="bitonic = psort.cc:167 (the metric); sample = psort.cc:203-375 redesigned")
    ap.add_argument("--no-alt", action="store_true",
                    help="N>1: skip the extra sample-sort timing reported under 'alt'")
    ap.add_argument("--no-t1", action="store_true",
                    help="N>1: skip the 1-GPU leg that scaling_eff is computed against")
    ap.add_argument("--cpu-sample-logn", type=int, default=None,
                    help="log2 keys of the CPU baseline sample (default: the workload, --logn)")
    ap.add_argument("--cpu-sweep", action="store_true",
                    help="also time the reference at P = 1, 2, 4, ... cores on u32 and on its own f64 "
                         "workload (BASELINE.md section 3), reported under cpu_sweep")
    ap.add_argument("--cpu-sweep-logn", type=int, default=27)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--watchdog-s", type=float, default=1200.0,
                    help="a rank still running after this many seconds prints every thread's stack and "
                         "exits (1): a hang ends as an error, as the reference's alarm(540) does "
                         "(psort.cc:17,56-65); each wait on a peer is bounded by MISORT_TIMEOUT_S too")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time without per-launch HIP events (roofline omitted)")
    ap.add_argument("--host-io", action="store_true",
                    help="also time the PCIe-inclusive path (host keys -> misort_sort_host -> host "
                         "keys), staged and overlapped vs one chunk; reported under 'host_io', "
                         "never as value")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher
def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, gpus, port):
    """The torchrun command that runs this file as `gpus` ranks (one per GPU)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            os.path.abspath(__file__), *argv]


def needs_launch(args, env=None):
    env = os.environ if env is None else env
    return args.gpus > 1 and "WORLD_SIZE" not in env


# ------------------------------------------------------------- CPU baseline
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """CPUs this process may use: affinity mask, cgroup quota, MISORT_CPU_CORES."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    why = f"sched_getaffinity={n}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                cg = max(1, int(int(q) / int(per)))
                why += f", cgroup cpu.max={cg}"
                n = min(n, cg)
    except (OSError, ValueError):
        pass
    if os.environ.get("MISORT_CPU_CORES"):
        n = int(os.environ["MISORT_CPU_CORES"])
        why += f", MISORT_CPU_CORES={n}"
    return max(1, n), why


def pow2_floor(n):
    p = 1
    while p * 2 <= n:
        p *= 2
    return p


def run_reference(cmd, timeout):
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd[:4])}...: rc {r.returncode}: {r.stderr[-400:]}")
    return r.stdout


def ref_keys_time(logn, cores, dtype="u32"):
    """Reference parallel_bitonic_sort on SplitMix keys (our harness around the
    unmodified psort.cc); returns (sort seconds, errors)."""
    out = run_reference([MPIRUN, "-np", str(cores), REF_BIN, "--dtype", dtype, "--gen-splitmix",
                         hex(SEED), "--n", str(1 << logn)], timeout=900)
    m = re.search(r'"sort_s": ([0-9.eE+-]+)', out)
    errs = re.search(r"(\d+) errors in sorting", out)
    return float(m.group(1)), int(errs.group(1)) if errs else None


def ref_psort_time(logn, cores):
    """The reference binary's own run (`mpirun -np P psort N`, its generator,
    its doubles, its printed max-over-ranks parallel sort time)."""
    out = run_reference([MPIRUN, "-np", str(cores), REF_BIN, str(1 << logn)], timeout=900)
    m = re.search(r"parallel sort time = ([0-9.eE+-]+)", out)
    errs = re.search(r"(\d+) errors in sorting", out)
    return float(m.group(1)), int(errs.group(1)) if errs else None


def cpu_baseline(sample_logn, sweep, sweep_logn, dtype="u32"):
    """The reference sorter's parallel_bitonic_sort on this host's cores (u32
    keys carried as doubles, or f64 keys for an f64 workload)."""
    share, why = cpu_share()
    cores = pow2_floor(share)
    model = cpu_model()
    if not (os.path.exists(REF_BIN) and os.path.exists(MPIRUN)):
        # Loud: the reference harness is built in the build container
        # (__graft_entry__.build(), oracle/Makefile) and travels in-tree.
        msg = (f"cpu baseline: {REF_BIN} or {MPIRUN} missing -- falling back to the C restatement "
               f"(kind 'port', 1 thread); rebuild with __graft_entry__.build() where /root/reference exists")
        sys.stderr.write("WARNING " + msg + "\n")
        return port_baseline(min(sample_logn, 24), msg)
    res = {"unit": "Gkeys/s", "cores": cores, "kind": "reference",
           "cores_why": f"largest power of two <= CPUs available ({why}); psort.cc needs 2^d ranks",
           "cpu": model}
    try:
        kd = "f64" if dtype == "f64" else "u32"
        t, errs = ref_keys_time(sample_logn, cores, kd)
        what = ("f64 keys (SplitMix64 seed {:#x} top 53 bits as doubles in [0, 1), the bench workload)"
                if kd == "f64" else "u32 keys (SplitMix64 seed {:#x}, the bench workload) carried as doubles")
        res.update(value=(1 << sample_logn) / t / 1e9, sort_s=t, errors=errs,
                   sample=(f"2^{sample_logn} {what.format(SEED)} through the reference psort.cc "
                           f"parallel_bitonic_sort (oracle/_ref harness), mpirun -np {cores}; timed region "
                           f"psort.cc:633-653, max over ranks"))
    except (RuntimeError, subprocess.TimeoutExpired, OSError, AttributeError) as e:
        sys.stderr.write(f"WARNING cpu baseline failed: {e}\n")
        return port_baseline(min(sample_logn, 24), f"reference run failed: {e}")
    if sweep:
        rows = []
        p = 1
        while p <= cores:
            row = {"p": p}
            try:
                tu, eu = ref_keys_time(sweep_logn, p)
                tf, ef = ref_psort_time(sweep_logn, p)
                row.update(u32_s=tu, u32_gkeys=(1 << sweep_logn) / tu / 1e9, u32_errors=eu,
                           f64_s=tf, f64_gkeys=(1 << sweep_logn) / tf / 1e9, f64_errors=ef)
            except (RuntimeError, subprocess.TimeoutExpired, OSError, AttributeError) as e:
                row["error"] = str(e)[-200:]
            rows.append(row)
            p *= 2
        res["sweep"] = {"n": 1 << sweep_logn, "rows": rows,
                        "note": "u32: SplitMix keys as doubles through parallel_bitonic_sort; f64: the "
                                "reference binary's own generator and stdout time (bitonic swapped in)"}
    return res


def port_baseline(logn, why):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O
    n = 1 << logn
    x = O.splitmix(SEED, n, np.uint32)
    t0 = time.perf_counter()
    O.parallel_bitonic_sort(x, 1)
    t = time.perf_counter() - t0
    return {"value": n / t / 1e9, "unit": "Gkeys/s", "cores": 1, "kind": "port",
            "sample": f"2^{logn} u32 keys, oracle/oracle.c restatement, 1 thread", "sort_s": t,
            "fallback_reason": why}


CPU_JSON_ENV = "MISORT_BENCH_CPU_JSON"


def load_cpu_json(path):
    """The host-core baseline the launcher parent measured (or None)."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        cpu = json.load(f)
    if isinstance(cpu, dict):
        cpu["measured_by"] = "bench.py launcher parent, before the GPU ranks started"
    return cpu


def baseline_config(logn, dtype):
    """The BASELINE.json config a bench workload is (configs[1..4]; config 5 is
    u64 N = 2^29 - 3 / - 7 over 8 GPUs, so a 2^29 u64 line is its size only)."""
    if dtype == "u32" and logn in (24, 28, 30):
        return f"BASELINE config {({24: 2, 28: 3, 30: 4})[logn]}"
    if dtype == "u64" and logn == 29:
        return "BASELINE config 5's key type and size (N = 2^29, not 2^29 - 3 / - 7)"
    if dtype == "f64":
        return "the reference's own key type, psort.cc:565; not a BASELINE config"
    return "not a BASELINE config"


def load_traffic(workload):
    """Per-launch HBM bytes of this exact workload from the committed rocprofv3
    --pmc summary profiles/traffic_<workload>.json (tools/traffic.py), or None
    -- never another workload's figures."""
    p = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        t = json.load(f)
    return t if t.get("workload") == workload else None


LOCAL_KINDS = ("tile_sort", "global_pass", "tile_merge", "span_pass", "wide_pass", "run_merge", "run_mergek",
               "run_mergek_kernel")


def per_pass(trace, steps):
    """The local sort's HBM passes of one step, averaged over the profiled
    steps: [{"kind", "ms", "bytes", "kernel_ms"}] in pass order.  A multi-way
    pass (run_mergek) carries its k_mergek launch (recorded just before it) as
    kernel_ms; other passes are single kernels."""
    recs = [r for r in trace if r[0] in LOCAL_KINDS]
    if not recs or steps < 1 or len(recs) % steps:
        return []
    per = len(recs) // steps
    rows = None
    for st in range(steps):
        out, held = [], None
        for kind, ms, byt in recs[st * per:(st + 1) * per]:
            if kind == "run_mergek_kernel":
                held = ms
                continue
            out.append([kind, ms, byt, held if kind == "run_mergek" else None])
            held = None
        if rows is None:
            rows = out
        elif len(out) != len(rows) or any(a[0] != b[0] for a, b in zip(out, rows)):
            return []  # steps differ in shape: no per-pass average
        else:
            for a, b in zip(rows, out):
                a[1] += b[1]
                a[2] = b[2]
                if a[3] is not None:
                    a[3] += b[3]
    return [{"kind": k, "ms": ms / steps, "bytes": byt, "kernel_ms": None if km is None else km / steps}
            for k, ms, byt, km in rows]


def pass_rows(passes, traffic):
    """roofline.passes: per-pass achieved rate and fraction of the HBM peak;
    `traffic_ratio` = PMC bytes / algorithmic bytes of that pass when the
    committed capture has per-pass figures for this workload."""
    tp = (traffic or {}).get("passes") or []
    if len(tp) != len(passes):
        tp = [None] * len(passes)
    rows = []
    for i, (p, t) in enumerate(zip(passes, tp)):
        ach = p["bytes"] / (p["ms"] * 1e-3) / 1e9 if p["ms"] > 0 else None
        row = {"pass": i, "kind": p["kind"], "ms": p["ms"], "algorithmic_bytes": p["bytes"], "achieved": ach,
               "frac": ach / HBM_PEAK_GBS if ach else None}
        if p["kernel_ms"]:
            kach = p["bytes"] / (p["kernel_ms"] * 1e-3) / 1e9
            row["kernel"] = {"name": "k_mergek", "ms": p["kernel_ms"], "achieved": kach,
                             "frac": kach / HBM_PEAK_GBS}
        if t and t.get("kind") == p["kind"] and t.get("bytes"):
            row["traffic"] = t["bytes"]
            row["traffic_ratio"] = t["bytes"] / p["bytes"] if p["bytes"] else None
            if t.get("kernel_bytes") and "kernel" in row:
                row["kernel"]["traffic"] = t["kernel_bytes"]
                row["kernel"]["traffic_ratio"] = t["kernel_bytes"] / p["bytes"]
        rows.append(row)
    return rows


# -------------------------------------------------------------------- ranks
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if needs_launch(args):
        # one process per GPU; this process never touches the GPU.  It runs the
        # host-core baseline first (the reference under mpirun on this host's
        # cores) and hands it to rank 0 in a file, so the N-GPU line carries it.
        cmd = launch_command(argv, args.gpus, free_port())
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        path = None
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(args.logn if args.cpu_sample_logn is None else args.cpu_sample_logn,
                               args.cpu_sweep, args.cpu_sweep_logn, args.dtype)
            fd, path = tempfile.mkstemp(prefix="misort_bench_cpu_", suffix=".json")
            with os.fdopen(fd, "w") as f:
                json.dump(cpu, f)
            env[CPU_JSON_ENV] = path
        try:
            return subprocess.call(cmd, env=env)
        finally:
            if path:
                os.remove(path)

    if args.watchdog_s > 0:
        faulthandler.dump_traceback_later(args.watchdog_s, exit=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.gpus != world:
        sys.stderr.write(f"WARNING --gpus {args.gpus} but WORLD_SIZE {world}: running {world} ranks\n")

    # The CPU baseline runs first, before this process touches the GPU, on
    # rank 0 at every N (the other ranks wait in the process-group setup):
    # the reference's parallel_bitonic_sort under mpirun on the host cores,
    # or the launcher parent's measurement of it when there was one.
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = load_cpu_json(os.environ.get(CPU_JSON_ENV))
        if cpu is None:
            cpu = cpu_baseline(args.logn if args.cpu_sample_logn is None else args.cpu_sample_logn,
                               args.cpu_sweep, args.cpu_sweep_logn, args.dtype)

    # RCCL logs (its version banner too) go to stderr: stdout is the JSON line
    os.environ.setdefault("NCCL_DEBUG_FILE", "/dev/stderr")
    import numpy as np
    import torch
    import torch.distributed as dist
    import misort

    if world > 1:
        dist.init_process_group("gloo")  # host plumbing only: ids, barriers, max
    ndev = torch.cuda.device_count()
    shared = world > ndev  # several ranks on one GPU: RCCL over sockets (correctness mode)
    dev = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev)
    ctx = misort.Context(dev)
    if world > 1:
        ctx.comm_init_torch(share_gpu=shared)
    nranks = ctx.numprocs  # the ranks RCCL actually saw

    n_total = 1 << args.logn
    sizes = misort.block_sizes(n_total, nranks)
    loc, max_size = sizes[rank], n_total // nranks + 1
    g0 = sum(sizes[:rank])
    if args.dtype == "f64":
        kdt = torch.float64
    elif args.dtype == "u32":
        kdt = torch.uint32 if hasattr(torch, "uint32") else torch.int32
    else:
        kdt = torch.uint64 if hasattr(torch, "uint64") else torch.int64
    key_bytes = 4 if args.dtype == "u32" else 8

    def fill(t, g):
        if args.dtype == "f64":
            # SplitMix64 bits -> uniform doubles in [0, 1): the reference's key
            # type and (pre-skew) distribution, psort.cc:600-609
            z = torch.empty(t.numel(), dtype=torch.int64, device=t.device)
            ctx.fill_splitmix(z, SEED, g)
            t.copy_(((z >> 11) & ((1 << 53) - 1)).to(torch.float64) * 2.0 ** -53)
            del z
        else:
            ctx.fill_splitmix(t, SEED, g)

    d_in = torch.empty(max(loc, 1), dtype=kdt, device="cuda")
    d_out = torch.empty_like(d_in)
    stream = torch.cuda.current_stream()
    fill(d_in[:loc], g0)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    def run(algo):
        if algo == "sample":
            ctx.parallel_sample_sort(d_in, loc, max_size, out=d_out, stream=stream.cuda_stream)
        else:
            ctx.parallel_bitonic_sort(d_in, loc, max_size, out=d_out, stream=stream.cuda_stream)

    def max_over_ranks(v):
        t = torch.tensor([v], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

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
        return max_over_ranks(time.perf_counter() - t0)

    for _ in range(args.warmup):
        run(args.algo)
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
        run(args.algo)
    torch.cuda.synchronize()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    kern = ctx.profile_read() if events else {}
    passes = per_pass(ctx.profile_trace(), args.steps) if events else []
    nst = len(misort.schedule(nranks, rank))
    stages = ctx.profile_stages(nst) if events and nranks > 1 and args.algo == "bitonic" else []
    ctx.profile(False)
    xst = ctx.exchange_stats()
    errors = ctx.check_sort(d_out, loc)  # psort.cc:497-520 over all ranks

    stage_rows = None
    if stages:
        sched = misort.schedule(nranks, rank)
        d = int(np.log2(nranks))
        ij = [(i, j) for i in range(d) for j in range(i, -1, -1)]  # psort.cc:184-185
        stage_rows = []
        for st, (cnt, xms, mms, byt) in enumerate(stages):
            cnt = max(cnt, 1)
            x_max = max_over_ranks(xms / cnt)
            m_max = max_over_ranks(mms / cnt)
            b_max = max_over_ranks(byt / cnt)
            stage_rows.append({
                "stage": st, "i": ij[st][0], "j": ij[st][1], "partner_bit": ij[st][1],
                "rank0_partner": sched[st][0],
                "exchange_ms_max": x_max, "merge_split_ms_max": m_max,
                "exchange_bytes_max": b_max,
                # bytes one rank sends + receives over its links in the stage / stage time
                "xgmi_GBs": b_max / (x_max * 1e-3) / 1e9 if x_max > 0 else None})

    alt = None
    if nranks > 1 and args.algo == "bitonic" and not args.no_alt:
        # the redesigned sample sort (one RCCL all-to-all) on the same input, same contract
        ts = timed("sample", args.steps)
        alt = {"sample_sort": {"value": n_total * args.steps / ts / 1e9, "unit": "Gkeys/s",
                               "ms_per_step": ts / args.steps * 1e3,
                               "check_errors": ctx.check_sort(d_out, loc),
                               "note": "psort.cc:203-375 redesigned: samples, one all-to-all-v, "
                                       "merge tree, rebalance to the reference layout"}}

    t1 = None
    if nranks > 1 and not args.no_t1:
        # 1-GPU leg: rank 0 sorts ALL n_total keys alone on its GPU (a P = 1
        # context), same keys, same steps; scaling_eff = t1 / (P * tP)
        barrier()
        if rank == 0:
            solo = misort.Context(dev)
            a = torch.empty(n_total, dtype=kdt, device="cuda")
            b = torch.empty_like(a)
            if args.dtype == "f64":
                a.copy_(d_in[:loc]) if nranks == 1 else fill(a, 0)
            else:
                solo.fill_splitmix(a, SEED, 0)
            for _ in range(2):
                solo.parallel_bitonic_sort(a, n_total, n_total, out=b, stream=stream.cuda_stream)
            torch.cuda.synchronize()
            ts0 = time.perf_counter()
            for _ in range(args.steps):
                solo.parallel_bitonic_sort(a, n_total, n_total, out=b, stream=stream.cuda_stream)
            torch.cuda.synchronize()
            t1 = (time.perf_counter() - ts0) / args.steps
            assert solo.check_sort(b) == 0
            del a, b
            solo.close()
            torch.cuda.empty_cache()
        barrier()

    host_io = None
    if args.host_io:
        # host keys of the same workload; sorted through the pinned staging pipeline
        h_in = d_in[:loc].cpu().numpy()
        h_in = h_in if args.dtype == "f64" else h_in.view(np.uint32 if key_bytes == 4 else np.uint64)
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
                tt = max_over_ranks(time.perf_counter() - t0)
                best = tt if best is None else min(best, tt)
            res[name] = {"value": n_total / best / 1e9, "unit": "Gkeys/s", "ms": best * 1e3,
                         "chunk_keys": chunk}
            assert bool(np.all(h_out[1:] >= h_out[:-1])) if loc > 1 else True
        os.environ.pop("MISORT_STAGE_CHUNK", None)
        res["note"] = ("PCIe-inclusive: host numpy keys in, host keys out (pinned ring, H2D/D2H, "
                       "host copies); not the metric value")
        host_io = res

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        tile = misort.plan(loc, key_bytes)[0][1] + 1
        local_algo = (f"SORT tiles of 2^{tile} keys in LDS (bitonic network, top levels as in-LDS merge "
                      "levels), then multi-way merge passes of up to 4 merge levels per HBM pass (16-way, "
                      "runsk.hip; u32 with 64-bit fences, u64 with 128-bit) "
                      "(the reference's local std::sort, psort.cc:175)")
        out = {
            "metric": METRIC,
            "value": n_total * args.steps / elapsed / 1e9,
            "unit": "Gkeys/s",
            "n_gpus": nranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (SplitMix64 keys generated in HBM, seed 0x5EED0003)",
            "config": {"workload": f"bitonic sort 2^{args.logn} {args.dtype} keys "
                                   f"({baseline_config(args.logn, args.dtype)})",
                       "keys": n_total, "keys_per_gpu": loc,
                       "algo": args.algo, "local_sort": local_algo,
                       "parallelism": (f"hypercube bitonic, {nranks} GPU(s), RCCL compare-split"
                                       if args.algo == "bitonic" else
                                       f"sample sort, {nranks} GPU(s), RCCL all-to-all")},
            "check_errors": errors,
        }
        if shared:
            out["shared_gpu"] = ("several ranks on one GPU: RCCL over its socket transport "
                                 "(NCCL_HOSTID per rank) -- a correctness run, not an xGMI figure")
        if nranks > 1:
            out["exchange"] = {"stages_per_step": xst[0] / args.steps,
                               "rank0_bytes_per_step": xst[1] / args.steps,
                               "rank0_whole_block_bytes_per_step": xst[2] / args.steps}
            if stage_rows:
                out["exchange"]["stages"] = stage_rows
        if t1 is not None:
            out["t1_ms"] = t1 * 1e3
            out["scaling_eff"] = t1 / (nranks * elapsed / args.steps)
        if kern:
            per = {}
            for name, (nl, tms, byt) in kern.items():
                if nl:
                    per[name] = {"launches_per_step": nl / args.steps, "ms_per_step": tms / args.steps,
                                 "avg_launch_us": tms / nl * 1e3,
                                 "achieved_GBs": byt / (tms * 1e-3) / 1e9 if tms > 0 and byt > 0 else None}
            if "run_mergek_kernel" in per:
                per["run_mergek_kernel"]["note"] = "k_mergek alone, inside run_mergek (not added twice)"
            out["kernels"] = per
            # families (passes); run_mergek_kernel is nested inside run_mergek
            hbm = {k: v for k, v in kern.items() if k not in ("exchange", "run_mergek_kernel")}
            dom = max(hbm.items(), key=lambda kv: kv[1][1])
            fam = dom[0]
            # the dominant KERNEL: for a multi-way pass, k_mergek itself (rocprof's
            # k_mergek rows); the pass with its planning kernels is reported beside it
            name = "run_mergek_kernel" if fam == "run_mergek" and kern.get("run_mergek_kernel", (0,))[0] else fam
            nl, tms, byt = kern[name]
            wl = f"{args.dtype}_2e{args.logn}_n{nranks}"
            traffic = load_traffic(wl)
            tr = None
            if traffic and name in traffic and traffic[name].get("bytes_per_launch"):
                tr = traffic[name]["bytes_per_launch"]
            achieved = byt / (tms * 1e-3) / 1e9
            out["roofline"] = {"kernel": name, "bound": "hbm", "achieved": achieved,
                               "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                               "traffic": tr, "algorithmic_bytes_per_launch": byt / nl,
                               "avg_launch_us": tms / nl * 1e3,
                               "traffic_source": (f"profiles/traffic_{wl}.json ({traffic.get('source')})"
                                                  if traffic else None)}
            if passes:
                out["roofline"]["passes"] = pass_rows(passes, traffic)
            if name != fam:
                pnl, pms, pbyt = kern[fam]
                pach = pbyt / (pms * 1e-3) / 1e9
                ptr = traffic[fam]["bytes_per_launch"] if traffic and fam in traffic and \
                    traffic[fam].get("bytes_per_launch") else None
                out["roofline"]["pass"] = {"family": fam, "achieved": pach, "frac": pach / HBM_PEAK_GBS,
                                           "avg_launch_us": pms / pnl * 1e3, "traffic": ptr,
                                           "note": "the whole multi-way pass: k_mergek + fence merge, "
                                                   "counts, bounds, descriptors"}
            kt = sum(v[1] for k, v in hbm.items()) / args.steps
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
    return 0


if __name__ == "__main__":
    sys.exit(main())
