"""One rank of the real RCCL path at BASELINE sizes, and of its failure paths
(tests/test_gpu_rccl_large.py launches P of these with torch.distributed.run
on ONE GPU; every rank presents its own NCCL_HOSTID, so RCCL joins them over
its socket transport on loopback -- the RcclTransport code of runtime.cpp,
only the wire is not xGMI).

    rccl_large_worker.py config4 [raw]   2^30 u32 (seed 0x5EED0003) over P ranks;
                                         `raw`: MISORT_COMPRESS=0 + whole-block
                                         exchange, a 4*N/P-byte ncclSend per stage
    rccl_large_worker.py config5         u64 N = 2^29-3 and 2^29-7 ("ref" mix) at P = 8
    rccl_large_worker.py config5full     the same N with BASELINE config 5's own mix
                                         ("full": 5 % all-ones keys, the sentinel
                                         collision, crossing the real exchange)
    rccl_large_worker.py stall|dead      rank 1 stops taking part (sleeps / exits)
                                         after the communicator is up; rank 0 must
                                         get MISORT_E_RCCL within MISORT_TIMEOUT_S
    rccl_large_worker.py dead_user_stream both ranks queue a sort on the caller's
                                         stream; rank 1 exits before its last
                                         transfer ran; rank 0 drains the context's
                                         own (idle) stream, then check_sort on the
                                         caller's stream must still get
                                         MISORT_E_RCCL within MISORT_TIMEOUT_S

Results are checked against tests/golden/large.json (the oracle's outputs,
pinned by runs of the compiled reference): each rank writes its block to a
file in $MISORT_TEST_SPOOL, rank 0 hashes the concatenation in rank order.
Rank 0 prints one JSON line.
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))

import oracle_lib as O  # noqa: E402


def sha_files(paths):
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            while True:
                b = f.read(1 << 26)
                if not b:
                    break
                h.update(b)
    return h.hexdigest()


def main():
    mode = sys.argv[1]
    raw = len(sys.argv) > 2 and sys.argv[2] == "raw"
    import torch
    import torch.distributed as dist
    import misort

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    misort.set_shared_gpu_env(rank)
    torch.cuda.set_device(0)
    ctx = misort.Context(0)
    ctx.comm_init_torch(share_gpu=True)
    assert ctx.numprocs == world and ctx.myid == rank
    u32_t = torch.uint32 if hasattr(torch, "uint32") else torch.int32
    u64_t = torch.uint64 if hasattr(torch, "uint64") else torch.int64
    with open(os.path.join(HERE, "golden", "large.json")) as f:
        large = json.load(f)["cases"]
    spool = os.environ.get("MISORT_TEST_SPOOL", "/tmp")
    results = []

    def log(msg):
        sys.stderr.write(f"[rank {rank} {time.strftime('%H:%M:%S')}] {msg}\n")
        sys.stderr.flush()

    if mode in ("stall", "dead"):
        import faulthandler
        faulthandler.dump_traceback_later(90, exit=True)  # a hang shows where, then ends
        dist.barrier()
        log("communicator up, peer " + ("leaves" if mode == "dead" else "stalls"))
        if rank == 1:
            if mode == "dead":
                os._exit(0)  # no teardown: the peer just disappears
            time.sleep(float(os.environ.get("MISORT_TEST_STALL_S", "40")))
            os._exit(0)
        x = torch.arange(1 << 16, 0, -1, dtype=torch.int32, device="cuda").view(u32_t)
        t0 = time.perf_counter()
        code, msg = 0, ""
        try:
            ctx.parallel_bitonic_sort(x, x.numel(), x.numel())
            ctx.synchronize()
        except misort.MisortError as e:
            code, msg = e.code, str(e)
        el = time.perf_counter() - t0
        log(f"first call returned {code} after {el:.1f} s: {msg}")
        # the communicator is aborted: later calls fail at once, no hang
        t1 = time.perf_counter()
        code2 = 0
        try:
            ctx.parallel_bitonic_sort(x, x.numel(), x.numel())
        except misort.MisortError as e:
            code2 = e.code
        print(json.dumps({"world": world, "mode": mode, "code": code, "msg": msg, "elapsed_s": el,
                          "second_code": code2, "second_s": time.perf_counter() - t1}), flush=True)
        os._exit(0)

    if mode == "dead_user_stream":
        import faulthandler
        faulthandler.dump_traceback_later(90, exit=True)
        # a whole-block 2^25-key exchange: rank 1's send cannot have finished
        # when it leaves right after queuing it
        ctx.set_compress(False)
        ctx.set_full_exchange(True)
        n = 1 << 26
        buf = torch.empty(n // world, dtype=u32_t, device="cuda")
        ctx.fill_splitmix(buf, 0x5EED0003, rank * (n // world))
        user = torch.cuda.Stream()
        user.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        code, msg = 0, ""
        try:
            ctx.parallel_bitonic_sort(buf, buf.numel(), buf.numel(), stream=user.cuda_stream)
            if rank == 1:
                os._exit(0)  # the last transfer is queued, not done
            ctx.synchronize()  # the context's own stream: idle, drains at once
            ctx.check_sort(buf, buf.numel(), stream=user.cuda_stream)
        except misort.MisortError as e:
            code, msg = e.code, str(e)
        el = time.perf_counter() - t0
        log(f"check_sort on the caller's stream returned {code} after {el:.1f} s: {msg}")
        print(json.dumps({"world": world, "mode": mode, "code": code, "msg": msg, "elapsed_s": el,
                          "second_code": code, "second_s": 0.0}), flush=True)
        os._exit(0)

    def sort_and_check(name, n, kdt, fill, want_sha, want_err, want_sizes=None):
        sizes = misort.block_sizes(n, world)
        g0 = sum(sizes[:rank])
        mx = n // world + 1
        buf = torch.empty(mx, dtype=kdt, device="cuda")
        fill(buf[:sizes[rank]], g0, sizes[rank])
        out = torch.empty_like(buf)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        ctx.parallel_bitonic_sort(buf, sizes[rank], mx, out=out)
        ctx.synchronize()
        el = time.perf_counter() - t0
        st = ctx.exchange_stats()
        errs = ctx.check_sort(out, sizes[rank])
        path = os.path.join(spool, f"misort_rccl_{name}_{rank}.bin")
        out[:sizes[rank]].view(torch.uint8).cpu().numpy().tofile(path)
        del buf, out
        torch.cuda.empty_cache()
        dist.barrier()
        if rank == 0:
            paths = [os.path.join(spool, f"misort_rccl_{name}_{r}.bin") for r in range(world)]
            got = sha_files(paths)
            for p in paths:
                os.remove(p)
            ok = got == want_sha and errs == want_err and (want_sizes is None or sizes == want_sizes)
            results.append({"case": name, "ok": ok, "errors": errs, "sort_s": el,
                            "rank0_stage_bytes": st[1], "rank0_whole_block_bytes": st[2]})
        dist.barrier()

    if mode == "config4":
        c = [c for c in large if c["config"] == 4][0]
        if raw:
            ctx.set_compress(False)
            ctx.set_full_exchange(True)

        def fill(t, g0, cnt):
            ctx.fill_splitmix(t, c["seed"], g0)
        sort_and_check(f"config4_P{world}{'_raw' if raw else ''}", c["n"], u32_t, fill,
                       c["out_sha256"], c["errors"])
    elif mode in ("config5", "config5full"):
        variant = "ref" if mode == "config5" else "full"
        for c in large:
            if c["config"] != 5 or c["variant"] != variant or c["p"] != world:
                continue

            def fill(t, g0, cnt, c=c):
                x = O.u64mix(c["seed"], c["n"], int(c["top"], 16), g0, cnt)
                t.view(torch.int64).copy_(torch.from_numpy(x.view(np.int64)))
            sort_and_check(f"{mode}_N{c['n']}_P{world}", c["n"], u64_t, fill, c["out_sha256"], c["errors"],
                           c["sizes"])
    else:
        raise SystemExit(f"unknown mode {mode}")

    ctx.close()
    dist.barrier()
    if rank == 0:
        print(json.dumps({"world": world, "mode": mode, "raw": raw, "results": results}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
