import os, sys, time, json
sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "parallel-computing-mpi_amd"))
import numpy as np, torch, misort
ctx = misort.Context(0)
n = 1 << 30
d = torch.empty(n, dtype=torch.int32, device="cuda")
ctx.fill_splitmix(d, 0x5EED0003)
x = d.cpu().numpy().view(np.uint32)
for th in (8, 16, 32):
    for ch in (1 << 22, 1 << 24, 1 << 26):
        os.environ["MISORT_STAGE_CHUNK"] = str(ch)
        os.environ["MISORT_STAGE_THREADS"] = str(th)
        # thread count is read once per process -> run each thread count in its own process
        break
th = int(sys.argv[1])
os.environ["MISORT_STAGE_THREADS"] = str(th)
for ch in (1 << 22, 1 << 24, 1 << 26):
    os.environ["MISORT_STAGE_CHUNK"] = str(ch)
    y = ctx.sort_host(x)
    ts = []
    for _ in range(2):
        t0 = time.perf_counter(); y = ctx.sort_host(x); ts.append(time.perf_counter() - t0)
    print(json.dumps({"threads": th, "chunk": ch, "ms": min(ts) * 1e3}), flush=True)
t0 = time.perf_counter(); z = x.copy(); print("numpy copy 4GiB ms", (time.perf_counter()-t0)*1e3, flush=True)
