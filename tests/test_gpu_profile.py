"""Per-pass profiling of the local sort (runtime.cpp Profiler), which bench.py
reports as `kernels` and `roofline.passes`.  By default the passes are timed by
events their own kernels carry (hipExtLaunchKernelGGL: the dispatch timestamps,
no marker packets between kernels: stop events only with MISORT_PROF_BIND=2,
the default, start and stop with 1); MISORT_PROF_MARKERS=1 times them by
marker events around each pass (the knobs are read once per process: a child
process per setting).
Either way one sort yields, in pass order, tile_sort, then per multi-way pass
its k_mergek launch (run_mergek_kernel) and the pass (run_mergek), per 2-way
pass run_merge; every record is positive, a k_mergek launch is within its pass,
and the passes add up to no more than the sort's wall time.  A host-staged sort
(misort_sort_host) records each pass once, by its marker scope (k_mergek's own
record nests only under marker timing)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, time, torch
sys.path.insert(0, sys.argv[1])
import misort
ctx = misort.Context(0)
out = {}
for n, kb in ((1 << 24, 4), ((1 << 16) + 3, 4), ((1 << 21) + 5, 8), ((1 << 23) + 77, 4)):
    T = torch.int32 if kb == 4 else torch.int64
    d = torch.randint(-2**31, 2**31 - 1, (n,), dtype=T, device="cuda")
    if kb == 4 and hasattr(torch, "uint32"):
        d = d.view(torch.uint32)
    elif kb == 8 and hasattr(torch, "uint64"):
        d = d.view(torch.uint64)
    o = torch.empty_like(d)
    ctx.local_sort(d, o)  # warm
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.profile_reset()
    t0 = time.perf_counter()
    ctx.local_sort(d, o)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    tr = ctx.profile_trace()
    ctx.profile(False)
    out[f"{n}_{kb}"] = {"plan": [p[0] for p in misort.plan(n, kb)], "trace": tr, "wall_ms": wall}
# host staging (misort_sort_host): its passes are recorded by marker scopes,
# each exactly once, in plan order
import numpy as np
hn = (1 << 22) + 9
h = np.random.default_rng(1).integers(0, 2**32, hn, dtype=np.uint64).astype(np.uint32)
ctx.sort_host(h)  # warm
ctx.profile(True)
ctx.profile_reset()
t0 = time.perf_counter()
r = ctx.sort_host(h)
wall = (time.perf_counter() - t0) * 1e3
tr = ctx.profile_trace()
ctx.profile(False)
out["host"] = {"plan": [p[0] for p in misort.plan(hn, 4)], "trace": tr, "wall_ms": wall,
               "sorted": bool(np.array_equal(r, np.sort(h)))}
print("JSON", json.dumps(out))
ctx.close()
"""


@pytest.mark.gpu
@pytest.mark.parametrize("markers,bind,sysfence", [("0", "2", "0"), ("0", "1", "0"), ("1", "2", "0"), ("0", "2", "1")])
def test_pass_records(markers, bind, sysfence):
    # sysfence: MISORT_PROF_SYSFENCE=1 restores the system-scope release of the events
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "parallel-computing-mpi_amd")],
                       env=dict(os.environ, MISORT_PROF_MARKERS=markers, MISORT_PROF_BIND=bind,
                                MISORT_PROF_SYSFENCE=sysfence),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([x for x in r.stdout.splitlines() if x.startswith("JSON")][-1][5:])
    assert res["host"]["sorted"]
    for key, v in res.items():
        want = []
        # host staging nests k_mergek's record only under marker timing
        nest = key != "host" or markers == "1"
        for kind in v["plan"]:
            want += ["run_mergek_kernel", "run_mergek"] if kind == "run_mergek" and nest else [kind]
        trace = v["trace"]
        assert [t[0] for t in trace] == want, key
        assert all(t[1] > 0 for t in trace), (key, trace)
        for a, b in zip(trace, trace[1:]):
            if a[0] == "run_mergek_kernel":
                assert a[1] <= b[1] * 1.001, (key, a, b)
        passes = sum(t[1] for t in trace if t[0] != "run_mergek_kernel")
        assert passes <= v["wall_ms"] * 1.02 + 0.01, (key, passes, v["wall_ms"])
