"""GPU parity of the wide ROWS pass (bitonic.h k_rows_wide: 2^16-key register
tile, one LDS transpose) -- one pass of the bitonic network that replaces the
reference's local std::sort (psort.cc:175).

Each pass shape (hi, R, flip) runs once through misort_pass_probe and is
compared bit for bit with
  * a numpy replay of the same network stages (flip i <-> i ^ (2^(hi+1)-1),
    half-cleaners i <-> i ^ 2^b, minimum to the lower index, indices >= n
    read as all-ones and never stored), and
  * the LDS-tile ROWS pass (k_stream<ROWS>) of the same shape.
Full sorts with the planner's wide passes forced on and off run in child
processes (the planner knobs are read once per process)."""
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import misort  # noqa: E402

pytestmark = pytest.mark.gpu

U32_T = torch.uint32 if hasattr(torch, "uint32") else torch.int32
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = misort.Context(0)
    yield c
    c.close()


def ceil_log2(n):
    return max(0, int(n - 1).bit_length())


def replay(keys, hi, r, flip):
    """The pass's stages on the virtually padded array; returns the first n keys."""
    n = keys.size
    x = np.full(1 << ceil_log2(n), 0xFFFFFFFF, dtype=np.uint32)
    x[:n] = keys
    i = np.arange(x.size)
    for b in range(hi, hi - r, -1):
        j = i ^ ((1 << (hi + 1)) - 1) if (flip and b == hi) else i ^ (1 << b)
        lo = i < j
        a, c = x[i[lo]], x[j[lo]]
        x[i[lo]] = np.minimum(a, c)
        x[j[lo]] = np.maximum(a, c)
    return x[:n]


def run(ctx, keys, kind, hi, r, flip):
    d_in = torch.from_numpy(keys.view(np.int32)).cuda().view(U32_T)
    d_out = torch.empty_like(d_in)
    ctx.pass_probe(d_in, d_out, kind, hi, r, flip, reps=1)
    torch.cuda.synchronize()
    return d_out.view(torch.int32).cpu().numpy().view(np.uint32)


SHAPES = [(hi, r, f) for hi in (15, 16, 17, 19) for r in range(4, 11) for f in (False, True)]


@pytest.mark.parametrize("n", [1 << 20, (1 << 20) - 12345, (1 << 19) + 7])
def test_wide_pass_matches_network(ctx, n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    keys[rng.integers(0, n, size=n // 8)] = 7  # duplicates
    k = ceil_log2(n)
    checked = 0
    for hi, r, flip in SHAPES:
        if hi + 1 > k:
            continue
        got = run(ctx, keys, "wide_pass", hi, r, flip)
        want = replay(keys, hi, r, flip)
        assert np.array_equal(got, want), (n, hi, r, flip)
        lds = run(ctx, keys, "global_pass", hi, r, flip)
        assert np.array_equal(got, lds), (n, hi, r, flip)
        checked += 1
    assert checked >= 28


def test_wide_pass_rejects_bad_shapes(ctx):
    keys = np.arange(1 << 16, dtype=np.uint32)
    for hi, r in ((15, 3), (15, 11), (16, 3), (17, 12)):
        with pytest.raises(misort.MisortError):
            run(ctx, keys, "wide_pass", hi, r, False)


CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import misort
n = int(sys.argv[2])
ctx = misort.Context(0)
plan = misort.plan(n, 4)
rng = np.random.default_rng(n)
keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
keys[: n // 5] = keys[n // 7]
T = torch.uint32 if hasattr(torch, "uint32") else torch.int32
d = torch.from_numpy(keys.view(np.int32)).cuda().view(T)
out = torch.empty_like(d)
ctx.parallel_bitonic_sort(d, n, n, out=out)
torch.cuda.synchronize()
got = out.view(torch.int32).cpu().numpy().view(np.uint32)
ok = np.array_equal(got, np.sort(keys))
print("WIDE_PASSES", sum(1 for p in plan if p[0] == "wide_pass"), "OK" if ok else "MISMATCH")
ctx.close()
"""


@pytest.mark.parametrize("wide", ["0", "1"])
@pytest.mark.parametrize("n", [1 << 24, (1 << 23) + 4099])
def test_full_sort_with_and_without_wide_passes(wide, n):
    env = dict(os.environ, MISORT_WIDE=wide, MISORT_MERGE_FROM="0")  # the network path
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "parallel-computing-mpi_amd"), str(n)],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("WIDE_PASSES")][-1]
    _, count, verdict = line.split()
    assert verdict == "OK", line
    if wide == "0":
        assert int(count) == 0
