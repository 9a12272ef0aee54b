"""The merge-level partition (runs.hip k_runs_partition) is a 32-ary search: each
round 32 lanes test the co-rank predicate A[x] <= B[d-1-x] at evenly spaced
points and keep the step around the first false one.  This CPU test runs a
line-for-line numpy model of those rounds against the plain definition (the
number of A keys among the first d outputs of merge(A, B), A first on ties) on
random, duplicate-heavy and disjoint runs, including ragged last pairs.  The GPU
tests (test_gpu_runs.py) run the kernel itself."""
import numpy as np
import pytest

LANES = 32


def model(A, B, d):
    na, nb = A.size, B.size
    lo, hi = (d - nb if d > nb else 0), (d if d < na else na)
    rounds = 0
    while lo < hi:
        rounds += 1
        step = (hi - lo + LANES - 1) // LANES
        x = lo + np.arange(LANES, dtype=np.int64) * step
        t = np.zeros(LANES, bool)
        v = x < hi
        t[v] = A[x[v]] <= B[d - 1 - x[v]]
        c = int(t.sum())
        assert np.all(t[:c])  # the true points are a prefix
        nhi = lo + c * step
        lo = lo + (c - 1) * step + 1 if c > 0 else lo
        hi = min(nhi, hi)
    return lo, rounds


def reference(A, B, d):
    """A first on ties: the largest i <= d with A[i-1] <= B[d-i] (merge path)."""
    best = max(0, d - B.size)
    for i in range(max(0, d - B.size), min(d, A.size) + 1):
        if i == 0 or d - i >= B.size or A[i - 1] <= B[d - i]:
            best = i
        else:
            break
    return best


@pytest.mark.parametrize("seed", range(6))
def test_partition_model_matches_merge_path(seed):
    rng = np.random.default_rng(seed)
    for na, nb in [(1000, 1000), (1000, 37), (5, 900), (4096, 4096), (3000, 0)]:
        for kind in ("spread", "dups", "disjoint_lo", "disjoint_hi"):
            if kind == "spread":
                A = np.sort(rng.integers(0, 2**32, na, dtype=np.uint64))
                B = np.sort(rng.integers(0, 2**32, nb, dtype=np.uint64))
            elif kind == "dups":
                A = np.sort(rng.integers(0, 4, na, dtype=np.uint64))
                B = np.sort(rng.integers(0, 4, nb, dtype=np.uint64))
            elif kind == "disjoint_lo":
                A = np.arange(na, dtype=np.uint64)
                B = np.arange(nb, dtype=np.uint64) + np.uint64(na)
            else:
                A = np.arange(na, dtype=np.uint64) + np.uint64(nb)
                B = np.arange(nb, dtype=np.uint64)
            for d in sorted(set([0, 1, na, nb, na + nb, (na + nb) // 2] + list(rng.integers(0, na + nb + 1, 8)))):
                got, rounds = model(A, B, int(d))
                assert got == reference(A, B, int(d))
                assert rounds <= 3  # ranges here are < 32^3


def test_rounds_for_a_2_23_pair():
    # 2^23-key runs (u64 fences of a 2^30 sort): 5 rounds instead of 23 bisection steps
    A = np.arange(1 << 23, dtype=np.uint64) * np.uint64(2)
    B = A + np.uint64(1)
    got, rounds = model(A, B, (1 << 23) + 12345)
    assert got == ((1 << 23) + 12345 + 1) // 2 and rounds == 5
