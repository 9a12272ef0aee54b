"""The compare-split bracket computed on the device (kernels.hip
k_exchange_count) must give exactly the host's misort_exchange_count (runtime.cpp
corank_lower), or the partners would disagree on the exchange size k.

The kernel narrows [lo, hi] by evaluating the (true-then-false) predicate at
EXN evenly spaced points per round instead of bisecting.  This CPU test runs a
line-for-line numpy model of those rounds against the library's host function
on random, duplicate-heavy, disjoint and ragged sample sets (u32 and u64, the
reference's block sizes psort.cc:556-562 among them).  The GPU tests
(test_gpu_multirank.py: coded vs raw exchange, golden SHA at P = 2/4/8) run the
kernel itself."""
import functools

import numpy as np
import pytest

import misort

EXN = 1024


def stride(n):
    return max(256, (n + 32767) // 32768)


def count(n):
    return 0 if n <= 0 else (n + stride(n) - 1) // stride(n) + 1


def device_model(sa, na, sb, nb):
    """k_exchange_count: i_lo by rounds of EXN probes (returns k = na - i_lo)."""
    Sa, Sb, ca, cb = stride(na), stride(nb), len(sa), len(sb)

    def certain(i):  # vectorised over the EXN points of a round
        return sa[np.minimum(i // Sa + 1, ca - 1)] <= sb[np.minimum((na - 1 - i) // Sb, cb - 1)]

    lo, hi = (na - nb if na > nb else 0), na
    if na == 0:
        lo = hi = 0
    elif nb == 0:
        lo = hi = na
    rounds = 0
    while lo < hi:
        rounds += 1
        step = (hi - lo + EXN - 1) // EXN
        x = lo + np.arange(EXN, dtype=np.int64) * step
        x = x[x < hi]
        c = int(np.count_nonzero(certain(x)))
        assert np.all(certain(x)[:c])  # the true points are a prefix (monotone predicate)
        if step == 1:
            lo += c
            break
        nlo = lo + (c - 1) * step + 1 if c > 0 else lo
        xc = lo + c * step
        hi = min(xc, hi)
        lo = nlo
    assert rounds <= 4  # 2^31 keys: three rounds of 1024 and a last exact one
    return na - lo


def samples(block):
    n = block.size
    idx = np.minimum(np.arange(count(n), dtype=np.int64) * stride(n), n - 1)
    return block[idx]


@functools.lru_cache(maxsize=1)
def cases():
    rng = np.random.default_rng(7)
    out = []
    for dt in (np.uint32, np.uint64):
        top = np.iinfo(dt).max
        for na, nb in [(100003, 100003), (1 << 20, 1 << 20), ((1 << 22) + 5, (1 << 22) + 4), (5000, 300),
                       (300, 5000), (1 << 21, 17)]:
            a = np.sort(rng.integers(0, top, size=na, dtype=dt, endpoint=True))
            b = np.sort(rng.integers(0, top, size=nb, dtype=dt, endpoint=True))
            out.append((a, b))
            out.append((np.sort(rng.integers(0, 8, size=na, dtype=dt)), np.sort(rng.integers(0, 8, size=nb, dtype=dt))))
            out.append((np.full(na, 3, dt), np.full(nb, 3, dt)))  # all equal
            out.append((np.arange(na, dtype=dt), np.arange(nb, dtype=dt) + dt(na)))  # A below B: k = 0
            out.append((np.arange(na, dtype=dt) + dt(nb), np.arange(nb, dtype=dt)))  # A above B: k = min
    return out


@pytest.mark.parametrize("i", range(60))
def test_device_bracket_model_equals_host(i):
    cs = cases()
    if i >= len(cs):
        pytest.skip()
    a, b = cs[i]
    sa, sb = samples(a), samples(b)
    host = misort.exchange_count(sa, a.size, sb, b.size)
    assert device_model(sa, a.size, sb, b.size) == host
    assert 0 <= host <= min(a.size, b.size)
