"""numpy model of the K-way merge pass's chunking (runsk.hip), CPU only.

Mirrors the kernels' constants and rules: fences every FG keys of each run,
packed (key, run, position/FG) so that u64 order is the total order; the
group's fences merged; every FM-th one starts a chunk whose start in each run
is that run's count of keys before the fence; chunks are then merged
independently.  Checks the properties the kernels rely on: chunks tile each
group exactly, no chunk exceeds CAP keys nor the load rows (RW keys of one
segment, NROWS per chunk), every chunk's keys precede the next chunk's, and
the chunk/slot indexing (chunks per full group = ceil(fences / FM)) matches
the bounds layout.  K = 2^lk, lk = 1..4."""
import numpy as np
import pytest

FG_LOG2, CAP = 7, 8192
NT, IT = 512, 18  # k_mergek lanes and keys per lane
FG = 1 << FG_LOG2


def shape(lk):
    """(K, FM, RW, NROWS) of runsk.hip's Shape<lk>."""
    K = 1 << lk
    rw = 64 if lk == 4 else 128 if lk == 3 else 256
    return K, CAP // FG - K, rw, IT * NT // rw


def fences(x, lw, lk, n):
    p = np.arange(0, n, FG, dtype=np.int64)
    r = (p >> lw) & ((1 << lk) - 1)
    j = (p & ((1 << lw) - 1)) >> FG_LOG2
    return ((x[p].astype(np.uint64) << np.uint64(32)) | (r.astype(np.uint64) << np.uint64(32 - lk))
            | j.astype(np.uint64))


def chunk_bounds(x, lw, lk, g, F):
    """Start of every chunk of group g in each run (+ the end slot), as k_bounds."""
    K, FM, _, _ = shape(lk)
    n, W = x.size, 1 << lw
    base = g << (lw + lk)
    lens = [max(0, min(W, n - base - r * W)) for r in range(K)]
    f0, f1 = base >> FG_LOG2, (min(n, base + K * W) + FG - 1) >> FG_LOG2
    M = np.sort(F[f0:f1])
    out = []
    for t in range(0, (f1 - f0 + FM - 1) // FM):
        f = int(M[t * FM])
        v, r0, j0 = f >> 32, (f >> (32 - lk)) & (K - 1), f & ((1 << (32 - lk)) - 1)
        st = []
        for r in range(K):
            if r == r0:
                st.append(j0 << FG_LOG2)
                continue
            run = x[base + r * W: base + r * W + lens[r]]
            want = int(np.searchsorted(run, v, side="right" if r < r0 else "left"))
            st.append(want)
            if lens[r] == 0:
                continue
            # k_bounds' two-stage search: fences of run r before f, then the
            # FG positions between two of them
            fr = F[(base + r * W) >> FG_LOG2: ((base + r * W) >> FG_LOG2) + ((lens[r] + FG - 1) >> FG_LOG2)]
            lo = int(np.searchsorted(fr, np.uint64(f), side="left"))
            got = 0 if lo == 0 else refine(run, fr, lo, lens[r], v, r < r0)
            assert got == want
        out.append(st)
    out.append(lens)
    return out, lens


def refine(run, fr, lo, ln, v, le):
    """k_bounds' window search: the first position in [a, b] whose key is not
    before the fence (key > v if le, key >= v otherwise), guessed by
    interpolating v between the window's fence keys, bracketed by galloping
    from the guess, then binary-searched."""
    def before(q):
        return run[q] <= v if le else run[q] < v
    a, b = ((lo - 1) << FG_LOG2) + 1, min(lo << FG_LOG2, ln)
    ka = int(fr[lo - 1]) >> 32
    p = a + ((b - a) >> 1)
    if (lo << FG_LOG2) < ln:
        kb = int(fr[lo]) >> 32
        if kb > ka:
            p = a + ((v - ka) * (b - a)) // (kb - ka)
    p = min(max(p, a), b)
    if p < b and before(p):
        lo_b, hi_b, step = p + 1, b, 4
        while lo_b + step - 1 < hi_b:
            x = lo_b + step - 1
            if before(x):
                lo_b, step = x + 1, step * 2
            else:
                hi_b = x
                break
    else:
        lo_b, hi_b, step = a, p, 4
        while hi_b - step >= lo_b:
            x = hi_b - step
            if not before(x):
                hi_b, step = x, step * 2
            else:
                lo_b = x + 1
                break
    while lo_b < hi_b:
        mid = (lo_b + hi_b) >> 1
        if before(mid):
            lo_b = mid + 1
        else:
            hi_b = mid
    return lo_b


@pytest.mark.parametrize("lk", [1, 2, 3, 4])
@pytest.mark.parametrize("lw", [15, 16])
@pytest.mark.parametrize("n_groups,tail", [(2, 0), (1, 3 * (1 << 15) + 5), (1, 777), (0, (1 << 15) * 2 + 1)])
@pytest.mark.parametrize("kind", ["uniform", "dup", "equal", "interleaved"])
def test_chunks_tile_and_bound(lk, lw, n_groups, tail, kind):
    K, FM, RW, NROWS = shape(lk)
    W = 1 << lw
    n = n_groups * K * W + tail
    rng = np.random.default_rng(lw + n)
    if kind == "uniform":
        x = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    elif kind == "dup":
        x = rng.integers(0, 7, n).astype(np.uint32)
    elif kind == "equal":
        x = np.full(n, 0xFFFFFFFF, np.uint32)
    else:
        x = (np.arange(n) % K * 1000 + np.arange(n) // K).astype(np.uint32)
    for s in range(0, n, W):
        x[s:s + W].sort()
    F = fences(x, lw, lk, n)
    ngroups = (n + K * W - 1) // (K * W)
    kf = ((K * W >> FG_LOG2) + FM - 1) // FM
    for g in range(ngroups):
        bounds, lens = chunk_bounds(x, lw, lk, g, F)
        if (g + 1) * K * W <= n:
            assert len(bounds) - 1 == kf
        base = g << (lw + lk)
        merged = []
        prev_max = None
        assert bounds[0] == [0] * K
        for a, b in zip(bounds[:-1], bounds[1:]):
            seg = [x[base + r * W + a[r]: base + r * W + b[r]] for r in range(K)]
            size = sum(s.size for s in seg)
            assert all(b[r] >= a[r] for r in range(K)) and size <= CAP
            # load rows: each row of RW keys inside one segment, NROWS per chunk
            assert sum(-(-s.size // RW) for s in seg) <= NROWS
            chunk = np.sort(np.concatenate(seg))
            if chunk.size and prev_max is not None:
                assert chunk[0] >= prev_max
            if chunk.size:
                prev_max = chunk[-1]
            merged.append(chunk)
        want = np.sort(x[base: base + sum(lens)])
        np.testing.assert_array_equal(np.concatenate(merged), want)
