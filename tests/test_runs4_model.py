"""numpy model of the 4-way merge pass's chunking (runs4.hip), CPU only.

Mirrors the kernels' constants and rules: fences every FG keys of each run,
packed (key, run, position/FG) so that u64 order is the total order; the
group's fences merged; every FM-th one starts a chunk whose start in each run
is that run's count of keys before the fence; chunks are then merged
independently.  Checks the properties the kernels rely on: chunks tile each
group exactly, no chunk exceeds CAP keys, every chunk's keys precede the next
chunk's, and the chunk/slot indexing (chunks per full group = ceil(fences /
FM)) matches the bounds layout."""
import numpy as np
import pytest

FG_LOG2, FM = 8, 28
NT, IT = 256, 36  # k_merge4 lanes and load rows
FG = 1 << FG_LOG2
CAP = (FM + 4) * FG


def fences(x, lw, n):
    p = np.arange(0, n, FG, dtype=np.int64)
    r = (p >> lw) & 3
    j = (p & ((1 << lw) - 1)) >> FG_LOG2
    return (x[p].astype(np.uint64) << np.uint64(32)) | (r.astype(np.uint64) << np.uint64(30)) | j.astype(np.uint64)


def chunk_bounds(x, lw, g, F):
    """Start of every chunk of group g in each run (+ the end slot), as k_bounds4."""
    n, W = x.size, 1 << lw
    base = g << (lw + 2)
    lens = [max(0, min(W, n - base - r * W)) for r in range(4)]
    f0, f1 = base >> FG_LOG2, (min(n, base + 4 * W) + FG - 1) >> FG_LOG2
    M = np.sort(F[f0:f1])
    out = []
    for t in range(0, (f1 - f0 + FM - 1) // FM):
        f = int(M[t * FM])
        v, r0, j0 = f >> 32, (f >> 30) & 3, f & ((1 << 30) - 1)
        st = []
        for r in range(4):
            if r == r0:
                st.append(j0 << FG_LOG2)
                continue
            run = x[base + r * W: base + r * W + lens[r]]
            want = int(np.searchsorted(run, v, side="right" if r < r0 else "left"))
            st.append(want)
            if lens[r] == 0:
                continue
            # k_bounds4's two-stage search: fences of run r before f, then the
            # FG positions between two of them
            fr = F[(base + r * W) >> FG_LOG2: ((base + r * W) >> FG_LOG2) + ((lens[r] + FG - 1) >> FG_LOG2)]
            lo = int(np.searchsorted(fr, np.uint64(f), side="left"))
            if lo == 0:
                got = 0
            else:
                a, b = ((lo - 1) << FG_LOG2) + 1, min(lo << FG_LOG2, lens[r])
                while a < b:
                    mid = (a + b) >> 1
                    before = run[mid] <= v if r < r0 else run[mid] < v
                    if before:
                        a = mid + 1
                    else:
                        b = mid
                got = a
            assert got == want
        out.append(st)
    out.append(lens)
    return out, lens


@pytest.mark.parametrize("lw", [15, 16])
@pytest.mark.parametrize("n_groups,tail", [(2, 0), (1, 3 * (1 << 15) + 5), (1, 777), (0, (1 << 15) * 2 + 1)])
@pytest.mark.parametrize("kind", ["uniform", "dup", "equal", "interleaved"])
def test_chunks_tile_and_bound(lw, n_groups, tail, kind):
    W = 1 << lw
    n = n_groups * 4 * W + tail
    rng = np.random.default_rng(lw + n)
    if kind == "uniform":
        x = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    elif kind == "dup":
        x = rng.integers(0, 7, n).astype(np.uint32)
    elif kind == "equal":
        x = np.full(n, 0xFFFFFFFF, np.uint32)
    else:
        x = (np.arange(n) % 4 * 1000 + np.arange(n) // 4).astype(np.uint32)
    for s in range(0, n, W):
        x[s:s + W].sort()
    F = fences(x, lw, n)
    ngroups = (n + 4 * W - 1) // (4 * W)
    kf = ((4 * W >> FG_LOG2) + FM - 1) // FM
    for g in range(ngroups):
        bounds, lens = chunk_bounds(x, lw, g, F)
        if (g + 1) * 4 * W <= n:
            assert len(bounds) - 1 == kf
        base = g << (lw + 2)
        merged = []
        prev_max = None
        assert bounds[0] == [0, 0, 0, 0]
        for a, b in zip(bounds[:-1], bounds[1:]):
            seg = [x[base + r * W + a[r]: base + r * W + b[r]] for r in range(4)]
            size = sum(s.size for s in seg)
            assert all(b[r] >= a[r] for r in range(4)) and size <= CAP
            # load rows: each row of NT keys inside one segment, IT rows per chunk
            assert sum(-(-s.size // NT) for s in seg) <= IT
            chunk = np.sort(np.concatenate(seg))
            if chunk.size and prev_max is not None:
                assert chunk[0] >= prev_max
            if chunk.size:
                prev_max = chunk[-1]
            merged.append(chunk)
        want = np.sort(x[base: base + sum(lens)])
        np.testing.assert_array_equal(np.concatenate(merged), want)
