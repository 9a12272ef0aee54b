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


def fence_rank_model(F, nf, wf_log2, lk, fm, nt=256):
    """k_fence_rank (runsk.hip) on a flat fence array: blocks of nt threads own
    nt - 1 fences each (thread 0 ranks the fence before them); returns the
    merged fences M and the per-(chunk, run) counts P exactly as the kernel
    writes them (-1 = never written)."""
    K, wf, gl = 1 << lk, 1 << wf_log2, wf_log2 + lk
    ngroups = (nf + (1 << gl) - 1) >> gl
    fences_per_group = 1 << gl
    kf = (fences_per_group + fm - 1) // fm
    nch_of = [kf if (g + 1) << gl <= nf else (min(nf - (g << gl), fences_per_group) + fm - 1) // fm
              for g in range(ngroups)]
    M = np.zeros(nf, np.uint64)
    P = np.full((ngroups * kf + 1) * K, -1, np.int64)
    nblocks = (nf + nt - 2) // (nt - 1)
    for b in range(nblocks):
        sp = [-1] * nt
        info = [None] * nt
        for tid in range(nt):
            e = b * (nt - 1) - 1 + tid
            if e < 0 or e >= nf:
                continue
            g = e >> gl
            gbase = g << gl
            nfg = min(nf - gbase, 1 << gl)
            gi = e - gbase
            q, i = gi >> wf_log2, gi & (wf - 1)
            v = F[e]
            p = i
            for r in range(K):
                ln = 0 if r == q else max(0, min(nfg - r * wf, wf))
                pos, st = 0, wf
                while st > 0:  # the kernel's power-of-two lower bound
                    if pos + st <= ln and F[gbase + r * wf + pos + st - 1] < v:
                        pos += st
                    st >>= 1
                p += pos
            M[gbase + p] = v
            sp[tid] = p
            info[tid] = (g, gbase, nfg, gi, q, i, p)
        for tid in range(1, nt):
            if info[tid] is None:
                continue
            g, gbase, nfg, gi, q, i, p = info[tid]
            c0, nch = g * kf, nch_of[g]
            lq = min(nfg - q * wf, wf)
            t0 = 0 if i == 0 else sp[tid - 1] // fm + 1
            t1 = p // fm
            for t in range(t0, t1 + 1):
                P[(c0 + t) * K + q] = i
            if i == lq - 1:
                for t in range(t1 + 1, nch):
                    P[(c0 + t) * K + q] = i + 1
            nruns = (nfg + wf - 1) >> wf_log2
            if gi < nch:
                for r in range(nruns, K):
                    P[(c0 + gi) * K + r] = 0
    return M, P, nch_of, kf


@pytest.mark.parametrize("lk,wf_log2,nf,fm", [(3, 5, 3 * 256 + 40, 7), (3, 5, 256 * 2, 60), (2, 6, 256 + 64 * 2 + 3, 9),
                                              (4, 3, 16 * 8 * 3 + 17, 5), (1, 7, 700, 13), (3, 8, 2048 + 1, 66)])
@pytest.mark.parametrize("kind", ["uniform", "dup", "interleaved"])
def test_fence_rank_counts(lk, wf_log2, nf, fm, kind):
    """k_fence_rank's merged order and counts equal the sorted group fences and
    the direct per-(chunk, run) counts, tail groups with short and missing runs
    included."""
    K, wf, gl = 1 << lk, 1 << wf_log2, wf_log2 + lk
    rng = np.random.default_rng(nf + fm)
    if kind == "uniform":
        keys = rng.integers(0, 2**20, nf)
    elif kind == "dup":
        keys = rng.integers(0, 3, nf)
    else:
        keys = np.arange(nf) % wf * K + (np.arange(nf) // wf) % K
    F = np.zeros(nf, np.uint64)
    for s in range(0, nf, wf):  # per run: sorted keys packed with (run, position) as the fences are
        e = np.arange(s, min(s + wf, nf))
        run = (e >> wf_log2) & (K - 1)
        F[s:s + e.size] = ((np.sort(keys[s:s + e.size]).astype(np.uint64) << np.uint64(32))
                           | (run.astype(np.uint64) << np.uint64(32 - lk)) | (e & (wf - 1)).astype(np.uint64))
    M, P, nch_of, kf = fence_rank_model(F, nf, wf_log2, lk, fm)
    for g in range(len(nch_of)):
        gbase = g << gl
        nfg = min(nf - gbase, 1 << gl)
        want = np.sort(F[gbase:gbase + nfg])
        np.testing.assert_array_equal(M[gbase:gbase + nfg], want)
        for t in range(nch_of[g]):
            start = int(want[t * fm])
            for r in range(K):
                run = F[gbase + r * wf: gbase + min(nfg, (r + 1) * wf)] if r * wf < nfg else F[:0]
                assert P[(g * kf + t) * K + r] == int(np.sum(run < start)), (g, t, r)
