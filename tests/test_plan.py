"""The local-sort plan (bitonic.h plan_uncached) on the CPU.

A local sort (the reference's std::sort, psort.cc:175) is one SORT pass of
2^LT-key tiles (u32: 2^14 or 2^15 by size, u64: 2^13; the plan's SORT record
carries it as hi = LT - 1) followed by merge passes:
2^lk-way passes of lk levels each (runsk.hip) and 2-way passes of one level
(runs.hip).  A plan is right when
  * it starts with the SORT pass and its merge passes finish exactly the levels
    LT+1 .. ceil(log2 n), in order, and
  * replaying it on a numpy model (sort every 2^LT tile, then merge neighbouring
    runs level by level, all-ones padding for non-power-of-two n) sorts random
    keys like np.sort.
No device is touched: misort_plan is host-only."""
import numpy as np
import pytest

import misort

KIND_SORT = "tile_sort"
KIND_RUNS = "run_merge"  # one merge level (runs.hip): runs of 2^hi -> 2^(hi+1)
KIND_RUNSK = "run_mergek"  # R merge levels in one pass (runsk.hip): runs of 2^hi -> 2^(hi+R)
MERGES = (KIND_RUNS, KIND_RUNSK)


def ceil_log2(n):
    return max(0, int(n - 1).bit_length())


def merge_levels(plan):
    """Levels (input run log2) the merge passes finish, in order."""
    out = []
    for kind, hi, r, _ in plan[1:]:
        assert kind in MERGES
        out += list(range(hi, hi + r)) if kind == KIND_RUNSK else [hi]
    return out


def replay(keys, plan):
    """The plan on a numpy model: the SORT pass sorts every 2^lt tile, each
    merge pass sorts neighbouring groups of runs (all-ones padding to 2^k)."""
    lt = plan[0][1] + 1
    n = keys.size
    k = max(ceil_log2(n), lt)
    x = np.full(1 << k, np.iinfo(keys.dtype).max, dtype=keys.dtype)
    x[:n] = keys
    for kind, hi, r, _ in plan:
        up = lt if kind == KIND_SORT else (hi + r if kind == KIND_RUNSK else hi + 1)
        x = np.sort(x.reshape(-1, 1 << up), axis=1).reshape(-1)
    return x[:n]


def widths(L, cap=4):
    """plan_uncached's multi-way pass widths for L levels (fewest passes of
    <= cap levels, the larger ones first; one level alone is a 2-way pass)."""
    if L < 2:
        return []
    np_ = -(-L // cap)
    return [L // np_ + (1 if i < L % np_ else 0) for i in range(np_)]


def expected_tile_u32(k):
    """sort_tile_u32 (bitonic.h): the 2^14 merge-level tile except for tiny
    sorts and, below 2^25, where only its plan has a 16-way pass."""
    if k <= 15:
        return 15
    if k >= 25:
        return 14
    has16 = lambda lt: 4 in widths(min(k, 30) - lt)
    return 15 if has16(14) and not has16(15) else 14


SIZES = [1, 2, 31, 1000, (1 << 13) + 1, (1 << 15) - 3, 1 << 15, (1 << 15) + 1, 1 << 16, 100003, 1 << 18,
         (1 << 20) - 7, 1 << 23, 1 << 24, 1 << 28, (1 << 29) - 3, 1 << 30, 1 << 31]


@pytest.mark.parametrize("key_bytes", [4, 8])
@pytest.mark.parametrize("n", SIZES)
def test_plan_covers_the_levels(n, key_bytes):
    assert misort.tile_log2(key_bytes) == (15 if key_bytes == 4 else 13)  # the largest tile
    p = misort.plan(n, key_bytes)
    assert p[0][0] == KIND_SORT
    lt = p[0][1] + 1
    k = ceil_log2(n)
    assert lt == (expected_tile_u32(k) if key_bytes == 4 else 13)
    assert merge_levels(p) == list(range(lt, k))
    lwk_max = 30 if key_bytes == 4 else 29  # 32-bit row offsets of a multi-way group
    for kind, hi, r, _ in p[1:]:
        if kind == KIND_RUNSK:
            assert 1 <= r <= 4 and hi >= lt and hi + r <= lwk_max


def test_plan_pass_counts():
    # 2^30 u32: 2^14-key SORT tiles + four 16-way passes (levels 15..30; one
    # 2-way merge pass per level would be 1 + 16)
    p30 = misort.plan(1 << 30, 4)
    assert tuple(p30[0][:2]) == (KIND_SORT, 13)
    assert [tuple(q[:3]) for q in p30[1:]] == [(KIND_RUNSK, 14, 4), (KIND_RUNSK, 18, 4), (KIND_RUNSK, 22, 4),
                                                (KIND_RUNSK, 26, 4)]
    # the fewest passes of at most four levels (16-way) at every size
    # (profiles/r04/mw: faster than 8-way passes from 2^26 to 2^31); the
    # 2^14 tile (profiles/r04/tile: 2^27 takes four passes on it and is 4 %
    # faster than three on 2^15 tiles)
    assert [q[2] for q in misort.plan(1 << 28, 4)[1:]] == [4, 4, 3, 3]
    assert [q[2] for q in misort.plan(1 << 29, 4)[1:]] == [4, 4, 4, 3]
    assert [q[1] for q in misort.plan(1 << 27, 4)] == [13, 14, 18, 21, 24]
    assert [q[2] for q in misort.plan(1 << 25, 4)[1:]] == [4, 4, 3]
    assert [q[2] for q in misort.plan(1 << 26, 4)[1:]] == [4, 4, 4]
    # 2^24: 2^15 tiles (3,3,3): the 2^14 tile's plan (4,3,3) has a 16-way pass
    assert misort.plan(1 << 24, 4)[0][1] == 14 and [q[2] for q in misort.plan(1 << 24, 4)[1:]] == [3, 3, 3]
    # 2^31: a multi-way pass may end at 2^30 at most (32-bit row offsets); one 2-way pass after
    assert [q[0] for q in misort.plan(1 << 31, 4)] == [KIND_SORT] + [KIND_RUNSK] * 4 + [KIND_RUNS]
    # small u32 sorts take the merge passes too (round 3: they beat the bitonic
    # network's ROWS/SPAN/MERGE passes at every size, profiles/r03/small_u32)
    assert [q[0] for q in misort.plan(1 << 23, 4)] == [KIND_SORT] + [KIND_RUNSK] * 3  # 2^14 tiles: 3 x 8-way
    assert [q[0] for q in misort.plan(1 << 24, 4)] == [KIND_SORT] + [KIND_RUNSK] * 3  # 2^24: 3 x 8-way (9 levels)
    assert [q[0] for q in misort.plan(1 << 16, 4)] == [KIND_SORT, KIND_RUNSK]  # 2^14 tiles, one 4-way pass
    assert [q[0] for q in misort.plan(1 << 15, 4)] == [KIND_SORT]  # one tile
    assert [q[0] for q in misort.plan(1 << 18, 4)] == [KIND_SORT, KIND_RUNSK]  # 2^15 tiles, one 8-way pass
    # u64: 2^13-key SORT tiles, then 16 levels in four 16-way passes
    # (128-bit fences; 2-way passes would be 1 + 16)
    p29 = misort.plan((1 << 29) - 3, 8)
    assert p29[0][0] == KIND_SORT and [q[0] for q in p29[1:]] == [KIND_RUNSK] * 4
    assert [q[2] for q in p29[1:]] == [4, 4, 4, 4]
    assert [q[2] for q in misort.plan(1 << 26, 8)[1:]] == [4, 3, 3, 3]
    # a u64 multi-way pass ends at 2^29 at most (32-bit row offsets of 8-byte keys)
    assert [q[0] for q in misort.plan(1 << 30, 8)] == [KIND_SORT] + [KIND_RUNSK] * 4 + [KIND_RUNS]
    assert [q[0] for q in misort.plan(1 << 14, 8)] == [KIND_SORT, KIND_RUNS]  # one level: 2-way


@pytest.mark.parametrize("key_bytes", [4, 8])
@pytest.mark.parametrize("n", [1000, (1 << 15) + 1, 1 << 16, 100003, (1 << 18) - 5, 1 << 19, (1 << 21) + 3])
def test_plan_replay_sorts(n, key_bytes):
    dt = np.uint32 if key_bytes == 4 else np.uint64
    rng = np.random.default_rng(n)
    keys = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt, endpoint=True)
    keys[::7] = keys[3]  # duplicates
    got = replay(keys, misort.plan(n, key_bytes))
    np.testing.assert_array_equal(got, np.sort(keys))


PLAN_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import misort
print(json.dumps({f"{n}_{kb}": misort.plan(n, kb) for n in map(int, sys.argv[2].split(",")) for kb in (4, 8)}))
"""


@pytest.mark.parametrize("mw", ["0", "2", "3", "4"])
def test_pass_width_knobs(mw):
    """MISORT_MULTIWAY / MISORT_MULTIWAY_U64 (read once per process: a child
    process per value) cap the levels per multi-way pass; 0: 2-way passes only."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sizes = [(1 << 20) + 3, 1 << 24, 1 << 30]
    r = subprocess.run([sys.executable, "-c", PLAN_CHILD, os.path.join(root, "parallel-computing-mpi_amd"),
                        ",".join(map(str, sizes))], env=dict(os.environ, MISORT_MULTIWAY=mw, MISORT_MULTIWAY_U64=mw),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plans = json.loads(r.stdout.strip().splitlines()[-1])
    for n in sizes:
        for kb in (4, 8):
            p = plans[f"{n}_{kb}"]
            assert p[0][0] == KIND_SORT
            assert merge_levels(p) == list(range(p[0][1] + 1, ceil_log2(n)))
            widths = [q[2] for q in p[1:] if q[0] == KIND_RUNSK]
            if int(mw) < 2:
                assert not widths
            else:
                assert widths and max(widths) <= int(mw)


@pytest.mark.parametrize("tile", ["14", "15"])
def test_sort_tile_knob(tile):
    """MISORT_SORT_TILE_U32 pins the u32 SORT tile at every size."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sizes = [(1 << 14) + 1, (1 << 18) + 3, 1 << 24, 1 << 27, 1 << 30]
    r = subprocess.run([sys.executable, "-c", PLAN_CHILD, os.path.join(root, "parallel-computing-mpi_amd"),
                        ",".join(map(str, sizes))], env=dict(os.environ, MISORT_SORT_TILE_U32=tile),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plans = json.loads(r.stdout.strip().splitlines()[-1])
    for n in sizes:
        p = plans[f"{n}_4"]
        assert p[0][1] + 1 == int(tile)
        assert merge_levels(p) == list(range(int(tile), ceil_log2(n)))
        assert plans[f"{n}_8"][0][1] == 12
