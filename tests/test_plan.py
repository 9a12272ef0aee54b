"""The HBM pass planner (bitonic.h plan_span / plan_levels) on the CPU.

Every plan misort_plan() returns is replayed stage by stage on a numpy model of
the flip-formulation bitonic network (the network local_sort runs in place of
the reference's std::sort, psort.cc:175).  A plan is right when
  * its stages, concatenated, are exactly the network's stage sequence, and
  * replaying them (with the virtual all-ones padding for non-power-of-two n)
    sorts random keys like np.sort.
No device is touched: misort_plan is host-only."""
import numpy as np
import pytest

import misort

KIND_SORT, KIND_ROWS, KIND_MERGE, KIND_SPAN = "tile_sort", "global_pass", "tile_merge", "span_pass"
KIND_WIDE = "wide_pass"  # ROWS stages in the 2^16-key register tile (u32)
KIND_RUNS = "run_merge"  # one merge level (runs.hip): runs of 2^hi -> 2^(hi+1)
KIND_RUNSK = "run_mergek"  # R merge levels in one pass (runsk.hip): runs of 2^hi -> 2^(hi+R)
MERGES = (KIND_RUNS, KIND_RUNSK)


def merge_levels(runs):
    """Levels (input run log2) the merge passes finish, in order."""
    out = []
    for kind, hi, r, _ in runs:
        out += list(range(hi, hi + r)) if kind == KIND_RUNSK else [hi]
    return out


def ceil_log2(n):
    return max(0, int(n - 1).bit_length())


def network(k, lt):
    """The stage sequence after the SORT pass: (level m, bit b), flip when b = m-1."""
    return [(m, b) for m in range(lt + 1, k + 1) for b in range(m - 1, -1, -1)]


def split_runs(plan):
    """(network passes, merge-level passes): merge levels come last."""
    i = next((j for j, q in enumerate(plan) if q[0] in MERGES), len(plan))
    assert all(q[0] in MERGES for q in plan[i:])
    return plan[:i], plan[i:]


def merge_from(plan, k):
    """First level the merge passes finish (k + 1: none)."""
    _, runs = split_runs(plan)
    return runs[0][1] if runs else k


def plan_stages(plan, lt):
    """Network stages the plan's passes run after the SORT pass, as (level, bit)."""
    out = []
    for kind, hi, r, flip in split_runs(plan)[0][1:]:
        if kind in (KIND_ROWS, KIND_WIDE):
            # a ROWS pass runs bits hi..hi-R+1 of the level whose stages they are;
            # the level is known from the flip (hi = m-1) or from the sequence so far
            m = hi + 1 if flip else out[-1][0]
            out += [(m, b) for b in range(hi, hi - r, -1)]
        elif kind == KIND_MERGE:
            m = out[-1][0] if out else lt + 1
            out += [(m, b) for b in range(lt - 1, -1, -1)]
        elif kind == KIND_SPAN:
            m = hi  # tail of level hi, then the head of level hi + 1
            out += [(m, b) for b in range(lt - r - 1, -1, -1)]
            out += [(m + 1, b) for b in range(m, m - r, -1)]
        else:
            raise AssertionError(kind)
    return out


def stage(x, m, b):
    """One network stage on the padded array x (length 2^k): flip (b = m-1) pairs i
    with i ^ (2^m - 1), a half-cleaner pairs i with i ^ 2^b; min to the lower index."""
    n = x.size
    i = np.arange(n)
    j = i ^ ((1 << m) - 1) if b == m - 1 else i ^ (1 << b)
    lo = i < j
    a, c = x[i[lo]], x[j[lo]]
    x[i[lo]] = np.minimum(a, c)
    x[j[lo]] = np.maximum(a, c)


def replay(keys, plan, lt):
    k = ceil_log2(keys.size)
    x = np.full(1 << k, np.iinfo(keys.dtype).max, dtype=keys.dtype)
    x[: keys.size] = keys
    # SORT pass: levels 1..min(lt, k) inside each 2^lt tile
    for m in range(1, min(lt, k) + 1):
        for b in range(m - 1, -1, -1):
            stage(x, m, b)
    for m, b in plan_stages(plan, lt):
        stage(x, m, b)
    for kind, hi, r, _ in split_runs(plan)[1]:
        # merge pass: every run of 2^hi is sorted, each pair (2-way) or group of
        # 2^r runs (multi-way) is merged
        runs = x.reshape(-1, 1 << hi)
        assert np.all(runs[:, 1:] >= runs[:, :-1])
        up = r if kind == KIND_RUNSK else 1
        x = np.sort(x.reshape(-1, 1 << (hi + up)), axis=1).reshape(-1)
    return x[: keys.size]


SIZES = [1, 2, 31, 1000, (1 << 15) - 3, 1 << 15, (1 << 15) + 1, 1 << 16, 100003, 1 << 18,
         (1 << 20) - 7, 1 << 24, 1 << 28, (1 << 29) - 3, 1 << 30, 1 << 31]


@pytest.mark.parametrize("key_bytes", [4, 8])
@pytest.mark.parametrize("n", SIZES)
def test_plan_covers_network(n, key_bytes):
    lt = misort.tile_log2(key_bytes)
    p = misort.plan(n, key_bytes)
    assert p[0][0] == KIND_SORT
    k = ceil_log2(n)
    m0 = merge_from(p, k)
    assert plan_stages(p, lt) == network(min(k, max(m0, lt)), lt)
    assert merge_levels(split_runs(p)[1]) == list(range(m0, k)) if m0 < k else True
    for kind, hi, r, flip in p[1:]:
        if kind in (KIND_ROWS, KIND_SPAN):
            assert 1 <= r <= lt - 5  # rows keep >= 32 consecutive keys (128 B for u32)
        if kind == KIND_WIDE:
            assert key_bytes == 4 and 4 <= r <= 10 and hi >= 15  # >= 64-key rows of a 2^16 tile


def test_plan_pass_counts():
    # 2^30 u32: 1 SORT + five 8-way passes (levels 16..30, three per pass; one
    # 2-way merge pass per level would be 1 + 15; the network alone needs
    # 1 + 28 with wide ROWS passes, 1 + 29 without)
    p30 = misort.plan(1 << 30, 4)
    assert p30[0][0] == KIND_SORT
    assert [tuple(q[:3]) for q in p30[1:]] == [(KIND_RUNSK, 15 + 3 * i, 3) for i in range(5)]
    # 13 and 14 levels: four passes, one or two of them 16-way (fewer passes win
    # unless the levels split into 8-way passes exactly); 12 levels: four 8-way
    assert [q[2] for q in misort.plan(1 << 28, 4)[1:]] == [4, 3, 3, 3]
    assert [q[2] for q in misort.plan(1 << 29, 4)[1:]] == [4, 4, 3, 3]
    assert [q[2] for q in misort.plan(1 << 27, 4)[1:]] == [3, 3, 3, 3]
    assert [q[2] for q in misort.plan(1 << 25, 4)[1:]] == [4, 3, 3]
    # 2^31: a multi-way pass may end at 2^30 at most (32-bit row offsets); one 2-way pass after
    assert [q[0] for q in misort.plan(1 << 31, 4)] == [KIND_SORT] + [KIND_RUNSK] * 5 + [KIND_RUNS]
    assert len(misort.plan(1 << 23, 4)) == 13  # cache-resident u32 sizes stay on the network
    assert [q[0] for q in misort.plan(1 << 24, 4)] == [KIND_SORT] + [KIND_RUNSK] * 3  # 2^24: 3 x 8-way
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
@pytest.mark.parametrize("n", [(1 << 15) + 1, 1 << 16, 100003, (1 << 18) - 5, 1 << 19])
def test_plan_replay_sorts(n, key_bytes):
    lt = misort.tile_log2(key_bytes)
    dt = np.uint32 if key_bytes == 4 else np.uint64
    rng = np.random.default_rng(n)
    keys = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt, endpoint=True)
    keys[::7] = keys[3]  # duplicates
    got = replay(keys, misort.plan(n, key_bytes), lt)
    np.testing.assert_array_equal(got, np.sort(keys))


WIDE_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
import misort
print(json.dumps({str(n): misort.plan(n, kb) for n in map(int, sys.argv[2].split(",")) for kb in (4,)}))
"""


@pytest.mark.parametrize("wide", ["0", "1"])
def test_plans_with_and_without_wide_passes(wide):
    """Plans under MISORT_WIDE=0/1 (knobs are read once per process: a child
    process) cover the network exactly and sort when replayed."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sizes = [(1 << 16) + 3, 100003, (1 << 18) - 5, 1 << 20, 1 << 24, 1 << 28, 1 << 30, 1 << 31]
    r = subprocess.run([sys.executable, "-c", WIDE_CHILD, os.path.join(root, "parallel-computing-mpi_amd"),
                        ",".join(map(str, sizes))], env=dict(os.environ, MISORT_WIDE=wide, MISORT_MERGE_FROM="0"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plans = {int(k): [tuple(p) for p in v] for k, v in json.loads(r.stdout).items()}
    lt = misort.tile_log2(4)
    n_wide = 0
    for n, p in plans.items():
        assert plan_stages(p, lt) == network(ceil_log2(n), lt)
        n_wide += sum(1 for q in p if q[0] == KIND_WIDE)
        for kind, hi, rr, flip in p:
            if kind == KIND_WIDE:
                assert 4 <= rr <= 10 and hi >= 15
        if n <= 1 << 18:
            rng = np.random.default_rng(n)
            keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
            np.testing.assert_array_equal(replay(keys, p, lt), np.sort(keys))
    if wide == "1":
        assert n_wide > 0 and len(plans[1 << 30]) <= 30
    else:
        assert n_wide == 0


@pytest.mark.parametrize("mfrom", ["0", "15", "19", "23"])
def test_plans_merge_from(mfrom):
    """Network-then-merge plans under MISORT_MERGE_FROM (0: network only, the
    pass counts of the pure network plan): the network part covers the network
    up to the merge level, merge passes cover each remaining level once, and
    small plans replay to a sort."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sizes = [(1 << 16) + 3, 100003, (1 << 18) - 5, 1 << 20, 1 << 24, 1 << 28, 1 << 30]
    r = subprocess.run([sys.executable, "-c", WIDE_CHILD, os.path.join(root, "parallel-computing-mpi_amd"),
                        ",".join(map(str, sizes))], env=dict(os.environ, MISORT_MERGE_FROM=mfrom),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plans = {int(k): [tuple(p) for p in v] for k, v in json.loads(r.stdout).items()}
    lt = misort.tile_log2(4)
    for n, p in plans.items():
        k = ceil_log2(n)
        m0 = merge_from(p, k)
        if mfrom == "0":
            assert m0 == k
        else:
            assert m0 == (int(mfrom) if int(mfrom) < k and k > 23 else k)  # MISORT_MERGE_MIN_LOG2 = 23
        assert plan_stages(p, lt) == network(min(k, m0), lt)
        if n <= 1 << 18:
            rng = np.random.default_rng(n)
            keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
            np.testing.assert_array_equal(replay(keys, p, lt), np.sort(keys))
    if mfrom == "0":
        # the pure network plan: 1 SORT + 28 passes at 2^30 (wide ROWS passes)
        assert len(plans[1 << 30]) == 29 and len(plans[1 << 28]) == 24 and len(plans[1 << 24]) == 15
