"""GPU parity of the merge levels (runs.hip) -- the passes that finish the
local sort replacing the reference's std::sort (psort.cc:175) once runs leave
the SORT tile: 2-way levels (runs.hip) and 2^lk-way passes of lk levels each
(runsk.hip, lk = 1..4).

* One merge level (misort_pass_probe, kind run_merge) on inputs made of
  ascending runs of 2^hi keys, ragged tails included, is compared bit for bit
  with numpy: each pair of runs sorted.
* Full local sorts (SORT tile, then merge passes) under the pass-width knobs
  MISORT_MULTIWAY / MISORT_MULTIWAY_U64 and the merge tile knobs MISORT_RUN_IT
  / MISORT_RUN_NT / MISORT_RUN_FUSE, MISORT_PLAN_FUSE and MISORT_PLAN_SCAN run in child processes (the planner knobs are read once per
  process) against np.sort."""
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import misort  # noqa: E402

pytestmark = pytest.mark.gpu

U32_T = torch.uint32 if hasattr(torch, "uint32") else torch.int32
U64_T = torch.uint64 if hasattr(torch, "uint64") else torch.int64
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = misort.Context(0)
    yield c
    c.close()


def runs_input(n, hi, dt, seed, dup=False):
    rng = np.random.default_rng(seed)
    top = 64 if dup else np.iinfo(dt).max
    x = rng.integers(0, top, size=n, dtype=dt, endpoint=not dup)
    if not dup:
        x[::11] = np.iinfo(dt).max  # all-ones keys (the padding value) inside the data
        x[5::13] = 0
    w = 1 << hi
    for s in range(0, n, w):
        x[s:s + w].sort()
    return x


def expect(x, hi):
    out = x.copy()
    w2 = 2 << hi
    for s in range(0, x.size, w2):
        out[s:s + w2].sort()
    return out


def expectk(x, hi, lk):
    out = x.copy()
    wk = 1 << (hi + lk)
    for s in range(0, x.size, wk):
        out[s:s + wk].sort()
    return out


def run_level(ctx, x, hi, kind="run_merge", lk=0):
    if x.dtype == np.uint32:
        d_in = torch.from_numpy(x.view(np.int32)).cuda().view(U32_T)
    else:
        d_in = torch.from_numpy(x.view(np.int64)).cuda().view(U64_T)
    d_out = torch.empty_like(d_in)
    ctx.pass_probe(d_in, d_out, kind, hi, lk, False, reps=1)
    torch.cuda.synchronize()
    if x.dtype == np.uint32:
        return d_out.view(torch.int32).cpu().numpy().view(np.uint32)
    return d_out.view(torch.int64).cpu().numpy().view(np.uint64)


@pytest.mark.parametrize("dt", [np.uint32, np.uint64])
@pytest.mark.parametrize("hi", [13, 15, 17])
@pytest.mark.parametrize("n", [(1 << 19), (1 << 19) - 4097, (1 << 18) + 3, 5000, 12345])
def test_merge_level_matches_numpy(ctx, dt, hi, n):
    if dt == np.uint32 and hi < 13:
        pytest.skip()
    x = runs_input(n, hi, dt, n + hi)
    np.testing.assert_array_equal(run_level(ctx, x, hi), expect(x, hi))


@pytest.mark.parametrize("dt", [np.uint32, np.uint64])
def test_merge_level_duplicates_and_single_run(ctx, dt):
    # duplicate-heavy pairs, and n < 2^(hi+1) (one pair, ragged B) and n <= 2^hi (copy)
    for n, hi in [(1 << 18, 14), (40000, 15), (30000, 15), (4096, 13)]:
        x = runs_input(n, hi, dt, n, dup=True)
        np.testing.assert_array_equal(run_level(ctx, x, hi), expect(x, hi))


@pytest.mark.parametrize("lk", [1, 2, 3, 4])
@pytest.mark.parametrize("dt,hi", [(np.uint32, 14), (np.uint32, 15), (np.uint32, 16), (np.uint32, 17),
                                   (np.uint64, 13), (np.uint64, 14), (np.uint64, 16)])
@pytest.mark.parametrize("n", [(1 << 20) + 3, (1 << 19), (1 << 19) - 4097, 3 * (1 << 17) + 5, 5000, 12345, 2049])
def test_mergek_level_matches_numpy(ctx, lk, dt, hi, n):
    """One 2^lk-way pass (runsk.hip): groups of 2^lk runs merged, ragged last
    group (1 to 2^lk runs, the last one short), fences gathered from the runs;
    u32 keys with 64-bit fences, u64 keys with 128-bit fences."""
    x = runs_input(n, hi, dt, n + hi + lk)
    np.testing.assert_array_equal(run_level(ctx, x, hi, "run_mergek", lk), expectk(x, hi, lk))


@pytest.mark.parametrize("lk", [1, 2, 3, 4])
@pytest.mark.parametrize("dt,hi", [(np.uint32, 14), (np.uint32, 16), (np.uint32, 21), (np.uint64, 13),
                                   (np.uint64, 16), (np.uint64, 19)])
def test_mergek_level_ties_and_edges(ctx, lk, dt, hi):
    """Duplicate-heavy, all-equal (every fence the same key: chunks cut by
    (run, position)), presorted and interleaved runs; hi = 21 (u32) / 19 (u64)
    merges the fences with lk fence merge levels instead of in LDS.  u64
    cases put distinct high words above equal low words, so a fence that
    compared only 32 bits of the key would cut the chunks wrongly."""
    K = 1 << lk
    n = (K << hi) + ((K - 1) << hi) + 1000  # one full group + a (K-1)-run tail
    top = np.iinfo(dt).max
    cases = [runs_input(n, hi, dt, hi, dup=True), np.full(n, 7, dt), np.arange(n, dtype=dt), np.full(n, top, dt)]
    inter = np.arange(n, dtype=dt)  # run r holds r, r+K, r+2K, ... of its group
    w = 1 << hi
    for g in range(0, n, K * w):
        for r in range(K):
            seg = inter[g + r * w: g + (r + 1) * w]
            seg[:] = np.arange(seg.size, dtype=dt) * K + r
    cases.append(inter)
    if dt == np.uint64:
        cases.append((inter << np.uint64(32)) | np.uint64(5))
        hiw = inter.copy()  # run r: keys r << 32 .. with equal low words: only the high word orders them
        for g in range(0, n, K * w):
            for r in range(K):
                seg = hiw[g + r * w: g + (r + 1) * w]
                seg[:] = (np.arange(seg.size, dtype=np.uint64) // 3 * K + r) << np.uint64(32)
        cases.append(hiw)
    for x in cases:
        np.testing.assert_array_equal(run_level(ctx, x, hi, "run_mergek", lk), expectk(x, hi, lk))


def test_merge_level_rejects_bad_shapes(ctx):
    x = np.arange(1 << 16, dtype=np.uint32)
    for hi in (5, 11):  # runs shorter than the merge tile
        with pytest.raises(misort.MisortError):
            run_level(ctx, x, hi)
    for hi, lk in ((11, 2), (13, 2), (15, 5)):  # multi-way: runs shorter than the 2^14 SORT tile; lk > 4
        with pytest.raises(misort.MisortError):
            run_level(ctx, x, hi, "run_mergek", lk)
    x64 = np.arange(1 << 16, dtype=np.uint64)
    for hi, lk in ((12, 2), (13, 5)):  # u64: runs shorter than the 2^13 SORT tile; lk > 4
        with pytest.raises(misort.MisortError):
            run_level(ctx, x64, hi, "run_mergek", lk)


CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import misort
n, kb = int(sys.argv[2]), int(sys.argv[3])
ctx = misort.Context(0)
plan = misort.plan(n, kb)
rng = np.random.default_rng(n)
dt = np.uint32 if kb == 4 else np.uint64
keys = rng.integers(0, np.iinfo(dt).max, size=n, dtype=dt, endpoint=True)
keys[: n // 5] = keys[n // 7]
keys[n // 3: n // 3 + 999] = np.iinfo(dt).max
if kb == 4:
    T = torch.uint32 if hasattr(torch, "uint32") else torch.int32
    d = torch.from_numpy(keys.view(np.int32)).cuda().view(T)
else:
    T = torch.uint64 if hasattr(torch, "uint64") else torch.int64
    d = torch.from_numpy(keys.view(np.int64)).cuda().view(T)
out = torch.empty_like(d)
ctx.parallel_bitonic_sort(d, n, n, out=out)
ctx.local_sort(d)  # in place (ping-pong through the context's scratch)
ctx.synchronize()  # raises MISORT_E_INTERNAL if a merge pass rejected a chunk
torch.cuda.synchronize()
iv = torch.int32 if kb == 4 else torch.int64
a = out.view(iv).cpu().numpy().view(dt)
b = d.view(iv).cpu().numpy().view(dt)
ref = np.sort(keys)
ok = np.array_equal(a, ref) and np.array_equal(b, ref)
print("TILE", plan[0][1] + 1, "RUNS", sum(1 for p in plan if p[0] == "run_merge") + sum(p[2] for p in plan if p[0] == "run_mergek"),
      "RUNSK", sum(1 for p in plan if p[0] == "run_mergek"), "OK" if ok else "MISMATCH")
ctx.close()
"""


@pytest.mark.parametrize("kb,env,n", [
    (4, {}, (1 << 22) + 4099),
    (4, {}, 1 << 23),
    (4, {"MISORT_RUN_IT": "32"}, (1 << 21) + 77),
    (4, {"MISORT_RUN_NT": "256"}, (1 << 21) + 77),
    (4, {"MISORT_RUN_NT": "1024"}, (1 << 22) + 8191),
    (4, {"MISORT_MULTIWAY": "0"}, (1 << 22) + 4099),
    (4, {"MISORT_MULTIWAY": "2"}, (1 << 22) + 4099),
    (4, {"MISORT_MULTIWAY": "3"}, (1 << 26) + 12345),  # chained 8-way passes, u64 fence merges
    (4, {}, (1 << 27) + 777),  # the default: 2^14 tiles, four 16-way passes
    (4, {}, (1 << 26) + 777),  # 2^14 tiles, 4 + 3 + 3 + 3 levels
    (4, {}, (1 << 23) + 5),  # 2^15 tiles (2^14 ones would need a 16-way pass): three 8-way passes
    (4, {}, (1 << 17) + 9),  # 2^15 tiles, one 8-way pass
    (4, {}, (1 << 25) + 3),  # 2^14 merge-level tiles, 4 + 4 + 4 levels
    (4, {"MISORT_SORT_TILE_U32": "15"}, (1 << 25) + 3),  # 2^15 tiles, 4 + 4 + 3 levels
    (4, {"MISORT_SORT_TILE_U32": "14"}, (1 << 23) + 4099),  # 2^14 tiles at a size that defaults to 2^15
    (4, {"MISORT_SORT_TILE_U32": "14"}, (1 << 14) + 1),  # one level past the 2^14 tile: a 2-way pass
    (4, {"MISORT_SORT_TILE_U32": "14"}, 3 * (1 << 14) - 5),  # a full tile + a partial one
    (4, {"MISORT_SORT_TILE_U32": "14", "MISORT_MULTIWAY": "3"}, (1 << 24) + 12345),
    (4, {}, 3 * (1 << 23) + 5),
    (4, {}, (1 << 17) + 1),  # one level past the tile: a 2-way pass
    (4, {}, (1 << 16) + 3),
    (4, {"MISORT_RUN_FUSE": "0", "MISORT_PLAN_FUSE": "0"}, (1 << 24) + 999),  # k_runs_partition, k_bounds
    (4, {"MISORT_PLAN_FUSE": "2"}, (1 << 26) + 12345),  # bounds inside k_chunk_desc<16>
    (4, {"MISORT_PLAN_SCAN": "0", "MISORT_FENCE_RANK_MAX": "0"}, (1 << 23) + 77),  # fused bounds, k_scan_totals
    # fence ranks and counts in one launch (k_fence_rank; the default for fused
    # passes of <= 2^14 fences per run): off, and forced on larger runs
    (4, {"MISORT_FENCE_RANK_MAX": "0"}, (1 << 24) + 999),
    (4, {"MISORT_FENCE_RANK_MAX": "20", "MISORT_PLAN_FUSE": "2"}, (1 << 26) + 12345),
    (8, {"MISORT_FENCE_RANK_MAX": "20", "MISORT_PLAN_FUSE": "2"}, (1 << 25) + 12345),
    (4, {"MISORT_FC_SLICES_MAX": "0", "MISORT_FENCE_RANK_MAX": "0"}, (1 << 23) + 77),  # coalesced fence counts
    (8, {"MISORT_FC_SLICES_MAX": "0", "MISORT_FENCE_RANK_MAX": "0"}, (1 << 22) + 3),
    (4, {"MISORT_RUN_FUSE": "2", "MISORT_MULTIWAY": "0"}, (1 << 22) + 4099),  # every 2-way level fused
    # fence merges as one nested u64 multi-way pass (the default from 2^21
    # fences, i.e. 2^28 keys): 4 levels, 3 + 3 levels, 8-way passes
    (4, {"MISORT_FENCE_NEST_MIN": "12"}, (1 << 26) + 12345),
    (4, {"MISORT_FENCE_NEST_MIN": "12"}, (1 << 27) + 777),
    (4, {"MISORT_FENCE_NEST_MIN": "12", "MISORT_MULTIWAY": "3"}, (1 << 26) + 12345),
    (4, {"MISORT_FENCE_NEST_MIN": "0"}, (1 << 27) + 777),  # never nested
    # 64-key fences (runsk_fg6.hip; the default from 2^29 u64 keys, forced here for u32)
    (4, {"MISORT_FENCE_FG6_MIN": "20"}, (1 << 26) + 12345),
    (4, {"MISORT_FENCE_FG6_MIN": "20"}, (1 << 27) + 777),
    (4, {"MISORT_FENCE_FG6_MIN": "20", "MISORT_FENCE_NEST_MIN": "12"}, (1 << 26) + 12345),
    (4, {"MISORT_FENCE_FG6_MIN": "20", "MISORT_MULTIWAY": "3"}, (1 << 24) + 12345),
    (8, {"MISORT_FENCE_FG6_MIN_U64": "20"}, (1 << 25) + 12345),
    (8, {"MISORT_FENCE_FG6_MIN_U64": "20"}, (1 << 22) + 3),
    # the capacity split (merge_pass): far more fences per chunk than the
    # defaults, so most chunks exceed CAP and run as two halves
    # (k_split_desc, k_mergek_ovf); u32 16-way, 8-way, 64-key fences, nested
    # fence passes, u64
    (4, {"MISORT_MK_FM_ADD": "80"}, (1 << 26) + 12345),
    (4, {"MISORT_MK_FM_ADD": "84"}, (1 << 27) + 777),
    (4, {"MISORT_MK_FM_ADD": "30", "MISORT_MULTIWAY": "3"}, (1 << 26) + 12345),
    (4, {"MISORT_MK_FM_ADD": "40", "MISORT_FENCE_FG6_MIN": "20"}, (1 << 26) + 12345),
    (4, {"MISORT_MK_FM_ADD": "60", "MISORT_FENCE_NEST_MIN": "12"}, (1 << 27) + 777),
    (4, {"MISORT_MK_FM_ADD": "0"}, (1 << 26) + 777),  # no split: the worst-case chunk bound
    # k_mergek's probe launches (MISORT_MK_PROBE: no-merge / first-level /
    # co-rank-only copies of every pass into a scratch buffer) leave the sort intact
    (4, {"MISORT_MK_PROBE": "1"}, (1 << 26) + 12345),
    # the network SORT tiles one tile per workgroup, and the persistent grid at twice the resident capacity
    (4, {"MISORT_PERSIST": "0"}, (1 << 23) + 5),
    (4, {"MISORT_GRID_MULT": "2"}, (1 << 23) + 5),
    (8, {"MISORT_PERSIST_U64": "0"}, (1 << 21) + 4099),
    (8, {"MISORT_MK_FM_ADD": "40"}, (1 << 25) + 12345),
    (8, {}, (1 << 21) + 4099),
    (8, {"MISORT_RUN_IT": "32"}, (1 << 20) + 5),
    (8, {"MISORT_RUN_NT": "512"}, (1 << 20) + 5),
    (8, {"MISORT_MULTIWAY_U64": "0"}, (1 << 21) + 4099),  # 2-way passes
    (8, {"MISORT_MULTIWAY_U64": "2"}, (1 << 21) + 4099),
    (8, {"MISORT_MULTIWAY_U64": "3"}, (1 << 22) + 3),
    (8, {}, (1 << 25) + 12345),  # chained passes, u128 fence merges
    (8, {"MISORT_RUN_FUSE": "2", "MISORT_MULTIWAY_U64": "0"}, (1 << 21) + 4099),
    (8, {"MISORT_PLAN_FUSE": "0"}, (1 << 22) + 3),
    (8, {"MISORT_PLAN_FUSE": "2"}, (1 << 25) + 12345),
])
def test_full_sort_merge_passes(kb, env, n):
    """The whole local sort (SORT tile, then merge passes) under the planner
    knobs, against np.sort; the plan has the fewest multi-way passes for the
    levels past the tile (u32: 2^14 or 2^15 keys by size, sort_tile_u32;
    u64: 2^13)."""
    r = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "parallel-computing-mpi_amd"), str(n),
                        str(kb)], env=dict(os.environ, **env), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("TILE")][-1]
    _, tile, _, count, _, countk, verdict = line.split()
    assert verdict == "OK", line
    if kb == 4:  # default: the fewest passes of up to 16-way
        cap = int(env["MISORT_MULTIWAY"]) if "MISORT_MULTIWAY" in env else 4
    else:
        cap = int(env.get("MISORT_MULTIWAY_U64", "4"))
    if cap >= 2 and int(count) >= 2:
        assert int(countk) == -(-int(count) // cap)  # the fewest multi-way passes
    else:
        assert int(countk) == 0
    if kb == 8:
        assert int(tile) == 13
    elif "MISORT_SORT_TILE_U32" in env:
        assert int(tile) == int(env["MISORT_SORT_TILE_U32"])
    elif not env:
        assert int(tile) == misort.plan(n, 4)[0][1] + 1  # this process has the default knobs
    else:
        assert int(tile) in (14, 15)
    assert int(count) == max(0, (n - 1).bit_length() - int(tile))
