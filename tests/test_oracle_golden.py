"""Pin the CPU oracle (oracle/oracle.c) against fixtures produced by the
compiled, unmodified reference (tests/golden/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLD_DIR, "golden.json")) as f:
    GOLD = json.load(f)["cases"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


PSORT = [c for c in GOLD if c["mode"] == "psort" and c.get("algo", "bitonic") == "bitonic"]
KEYS = [c for c in GOLD if c["mode"] == "keys" and c.get("algo", "bitonic") == "bitonic"]
QPSORT = [c for c in GOLD if c["mode"] == "psort" and c.get("algo") == "quick"]
QKEYS = [c for c in GOLD if c["mode"] == "keys" and c.get("algo") == "quick"]


@pytest.mark.parametrize("case", PSORT, ids=lambda c: f"N{c['n']}_P{c['p']}")
def test_psort_generator_and_sort(case):
    n, p = case["n"], case["p"]
    x = O.generate_f64(n)  # psort.cc:587-614
    assert sha(x) == case["in_sha256"]
    assert list(O.block_sizes(n, p)) == case["sizes"]  # psort.cc:556-562
    y = O.parallel_bitonic_sort(x, p)  # psort.cc:167-201
    assert sha(y) == case["out_sha256"]
    assert O.check_sort(y, p) == case["errors"]  # psort.cc:497-520
    full = os.path.join(GOLD_DIR, f"psort_out_N{n}_P{p}.f64")
    if os.path.exists(full):
        np.testing.assert_array_equal(np.fromfile(full).view(np.uint64), y.view(np.uint64))


def test_generator_block_offsets_are_p_independent():
    # The reference passes the erand48 state rank to rank (psort.cc:591-614);
    # the restatement addresses any block by its global offset.
    n = 70001
    whole = O.generate_f64(n)
    for g0, cnt in [(0, 5), (65530, 20), (69990, 11)]:
        np.testing.assert_array_equal(O.generate_f64(n, g0, cnt), whole[g0:g0 + cnt])


def _keys_input(case):
    if case["dtype"] == "u32":
        return O.splitmix(0x5EED0001, case["n"], np.uint32)
    return np.fromfile(os.path.join(GOLD_DIR, f"keys_{case['name']}.in"), dtype=np.uint64)


@pytest.mark.parametrize("case", KEYS, ids=lambda c: f"{c['name']}_P{c['p']}")
def test_keys_cases(case):
    x = _keys_input(case)
    assert sha(x) == case["in_sha256"]
    y = O.parallel_bitonic_sort(x, case["p"])
    assert sha(y) == case["out_sha256"]
    assert O.check_sort(y, case["p"]) == case["errors"]


@pytest.mark.parametrize("case", QPSORT, ids=lambda c: f"N{c['n']}_P{c['p']}")
def test_psort_quick_sort(case):
    # psort.cc:377-490 as shipped: per-rank sizes are data-dependent.
    n, p = case["n"], case["p"]
    x = O.generate_f64(n)
    assert sha(x) == case["in_sha256"]
    y, sizes = O.parallel_quick_sort(x, p)
    assert sizes.tolist() == case["sizes"]
    assert sha(y) == case["out_sha256"]
    full = os.path.join(GOLD_DIR, f"psort_quick_out_N{n}_P{p}.f64")
    if os.path.exists(full):
        np.testing.assert_array_equal(np.fromfile(full).view(np.uint64), y.view(np.uint64))


@pytest.mark.parametrize("case", QKEYS, ids=lambda c: f"{c['name']}_P{c['p']}")
def test_keys_quick_cases(case):
    x = _keys_input(case)
    y, sizes = O.parallel_quick_sort(x, case["p"])
    assert sizes.tolist() == case["sizes"]
    assert sha(y) == case["out_sha256"]


def test_non_power_of_two_rejected():
    with pytest.raises(ValueError):
        O.parallel_bitonic_sort(np.arange(10, dtype=np.uint32), 3)
    with pytest.raises(ValueError):
        O.parallel_quick_sort(np.arange(10, dtype=np.uint32), 6)


def test_schedule_matches_reference_loop():
    # psort.cc:184-194: d(d+1)/2 stages, partner myid^2^j.
    for p in (1, 2, 4, 8, 16):
        d = p.bit_length() - 1
        for r in range(p):
            s = O.schedule(p, r)
            assert len(s) == d * (d + 1) // 2
            k = 0
            for i in range(d):
                for j in range(i, -1, -1):
                    ib, jb = (r >> (i + 1)) & 1, (r >> j) & 1
                    assert s[k] == (r ^ (1 << j), int(ib != jb))
                    k += 1


def test_defective_layout_is_reproduced():
    # uneven blocks with P>=4 are not globally sorted by the
    # reference; the fixtures hold nonzero error counts and the oracle matches.
    bad = [c for c in GOLD if c["errors"] > 0]
    assert bad and all(c["p"] >= 4 and c.get("algo", "bitonic") == "bitonic" for c in bad)


def test_large_fixtures_pinned_by_reference():
    """tests/golden/large.json: every reference run recorded by
    make_golden_large.py hashed exactly like the oracle's output."""
    with open(os.path.join(GOLD_DIR, "large.json")) as f:
        cases = json.load(f)["cases"]
    assert {c["config"] for c in cases} == {3, 4, 5}
    for c in cases:
        for pin in c.get("pinned_by_reference", []):
            assert pin["out_sha256"] == c["out_sha256"] and pin["errors"] == c["errors"]
    assert all(c.get("pinned_by_reference") for c in cases if c["dtype"] == "u32" or c["variant"] == "ref")


def test_large_config3_oracle_sha():
    """The oracle reproduces the reference-pinned 2^28 u32 hash (config 3)."""
    with open(os.path.join(GOLD_DIR, "large.json")) as f:
        c = [c for c in json.load(f)["cases"] if c["config"] == 3][0]
    x = O.splitmix(c["seed"], c["n"], np.uint32)
    assert hashlib.sha256(x.tobytes()).hexdigest() == c["in_sha256"]
    y = O.local_sort(x)
    del x
    assert hashlib.sha256(y.tobytes()).hexdigest() == c["out_sha256"]


def test_u64mix_is_split_invariant_and_mixed():
    n = 100003
    x = O.u64mix(0x5EED0005, n)
    parts = np.concatenate([O.u64mix(0x5EED0005, n, g0=g, cnt=min(7777, n - g)) for g in range(0, n, 7777)])
    np.testing.assert_array_equal(x, parts)
    assert 0.03 < np.mean(x == 0) < 0.07 and 0.03 < np.mean(x == np.uint64(O.ALL_ONES)) < 0.07
    r = O.u64mix(0x5EED0005, n, top=O.REF_TOP)
    assert r.max() <= np.uint64(O.REF_TOP)


F64Z = json.load(open(os.path.join(GOLD_DIR, "f64zero.json")))["cases"]


@pytest.mark.parametrize("case", F64Z, ids=lambda c: f"P{c['p']}")
def test_f64_signed_zero_fixtures(case):
    """The oracle on the reference's +-0.0 fixtures (make_golden_f64zero.py):
    equal as doubles at every position, bit-exact wherever the value is not
    zero, the same check_sort count; only the zeros' sign order is the
    reference's implementation-defined one (parity unpinned for those bits)."""
    x = np.fromfile(os.path.join(GOLD_DIR, "f64zero.in"))
    ref = np.fromfile(os.path.join(GOLD_DIR, f"f64zero_P{case['p']}.out"))
    assert sha(ref) == case["out_sha256"]
    y = O.parallel_bitonic_sort(x, case["p"])
    assert np.array_equal(y, ref)
    nz = ref != 0
    np.testing.assert_array_equal(y.view(np.uint64)[nz], ref.view(np.uint64)[nz])
    assert O.check_sort(y, case["p"]) == case["errors"]
    assert int(np.count_nonzero(ref == 0)) == case["zeros"]
