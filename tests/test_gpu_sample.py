"""Sample sort (psort.cc:203-375 redesigned: regular samples, (key, rank,
position) splitters, one all-to-all-v, merge tree, rebalance to the reference
block layout) on the GPU, P ranks as threads of one process (misort.Group).

The reference's sample sorts are not well defined (uninitialised splitter at
psort.cc:318, MPI_INT for doubles at :224/:269), so parity is anchored on the
sorted sequence: the output must equal the reference's bitonic output wherever
that one is globally sorted (golden cases with 0 errors), and the oracle's
sort of the input in the reference block layout everywhere."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O

torch = pytest.importorskip("torch")
import misort  # noqa: E402

pytestmark = pytest.mark.gpu

GOLD_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
with open(os.path.join(GOLD_DIR, "golden.json")) as f:
    GOLD = json.load(f)["cases"]
CLEAN = [c for c in GOLD if c.get("algo", "bitonic") == "bitonic" and c["errors"] == 0 and c["p"] > 1]

U32_T = torch.uint32 if hasattr(torch, "uint32") else torch.int32
U64_T = torch.uint64 if hasattr(torch, "uint64") else torch.int64


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def to_dev(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        return torch.from_numpy(a.view(np.int32)).cuda().view(U32_T)
    if a.dtype == np.uint64:
        return torch.from_numpy(a.view(np.int64)).cuda().view(U64_T)
    return torch.from_numpy(a).cuda()


def to_host(t, dtype):
    if dtype == np.uint32:
        return t.view(torch.int32).cpu().numpy().view(np.uint32)
    if dtype == np.uint64:
        return t.view(torch.int64).cpu().numpy().view(np.uint64)
    return t.cpu().numpy()


def group_sample(x, p):
    sizes = misort.block_sizes(x.size, p)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    mx = x.size // p + 1
    blocks = [np.ascontiguousarray(x[offs[r]:offs[r + 1]]) for r in range(p)]

    def rank_fn(r, ctx):
        buf = to_dev(np.concatenate([blocks[r], np.zeros(mx - sizes[r], x.dtype)]))
        out = torch.empty_like(buf)
        torch.cuda.synchronize()
        ctx.parallel_sample_sort(buf, sizes[r], mx, out=out, stream=ctx.native_stream)
        ctx.synchronize()
        np.testing.assert_array_equal(to_host(buf[:sizes[r]], x.dtype), blocks[r])
        errs = ctx.check_sort(out, sizes[r], stream=ctx.native_stream)
        return to_host(out[:sizes[r]], x.dtype), errs

    g = misort.Group(p)
    try:
        res = g.run(rank_fn)
    finally:
        g.close()
    return np.concatenate([r[0] for r in res]), [r[1] for r in res]


def _golden_input(case):
    if case["mode"] == "psort":
        return O.generate_f64(case["n"])
    if case["dtype"] == "u32":
        return O.splitmix(0x5EED0001, case["n"], np.uint32)
    return np.fromfile(os.path.join(GOLD_DIR, f"keys_{case['name']}.in"), dtype=np.uint64)


@pytest.mark.parametrize("case", CLEAN, ids=lambda c: f"{c['mode']}_{c.get('name', '')}N{c['n']}_P{c['p']}")
def test_sample_sort_equals_reference_bitonic(case):
    y, errs = group_sample(_golden_input(case), case["p"])
    assert sha(y) == case["out_sha256"]
    assert errs == [0] * case["p"]


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("kind", ["u32", "u64", "f64", "dups", "constant", "sorted", "reversed", "tiny"])
def test_sample_sort_matches_oracle(p, kind):
    rng = np.random.default_rng(11)
    n = 200003
    x = {"u32": lambda: O.splitmix(0x5EED0003, n, np.uint32),
         "u64": lambda: O.splitmix(0x5EED0004, n, np.uint64),
         "f64": lambda: O.generate_f64(n),
         "dups": lambda: rng.integers(0, 5, n).astype(np.uint32),
         "constant": lambda: np.full(n, 0xFFFFFFFF, dtype=np.uint32),
         "sorted": lambda: np.arange(n, dtype=np.uint64),
         "reversed": lambda: np.arange(n, 0, -1).astype(np.uint32),
         "tiny": lambda: np.array([5, 3, 9], dtype=np.uint32)}[kind]()
    y, errs = group_sample(x, p)
    np.testing.assert_array_equal(y, O.local_sort(x))  # globally sorted, reference layout
    assert sum(errs) == 0 or x.size < p


def test_sample_sort_rejects_in_place():
    g = misort.Group(2)
    try:
        def fn(r, ctx):
            b = to_dev(np.arange(10, dtype=np.uint32))
            with pytest.raises(misort.MisortError):
                ctx.parallel_sample_sort(b, 10, 10, out=b)
            return True
        assert g.run(fn) == [True, True]
    finally:
        g.close()
