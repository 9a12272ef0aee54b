"""parallel_quick_sort (psort.cc:377-490, the reference binary's shipped sort)
on the GPU: P ranks as threads of one process (misort.Group; the exchange is a
device copy instead of ncclSend/ncclRecv), compared with the golden fixtures
of the compiled reference -- per-rank sizes and bytes -- and with the oracle."""
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
QPSORT = [c for c in GOLD if c["mode"] == "psort" and c.get("algo") == "quick"]
QKEYS = [c for c in GOLD if c["mode"] == "keys" and c.get("algo") == "quick"]

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


def group_quick(x, p):
    sizes = misort.block_sizes(x.size, p)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    blocks = [np.ascontiguousarray(x[offs[r]:offs[r + 1]]) for r in range(p)]

    def rank_fn(r, ctx):
        buf = to_dev(np.concatenate([blocks[r], np.zeros(1, x.dtype)]))
        torch.cuda.synchronize()
        out, n = ctx.parallel_quick_sort(buf, sizes[r], stream=ctx.native_stream)
        ctx.synchronize()
        # the input block is left unchanged
        np.testing.assert_array_equal(to_host(buf[:sizes[r]], x.dtype), blocks[r])
        return to_host(out[:n], x.dtype), n

    g = misort.Group(p)
    try:
        res = g.run(rank_fn)
    finally:
        g.close()
    return np.concatenate([r[0] for r in res]), [r[1] for r in res]


@pytest.mark.parametrize("case", QPSORT, ids=lambda c: f"N{c['n']}_P{c['p']}")
def test_psort_quick_matches_reference(case):
    x = O.generate_f64(case["n"])
    y, sizes = group_quick(x, case["p"])
    assert sizes == case["sizes"]
    assert sha(y) == case["out_sha256"]


@pytest.mark.parametrize("case", QKEYS, ids=lambda c: f"{c['name']}_P{c['p']}")
def test_keys_quick_matches_reference(case):
    if case["dtype"] == "u32":
        x = O.splitmix(0x5EED0001, case["n"], np.uint32)
    else:
        x = np.fromfile(os.path.join(GOLD_DIR, f"keys_{case['name']}.in"), dtype=np.uint64)
    y, sizes = group_quick(x, case["p"])
    assert sizes == case["sizes"]
    assert sha(y) == case["out_sha256"]


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("kind", ["dups", "sorted", "reversed", "constant"])
def test_quick_edge_inputs_match_oracle(p, kind):
    # duplicate-heavy, presorted, reversed and all-equal inputs (pivot ties,
    # lower_bound at 0 / n, ranks that end up empty)
    n = 50011
    rng = np.random.default_rng(7)
    x = {"dups": rng.integers(0, 7, n).astype(np.uint64),
         "sorted": np.arange(n, dtype=np.uint64),
         "reversed": np.arange(n, 0, -1).astype(np.uint64),
         "constant": np.full(n, 5, dtype=np.uint64)}[kind]
    y, sizes = group_quick(x, p)
    want, wsizes = O.parallel_quick_sort(x, p)
    assert sizes == wsizes.tolist()
    np.testing.assert_array_equal(y, want)


def test_quick_single_rank_is_local_sort():
    x = O.splitmix(0x5EED0002, 100003, np.uint32)
    y, sizes = group_quick(x, 1)
    assert sizes == [x.size]
    np.testing.assert_array_equal(y, np.sort(x))


def test_quick_rejects_non_power_of_two():
    g = misort.Group(4)
    try:
        def fn(r, ctx):
            return ctx.numprocs
        assert g.run(fn) == [4] * 4
    finally:
        g.close()
    with pytest.raises(misort.NotPowerOfTwo):
        misort.Group(3)
