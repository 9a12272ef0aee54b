"""The P-rank path of parallel_bitonic_sort (psort.cc:167-201) on one GPU.

P ranks run as P threads of this process, each with its own misort context
and stream (misort.Group).  Everything the RCCL build does per rank runs here
too -- size all-gather, hypercube schedule, splitter-sample exchange, the
bracketed partial exchange, device merge-split, buffer rotation, check_sort --
except that the byte transfer is a device-to-device copy instead of
ncclSend/ncclRecv (RCCL refuses two ranks on one GPU).  Results are compared
with the golden fixtures of the compiled reference and with the oracle."""
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


def group_sort(x, p, full_exchange=False, out_of_place=False, relay=True, compress=True, raw=None, kinds=None,
               setters=True):
    """Each rank sorts its reference-layout block; returns (concatenated
    result, check_sort count of every rank, exchange stats of every rank).
    raw (a dict) receives each rank's uncoded exchange bytes; kinds (a dict)
    each rank's profiled launches per kernel kind."""
    sizes = misort.block_sizes(x.size, p)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    max_size = x.size // p + 1
    blocks = [np.ascontiguousarray(x[offs[r]:offs[r + 1]]) for r in range(p)]

    def rank_fn(r, ctx):
        if setters:  # else the environment's defaults (MISORT_FULL_EXCHANGE, MISORT_RELAY, MISORT_COMPRESS)
            ctx.set_full_exchange(full_exchange)
            ctx.set_relay(relay)
            ctx.set_compress(compress)
        buf = to_dev(np.concatenate([blocks[r], np.zeros(max_size - sizes[r], x.dtype)]))
        out = torch.empty_like(buf) if out_of_place else None
        torch.cuda.synchronize()
        if kinds is not None:
            ctx.profile(True)
            ctx.profile_reset()
        res = ctx.parallel_bitonic_sort(buf, sizes[r], max_size, out=out, stream=ctx.native_stream)
        ctx.synchronize()
        if kinds is not None:
            kinds[r] = {k: v[0] for k, v in ctx.profile_read().items()}
            ctx.profile(False)
        errs = ctx.check_sort(res, sizes[r], stream=ctx.native_stream)
        if out_of_place:  # input left unchanged
            np.testing.assert_array_equal(to_host(buf[:sizes[r]], x.dtype), blocks[r])
        st = ctx.exchange_stats()
        if raw is not None:
            raw[r] = ctx.exchange_raw_bytes()
        return to_host(res[:sizes[r]], x.dtype), errs, st

    g = misort.Group(p)
    try:
        res = g.run(rank_fn)
    finally:
        g.close()
    y = np.concatenate([r[0] for r in res]) if res else np.empty(0, x.dtype)
    return y, [r[1] for r in res], [r[2] for r in res]


PSORT = [c for c in GOLD if c["mode"] == "psort" and c["p"] > 1 and c.get("algo", "bitonic") == "bitonic"]
KEYS = [c for c in GOLD if c["mode"] == "keys" and c["p"] > 1 and c.get("algo", "bitonic") == "bitonic"]


@pytest.mark.parametrize("case", PSORT, ids=lambda c: f"N{c['n']}_P{c['p']}")
def test_golden_psort_group(case):
    x = O.generate_f64(case["n"])
    y, errs, _ = group_sort(x, case["p"])
    assert sha(y) == case["out_sha256"]
    assert errs == [case["errors"]] * case["p"]


@pytest.mark.parametrize("case", KEYS, ids=lambda c: f"{c['name']}_P{c['p']}")
def test_golden_keys_group(case):
    if case["dtype"] == "u32":
        x = O.splitmix(0x5EED0001, case["n"], np.uint32)
    else:
        x = np.fromfile(os.path.join(GOLD_DIR, f"keys_{case['name']}.in"), dtype=np.uint64)
    y, errs, _ = group_sort(x, case["p"], out_of_place=True)
    assert sha(y) == case["out_sha256"]
    assert errs == [case["errors"]] * case["p"]


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("n", [(1 << 22) + 5, (1 << 20)])
def test_u32_partial_vs_full_exchange(p, n):
    x = O.splitmix(0xABC + n + p, n, np.uint32)
    want = O.parallel_bitonic_sort(x, p)
    y1, e1, st1 = group_sort(x, p)
    y2, e2, st2 = group_sort(x, p, full_exchange=True)
    np.testing.assert_array_equal(y1, want)
    np.testing.assert_array_equal(y2, want)
    assert e1 == e2 == [O.check_sort(want, p)] * p
    moved = sum(s[1] for s in st1)
    assert moved < sum(s[1] for s in st2)  # the bracket saves bytes
    assert sum(s[1] for s in st2) == sum(s[2] for s in st2)


@pytest.mark.parametrize("p", [4, 8])
@pytest.mark.parametrize("full", [False, True])
def test_relayed_exchange_equals_direct(p, full):
    # the xGMI relay (messages cut into P parts, P-2 of them two hops through
    # the other GPUs) delivers the same bytes as the direct pair exchange,
    # including asymmetric whole-block messages (N % P != 0) and k = 0 stages
    x = O.splitmix(0x5EED0009 + p, (1 << 21) + 3, np.uint32)
    y1, e1, st1 = group_sort(x, p, full_exchange=full, relay=True)
    y2, e2, st2 = group_sort(x, p, full_exchange=full, relay=False)
    np.testing.assert_array_equal(y1, y2)
    np.testing.assert_array_equal(y1, O.parallel_bitonic_sort(x, p))
    assert e1 == e2 and st1 == st2


@pytest.mark.parametrize("p", [2, 4, 8])
def test_u64_mixed_uneven_group(p):
    # BASELINE config 5 shape: N % P != 0, duplicates, zeros, all-ones keys.
    rng = np.random.default_rng(p)
    n = (1 << 19) - 3
    alpha = rng.integers(0, 2**63, size=1024, dtype=np.uint64)
    x = np.concatenate([alpha[rng.integers(0, 1024, n // 2)],
                        np.zeros(n // 8, np.uint64), np.full(n // 8, 2**64 - 1, np.uint64)])
    x = np.concatenate([x, rng.integers(0, 2**64 - 1, n - x.size, dtype=np.uint64)])
    rng.shuffle(x)
    y, errs, _ = group_sort(x, p)
    want = O.parallel_bitonic_sort(x, p)
    np.testing.assert_array_equal(y, want)
    assert errs == [O.check_sort(want, p)] * p


@pytest.mark.parametrize("n,p", [(5, 8), (3, 4), (8, 8), (9, 8), (17, 2)])
def test_tiny_and_empty_blocks(n, p):
    x = O.splitmix(n, n, np.uint32)
    y, _, _ = group_sort(x, p)
    np.testing.assert_array_equal(y, O.parallel_bitonic_sort(x, p))


def test_presorted_reversed_and_equal_keys():
    # Sorted input is not a no-op for bitonic: its first stages make every
    # other block descending, so some pairs swap whole blocks (k = n) while
    # others move nothing (k = 0, the stage is skipped on both sides).
    n, p = 1 << 20, 4
    for x in [np.arange(n, dtype=np.uint32), np.arange(n, dtype=np.uint32)[::-1].copy(),
              np.full(n, 42, np.uint32)]:
        y, _, st = group_sort(x, p)
        np.testing.assert_array_equal(y, np.sort(x))
        assert all(s[1] <= s[2] for s in st)


def test_f64_psort_generator_group_p8_large():
    n = (1 << 21) - 3
    x = O.generate_f64(n)
    y, errs, _ = group_sort(x, 8)
    want = O.parallel_bitonic_sort(x, 8)
    np.testing.assert_array_equal(y.view(np.uint64), want.view(np.uint64))
    assert errs == [O.check_sort(want, 8)] * 8


@pytest.mark.parametrize("kind", ["u32", "f64"])
def test_tail_merges_vs_whole_block(monkeypatch, kind):
    """The hypercube stages with the in-place small-bracket compare-split
    (MISORT_TAIL_DIV = 8, the default: k <= loc / 8) and with whole-block
    merges only (0) write the same bytes as the oracle (psort.cc:116-201), for
    u32 and for f64 (the stages merge the ordered form; the last one maps back
    to double bits); the default run takes the tail path at least once."""
    p = 8
    n = (1 << 20) + 5
    x = O.splitmix(0x5EED7A11, n, np.uint32) if kind == "u32" else O.generate_f64(n)
    want = O.parallel_bitonic_sort(x, p)
    w = np.uint64 if kind == "f64" else np.uint32
    for div, tail in (("0", False), ("8", True)):
        monkeypatch.setenv("MISORT_TAIL_DIV", div)
        kinds = {}
        y, errs, _ = group_sort(x, p, kinds=kinds)
        np.testing.assert_array_equal(y.view(w), want.view(w))
        assert errs == [O.check_sort(want, p)] * p
        ntail = sum(k.get("merge_split_tail", 0) for k in kinds.values())
        assert (ntail > 0) == tail, (div, ntail)


def test_exchange_switches_from_environment(monkeypatch):
    """MISORT_FULL_EXCHANGE=1, MISORT_RELAY=0, MISORT_COMPRESS=0 as the
    contexts' defaults: whole blocks each way every stage (the reference's
    MPI_Sendrecv, psort.cc:121-122,146-147), the same bytes as the oracle."""
    monkeypatch.setenv("MISORT_FULL_EXCHANGE", "1")
    monkeypatch.setenv("MISORT_RELAY", "0")
    monkeypatch.setenv("MISORT_COMPRESS", "0")
    n, p = (1 << 18) + 3, 4
    x = O.splitmix(0x5EED0EE1, n, np.uint32)
    y, errs, st = group_sort(x, p, setters=False)
    want = O.parallel_bitonic_sort(x, p)
    np.testing.assert_array_equal(y, want)
    assert all(s[1] == s[2] and s[1] > 0 for s in st), st  # every stage moved whole blocks


def _u64_mix(n, seed):
    rng = np.random.default_rng(seed)
    alpha = rng.integers(0, 2**63, size=1024, dtype=np.uint64)
    x = np.concatenate([alpha[rng.integers(0, 1024, n // 2)],
                        np.zeros(n // 8, np.uint64), np.full(n // 8, 2**64 - 1, np.uint64)])
    x = np.concatenate([x, rng.integers(0, 2**64 - 1, n - x.size, dtype=np.uint64)])
    rng.shuffle(x)
    return x


@pytest.mark.parametrize("p", [2, 4, 8])
@pytest.mark.parametrize("relay", [True, False])
@pytest.mark.parametrize("kind", ["u32", "u64mix", "f64", "u32dup"])
def test_coded_exchange_equals_raw(p, relay, kind):
    """Delta-coded compare-split messages (codec.hip) deliver the same keys as
    raw ones: u32 uniform (coded ~4x smaller), u64 with 64-bit gaps (0 and
    all-ones sentinels: width 64, sent raw or coded), the reference's f64
    generator, and all-duplicate runs (width 0)."""
    n = (1 << 20) + 7
    if kind == "u32":
        x = O.splitmix(0xC0DE + p, n, np.uint32)
    elif kind == "u32dup":
        x = (O.splitmix(0xC0DF + p, n, np.uint32) & np.uint32(7)).astype(np.uint32)
    elif kind == "u64mix":
        x = _u64_mix(n, p)
    else:
        x = O.generate_f64(n)
    raw_c, raw_r = {}, {}
    y1, e1, st1 = group_sort(x, p, relay=relay, compress=True, raw=raw_c)
    y2, e2, st2 = group_sort(x, p, relay=relay, compress=False, raw=raw_r)
    want = O.parallel_bitonic_sort(x, p)
    np.testing.assert_array_equal(y1.view(np.uint8), want.view(np.uint8))
    np.testing.assert_array_equal(y2.view(np.uint8), want.view(np.uint8))
    assert e1 == e2
    assert raw_c == raw_r == {r: s[1] for r, s in enumerate(st2)}  # what the raw run moved
    coded, uncoded = sum(s[1] for s in st1), sum(s[1] for s in st2)
    assert coded <= uncoded
    if kind == "u32":  # 2^19 keys per rank: gaps ~2^13, ~16-bit fields
        assert coded < 0.7 * uncoded
    if kind == "u32dup":  # gaps 0..7: 3-bit fields
        assert coded * 5 < uncoded
