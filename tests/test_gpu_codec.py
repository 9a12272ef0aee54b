"""The exchange codec (codec.hip) on its own: a sorted run encoded (width,
scans, pack) and decoded must give back the run, and the coded size must be
the stream format's: 4 header words per 1024-key block plus each block's gaps
packed at the width of its largest gap.  The reference ships
uncoded blocks (psort.cc:121-122,146-147); the codec is this framework's own,
so the expected sizes come from the format, computed here with numpy."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
import misort  # noqa: E402

pytestmark = pytest.mark.gpu

CB = 1024  # keys per block (codec.hip)


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = misort.Context(0)
    yield c
    c.close()


def coded_bytes(x):
    """4 * (4 words per block + the payload words at each block's width)."""
    words = 0
    for k0 in range(0, x.size, CB):
        blk = x[k0:k0 + CB].astype(np.uint64)
        g = np.diff(blk)
        w = int(g.max()).bit_length() if g.size else 0
        words += 4 + ((blk.size - 1) * w + 31) // 32
    return 4 * words


def sorted_run(kind, n, dt, seed):
    rng = np.random.default_rng(seed)
    info = np.iinfo(dt)
    if kind == "uniform":
        x = rng.integers(0, info.max, size=n, dtype=dt, endpoint=True)
    elif kind == "dups":
        x = (rng.integers(0, 1 << 20, size=n, dtype=np.uint64) & np.uint64(7)).astype(dt)
    elif kind == "wide":  # full-width gaps: 0 and MAX sentinels among spread keys
        x = rng.integers(0, info.max, size=n, dtype=dt, endpoint=True)
        x[: n // 3] = 0
        x[-(n // 3):] = info.max
    else:  # "equal": width 0 everywhere, headers only
        x = np.full(n, 12345, dtype=dt)
    return np.sort(x)


@pytest.mark.parametrize("dt", [np.uint32, np.uint64])
@pytest.mark.parametrize("n", [1, 2, 1023, 1024, 1025, 3 * CB + 17, 65 * CB + 1, (1 << 20) + 7])
@pytest.mark.parametrize("kind", ["uniform", "dups", "wide", "equal"])
def test_codec_roundtrip_and_size(ctx, dt, n, kind):
    x = sorted_run(kind, n, dt, n * 7 + (dt == np.uint64))
    iv = torch.int32 if dt == np.uint32 else torch.int64
    d = torch.from_numpy(x.view(np.int32 if dt == np.uint32 else np.int64)).cuda()
    out = torch.empty_like(d)
    _, _, nbytes = ctx.codec_probe(d, out, reps=2)
    y = out.view(iv).cpu().numpy().view(dt)
    np.testing.assert_array_equal(y, x)
    assert nbytes == coded_bytes(x)


@pytest.mark.parametrize("dt", [np.uint32, np.uint64])
def test_codec_many_blocks(ctx, dt):
    """2^24 + 5 keys: 16385 blocks, 17 chunks of the payload-offset scan;
    repeated encodes into the same buffers."""
    n = (1 << 24) + 5
    kt = torch.int32 if dt == np.uint32 else torch.int64
    full = torch.empty(n, dtype=kt, device="cuda")
    ctx.fill_splitmix(full, 0xC0DEC)
    run = torch.empty_like(full)
    ctx.local_sort(full, run)
    dec = torch.empty_like(run)
    _, _, nbytes = ctx.codec_probe(run, dec, reps=3)
    assert torch.equal(run, dec)
    x = run.cpu().numpy().view(dt)
    assert nbytes == coded_bytes(x)
