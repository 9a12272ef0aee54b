"""Multi-process (world_size 2 and 4) CPU test of the N>1 host logic, over gloo.

Each process is one rank of psort.cc:167-201.  The ranks run the compare-split
protocol of the GPU build: the schedule and block layout come from
libmisort's C-ABI (misort_bitonic_schedule, misort_block_size), the splitter
samples and the exchange size k from misort_sample_count/stride and
misort_exchange_count (the same host functions the device path calls), and the
bytes travel over torch.distributed send/recv (gloo) where the GPU build uses
RCCL.  The local sort and keep-min/max merge are the oracle's, so the test
isolates the protocol: the result must equal the reference's whole-block
MPI_Sendrecv algorithm (oracle, pinned to golden fixtures) bit for bit."""
import json
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import oracle_lib as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ord(a):
    """Order-preserving u64 view of f64 keys (as the device path uses)."""
    b = a.view(np.uint64)
    return np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))


def _t(a):
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        return torch.from_numpy(a.view(np.int32).copy())
    return torch.from_numpy(a.view(np.int64).copy())


def _np(t, dtype):
    return t.numpy().view(dtype)


def _sendrecv(send, nrecv, dtype, peer):
    rbuf = torch.empty(nrecv, dtype=torch.int32 if np.dtype(dtype).itemsize == 4 else torch.int64)
    reqs = []
    if send.size:
        reqs.append(dist.isend(_t(send), peer))
    if nrecv:
        reqs.append(dist.irecv(rbuf, peer))
    for r in reqs:
        r.wait()
    return _np(rbuf, dtype)


def _make_input(kind, n):
    if kind == "u32":
        return O.splitmix(0xD157 + n, n, np.uint32)
    if kind == "f64":
        return O.generate_f64(n)
    rng = np.random.default_rng(n)
    x = rng.integers(0, 4096, size=n, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
    x[: n // 10] = 0
    x[n // 10: n // 5] = np.uint64(2**64 - 1)
    rng.shuffle(x)
    return x


def _worker(rank, world, port, kind, n, full, outdir):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "parallel-computing-mpi_amd"))
    sys.path.insert(0, HERE)
    import misort
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = _make_input(kind, n)
    sizes = misort.block_sizes(n, world)
    off = sum(sizes[:rank])
    block = O.local_sort(x[off:off + sizes[rank]])  # psort.cc:175
    dt = block.dtype
    stats = []
    for q, keep in misort.schedule(world, rank):  # psort.cc:184-194
        nq = sizes[q]
        me_s = block[misort.sample_indices(block.size)]
        pe_s = _sendrecv(me_s, int(len(misort.sample_indices(nq))), dt, q)
        if dt == np.float64:
            me_s, pe_s = _ord(me_s), _ord(pe_s)
        if full:
            k = -1
        elif keep:  # this rank is the keep-max side ("B")
            k = misort.exchange_count(pe_s, nq, me_s, block.size)
        else:
            k = misort.exchange_count(me_s, block.size, pe_s, nq)
        stats.append(k)
        if k == 0:
            continue
        if k < 0:
            recv = _sendrecv(block, nq, dt, q)
        else:
            send = block[:k] if keep else block[block.size - k:]
            recv = _sendrecv(send, k, dt, q)
        block = O.compare_split(block, recv, keep)  # psort.cc:116-164
    np.save(os.path.join(outdir, f"block_{rank}.npy"), block)
    with open(os.path.join(outdir, f"stats_{rank}.json"), "w") as f:
        json.dump(stats, f)
    dist.barrier()
    dist.destroy_process_group()


CASES = [("u32", 100003, 2), ("u32", 100003, 4), ("f64", 1000005, 4), ("u64", 65541, 2),
         ("u64", 65541, 4), ("u32", 7, 4)]


@pytest.mark.parametrize("full", [False, True])
@pytest.mark.parametrize("kind,n,world", CASES)
def test_protocol_over_gloo(tmp_path, kind, n, world, full):
    mp.spawn(_worker, args=(world, _free_port(), kind, n, full, str(tmp_path)), nprocs=world, join=True)
    y = np.concatenate([np.load(tmp_path / f"block_{r}.npy", allow_pickle=False) for r in range(world)])
    want = O.parallel_bitonic_sort(_make_input(kind, n), world)
    np.testing.assert_array_equal(y.view(np.uint8), want.view(np.uint8))
    ks = [json.load(open(tmp_path / f"stats_{r}.json")) for r in range(world)]
    # partners agree on k at every stage (the exchange sizes match on both sides)
    import misort
    for r in range(world):
        for st, (q, _) in enumerate(misort.schedule(world, r)):
            assert ks[r][st] == ks[q][st]
