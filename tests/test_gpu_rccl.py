"""The real RCCL transport (RcclTransport, runtime.cpp) at P = 2, 4, 8 on one GPU.

tests/rccl_worker.py runs as P processes under torch.distributed.run, each with
its own misort context and RCCL communicator.  RCCL refuses two ranks of one
host on one device, so every rank presents its own NCCL_HOSTID and RCCL joins
them through its socket transport on loopback: ncclSend/ncclRecv in groups
(compare-split, relay), ncclAllGather (sizes, samples) and the all-to-all-v of
the sample sort all execute; only the wire differs from xGMI.  Outputs are
compared with the compiled reference's golden fixtures on rank 0.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(400)
@pytest.mark.parametrize("p", [2, 4, 8])
def test_rccl_ranks_on_one_gpu(p):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", NCCL_SOCKET_IFNAME="lo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={p}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.join(HERE, "rccl_worker.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=360, env=env)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["world"] == p
    bad = [c for c in res["results"] if not c["ok"]]
    assert not bad, bad
    assert len(res["results"]) >= 10
