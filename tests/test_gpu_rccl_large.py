"""The real RCCL transport (RcclTransport, runtime.cpp) at BASELINE sizes and on
its failure paths, P processes on ONE GPU (RCCL's socket transport on loopback;
tests/rccl_large_worker.py).

* config 4, 2^30 u32 at P = 2 (delta-coded bracketed exchange) and P = 8
  (relayed over every peer), SHA-256-equal to tests/golden/large.json;
* config 4 at P = 2 with MISORT_COMPRESS=0 and whole-block exchange: one
  2 GiB ncclSend/ncclRecv each way, the reference's MPI_Sendrecv of the whole
  block (psort.cc:121-122, 146-147);
* config 5, u64 N = 2^29 - 3 (the reference's defective uneven output, 1 error)
  and 2^29 - 7 at P = 8, with keys the reference can take as doubles ("ref")
  and with BASELINE config 5's own mix ("full": 5 % all-ones keys, which
  collide with the merge passes' MAX sentinels, crossing the real exchange,
  psort.cc:121-122, 146-147);
* failure detection: a peer that stalls or dies after the communicator is up
  makes rank 0 fail with MISORT_E_RCCL within MISORT_TIMEOUT_S instead of
  hanging (the reference's alarm(540) watchdog + abort, psort.cc:17,56-65,170),
  and later calls fail at once; also when the sort was queued on the caller's
  stream and another stream drained before check_sort (the deadline follows
  the stream that holds the transfers).
"""
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MISORT_E_RCCL = -4


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(p, args, timeout, extra_env=None):
    """torchrun P ranks of rccl_large_worker.py in their own process group
    (killed whole on timeout, so no rank outlives the test); the ranks' output
    goes to files (MISORT_TEST_LOGDIR, default a temporary directory)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else None
    spool = tempfile.mkdtemp(prefix="misort_rccl_", dir=base)
    logdir = os.environ.get("MISORT_TEST_LOGDIR") or spool
    os.makedirs(logdir, exist_ok=True)
    tag = "_".join([f"P{p}", *args])
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", NCCL_SOCKET_IFNAME="lo", OMP_NUM_THREADS="2",
               MISORT_TEST_SPOOL=spool, **(extra_env or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={p}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.join(HERE, "rccl_large_worker.py"), *args]
    out_p, err_p = os.path.join(logdir, f"rccl_{tag}.out"), os.path.join(logdir, f"rccl_{tag}.err")
    try:
        with open(out_p, "w") as fo, open(err_p, "w") as fe:
            proc = subprocess.Popen(cmd, stdout=fo, stderr=fe, env=env, start_new_session=True)
            try:
                rc = proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait()
                rc = None
        with open(out_p) as f:
            stdout = f.read()
        with open(err_p) as f:
            stderr = f.read()
    finally:
        shutil.rmtree(spool, ignore_errors=True)
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert rc is not None, ("timed out", stdout[-3000:], stderr[-3000:])
    assert lines, (rc, stdout[-3000:], stderr[-3000:])
    return rc, json.loads(lines[-1])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("p,args", [(2, ["config4"]), (2, ["config4", "raw"]), (8, ["config4"]),
                                    (8, ["config5"]), (8, ["config5full"])],
                         ids=["config4_P2", "config4_P2_raw_whole_block", "config4_P8", "config5_P8",
                              "config5_full_P8"])
def test_rccl_baseline_size(p, args):
    rc, res = launch(p, args, timeout=280)
    assert rc == 0, res
    assert res["world"] == p and res["results"], res
    bad = [c for c in res["results"] if not c["ok"]]
    assert not bad, bad
    if "raw" in args:
        # whole blocks crossed: 2 x 2^29 keys x 4 B sent + received by rank 0
        assert res["results"][0]["rank0_stage_bytes"] == 2 * (1 << 29) * 4
    if args[0].startswith("config5"):
        assert len(res["results"]) == 2


@pytest.mark.timeout(200)
@pytest.mark.parametrize("mode", ["stall", "dead", "dead_user_stream"])
def test_rccl_failed_peer_errors_instead_of_hanging(mode):
    limit = 15
    rc, res = launch(2, [mode], timeout=120, extra_env={"MISORT_TIMEOUT_S": str(limit), "MISORT_TRACE": "1",
                                                       "MISORT_TEST_STALL_S": str(limit + 25)})
    assert res["mode"] == mode
    assert res["code"] == MISORT_E_RCCL, res
    assert res["elapsed_s"] < limit + 10, res
    assert res["second_code"] == MISORT_E_RCCL and res["second_s"] < 1.0, res
