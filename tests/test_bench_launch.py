"""bench.py's launcher (CPU only): `--gpus N` without a torchrun environment
must start N ranks through torch.distributed.run as a child process, before
anything touches a GPU, and pass every argument through."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_needs_launch_only_without_world_size():
    b = load_bench()
    a = b.parse_args(["--gpus", "8"])
    assert b.needs_launch(a, env={})
    assert not b.needs_launch(a, env={"WORLD_SIZE": "8"})
    assert not b.needs_launch(b.parse_args([]), env={})
    assert not b.needs_launch(b.parse_args(["--gpus", "1"]), env={})


def test_launch_command_shape():
    b = load_bench()
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    cmd = b.launch_command(argv, 4, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv


def test_main_relaunches_without_touching_the_gpu(monkeypatch):
    b = load_bench()
    calls = []

    def fake_call(cmd, env=None):
        calls.append((cmd, env))
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b.subprocess, "call", fake_call)
    monkeypatch.setattr(b, "cpu_baseline", lambda *a: {"value": 0.1, "kind": "reference", "cores": 16})
    # if main went past the launcher it would build contexts: make that fatal
    import misort
    monkeypatch.setattr(misort, "Context", lambda *a, **k: (_ for _ in ()).throw(AssertionError("GPU touched")))
    rc = b.main(["--gpus", "8", "--steps", "2"])
    assert rc == 7
    (cmd, env), = calls
    assert "--nproc-per-node=8" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "2"]
    assert env["MASTER_ADDR"] == "127.0.0.1"
    # the host-core baseline was measured by the parent and handed over
    # (the file is removed once the ranks have finished)
    assert b.CPU_JSON_ENV in env and not os.path.exists(env[b.CPU_JSON_ENV])


def test_parent_cpu_baseline_reaches_rank0(monkeypatch, tmp_path):
    """The N > 1 line carries the host-core baseline: the parent measures it
    (no HIP call: misort.Context is fatal here) and rank 0 loads it."""
    b = load_bench()
    seen = {}

    def fake_call(cmd, env=None):
        seen["cpu"] = b.load_cpu_json(env[b.CPU_JSON_ENV])
        return 0

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b.subprocess, "call", fake_call)
    monkeypatch.setattr(b, "cpu_baseline", lambda *a: {"value": 0.12, "kind": "reference", "cores": 16})
    import misort
    monkeypatch.setattr(misort, "Context", lambda *a, **k: (_ for _ in ()).throw(AssertionError("GPU touched")))
    assert b.main(["--gpus", "4"]) == 0
    assert seen["cpu"]["value"] == 0.12 and seen["cpu"]["kind"] == "reference"
    assert "launcher parent" in seen["cpu"]["measured_by"]
    assert b.load_cpu_json(None) is None and b.load_cpu_json(str(tmp_path / "missing.json")) is None


def test_cpu_share_and_pow2():
    b = load_bench()
    n, why = b.cpu_share()
    assert n >= 1 and "sched_getaffinity" in why
    assert [b.pow2_floor(v) for v in (1, 2, 3, 8, 15, 16, 63, 64)] == [1, 2, 2, 8, 8, 16, 32, 64]
