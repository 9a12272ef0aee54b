"""The host logic under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

build/asan/libmisort.so is libmisort with its host code sanitized (the
device code is the production build) and build/asan/liboracle.so the C
restatement, both from `make asan` (parallel-computing-mpi_amd/csrc,
oracle/; __graft_entry__.build() makes them).  This test reruns the host-logic
tests -- the C-ABI exports, the hypercube schedule and block layout, the pass
planner replayed stage by stage, the exchange-count bracket, the multi-way
chunk model and the oracle against the reference's golden vectors -- in a
child process with the sanitizer runtime preloaded, and checks with a
deliberate out-of-bounds read through the C-ABI that the instrumentation is
live.  tools/asan_cpu_suite.sh runs the whole CPU suite the same way.
"""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "build", "asan")
LIBS = [os.path.join(ASAN, "libmisort.so"), os.path.join(ASAN, "liboracle.so")]
RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))

pytestmark = pytest.mark.skipif(not RT or not all(os.path.exists(p) for p in LIBS),
                                reason="sanitized builds missing: make -C parallel-computing-mpi_amd/csrc asan "
                                       "&& make -C oracle asan")


def sanitized_env():
    return dict(os.environ, LD_PRELOAD=RT[-1], ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", MISORT_LIBRARY=LIBS[0],
                ORACLE_LIBRARY=LIBS[1])


@pytest.mark.timeout(900)
def test_host_logic_clean_under_asan_ubsan():
    files = ["test_abi.py", "test_plan.py", "test_exchange_bracket.py", "test_runsk_model.py",
             "test_runs_partition_model.py", "test_oracle_golden.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        *[os.path.join(ROOT, "tests", f) for f in files]],
                       capture_output=True, text=True, env=sanitized_env(), cwd=ROOT, timeout=850)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout and "Sanitizer" not in r.stderr


def test_instrumentation_is_live():
    """Negative control: misort_exchange_count told that a 2-key sample array
    holds the samples of a 2^20-key block reads past it -- ASan must stop it."""
    code = ("import ctypes, numpy as np, sys; sys.path.insert(0, %r); import misort; "
            "a = np.zeros(2, np.uint32); b = np.zeros(2, np.uint32); "
            "misort.exchange_count(a, 1 << 20, b, 1 << 20)" % os.path.join(ROOT, "parallel-computing-mpi_amd"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=sanitized_env(),
                       timeout=120)
    assert r.returncode != 0 and "AddressSanitizer" in r.stderr, (r.returncode, r.stderr[-2000:])
