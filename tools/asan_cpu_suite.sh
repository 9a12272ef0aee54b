#!/bin/bash
# The CPU suite (pytest -m "not gpu") against host-sanitized builds of
# libmisort (ASan + UBSan on its host code: schedule, block sizes, exchange
# count, planner, profiler, transports' host logic) and of the C oracle.
# CPU only (no GPU, no device sanitizer).  Usage: tools/asan_cpu_suite.sh [pytest args]
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$R/parallel-computing-mpi_amd/csrc" asan -j8
make -s -C "$R/oracle" asan
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$R"
LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
MISORT_LIBRARY="$R/build/asan/libmisort.so" ORACLE_LIBRARY="$R/build/asan/liboracle.so" \
  python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
