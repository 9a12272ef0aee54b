"""The drop-in boundary (include/misort.h) on the CPU: libmisort.so loads without
a GPU and exports every function the header declares, the header's enums agree
with the Python mirror, and the pure host entry points (schedule, block
layout, sample bracket, plan) answer without touching a device."""
import ctypes
import os
import re

import pytest

import misort

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "misort.h")


def header_text():
    with open(HEADER) as f:
        return re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)


def declared_functions():
    # "int misort_x(...);" / "int64_t misort_x(...);" / "void* misort_x(...);" / "const char* ..."
    return sorted(set(re.findall(r"\b(misort_\w+)\s*\(", header_text())))


def test_header_declares_the_hot_path():
    names = declared_functions()
    for fn in ("misort_parallel_bitonic_sort", "misort_parallel_bitonic_sort_oop", "misort_local_sort",
               "misort_merge_split", "misort_check_sort", "misort_comm_init", "misort_sort_host"):
        assert fn in names


def test_library_exports_every_declared_function():
    lib = ctypes.CDLL(misort.library_path())  # loads without a GPU (no HIP call at load)
    missing = [fn for fn in declared_functions() if not hasattr(lib, fn)]
    assert not missing, missing


def test_kind_enum_matches_python_names():
    kinds = {int(v): k for k, v in re.findall(r"\b(MISORT_K_\w+)\s*=\s*(\d+)", header_text())}
    assert sorted(kinds) == list(range(len(kinds)))
    assert len(misort.KIND_NAMES) == len(kinds)


def test_status_codes_are_negative_and_distinct():
    codes = [int(v) for v in re.findall(r"\bMISORT_E_\w+\s*=\s*(-\d+)", header_text())]
    assert codes and all(c < 0 for c in codes) and len(set(codes)) == len(codes)


def test_host_only_entry_points():
    lib = misort.lib()
    assert lib.misort_version() >= 1
    # psort.cc:556-562 block layout and psort.cc:182-196 schedule, no device
    assert misort.block_sizes(1031, 4) == [258, 258, 258, 257]
    # rank 0 of 8: partners 0^2^j for i in 0..2, j = i..0; rank 0 keeps the low half
    assert misort.schedule(8, 0) == [(1, 0), (2, 0), (1, 0), (4, 0), (2, 0), (1, 0)]
    with pytest.raises(misort.MisortError):
        misort.schedule(6, 0)  # psort.cc:168-172: 2^d ranks only
    assert misort.plan(1 << 30, 4)[0][0] == "tile_sort"
