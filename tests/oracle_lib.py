"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of /root/reference/Parallel-Sorting/src/psort.cc
(see oracle/oracle.c).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
REF_BIN = os.path.join(ORACLE_DIR, "_ref", "psort_ref")
MPIRUN = "/opt/conda/bin/mpirun"

U32, U64, F64 = 0, 1, 2
NP_DTYPE = {U32: np.uint32, U64: np.uint64, F64: np.float64}

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.environ.get("ORACLE_LIBRARY") or os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)
        L = ctypes.CDLL(path)
        i64, vp = ctypes.c_int64, ctypes.c_void_p
        L.orc_block_sizes.argtypes = [i64, ctypes.c_int, vp]
        L.orc_generate_f64.argtypes = [i64, i64, i64, vp]
        L.orc_splitmix_u32.argtypes = [ctypes.c_uint64, i64, i64, vp]
        L.orc_splitmix_u64.argtypes = [ctypes.c_uint64, i64, i64, vp]
        L.orc_u64mix.argtypes = [ctypes.c_uint64, i64, i64, i64, ctypes.c_uint64, vp]
        L.orc_sort.argtypes = [ctypes.c_int, vp, i64]
        L.orc_compare_split.argtypes = [ctypes.c_int, vp, i64, vp, i64, vp, ctypes.c_int]
        L.orc_parallel_bitonic_sort.argtypes = [ctypes.c_int, vp, i64, ctypes.c_int]
        L.orc_parallel_bitonic_sort.restype = ctypes.c_int
        L.orc_bitonic_schedule.argtypes = [ctypes.c_int, ctypes.c_int, vp, vp]
        L.orc_bitonic_schedule.restype = ctypes.c_int
        L.orc_parallel_quick_sort.argtypes = [ctypes.c_int, vp, i64, ctypes.c_int, vp, vp]
        L.orc_parallel_quick_sort.restype = ctypes.c_int
        L.orc_check_sort.argtypes = [ctypes.c_int, vp, i64, ctypes.c_int]
        L.orc_check_sort.restype = ctypes.c_int64
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def dtype_code(arr):
    return {np.dtype(np.uint32): U32, np.dtype(np.uint64): U64,
            np.dtype(np.float64): F64}[arr.dtype]


def block_sizes(n, p):
    out = np.zeros(p, dtype=np.int64)
    lib().orc_block_sizes(n, p, _ptr(out))
    return out


def generate_f64(n, g0=0, cnt=None):
    cnt = n - g0 if cnt is None else cnt
    out = np.empty(cnt, dtype=np.float64)
    lib().orc_generate_f64(n, g0, cnt, _ptr(out))
    return out


def splitmix(seed, n, dtype=np.uint32, g0=0):
    out = np.empty(n, dtype=dtype)
    if np.dtype(dtype) == np.uint32:
        lib().orc_splitmix_u32(seed, g0, n, _ptr(out))
    else:
        lib().orc_splitmix_u64(seed, g0, n, _ptr(out))
    return out


ALL_ONES = 0xFFFFFFFFFFFFFFFF
REF_TOP = 0x7FF0000000000000  # largest u64 the reference carries as an ordered double


def u64mix(seed, n, top=ALL_ONES, g0=0, cnt=None):
    """BASELINE config-5 mix (oracle.h orc_u64mix), keys [g0, g0+cnt) of n."""
    cnt = n - g0 if cnt is None else cnt
    out = np.empty(cnt, dtype=np.uint64)
    lib().orc_u64mix(seed, n, g0, cnt, top, _ptr(out))
    return out


def local_sort(keys):
    keys = np.ascontiguousarray(keys).copy()
    lib().orc_sort(dtype_code(keys), _ptr(keys), keys.size)
    return keys


def compare_split(local, recv, keep_max):
    out = np.empty_like(local)
    lib().orc_compare_split(dtype_code(local), _ptr(local), local.size, _ptr(recv),
                            recv.size, _ptr(out), int(keep_max))
    return out


def parallel_bitonic_sort(keys, p):
    """All P ranks of psort.cc:167-201 on one host array (rank blocks in order)."""
    keys = np.ascontiguousarray(keys).copy()
    rc = lib().orc_parallel_bitonic_sort(dtype_code(keys), _ptr(keys), keys.size, p)
    if rc != 0:
        raise ValueError("bitonic sort requires 2^d processors")
    return keys


def parallel_quick_sort(keys, p):
    """All P ranks of psort.cc:377-490: (rank-ordered output, per-rank sizes)."""
    keys = np.ascontiguousarray(keys)
    out = np.empty_like(keys)
    sizes = np.zeros(p, dtype=np.int64)
    rc = lib().orc_parallel_quick_sort(dtype_code(keys), _ptr(keys), keys.size, p, _ptr(out), _ptr(sizes))
    if rc != 0:
        raise ValueError("Quick sort requires 2^d processors")
    return out, sizes


def schedule(p, rank):
    partner = np.zeros(64, dtype=np.int32)
    keep = np.zeros(64, dtype=np.int32)
    s = lib().orc_bitonic_schedule(p, rank, _ptr(partner), _ptr(keep))
    return list(zip(partner[:s].tolist(), keep[:s].tolist()))


def check_sort(keys, p):
    keys = np.ascontiguousarray(keys)
    return int(lib().orc_check_sort(dtype_code(keys), _ptr(keys), keys.size, p))
