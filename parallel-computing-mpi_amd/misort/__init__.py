"""misort -- MI355X-native bitonic sort (Python host mirror of the C-ABI).

Mirrors the reference's sorter interface, /root/reference/Parallel-Sorting/src/
psort.cc:

* ``parallel_bitonic_sort(buffer, loc_buf_size, max_size)``   (psort.cc:167)
* ``compare_split(local, recv, keep_max)``                    (psort.cc:116-164)
* ``check_sort(local_numbers, local_size)``                   (psort.cc:497-520)
* ``block_sizes(n, p)``                                       (psort.cc:556-562)

with MPI ranks replaced by GPUs (one process per GPU, RCCL over xGMI) and the
keys held in HBM as torch tensors.  Every call goes through libmisort.so
(hand-written gfx950 HIP kernels); there is no CPU fallback: a missing
extension raises ``NativeLibraryMissing``.
"""
import ctypes
import os

__all__ = [
    "U32", "U64", "F64", "MisortError", "NotPowerOfTwo", "NativeLibraryMissing",
    "library_path", "lib", "Context", "Group", "block_sizes", "schedule", "tile_log2", "plan",
    "sample_indices", "exchange_count", "set_shared_gpu_env",
]

U32, U64, F64 = 0, 1, 2
KIND_NAMES = ["tile_sort", "global_pass", "tile_merge", "merge_split", "other", "span_pass",
              "wide_pass", "run_merge", "exchange", "run_mergek", "run_mergek_kernel", "merge_split_tail"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("MISORT_LIBRARY") or os.path.join(os.path.dirname(_HERE), "lib", "libmisort.so")
_lib = None


class MisortError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"misort error {code}: {msg}")
        self.code = code


class NotPowerOfTwo(MisortError):
    """psort.cc:168-172: 'bitonic sort requires 2^d processors'."""


class NativeLibraryMissing(RuntimeError):
    pass


def library_path():
    return _LIB_PATH


def lib():
    """Load libmisort.so (built in-tree by parallel-computing-mpi_amd/csrc/Makefile)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        raise NativeLibraryMissing(
            f"{_LIB_PATH} not built; run `make -C parallel-computing-mpi_amd/csrc` "
            "(or __graft_entry__.build())")
    L = ctypes.CDLL(_LIB_PATH)
    vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
    sig = {
        "misort_version": ([], i32),
        "misort_last_error": ([], ctypes.c_char_p),
        "misort_create": ([i32, ctypes.POINTER(vp)], i32),
        "misort_destroy": ([vp], i32),
        "misort_stream": ([vp], vp),
        "misort_synchronize": ([vp], i32),
        "misort_get_unique_id": ([vp], i32),
        "misort_comm_init": ([vp, i32, i32, vp], i32),
        "misort_comm_size": ([vp], i32),
        "misort_comm_rank": ([vp], i32),
        "misort_bitonic_schedule": ([i32, i32, vp, vp], i32),
        "misort_block_size": ([i64, i32, i32], i64),
        "misort_parallel_bitonic_sort": ([vp, i32, vp, i64, i64, vp], i32),
        "misort_parallel_bitonic_sort_oop": ([vp, i32, vp, vp, i64, i64, vp], i32),
        "misort_local_sort": ([vp, i32, vp, vp, i64, vp], i32),
        "misort_merge_split": ([vp, i32, vp, i64, vp, i64, vp, i32, vp], i32),
        "misort_merge_split_tail": ([vp, i32, vp, i64, vp, i64, i32, vp], i32),
        "misort_parallel_quick_sort": ([vp, i32, vp, i64, vp, i64, ctypes.POINTER(i64), vp], i32),
        "misort_parallel_sample_sort": ([vp, i32, vp, vp, i64, i64, vp], i32),
        "misort_check_sort": ([vp, i32, vp, i64, ctypes.POINTER(i64), vp], i32),
        "misort_sort_host": ([vp, i32, vp, vp, i64, i64], i32),
        "misort_fill_splitmix": ([vp, i32, vp, i64, ctypes.c_uint64, i64, vp], i32),
        "misort_profile_enable": ([vp, i32], i32),
        "misort_profile_reset": ([vp], i32),
        "misort_profile_read": ([vp, i32, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_double)], i32),
        "misort_tile_log2": ([i32], i32),
        "misort_profile_trace": ([vp, i32, ctypes.POINTER(i32), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double)], i32),
        "misort_profile_stage": ([vp, i32, ctypes.POINTER(i64), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)], i32),
        "misort_plan": ([ctypes.c_int64, i32, ctypes.POINTER(i32), i32], i32),
        "misort_pass_probe": ([vp, i32, vp, vp, i64, i32, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_float)], i32),
        "misort_group_create": ([i32, ctypes.POINTER(vp)], i32),
        "misort_group_destroy": ([vp], i32),
        "misort_comm_init_group": ([vp, vp, i32], i32),
        "misort_set_full_exchange": ([vp, i32], i32),
        "misort_set_relay": ([vp, i32], i32),
        "misort_set_compress": ([vp, i32], i32),
        "misort_codec_probe": ([vp, i32, vp, i64, i32, ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_float), ctypes.POINTER(i64), vp], i32),
        "misort_exchange_raw_bytes": ([vp, ctypes.POINTER(i64)], i32),
        "misort_sample_stride": ([i64], i64),
        "misort_sample_count": ([i64], i64),
        "misort_exchange_count": ([i32, vp, i64, vp, i64], i64),
        "misort_exchange_stats": ([vp, ctypes.POINTER(i64), ctypes.POINTER(i64),
                                   ctypes.POINTER(i64)], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _check(rc):
    if rc < 0:
        msg = lib().misort_last_error().decode()
        if rc == -2:
            raise NotPowerOfTwo(rc, msg)
        raise MisortError(rc, msg)
    return rc


def block_sizes(n, p):
    """psort.cc:556-562 block layout."""
    return [int(lib().misort_block_size(n, p, r)) for r in range(p)]


def schedule(p, rank):
    """psort.cc:182-196: [(partner, keep_max)] per stage for `rank`."""
    partner = (ctypes.c_int * 64)()
    keep = (ctypes.c_int * 64)()
    s = _check(lib().misort_bitonic_schedule(p, rank, partner, keep))
    return [(partner[i], keep[i]) for i in range(s)]


def sample_indices(n):
    """Indices of the splitter samples of a sorted n-key block."""
    import numpy as np
    if n <= 0:
        return np.zeros(0, dtype=np.int64)
    S, C = int(lib().misort_sample_stride(n)), int(lib().misort_sample_count(n))
    return np.minimum(np.arange(C, dtype=np.int64) * S, n - 1)


def exchange_count(samples_min, n_min, samples_max, n_max):
    """k keys each side sends in a compare-split (-1 = whole blocks)."""
    import numpy as np
    a, b = np.ascontiguousarray(samples_min), np.ascontiguousarray(samples_max)
    dt = U32 if a.dtype == np.uint32 else U64
    return int(lib().misort_exchange_count(dt, a.ctypes.data_as(ctypes.c_void_p), n_min,
                                           b.ctypes.data_as(ctypes.c_void_p), n_max))


def set_shared_gpu_env(rank):
    """RCCL environment for ranks that share one GPU (see Context.comm_init_torch);
    call before the first RCCL call of the process."""
    os.environ["NCCL_HOSTID"] = f"misort-shared-gpu-rank{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")


def tile_log2(key_bytes):
    return int(lib().misort_tile_log2(key_bytes))


def plan(n, key_bytes=4):
    """The HBM pass plan of a local sort of n keys: [(kind_name, hi, R, flip)]."""
    np_ = lib().misort_plan(n, key_bytes, None, 0)
    _check(np_ if np_ < 0 else 0)
    buf = (ctypes.c_int32 * (4 * max(np_, 1)))()
    lib().misort_plan(n, key_bytes, buf, np_)
    return [(KIND_NAMES[buf[4 * i]], buf[4 * i + 1], buf[4 * i + 2], bool(buf[4 * i + 3]))
            for i in range(np_)]


class Group:
    """In-process rank group: P ranks = P threads, one Context each (the
    exchange is a device-to-device copy; same schedule and merge-split as RCCL)."""

    def __init__(self, nranks):
        self._h = ctypes.c_void_p()
        _check(lib().misort_group_create(nranks, ctypes.byref(self._h)))
        self.nranks = nranks

    def close(self):
        if self._h:
            lib().misort_group_destroy(self._h)
            self._h = ctypes.c_void_p()

    def run(self, fn, devices=None):
        """Run fn(rank, ctx) on one thread per rank; returns the results."""
        import threading
        res, err = [None] * self.nranks, []
        ctxs = [Context((devices or [0])[r % len(devices or [0])]) for r in range(self.nranks)]
        for r, c in enumerate(ctxs):
            _check(lib().misort_comm_init_group(c._h, self._h, r))

        def body(r):
            try:
                import torch
                torch.cuda.set_device(ctxs[r].device)
                res[r] = fn(r, ctxs[r])
            except BaseException as e:  # noqa: BLE001 -- re-raised below
                err.append(e)

        th = [threading.Thread(target=body, args=(r,)) for r in range(self.nranks)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for c in ctxs:
            c.close()
        if err:
            raise err[0]
        return res


def _dtype_of(t):
    import torch
    m = {torch.int32: U32, torch.int64: U64, torch.float64: F64}
    if hasattr(torch, "uint32"):
        m[torch.uint32] = U32
    if hasattr(torch, "uint64"):
        m[torch.uint64] = U64
    if t.dtype not in m:
        raise TypeError(f"unsupported key dtype {t.dtype} (u32/u64/f64 keys)")
    return m[t.dtype]


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class Context:
    """One GPU (HIP device) = one reference MPI rank.

    ``dtype`` of a tensor selects the key type: uint32/int32 storage = u32 keys,
    uint64/int64 storage = u64 keys (compared unsigned), float64 = f64 keys.
    """

    def __init__(self, device=0):
        self._h = ctypes.c_void_p()
        _check(lib().misort_create(device, ctypes.byref(self._h)))
        self.device = device

    def close(self):
        if self._h:
            lib().misort_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream):
        if stream is None:
            import torch
            return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        return ctypes.c_void_p(stream)

    # ---- communicator (MPI_COMM_WORLD -> RCCL) ---------------------------------
    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(128)
        _check(lib().misort_get_unique_id(buf))
        return buf.raw

    def comm_init(self, nranks, rank, uid):
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        _check(lib().misort_comm_init(self._h, nranks, rank, buf))

    def comm_init_torch(self, group=None, share_gpu=None):
        """Create the RCCL communicator; the id travels over torch.distributed.

        share_gpu (default: env MISORT_SHARE_GPU=1): several ranks drive ONE
        GPU.  RCCL refuses two ranks on one device within a host, so each rank
        then presents its own host id (NCCL_HOSTID) and the ranks talk over
        RCCL's socket transport on loopback: the RCCL calls, schedule and
        merge-split are the production ones, the bandwidth is not xGMI's (a
        correctness mode for 1-GPU boxes, never a performance figure)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        if share_gpu is None:
            share_gpu = os.environ.get("MISORT_SHARE_GPU", "0") == "1"
        if share_gpu and world > 1:
            set_shared_gpu_env(rank)
        obj = [self.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        self.comm_init(world, rank, obj[0])

    @property
    def numprocs(self):
        return int(lib().misort_comm_size(self._h))

    @property
    def myid(self):
        return int(lib().misort_comm_rank(self._h))

    # ---- hot path ---------------------------------------------------------------
    def parallel_bitonic_sort(self, buffer, loc_buf_size=None, max_size=None, out=None,
                              stream=None):
        """psort.cc:167.  Sorts this rank's block `buffer[:loc_buf_size]` with the
        reference's hypercube schedule; returns the tensor holding the result
        (``buffer`` itself, or ``out`` when given: input left unchanged)."""
        loc = buffer.numel() if loc_buf_size is None else int(loc_buf_size)
        mx = 0 if max_size is None else int(max_size)  # 0: the largest block (collective)
        dt = _dtype_of(buffer)
        if out is None:
            _check(lib().misort_parallel_bitonic_sort(self._h, dt, _ptr(buffer), loc, mx,
                                                      self._stream(stream)))
            return buffer
        _check(lib().misort_parallel_bitonic_sort_oop(self._h, dt, _ptr(buffer), _ptr(out), loc,
                                                      mx, self._stream(stream)))
        return out

    def parallel_quick_sort(self, buffer, loc_buf_size=None, out=None, stream=None):
        """psort.cc:377 (the reference binary's shipped sort).  Returns
        ``(out, n)``: this rank's sorted keys are ``out[:n]``, n data-dependent.
        ``out`` defaults to the reference's capacity, (loc+1)*P keys."""
        import torch
        loc = buffer.numel() if loc_buf_size is None else int(loc_buf_size)
        if out is None:
            out = torch.empty((loc + 1) * self.numprocs, dtype=buffer.dtype, device=buffer.device)
        n = ctypes.c_int64()
        _check(lib().misort_parallel_quick_sort(self._h, _dtype_of(buffer), _ptr(buffer), loc, _ptr(out),
                                                out.numel(), ctypes.byref(n), self._stream(stream)))
        return out, int(n.value)

    def parallel_sample_sort(self, buffer, loc_buf_size=None, max_size=None, out=None, stream=None):
        """psort.cc:203-375 redesigned (RCCL all-to-all).  Same contract as
        parallel_bitonic_sort: the globally sorted keys in the reference block
        layout, out of place (``out`` defaults to a new tensor)."""
        import torch
        loc = buffer.numel() if loc_buf_size is None else int(loc_buf_size)
        mx = 0 if max_size is None else int(max_size)
        out = torch.empty_like(buffer) if out is None else out
        _check(lib().misort_parallel_sample_sort(self._h, _dtype_of(buffer), _ptr(buffer), _ptr(out), loc, mx,
                                                 self._stream(stream)))
        return out

    def local_sort(self, inp, out=None, n=None, stream=None):
        """psort.cc:175 (std::sort of the local block) on the GPU."""
        out = inp if out is None else out
        n = inp.numel() if n is None else int(n)
        _check(lib().misort_local_sort(self._h, _dtype_of(inp), _ptr(inp), _ptr(out), n,
                                       self._stream(stream)))
        return out

    def compare_split(self, local, recv, keep_max, out=None, stream=None, in_place_tail=False):
        """Device half of psort.cc:116-164 (no exchange).  in_place_tail: the
        small-bracket path of the hypercube stages (misort_merge_split_tail) on a
        copy of `local` in `out`."""
        import torch
        out = torch.empty_like(local) if out is None else out
        if in_place_tail:
            if out.data_ptr() != local.data_ptr():
                out[:local.numel()].copy_(local)
            _check(lib().misort_merge_split_tail(self._h, _dtype_of(local), _ptr(out), local.numel(),
                                                 _ptr(recv), recv.numel(), int(keep_max), self._stream(stream)))
            return out
        _check(lib().misort_merge_split(self._h, _dtype_of(local), _ptr(local), local.numel(),
                                        _ptr(recv), recv.numel(), _ptr(out), int(keep_max),
                                        self._stream(stream)))
        return out

    def check_sort(self, local_numbers, local_size=None, stream=None):
        """psort.cc:497-520: total error count over the communicator."""
        n = local_numbers.numel() if local_size is None else int(local_size)
        err = ctypes.c_int64()
        _check(lib().misort_check_sort(self._h, _dtype_of(local_numbers), _ptr(local_numbers), n,
                                       ctypes.byref(err), self._stream(stream)))
        return int(err.value)

    def sort_host(self, arr, max_size=None, out=None):
        """numpy block -> pinned staging ring -> GPU parallel sort -> numpy
        (chunked and overlapped; `out` may be a preallocated array)."""
        import numpy as np
        arr = np.ascontiguousarray(arr)
        dt = {np.dtype(np.uint32): U32, np.dtype(np.uint64): U64,
              np.dtype(np.float64): F64}[arr.dtype]
        if out is None:
            out = np.empty_like(arr)
        elif out.dtype != arr.dtype or out.size < arr.size or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous array of the input dtype and size")
        mx = 0 if max_size is None else int(max_size)
        _check(lib().misort_sort_host(self._h, dt, arr.ctypes.data_as(ctypes.c_void_p),
                                      out.ctypes.data_as(ctypes.c_void_p), arr.size, mx))
        return out

    def fill_splitmix(self, out, seed, g0=0, stream=None):
        _check(lib().misort_fill_splitmix(self._h, _dtype_of(out), _ptr(out), out.numel(), seed, g0,
                                          self._stream(stream)))
        return out

    def synchronize(self):
        _check(lib().misort_synchronize(self._h))

    @property
    def native_stream(self):
        """The context's own hipStream_t (int), for stream=..."""
        return int(lib().misort_stream(self._h) or 0)

    def set_full_exchange(self, on=True):
        _check(lib().misort_set_full_exchange(self._h, int(on)))

    def set_relay(self, on=True):
        """Spread compare-split exchanges over every xGMI link (P > 2)."""
        _check(lib().misort_set_relay(self._h, int(on)))

    def set_compress(self, on=True):
        """Delta-code compare-split messages (lossless; default on)."""
        _check(lib().misort_set_compress(self._h, int(on)))

    def codec_probe(self, keys, decoded=None, reps=3):
        """Exchange codec on a sorted device run: (encode ms, decode ms, coded bytes)."""
        a, b, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_int64()
        _check(lib().misort_codec_probe(self._h, _dtype_of(keys), _ptr(keys), keys.numel(), reps,
                                        ctypes.byref(a), ctypes.byref(b), ctypes.byref(n),
                                        _ptr(decoded) if decoded is not None else None))
        return a.value, b.value, int(n.value)

    def exchange_raw_bytes(self):
        """Bytes the exchanges since the last call would have moved uncoded; resets."""
        v = ctypes.c_int64()
        _check(lib().misort_exchange_raw_bytes(self._h, ctypes.byref(v)))
        return int(v.value)

    def exchange_stats(self):
        """(stages, bytes moved, bytes a whole-block exchange would move); resets."""
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _check(lib().misort_exchange_stats(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return int(a.value), int(b.value), int(c.value)

    # ---- profiling ----------------------------------------------------------------
    def profile(self, on=True):
        _check(lib().misort_profile_enable(self._h, int(on)))

    def profile_reset(self):
        _check(lib().misort_profile_reset(self._h))

    def pass_probe(self, inp, out, kind, hi, r, flip, reps=5, n=None):
        """Average ms of one HBM pass of a plan shape (tile_sort, run_merge or run_mergek)."""
        ms = ctypes.c_float()
        k = KIND_NAMES.index(kind) if isinstance(kind, str) else int(kind)
        _check(lib().misort_pass_probe(self._h, _dtype_of(inp), _ptr(inp), _ptr(out),
                                       inp.numel() if n is None else n, k, hi, r, int(flip), reps,
                                       ctypes.byref(ms)))
        return ms.value

    def profile_stages(self, nstages):
        """Per hypercube stage: [(sorts, exchange_ms, merge_ms, exchange_bytes)]."""
        res = []
        for st in range(nstages):
            n, xm, mm, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
            _check(lib().misort_profile_stage(self._h, st, ctypes.byref(n), ctypes.byref(xm),
                                              ctypes.byref(mm), ctypes.byref(b)))
            res.append((int(n.value), float(xm.value), float(mm.value), float(b.value)))
        return res

    def profile_trace(self):
        """[(kind_name, ms, algorithmic_bytes)] of every profiled record since the
        last reset, in completion order (a pass after the kernel nested in it)."""
        n = _check(lib().misort_profile_trace(self._h, 0, None, None, None))
        k = (ctypes.c_int32 * max(n, 1))()
        ms = (ctypes.c_double * max(n, 1))()
        b = (ctypes.c_double * max(n, 1))()
        _check(lib().misort_profile_trace(self._h, n, k, ms, b))
        return [(KIND_NAMES[k[i]], ms[i], b[i]) for i in range(n)]

    def profile_read(self):
        """{kind: (launches, total_ms, algorithmic_bytes)}."""
        res = {}
        for k, name in enumerate(KIND_NAMES):
            n, ms, b = ctypes.c_int64(), ctypes.c_double(), ctypes.c_double()
            _check(lib().misort_profile_read(self._h, k, ctypes.byref(n), ctypes.byref(ms),
                                             ctypes.byref(b)))
            res[name] = (int(n.value), float(ms.value), float(b.value))
        return res
