// runtime.cpp -- C-ABI runtime of libmisort.so (include/misort.h).
//
// Host side of the MI355X bitonic sort: device/stream setup, scratch buffers,
// the RCCL communicator that replaces MPI_COMM_WORLD, the hypercube schedule of
// psort.cc:182-196 with RCCL send/recv in place of MPI_Sendrecv
// (psort.cc:121,146), check_sort (psort.cc:497-520), pinned host staging and
// per-launch HIP-event profiling.  No exception crosses the C-ABI.
#include "misort.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) return fail(MISORT_E_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

#define NCCLCHK(x)                                                                            \
    do {                                                                                      \
        ncclResult_t r_ = (x);                                                                \
        if (r_ != ncclSuccess) return fail(MISORT_E_RCCL, "%s: %s", #x, ncclGetErrorString(r_)); \
    } while (0)

// psort.cc:81-86
int ilog2(int v) {
    int d = 0;
    for (v >>= 1; v != 0; v >>= 1) d++;
    return d;
}

size_t key_bytes(int dtype) { return dtype == MISORT_U32 ? 4 : 8; }
bool valid_dtype(int dtype) { return dtype == MISORT_U32 || dtype == MISORT_U64 || dtype == MISORT_F64; }

// HIP-event profiler: one event pair per kernel launch of a sort.
struct Profiler final : misort::LaunchHook {
    struct Rec {
        int kind;
        hipEvent_t a, b;
        double bytes;
    };
    std::vector<hipEvent_t> pool;
    std::vector<Rec> pending;
    int64_t launches[misort::KIND_COUNT] = {};
    double ms[misort::KIND_COUNT] = {};
    double bytes[misort::KIND_COUNT] = {};
    Rec cur{};
    bool on = false;

    hipEvent_t take() {
        if (pool.empty()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    void before(misort::Kind k, double b, hipStream_t s) override {
        cur = Rec{k, take(), take(), b};
        if (cur.a) (void)hipEventRecord(cur.a, s);
    }
    void after(misort::Kind, hipStream_t s) override {
        if (cur.b) (void)hipEventRecord(cur.b, s);
        pending.push_back(cur);
    }
    int collect() {
        for (auto& r : pending) {
            float t = 0.f;
            if (r.a && r.b) {
                HIPCHK(hipEventSynchronize(r.b));
                HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
            }
            launches[r.kind] += 1;
            ms[r.kind] += t;
            bytes[r.kind] += r.bytes;
            if (r.a) pool.push_back(r.a);
            if (r.b) pool.push_back(r.b);
        }
        pending.clear();
        return MISORT_OK;
    }
    void reset() {
        std::fill(std::begin(launches), std::end(launches), 0);
        std::fill(std::begin(ms), std::end(ms), 0.0);
        std::fill(std::begin(bytes), std::end(bytes), 0.0);
    }
    ~Profiler() override {
        for (auto& r : pending) {
            if (r.a) (void)hipEventDestroy(r.a);
            if (r.b) (void)hipEventDestroy(r.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int ensure(size_t want) {
        if (want <= bytes) return MISORT_OK;
        if (p) HIPCHK(hipFree(p));
        p = nullptr;
        bytes = 0;
        HIPCHK(hipMalloc(&p, want));
        bytes = want;
        return MISORT_OK;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct misort_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DevBuf work, recv, scratch, small;
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    Profiler prof;
};

namespace {

hipStream_t pick(misort_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }
misort::LaunchHook* hook(misort_ctx* c) { return c->prof.on ? &c->prof : nullptr; }

int do_local_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t n, bool ord_in,
                  hipStream_t s) {
    hipError_t e;
    if (dtype == MISORT_U32)
        e = misort::local_sort<uint32_t>((const uint32_t*)in, (uint32_t*)out, n, false, s, hook(c));
    else
        e = misort::local_sort<uint64_t>((const uint64_t*)in, (uint64_t*)out, n, ord_in, s, hook(c));
    if (e != hipSuccess) return fail(MISORT_E_HIP, "local_sort: %s", hipGetErrorString(e));
    return MISORT_OK;
}

int do_merge_split(misort_ctx* c, int dtype, const void* a, int64_t na, const void* b, int64_t nb,
                   void* out, int keep_max, hipStream_t s) {
    const int64_t ntiles = (na + 2047) / 2048 + 2;
    int rc = c->scratch.ensure((size_t)ntiles * sizeof(int64_t));
    if (rc) return rc;
    hipError_t e;
    if (dtype == MISORT_U32)
        e = misort::merge_split<uint32_t>((const uint32_t*)a, na, (const uint32_t*)b, nb,
                                          (uint32_t*)out, keep_max, (int64_t*)c->scratch.p, s, hook(c));
    else
        e = misort::merge_split<uint64_t>((const uint64_t*)a, na, (const uint64_t*)b, nb,
                                          (uint64_t*)out, keep_max, (int64_t*)c->scratch.p, s, hook(c));
    if (e != hipSuccess) return fail(MISORT_E_HIP, "merge_split: %s", hipGetErrorString(e));
    return MISORT_OK;
}

// Block sizes of every rank (the reference learns the partner's size from
// MPI_Get_count, psort.cc:125,150; one all-gather up front gives all of them).
int gather_sizes(misort_ctx* c, int64_t loc, std::vector<int64_t>& sizes, hipStream_t s) {
    sizes.assign(c->nranks, 0);
    if (c->nranks == 1) {
        sizes[0] = loc;
        return MISORT_OK;
    }
    int rc = c->small.ensure(sizeof(int64_t) * (c->nranks + 1));
    if (rc) return rc;
    int64_t* d = (int64_t*)c->small.p;
    HIPCHK(hipMemcpyAsync(d + c->nranks, &loc, sizeof(int64_t), hipMemcpyHostToDevice, s));
    NCCLCHK(ncclAllGather(d + c->nranks, d, 1, ncclInt64, c->comm, s));
    HIPCHK(hipMemcpyAsync(sizes.data(), d, sizeof(int64_t) * c->nranks, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MISORT_OK;
}

int parallel_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t loc,
                  int64_t max_size, hipStream_t s) {
    if (!valid_dtype(dtype)) return fail(MISORT_E_INVALID, "bad dtype %d", dtype);
    if (loc < 0 || max_size < loc) return fail(MISORT_E_INVALID, "loc_size %lld > max_size %lld",
                                               (long long)loc, (long long)max_size);
    const int p = c->nranks;
    if (p & (p - 1)) return fail(MISORT_E_NOT_POW2, "bitonic sort requires 2^d processors");
    std::vector<int64_t> sizes;
    int rc = gather_sizes(c, loc, sizes, s);
    if (rc) return rc;
    for (int r = 0; r < p; ++r)
        if (sizes[r] > max_size)
            return fail(MISORT_E_CAPACITY, "rank %d holds %lld keys > max_size %lld", r,
                        (long long)sizes[r], (long long)max_size);
    int partner[64], keep[64];
    const int nst = misort_bitonic_schedule(p, c->rank, partner, keep);
    const size_t w = key_bytes(dtype);
    const bool f64 = dtype == MISORT_F64;
    void* work = nullptr;
    if (nst > 0) {
        int64_t maxp = 0;
        for (int st = 0; st < nst; ++st) maxp = std::max(maxp, sizes[partner[st]]);
        if ((rc = c->work.ensure(std::max<size_t>(1, (size_t)loc * w)))) return rc;
        if ((rc = c->recv.ensure(std::max<size_t>(1, (size_t)maxp * w)))) return rc;
        work = c->work.p;
    }
    // The local sort writes where the stage parity leaves the result in `out`.
    void* cur = (nst & 1) ? work : out;
    if ((rc = do_local_sort(c, dtype, in, cur, loc, f64, s))) return rc;
    void* other = (cur == work) ? out : work;
    const ncclDataType_t nt = w == 4 ? ncclUint32 : ncclUint64;
    for (int st = 0; st < nst; ++st) {
        const int q = partner[st];
        NCCLCHK(ncclGroupStart());
        NCCLCHK(ncclSend(cur, (size_t)loc, nt, q, c->comm, s));
        NCCLCHK(ncclRecv(c->recv.p, (size_t)sizes[q], nt, q, c->comm, s));
        NCCLCHK(ncclGroupEnd());
        if ((rc = do_merge_split(c, dtype, cur, loc, c->recv.p, sizes[q], other, keep[st], s))) return rc;
        std::swap(cur, other);
    }
    if (f64) HIPCHK(misort::ord_to_f64((uint64_t*)out, loc, s));
    return MISORT_OK;
}

}  // namespace

extern "C" {

int misort_version(void) { return MISORT_VERSION; }
const char* misort_last_error(void) { return g_err.c_str(); }

int misort_create(int device, misort_ctx** out) try {
    if (!out) return fail(MISORT_E_INVALID, "null out");
    *out = nullptr;
    HIPCHK(hipSetDevice(device));
    auto* c = new misort_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(MISORT_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    *out = c;
    return MISORT_OK;
} catch (const std::bad_alloc&) {
    return fail(MISORT_E_INVALID, "out of host memory");
}

int misort_destroy(misort_ctx* c) {
    if (!c) return MISORT_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) ncclCommDestroy(c->comm);
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return MISORT_OK;
}

void* misort_stream(misort_ctx* c) { return c ? (void*)c->stream : nullptr; }

int misort_synchronize(misort_ctx* c) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    HIPCHK(hipStreamSynchronize(c->stream));
    return MISORT_OK;
}

int misort_get_unique_id(void* id) {
    if (!id) return fail(MISORT_E_INVALID, "null id");
    static_assert(sizeof(ncclUniqueId) == MISORT_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return MISORT_OK;
}

int misort_comm_init(misort_ctx* c, int nranks, int rank, const void* id) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(MISORT_E_INVALID, "bad communicator arguments");
    if (nranks & (nranks - 1)) return fail(MISORT_E_NOT_POW2, "bitonic sort requires 2^d processors");
    HIPCHK(hipSetDevice(c->device));
    if (c->comm) {
        ncclCommDestroy(c->comm);
        c->comm = nullptr;
    }
    if (nranks > 1) {
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        NCCLCHK(ncclCommInitRank(&c->comm, nranks, u, rank));
    }
    c->nranks = nranks;
    c->rank = rank;
    return MISORT_OK;
}

int misort_comm_size(misort_ctx* c) { return c ? c->nranks : MISORT_E_INVALID; }
int misort_comm_rank(misort_ctx* c) { return c ? c->rank : MISORT_E_INVALID; }

int misort_bitonic_schedule(int p, int rank, int* partner, int* keep_max) {
    if (p < 1 || rank < 0 || rank >= p || !partner || !keep_max)
        return fail(MISORT_E_INVALID, "bad schedule arguments");
    if (p & (p - 1)) return fail(MISORT_E_NOT_POW2, "bitonic sort requires 2^d processors");
    const int d = ilog2(p);
    int s = 0;
    for (int i = 0; i < d; ++i)      // psort.cc:184
        for (int j = i; j >= 0; --j) {  // psort.cc:185
            const int ibit = (rank & (1 << (i + 1))) != 0;  // psort.cc:186
            const int jbit = (rank & (1 << j)) != 0;        // psort.cc:187
            partner[s] = rank ^ (1 << j);                   // psort.cc:188
            keep_max[s] = ibit != jbit;                     // psort.cc:189-194
            ++s;
        }
    return s;
}

int64_t misort_block_size(int64_t n, int p, int rank) {
    if (p < 1 || rank < 0 || rank >= p || n < 0) return MISORT_E_INVALID;
    return n / p + (rank < n % p ? 1 : 0);  // psort.cc:556-562
}

int misort_local_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t n, void* stream) {
    if (!c || !valid_dtype(dtype) || n < 0 || (n > 0 && (!in || !out)))
        return fail(MISORT_E_INVALID, "bad local_sort arguments");
    hipStream_t s = pick(c, stream);
    int rc = do_local_sort(c, dtype, in, out, n, dtype == MISORT_F64, s);
    if (rc) return rc;
    if (dtype == MISORT_F64) HIPCHK(misort::ord_to_f64((uint64_t*)out, n, s));
    return MISORT_OK;
}

int misort_parallel_bitonic_sort_oop(misort_ctx* c, int dtype, const void* in, void* out,
                                     int64_t loc, int64_t max_size, void* stream) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    if (c->nranks > 1 && !c->comm) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    if (loc > 0 && (!in || !out)) return fail(MISORT_E_INVALID, "null buffer");
    return parallel_sort(c, dtype, in, out, loc, max_size, pick(c, stream));
}

int misort_parallel_bitonic_sort(misort_ctx* c, int dtype, void* keys, int64_t loc,
                                 int64_t max_size, void* stream) {
    return misort_parallel_bitonic_sort_oop(c, dtype, keys, keys, loc, max_size, stream);
}

int misort_merge_split(misort_ctx* c, int dtype, const void* local, int64_t nloc, const void* recv,
                       int64_t nrecv, void* out, int keep_max, void* stream) {
    if (!c || !valid_dtype(dtype) || nloc < 0 || nrecv < 0)
        return fail(MISORT_E_INVALID, "bad merge_split arguments");
    hipStream_t s = pick(c, stream);
    if (dtype != MISORT_F64)
        return do_merge_split(c, dtype, local, nloc, recv, nrecv, out, keep_max, s);
    // f64: order-preserving copies of both blocks, merge, map back.
    int rc;
    if ((rc = c->work.ensure(std::max<size_t>(8, (size_t)nloc * 8)))) return rc;
    if ((rc = c->recv.ensure(std::max<size_t>(8, (size_t)nrecv * 8)))) return rc;
    HIPCHK(hipMemcpyAsync(c->work.p, local, (size_t)nloc * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(c->recv.p, recv, (size_t)nrecv * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(misort::f64_to_ord((uint64_t*)c->work.p, nloc, s));
    HIPCHK(misort::f64_to_ord((uint64_t*)c->recv.p, nrecv, s));
    if ((rc = do_merge_split(c, dtype, c->work.p, nloc, c->recv.p, nrecv, out, keep_max, s))) return rc;
    HIPCHK(misort::ord_to_f64((uint64_t*)out, nloc, s));
    return MISORT_OK;
}

int misort_check_sort(misort_ctx* c, int dtype, const void* keys, int64_t n, int64_t* errors,
                      void* stream) {
    if (!c || !valid_dtype(dtype) || n < 0 || !errors) return fail(MISORT_E_INVALID, "bad check args");
    if (c->nranks > 1 && !c->comm) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    hipStream_t s = pick(c, stream);
    const int p = c->nranks;
    // Per rank: {local descents, n, first key bits, last key bits}.
    int rc = c->small.ensure(sizeof(uint64_t) * 4 * (p + 1) + 64);
    if (rc) return rc;
    uint64_t* d = (uint64_t*)c->small.p;
    uint64_t* mine = d + 4 * p;
    HIPCHK(hipMemsetAsync(mine, 0, sizeof(uint64_t) * 4, s));
    hipError_t e = hipSuccess;
    if (dtype == MISORT_U32) e = misort::count_descents<uint32_t>((const uint32_t*)keys, n, (unsigned long long*)mine, s);
    else if (dtype == MISORT_U64) e = misort::count_descents<uint64_t>((const uint64_t*)keys, n, (unsigned long long*)mine, s);
    else e = misort::count_descents<double>((const double*)keys, n, (unsigned long long*)mine, s);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "count_descents: %s", hipGetErrorString(e));
    const uint64_t nn = (uint64_t)n;
    HIPCHK(hipMemcpyAsync(mine + 1, &nn, 8, hipMemcpyHostToDevice, s));
    const size_t w = key_bytes(dtype);
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(mine + 2, keys, w, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(mine + 3, (const char*)keys + (size_t)(n - 1) * w, w, hipMemcpyDeviceToDevice, s));
    }
    std::vector<uint64_t> all(4 * (size_t)p);
    if (p > 1) {
        NCCLCHK(ncclAllGather(mine, d, 4, ncclUint64, c->comm, s));
        HIPCHK(hipMemcpyAsync(all.data(), d, sizeof(uint64_t) * 4 * p, hipMemcpyDeviceToHost, s));
    } else {
        HIPCHK(hipMemcpyAsync(all.data(), mine, sizeof(uint64_t) * 4, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    // psort.cc:498-516: local descents + (rank>0) last(rank-1) > first(rank), SUM.
    int64_t total = 0;
    bool have_prev = false;
    uint64_t prev = 0;
    auto gt = [&](uint64_t a, uint64_t b) {
        if (dtype == MISORT_F64) {
            double x, y;
            memcpy(&x, &a, 8);
            memcpy(&y, &b, 8);
            return x > y;
        }
        if (w == 4) return (uint32_t)a > (uint32_t)b;
        return a > b;
    };
    for (int r = 0; r < p; ++r) {
        const uint64_t* q = &all[4 * (size_t)r];
        total += (int64_t)q[0];
        if (q[1] == 0) continue;  // empty block: UB in the reference; forwards prev
        if (r > 0 && have_prev && gt(prev, q[2])) total++;
        prev = q[3];
        have_prev = true;
    }
    *errors = total;
    return MISORT_OK;
}

int misort_sort_host(misort_ctx* c, int dtype, const void* h_in, void* h_out, int64_t loc,
                     int64_t max_size) {
    if (!c || !valid_dtype(dtype) || loc < 0 || (loc > 0 && (!h_in || !h_out)))
        return fail(MISORT_E_INVALID, "bad sort_host arguments");
    const size_t bytes = (size_t)loc * key_bytes(dtype);
    if (bytes > c->pinned_bytes) {
        if (c->pinned) HIPCHK(hipHostFree(c->pinned));
        c->pinned = nullptr;
        c->pinned_bytes = 0;
        HIPCHK(hipHostMalloc(&c->pinned, std::max<size_t>(bytes, 64), hipHostMallocDefault));
        c->pinned_bytes = std::max<size_t>(bytes, 64);
    }
    DevBuf dev;
    int rc = dev.ensure(std::max<size_t>(bytes, 64));
    if (rc) return rc;
    memcpy(c->pinned, h_in, bytes);
    HIPCHK(hipMemcpyAsync(dev.p, c->pinned, bytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = parallel_sort(c, dtype, dev.p, dev.p, loc, max_size, c->stream))) return rc;
    HIPCHK(hipMemcpyAsync(c->pinned, dev.p, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    memcpy(h_out, c->pinned, bytes);
    return MISORT_OK;
}

int misort_fill_splitmix(misort_ctx* c, int dtype, void* out, int64_t n, uint64_t seed, int64_t g0,
                         void* stream) {
    if (!c || !valid_dtype(dtype) || n < 0) return fail(MISORT_E_INVALID, "bad fill arguments");
    hipStream_t s = pick(c, stream);
    if (dtype == MISORT_U32) HIPCHK(misort::fill_splitmix_u32((uint32_t*)out, n, seed, g0, s));
    else HIPCHK(misort::fill_splitmix_u64((uint64_t*)out, n, seed, g0, s));
    return MISORT_OK;
}

int misort_profile_enable(misort_ctx* c, int on) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    c->prof.on = on != 0;
    return MISORT_OK;
}

int misort_profile_reset(misort_ctx* c) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    int rc = c->prof.collect();
    c->prof.reset();
    return rc;
}

int misort_profile_read(misort_ctx* c, int kind, int64_t* launches, double* total_ms, double* bytes) {
    if (!c || kind < 0 || kind >= misort::KIND_COUNT) return fail(MISORT_E_INVALID, "bad kind");
    int rc = c->prof.collect();
    if (rc) return rc;
    if (launches) *launches = c->prof.launches[kind];
    if (total_ms) *total_ms = c->prof.ms[kind];
    if (bytes) *bytes = c->prof.bytes[kind];
    return MISORT_OK;
}

int misort_tile_log2(int key_bytes_) { return misort::tile_log2(key_bytes_); }

}  // extern "C"
