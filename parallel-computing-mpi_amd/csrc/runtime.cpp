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
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <set>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <new>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "kernels.h"

namespace {

thread_local std::string g_err;

// MISORT_TRACE=1: one stderr line per RCCL-side step (group calls, waits,
// aborts), to see where a multi-rank run stands when it stops.
bool trace_on() {
    static const bool on = getenv("MISORT_TRACE") && atoi(getenv("MISORT_TRACE")) != 0;
    return on;
}
#define TRACE(...)                                  \
    do {                                            \
        if (trace_on()) {                           \
            fprintf(stderr, "[misort] " __VA_ARGS__); \
            fputc('\n', stderr);                    \
            fflush(stderr);                         \
        }                                           \
    } while (0)

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

// Deadline of every wait on another rank (MISORT_TIMEOUT_S, default 120 s):
// the role of the reference's alarm(540) watchdog (psort.cc:17,56-65), per
// wait instead of per run, so a dead or desynchronised peer turns into an
// error instead of a hang.
double peer_timeout_s() {
    static const double t = [] {
        const char* e = getenv("MISORT_TIMEOUT_S");
        const double v = e ? atof(e) : 120.0;
        return v > 0 ? v : 120.0;
    }();
    return t;
}

// HIP-event profiler: one event pair per kernel launch of a sort.
struct Profiler final : misort::LaunchHook {
    struct Rec {
        int kind;
        hipEvent_t a, b;
        double bytes;
        int stage;  // hypercube stage of parallel_sort (-1: local sort / other)
        bool own_a = true, own_b = true;  // events another record shares are returned to the pool once
    };
    static constexpr int MAX_STAGES = 64;
    std::vector<hipEvent_t> pool;
    std::vector<Rec> pending;
    int64_t launches[misort::KIND_COUNT] = {};
    double ms[misort::KIND_COUNT] = {};
    double bytes[misort::KIND_COUNT] = {};
    // per hypercube stage: [0] exchange leg, [1] merge-split kernels
    int64_t st_count[MAX_STAGES] = {};
    double st_ms[MAX_STAGES][2] = {};
    double st_bytes[MAX_STAGES] = {};
    int stage = -1;
    // every collected record in completion order (an enclosing pass after the
    // kernels nested in it), for per-pass figures; capped
    struct Trace {
        int kind;
        float ms;
        double bytes;
    };
    static constexpr size_t MAX_TRACE = (size_t)1 << 20;
    std::vector<Trace> trace;
    Rec cur{-1, nullptr, nullptr, 0.0, -1};             // the innermost open record (the exchange leg sets its bytes)
    std::vector<Rec> open;   // enclosing records (a pass around its kernel)
    bool on = false;

    // Timing-only events skip the system-scope release a default event's
    // record performs: that write-back of the L2s put ~5 us of idle time behind
    // every record (2^24 u32: 73 us of a 403 us sort between kernels, rocprofv3
    // kernel trace, profiles/r03/timeline).  MISORT_PROF_SYSFENCE=1 restores it.
    hipEvent_t take() {
        static const unsigned flags =
            getenv("MISORT_PROF_SYSFENCE") && atoi(getenv("MISORT_PROF_SYSFENCE")) ? 0u : hipEventDisableSystemFence;
        if (pool.empty()) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, flags) != hipSuccess) return nullptr;
            return e;
        }
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    void before(misort::Kind k, double b, hipStream_t s) override {
        if (cur.kind >= 0) open.push_back(cur);
        cur = Rec{k, take(), take(), b, stage};
        if (cur.a) (void)hipEventRecord(cur.a, s);
    }
    // Kernel-bound records (the local sort's passes): see LaunchHook.
    // MISORT_PROF_MARKERS=1 times them by marker events instead.
    // MISORT_PROF_BIND: 1 = a record's launch carries a start and a stop
    // event; 2 (default) = launches carry stop events only and a record starts
    // at the previous stop (its kernel's at the stop of the launch before it,
    // bound as a tick; a pass's at the end of the previous pass).
    hipEvent_t last = nullptr;        // the stop of the last bound launch of the current sort
    hipEvent_t pass_start = nullptr;  // the end of the current sort's previous pass
    std::vector<hipEvent_t> live;     // bound events, back to the pool at collect()
    static int bind_mode() {
        static const int m = getenv("MISORT_PROF_BIND") ? atoi(getenv("MISORT_PROF_BIND")) : 2;
        return m == 1 ? 1 : 2;
    }
    bool binds() const override {
        static const bool markers = getenv("MISORT_PROF_MARKERS") && atoi(getenv("MISORT_PROF_MARKERS"));
        return !markers;
    }
    void bind_reset() override { last = pass_start = nullptr; }
    bool bind(int kk, int pk, double b, hipEvent_t* a, hipEvent_t* z) override {
        *a = *z = nullptr;
        const bool ticks = bind_mode() == 2;
        if (kk < 0 && pk < 0 && !ticks) return false;  // a tick: only stop-only binding uses them
        const bool need_a = (kk >= 0 && (!ticks || !last)) || (pk >= 0 && !pass_start);
        hipEvent_t ea = need_a ? take() : nullptr, eb = take();
        if (!eb || (need_a && !ea)) {
            if (ea) pool.push_back(ea);
            if (eb) pool.push_back(eb);
            return false;
        }
        if (ea) live.push_back(ea);
        live.push_back(eb);
        if (kk >= 0) pending.push_back(Rec{kk, ticks && last ? last : ea, eb, b, stage, false, false});
        if (pk >= 0) pending.push_back(Rec{pk, pass_start ? pass_start : ea, eb, b, stage, false, false});
        last = eb;
        if (pk >= 0 || kk == misort::KIND_TILE_SORT) pass_start = eb;
        *a = ea;
        *z = eb;
        return true;
    }
    void after(misort::Kind, hipStream_t s) override {
        if (cur.b) (void)hipEventRecord(cur.b, s);
        pending.push_back(cur);
        if (!open.empty()) {
            cur = open.back();
            open.pop_back();
        } else {
            cur = Rec{-1, nullptr, nullptr, 0.0, -1};
        }
    }
    int collect() {
        for (auto& r : pending) {
            float t = 0.f;
            if (r.a && r.b) {
                HIPCHK(hipEventSynchronize(r.b));
                HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
            }
            if (r.kind < 0 || r.kind >= misort::KIND_COUNT) continue;
            launches[r.kind] += 1;
            ms[r.kind] += t;
            bytes[r.kind] += r.bytes;
            if (trace.size() < MAX_TRACE) trace.push_back(Trace{r.kind, t, r.bytes});
            if (r.stage >= 0 && r.stage < MAX_STAGES) {
                const bool xg = r.kind == misort::KIND_EXCHANGE;
                st_ms[r.stage][xg ? 0 : 1] += t;
                if (xg) {
                    st_count[r.stage] += 1;
                    st_bytes[r.stage] += r.bytes;
                }
            }
            if (r.a && r.own_a) pool.push_back(r.a);
            if (r.b && r.own_b) pool.push_back(r.b);
        }
        pending.clear();
        for (auto e : live) pool.push_back(e);
        live.clear();
        last = pass_start = nullptr;  // back in the pool
        return MISORT_OK;
    }
    void reset() {
        std::fill(std::begin(launches), std::end(launches), 0);
        std::fill(std::begin(ms), std::end(ms), 0.0);
        std::fill(std::begin(bytes), std::end(bytes), 0.0);
        std::fill(std::begin(st_count), std::end(st_count), 0);
        std::fill(&st_ms[0][0], &st_ms[0][0] + 2 * MAX_STAGES, 0.0);
        std::fill(std::begin(st_bytes), std::end(st_bytes), 0.0);
        trace.clear();
    }
    ~Profiler() override {
        for (auto& r : pending) {
            if (r.a && r.own_a) (void)hipEventDestroy(r.a);
            if (r.b && r.own_b) (void)hipEventDestroy(r.b);
        }
        for (auto e : live) (void)hipEventDestroy(e);
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

// The context's small device words (sizes, counts, check_sort's words) are
// one buffer of this size from its first use: growing it would hipFree the
// old one, which waits for the whole device -- with no deadline behind a
// transfer from a dead peer.
constexpr size_t kSmallBytes = 256;

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
    void swap(DevBuf& o) {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
    }
};

// ---------------------------------------------------------------- transport
//
// The exchange step of compare_split (MPI_Sendrecv, psort.cc:121,146) and the
// two small all-gathers the driver needs, behind one interface:
//   RcclTransport   one process per GPU, ncclSend/ncclRecv over xGMI;
//   LocalTransport  ranks are threads of one process (misort_group), the
//                   exchange is a device-to-device copy ordered by HIP events.
struct Transport {
    int nranks = 1, rank = 0;
    uint64_t calls = 0;  // collective calls made (entry points abort only after the first)
    virtual ~Transport() = default;
    // all ranks' int64 value, host-visible on return
    virtual int allgather_i64(const int64_t* mine, int count, std::vector<int64_t>& all,
                              hipStream_t s) = 0;
    // the same from `count` int64 values already in device memory (d_mine),
    // so a size computed on the device needs no host round trip before it
    virtual int allgather_i64_dev(const int64_t* d_mine, int count, std::vector<int64_t>& all, hipStream_t s) = 0;
    // device buffers; both sides know both byte counts
    virtual int sendrecv(const void* send, size_t send_bytes, void* recv, size_t recv_bytes, int peer,
                         hipStream_t s) = 0;
    // one group of point-to-point transfers (no self transfers; at most one
    // message per (sender, receiver) pair; both sides post matching sizes)
    struct Op {
        int peer;
        bool send;
        const void* sptr;
        void* rptr;
        size_t bytes;
    };
    virtual int group_p2p(const std::vector<Op>& ops, hipStream_t s) = 0;
    // all-to-all-v on device buffers: to rank q go send[soff[q], +scnt[q]) bytes,
    // from rank q come recv[roff[q], +rcnt[q]); every rank knows its own counts
    virtual int alltoallv(const void* send, const int64_t* soff, const int64_t* scnt, void* recv,
                          const int64_t* roff, const int64_t* rcnt, hipStream_t s) = 0;
    // Wait for stream s, whose queue may hold transfers from other ranks,
    // within peer_timeout_s().
    virtual int wait(hipStream_t s) = 0;
    // Stream s may hold a transfer from another rank (a copy from pageable
    // host memory enqueued behind it would block the host with no deadline).
    virtual bool busy(hipStream_t) const { return false; }
    // A rank failed inside a collective call: make the failure collective
    // (the reference MPI_Abort's, psort.cc:170), so the other ranks error out
    // instead of waiting for this one.  The transport is unusable afterwards.
    virtual void abort_all(const char* why) = 0;
};

// Host-side watchdog for RCCL calls that can block the calling thread
// (communicator setup, the first connection to a peer inside ncclGroupEnd):
// armed around each such call; if the call outlives the deadline, the process
// prints why and aborts -- the reference's SIGALRM -> program_trap -> abort()
// (psort.cc:56-65).  Waits on the stream never block here: they poll with
// their own deadline (RcclTransport::wait).  The thread starts on first use.
struct CallWatchdog {
    std::mutex mu;
    std::condition_variable cv;
    std::thread th;
    bool stop = false, armed = false;
    const char* what = "";
    std::chrono::steady_clock::time_point deadline;
    void arm(const char* w) {
        std::lock_guard<std::mutex> lk(mu);
        if (!th.joinable()) th = std::thread([this] { loop(); });
        what = w;
        deadline = std::chrono::steady_clock::now() +
                   std::chrono::microseconds((int64_t)(peer_timeout_s() * 1e6));
        armed = true;
        cv.notify_all();
    }
    void disarm() {
        std::lock_guard<std::mutex> lk(mu);
        armed = false;
    }
    void loop() {
        std::unique_lock<std::mutex> lk(mu);
        while (!stop) {
            if (!armed) {
                cv.wait(lk);
                continue;
            }
            if (cv.wait_until(lk, deadline) == std::cv_status::timeout && armed && !stop &&
                std::chrono::steady_clock::now() >= deadline) {
                // the blocked call holds the communicator, so it cannot be
                // aborted safely from here: end the process (no core dump)
                fprintf(stderr, "misort: RCCL call %s blocked for more than MISORT_TIMEOUT_S=%.0f s; exiting\n",
                        what, peer_timeout_s());
                fflush(stderr);
                _exit(EXIT_FAILURE);
            }
        }
    }
    ~CallWatchdog() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        if (th.joinable()) th.join();
    }
};

struct RcclTransport final : Transport {
    ncclComm_t comm = nullptr;
    bool dead = false;  // aborted: every later call fails with MISORT_E_RCCL
    std::string dead_why;
    DevBuf buf;
    CallWatchdog dog;
    ~RcclTransport() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    int usable() {
        if (dead || !comm) return fail(MISORT_E_RCCL, "RCCL communicator aborted earlier (%s)", dead_why.c_str());
        return MISORT_OK;
    }
    void abort_all(const char* why) override {
        if (dead) return;
        dead = true;
        dead_why = why;
        TRACE("rank %d: aborting the communicator (%s)", rank, why);
        if (comm) (void)ncclCommAbort(comm);  // peers' pending transfers fail or time out
        TRACE("rank %d: communicator aborted", rank);
        comm = nullptr;
    }
    // An RCCL error: abort the communicator, keep the first message.
    int rccl_fail(const char* what, ncclResult_t r) {
        char why[512];
        snprintf(why, sizeof why, "%s: %s", what, ncclGetErrorString(r));
        abort_all(why);
        return fail(MISORT_E_RCCL, "%s", why);
    }
    // Polls the stream and the communicator's asynchronous error state; a
    // remote failure or the deadline aborts the communicator and returns
    // MISORT_E_RCCL.  Spins briefly (stage waits are usually short), then
    // sleeps between polls.
    // Streams with a transport call queued since they last drained under
    // wait(): a caller may queue a sort on its own stream and drain another
    // one first, so the record is per stream (one per transport would let the
    // other stream's drain clear this one's, and a dead peer would then hang
    // the plain synchronisation below).
    std::set<hipStream_t> pending;
    bool busy(hipStream_t s) const override { return pending.count(s) != 0; }
    int wait(hipStream_t s) override {
        int rc = usable();
        if (rc) return rc;
        if (!pending.count(s)) {
            // no transport call on s since it last drained: only local work
            // is queued (it may legitimately run longer than the peer deadline,
            // e.g. under a counter-collecting profiler), so no deadline and no abort
            HIPCHK(hipStreamSynchronize(s));
            return MISORT_OK;
        }
        TRACE("rank %d: waiting on the stream (deadline %.0f s)", rank, peer_timeout_s());
        const auto t0 = std::chrono::steady_clock::now();
        const double lim = peer_timeout_s();
        for (int it = 0;; ++it) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess) {
                pending.erase(s);
                return MISORT_OK;
            }
            if (q != hipErrorNotReady) {
                abort_all("stream error while waiting for peers");
                return fail(MISORT_E_HIP, "hipStreamQuery: %s", hipGetErrorString(q));
            }
            ncclResult_t ar = ncclSuccess;
            const ncclResult_t gr = ncclCommGetAsyncError(comm, &ar);
            if (gr != ncclSuccess) return rccl_fail("ncclCommGetAsyncError", gr);
            if (ar != ncclSuccess && ar != ncclInProgress) return rccl_fail("asynchronous RCCL error", ar);
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (el > lim) {
                char why[160];
                snprintf(why, sizeof why, "no progress from peers within MISORT_TIMEOUT_S=%.0f s", lim);
                abort_all(why);
                return fail(MISORT_E_RCCL, "%s", why);
            }
            if (it < 2000) std::this_thread::yield();
            else std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
    }
    // ncclGroupStart ... ncclGroupEnd that always closes the group, also when
    // a call inside it fails, under the call watchdog.
    template <typename F>
    int grouped(const char* what, hipStream_t s, F&& body) {
        ++calls;
        int rc = usable();
        if (rc) return rc;
        pending.insert(s);
        ncclResult_t r = ncclGroupStart();
        if (r != ncclSuccess) return rccl_fail("ncclGroupStart", r);
        ncclResult_t inner = body();
        TRACE("rank %d: ncclGroupEnd (%s)", rank, what);
        dog.arm(what);
        r = ncclGroupEnd();
        dog.disarm();
        TRACE("rank %d: ncclGroupEnd returned %d", rank, (int)r);
        if (inner != ncclSuccess) return rccl_fail(what, inner);
        if (r != ncclSuccess) return rccl_fail(what, r);
        return MISORT_OK;
    }
    // Connects every path a sort uses -- the collective ring and a send and a
    // receive with every peer, large enough to open all of RCCL's point-to-
    // point channels -- right after ncclCommInitRank, under the call
    // watchdog.  RCCL connects lazily, inside ncclGroupEnd, with the peer's
    // cooperation, so without this the first exchange with a dead or stalled
    // peer would block the host in a call that cannot be aborted safely;
    // afterwards a failed peer shows as a stream that does not drain, which
    // wait() detects and aborts.
    int connect_all(hipStream_t s) {
        const size_t per = (size_t)8 << 20;
        DevBuf tmp;
        int rc = tmp.ensure(per * 2 * (size_t)nranks);
        if (rc) return rc;
        HIPCHK(hipMemsetAsync(tmp.p, 0, tmp.bytes, s));
        char* b = (char*)tmp.p;
        rc = grouped("connect: ncclSend/ncclRecv with every peer", s, [&] {
            ncclResult_t r = ncclSuccess;
            for (int k = 1; k < nranks && r == ncclSuccess; ++k) {
                const int to = (rank + k) % nranks, from = (rank - k + nranks) % nranks;
                r = ncclSend(b + per * to, per, ncclUint8, to, comm, s);
                if (r == ncclSuccess) r = ncclRecv(b + per * (nranks + from), per, ncclUint8, from, comm, s);
            }
            return r;
        });
        if (rc) return rc;
        if ((rc = buf.ensure(sizeof(int64_t) * 2 * (nranks + 1)))) return rc;
        std::vector<int64_t> all;
        const int64_t v[2] = {rank, nranks};
        if ((rc = allgather_i64(v, 2, all, s))) return rc;
        for (int r = 0; r < nranks; ++r)
            if (all[2 * r] != r || all[2 * r + 1] != nranks) return fail(MISORT_E_RCCL, "connect: bad all-gather");
        return wait(s);
    }
    int allgather_dev(const int64_t* d_src, int count, std::vector<int64_t>& all, hipStream_t s) {
        int64_t* d = (int64_t*)buf.p;
        int rc = grouped("ncclAllGather", s, [&] { return ncclAllGather(d_src, d, count, ncclInt64, comm, s); });
        if (rc) return rc;
        // drain the stream under the deadline first: a device-to-host copy
        // into pageable memory would block on it without one
        if ((rc = wait(s))) return rc;
        all.resize((size_t)count * nranks);
        HIPCHK(hipMemcpyAsync(all.data(), d, sizeof(int64_t) * count * nranks, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return MISORT_OK;
    }
    int allgather_i64(const int64_t* mine, int count, std::vector<int64_t>& all, hipStream_t s) override {
        int rc = usable();
        if (rc || (rc = buf.ensure(sizeof(int64_t) * (size_t)count * (nranks + 1)))) return rc;
        // the copy below is from pageable memory: behind a transfer from a
        // dead peer it would block with no deadline, so drain under one first
        if (busy(s) && (rc = wait(s))) return rc;
        int64_t* d = (int64_t*)buf.p;
        HIPCHK(hipMemcpyAsync(d + (size_t)count * nranks, mine, sizeof(int64_t) * count,
                              hipMemcpyHostToDevice, s));
        return allgather_dev(d + (size_t)count * nranks, count, all, s);
    }
    int allgather_i64_dev(const int64_t* d_mine, int count, std::vector<int64_t>& all, hipStream_t s) override {
        int rc = usable();
        if (rc || (rc = buf.ensure(sizeof(int64_t) * (size_t)count * (nranks + 1)))) return rc;
        return allgather_dev(d_mine, count, all, s);
    }
    int sendrecv(const void* send, size_t sb, void* recv, size_t rb, int peer, hipStream_t s) override {
        return grouped("ncclSend/ncclRecv", s, [&] {
            ncclResult_t r = ncclSuccess;
            if (sb) r = ncclSend(send, sb, ncclUint8, peer, comm, s);
            if (r == ncclSuccess && rb) r = ncclRecv(recv, rb, ncclUint8, peer, comm, s);
            return r;
        });
    }
    int group_p2p(const std::vector<Op>& ops, hipStream_t s) override {
        return grouped("grouped ncclSend/ncclRecv", s, [&] {
            ncclResult_t r = ncclSuccess;
            for (const Op& o : ops) {
                if (!o.bytes || r != ncclSuccess) continue;
                r = o.send ? ncclSend(o.sptr, o.bytes, ncclUint8, o.peer, comm, s)
                           : ncclRecv(o.rptr, o.bytes, ncclUint8, o.peer, comm, s);
            }
            return r;
        });
    }
    // One grouped call: every peer pair moves over its own xGMI link at once.
    int alltoallv(const void* send, const int64_t* soff, const int64_t* scnt, void* recv, const int64_t* roff,
                  const int64_t* rcnt, hipStream_t s) override {
        if (scnt[rank] != rcnt[rank]) return fail(MISORT_E_INVALID, "alltoallv self count mismatch");
        if (scnt[rank])
            HIPCHK(hipMemcpyAsync((char*)recv + roff[rank], (const char*)send + soff[rank], (size_t)scnt[rank],
                                  hipMemcpyDeviceToDevice, s));
        return grouped("all-to-all-v ncclSend/ncclRecv", s, [&] {
            ncclResult_t r = ncclSuccess;
            for (int k = 1; k < nranks && r == ncclSuccess; ++k) {
                const int to = (rank + k) % nranks, from = (rank - k + nranks) % nranks;
                if (scnt[to]) r = ncclSend((const char*)send + soff[to], (size_t)scnt[to], ncclUint8, to, comm, s);
                if (r == ncclSuccess && rcnt[from])
                    r = ncclRecv((char*)recv + roff[from], (size_t)rcnt[from], ncclUint8, from, comm, s);
            }
            return r;
        });
    }
};

}  // namespace

// In-process rank group: one thread (and one misort_ctx) per rank.
struct misort_group {
    int n;
    std::mutex mu;
    std::condition_variable cv;
    // Exchanges are matched per partner pair: posted[q]/finished[q] count this
    // rank's exchanges with rank q, which both sides advance in the same order
    // (a stage that moves nothing skips on both sides).
    struct Slot {
        const void* ptr = nullptr;
        size_t bytes = 0;
        hipEvent_t ready = nullptr, done = nullptr;
        std::vector<uint64_t> posted, finished;
        std::vector<int64_t> vals;
        std::vector<int64_t> a2a_off, a2a_cnt;  // alltoallv: this rank's send slices
        std::vector<std::pair<const void*, size_t>> p2p_send;  // group_p2p: message to each rank
    };
    std::vector<Slot> slots;
    uint64_t bar_count = 0, bar_gen = 0;
    bool failed = false;  // a rank failed inside a collective call: every wait ends
    explicit misort_group(int n_) : n(n_), slots(n_) {
        for (auto& sl : slots) {
            sl.posted.assign(n_, 0);
            sl.finished.assign(n_, 0);
        }
    }
    // Waits (lock held) until pred() or a failure of the group, at most
    // peer_timeout_s(); true iff pred() holds.
    template <typename Pred>
    bool wait_for(std::unique_lock<std::mutex>& lk, Pred pred) {
        cv.wait_for(lk, std::chrono::microseconds((int64_t)(peer_timeout_s() * 1e6)),
                    [&] { return failed || pred(); });
        return !failed && pred();
    }
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) return false;
        const uint64_t gen = bar_gen;
        if (++bar_count == (uint64_t)n) {
            bar_count = 0;
            ++bar_gen;
            cv.notify_all();
            return true;
        }
        return wait_for(lk, [&] { return bar_gen != gen; });
    }
    void fail_all() {
        {
            std::lock_guard<std::mutex> lk(mu);
            failed = true;
        }
        cv.notify_all();
    }
};

namespace {

struct LocalTransport final : Transport {
    misort_group* g = nullptr;
    std::vector<uint64_t> epoch;  // exchanges with each peer so far
    ~LocalTransport() override {
        auto& me = g->slots[rank];
        if (me.ready) (void)hipEventDestroy(me.ready);
        if (me.done) (void)hipEventDestroy(me.done);
        me.ready = me.done = nullptr;
    }
    int wait(hipStream_t s) override {
        HIPCHK(hipStreamSynchronize(s));
        return MISORT_OK;
    }
    void abort_all(const char*) override { g->fail_all(); }
    int allgather_i64_dev(const int64_t* d_mine, int count, std::vector<int64_t>& all, hipStream_t s) override {
        std::vector<int64_t> mine((size_t)count);
        HIPCHK(hipMemcpyAsync(mine.data(), d_mine, sizeof(int64_t) * count, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        return allgather_i64(mine.data(), count, all, s);
    }
    int allgather_i64(const int64_t* mine, int count, std::vector<int64_t>& all, hipStream_t) override {
        ++calls;
        {
            std::lock_guard<std::mutex> lk(g->mu);
            g->slots[rank].vals.assign(mine, mine + count);
        }
        if (!g->barrier()) return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        all.clear();
        {
            std::lock_guard<std::mutex> lk(g->mu);
            for (int r = 0; r < nranks; ++r)
                all.insert(all.end(), g->slots[r].vals.begin(), g->slots[r].vals.end());
        }
        if (!g->barrier())  // nobody overwrites vals before everyone has read them
            return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        return MISORT_OK;
    }
    int sendrecv(const void* send, size_t sb, void* recv, size_t rb, int peer, hipStream_t s) override {
        auto& me = g->slots[rank];
        ++calls;
        auto& pe = g->slots[peer];
        const uint64_t e = ++epoch[peer];
        HIPCHK(hipEventRecord(me.ready, s));
        {
            std::lock_guard<std::mutex> lk(g->mu);
            me.ptr = send;
            me.bytes = sb;
            me.posted[peer] = e;
        }
        g->cv.notify_all();
        {
            std::unique_lock<std::mutex> lk(g->mu);
            if (!g->wait_for(lk, [&] { return pe.posted[rank] >= e; }))
                return fail(MISORT_E_INVALID, "group exchange %d<->%d failed or timed out", rank, peer);
        }
        if (pe.bytes != rb)
            return fail(MISORT_E_INVALID, "sendrecv size mismatch with rank %d (%zu vs %zu)", peer,
                        pe.bytes, rb);
        HIPCHK(hipStreamWaitEvent(s, pe.ready, 0));
        if (rb) HIPCHK(hipMemcpyAsync(recv, pe.ptr, rb, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipEventRecord(me.done, s));
        {
            std::lock_guard<std::mutex> lk(g->mu);
            me.finished[peer] = e;
        }
        g->cv.notify_all();
        {
            std::unique_lock<std::mutex> lk(g->mu);
            if (!g->wait_for(lk, [&] { return pe.finished[rank] >= e; }))
                return fail(MISORT_E_INVALID, "group exchange %d<->%d failed or timed out", rank, peer);
        }
        // the peer has read my send buffer before this stream reuses it
        HIPCHK(hipStreamWaitEvent(s, pe.done, 0));
        return MISORT_OK;
    }
    int group_p2p(const std::vector<Op>& ops, hipStream_t s) override {
        auto& me = g->slots[rank];
        ++calls;
        HIPCHK(hipEventRecord(me.ready, s));
        {
            std::lock_guard<std::mutex> lk(g->mu);
            me.p2p_send.assign(nranks, {nullptr, 0});
            for (const Op& o : ops)
                if (o.send) me.p2p_send[o.peer] = {o.sptr, o.bytes};
        }
        if (!g->barrier()) return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        for (const Op& o : ops) {
            if (o.send) continue;
            const auto& pe = g->slots[o.peer];
            if (pe.p2p_send[rank].second != o.bytes)
                return fail(MISORT_E_INVALID, "group_p2p size mismatch from rank %d (%zu vs %zu)", o.peer,
                            pe.p2p_send[rank].second, o.bytes);
            if (!o.bytes) continue;
            HIPCHK(hipStreamWaitEvent(s, pe.ready, 0));
            HIPCHK(hipMemcpyAsync(o.rptr, pe.p2p_send[rank].first, o.bytes, hipMemcpyDeviceToDevice, s));
        }
        HIPCHK(hipStreamSynchronize(s));
        if (!g->barrier()) return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        return MISORT_OK;
    }
    int alltoallv(const void* send, const int64_t* soff, const int64_t* scnt, void* recv, const int64_t* roff,
                  const int64_t* rcnt, hipStream_t s) override {
        auto& me = g->slots[rank];
        ++calls;
        HIPCHK(hipEventRecord(me.ready, s));
        {
            std::lock_guard<std::mutex> lk(g->mu);
            me.ptr = send;
            me.a2a_off.assign(soff, soff + nranks);
            me.a2a_cnt.assign(scnt, scnt + nranks);
        }
        if (!g->barrier()) return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        for (int q = 0; q < nranks; ++q) {
            const auto& pe = g->slots[q];
            if (pe.a2a_cnt[rank] != rcnt[q])
                return fail(MISORT_E_INVALID, "alltoallv size mismatch with rank %d (%lld vs %lld)", q,
                            (long long)pe.a2a_cnt[rank], (long long)rcnt[q]);
            if (!rcnt[q]) continue;
            HIPCHK(hipStreamWaitEvent(s, pe.ready, 0));
            HIPCHK(hipMemcpyAsync((char*)recv + roff[q], (const char*)pe.ptr + pe.a2a_off[rank], (size_t)rcnt[q],
                                  hipMemcpyDeviceToDevice, s));
        }
        // every reader is done with every send buffer before anyone reuses it
        HIPCHK(hipStreamSynchronize(s));
        if (!g->barrier()) return fail(MISORT_E_INVALID, "group barrier failed or timed out");
        return MISORT_OK;
    }
};

// MISORT_TAIL_DIV: a stage whose k received keys are at most 1/tail_div of the
// block merges in place at the block's end (0 = never); clamped to [0, 2^20]
// so the bracket test cannot overflow.
int64_t env_tail_div() {
    const char* v = getenv("MISORT_TAIL_DIV");
    if (!v) return 8;
    const long long d = atoll(v);
    return d < 0 ? 0 : d > (1 << 20) ? (1 << 20) : (int64_t)d;
}

}  // namespace

struct misort_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    Transport* tr = nullptr;
    int nranks = 1, rank = 0;
    DevBuf work, recv, scratch, small, samp_me, samp_peer, pong;
    DevBuf qa, qb, qcnt;  // quick sort: current run, merge target, exchanged counts
    void* pinned = nullptr;
    size_t pinned_bytes = 0;
    // host staging (misort_sort_host): device keys, pinned ring, copy stream
    DevBuf host_keys;
    static constexpr int RING = 3;
    void* ring[RING] = {};
    size_t ring_bytes = 0;
    hipEvent_t ring_ev[RING] = {};
    bool ring_busy[RING] = {};
    hipStream_t copy_stream = nullptr;
    Profiler prof;
    int64_t xchg_bytes = 0, xchg_stages = 0, xchg_full_bytes = 0;
    bool full_exchange = getenv("MISORT_FULL_EXCHANGE") != nullptr;
    // relay compare-split exchanges through the other GPUs (P > 2): MISORT_RELAY=0 disables
    bool relay = !getenv("MISORT_RELAY") || atoi(getenv("MISORT_RELAY")) != 0;
    DevBuf relay_buf;
    // delta-coded exchange (codec.hip): MISORT_COMPRESS=0 / misort_set_compress(ctx, 0) disables
    bool compress = !getenv("MISORT_COMPRESS") || atoi(getenv("MISORT_COMPRESS")) != 0;
    // a stage whose message is at most 1/tail_div of the block merges in place
    // at the block's end (misort::merge_split_tail); 0 = always the
    // whole-block merge (MISORT_TAIL_DIV)
    int64_t tail_div = env_tail_div();
    DevBuf enc_send, enc_recv, codec_scr;
    int64_t xchg_raw_bytes = 0;  // what the coded stages would have moved uncoded
    ~misort_ctx() {
        delete tr;
        for (int i = 0; i < RING; ++i) {
            if (ring[i]) (void)hipHostFree(ring[i]);
            if (ring_ev[i]) (void)hipEventDestroy(ring_ev[i]);
        }
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
    }
};

namespace {

hipStream_t pick(misort_ctx* c, void* s) { return s ? (hipStream_t)s : c->stream; }
misort::LaunchHook* hook(misort_ctx* c) { return c->prof.on ? &c->prof : nullptr; }

// Host wait on a stream whose queue may hold transfers from other ranks: with
// a communicator, bounded by peer_timeout_s() (RCCL: polled, aborted on a
// remote error or the deadline); a lone rank waits plainly.
int sync(misort_ctx* c, hipStream_t s) {
    if (c->tr) return c->tr->wait(s);
    HIPCHK(hipStreamSynchronize(s));
    return MISORT_OK;
}

// A small host -> device copy from pageable memory on stream s: such a copy
// blocks the host until the stream reaches it, so a stream that may hold a
// transfer from another rank is drained under the peer deadline first.
int h2d(misort_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t s) {
    if (c->tr && c->tr->busy(s)) {
        const int rc = c->tr->wait(s);
        if (rc) return rc;
    }
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return MISORT_OK;
}

// Small device -> host copies after work that may include transfers from
// other ranks: the stream is drained first by the bounded wait (a copy into
// pageable memory would block on an undrained stream with no deadline).
struct D2H {
    void* dst;
    const void* src;
    size_t bytes;
};
int fetch(misort_ctx* c, hipStream_t s, std::initializer_list<D2H> cps) {
    int rc = sync(c, s);
    if (rc) return rc;
    for (const D2H& x : cps) HIPCHK(hipMemcpyAsync(x.dst, x.src, x.bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return MISORT_OK;
}

// The merge passes' device error word of stream s (k_chunk_desc rejected a
// chunk): the stream is synchronised.
int planning_check(hipStream_t s) {
    const int e0 = misort::mergek_take_error(s), e1 = misort::mergek_take_error_fg6(s);
    const int e = e0 < 0 || e1 < 0 ? -1 : (e0 | e1);
    if (e < 0) return fail(MISORT_E_HIP, "reading the merge passes' error word failed");
    if (e > 0) return fail(MISORT_E_INTERNAL, "a merge pass rejected its chunk bounds: the sorted output is incomplete");
    return MISORT_OK;
}

// Result of a collective entry point: a failure after the first transport
// call is made collective -- the communicator is aborted, so the other ranks
// fail instead of waiting for this one (the reference MPI_Abort's,
// psort.cc:170).  Argument errors found before any transport call stay local.
int collective_result(misort_ctx* c, uint64_t calls0, int rc) {
    if (rc != MISORT_OK && c->tr && c->nranks > 1 && c->tr->calls != calls0) {
        const std::string why = g_err;
        c->tr->abort_all(why.c_str());
        g_err = why;
    }
    return rc;
}

int do_local_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t n, bool ord_in,
                  hipStream_t s, const misort::StageIO* io = nullptr, bool ord_out = false) {
    // scratch for the ping-pong passes (grown on demand, kept for the context)
    int rc = c->pong.ensure(std::max<size_t>(16, (size_t)n * key_bytes(dtype)));
    if (rc) return rc;
    hipError_t e;
    if (dtype == MISORT_U32)
        e = misort::local_sort<uint32_t>((const uint32_t*)in, (uint32_t*)out, n, false, (uint32_t*)c->pong.p, s,
                                         hook(c), io);
    else
        e = misort::local_sort<uint64_t>((const uint64_t*)in, (uint64_t*)out, n, ord_in, (uint64_t*)c->pong.p, s,
                                         hook(c), io, ord_out);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "local_sort: %s", hipGetErrorString(e));
    return MISORT_OK;
}

int do_merge_split(misort_ctx* c, int dtype, const void* a, int64_t na, const void* b, int64_t nb,
                   void* out, int keep_max, hipStream_t s, bool ord_out = false) {
    const int64_t ntiles = (na + 2047) / 2048 + 2;
    int rc = c->scratch.ensure((size_t)ntiles * sizeof(int64_t));
    if (rc) return rc;
    hipError_t e;
    if (dtype == MISORT_U32)
        e = misort::merge_split<uint32_t>((const uint32_t*)a, na, (const uint32_t*)b, nb,
                                          (uint32_t*)out, keep_max, (int64_t*)c->scratch.p, s, hook(c));
    else
        e = misort::merge_split<uint64_t>((const uint64_t*)a, na, (const uint64_t*)b, nb,
                                          (uint64_t*)out, keep_max, (int64_t*)c->scratch.p, s, hook(c), ord_out);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "merge_split: %s", hipGetErrorString(e));
    return MISORT_OK;
}

// The compare-split in place in `a` (psort.cc:116-164 keep-n semantics): only
// the end of the block the k received keys reach is rewritten, staged through
// `stage` (a block-sized buffer).
int do_merge_split_tail(misort_ctx* c, int dtype, void* a, int64_t na, const void* b, int64_t nb, void* stage,
                        int keep_max, hipStream_t s) {
    const int64_t ntiles = (na + 2047) / 2048 + 6;
    int rc = c->scratch.ensure((size_t)ntiles * sizeof(int64_t));
    if (rc) return rc;
    hipError_t e;
    if (dtype == MISORT_U32)
        e = misort::merge_split_tail<uint32_t>((uint32_t*)a, na, (const uint32_t*)b, nb, keep_max, (uint32_t*)stage,
                                               (int64_t*)c->scratch.p, s, hook(c));
    else
        e = misort::merge_split_tail<uint64_t>((uint64_t*)a, na, (const uint64_t*)b, nb, keep_max, (uint64_t*)stage,
                                               (int64_t*)c->scratch.p, s, hook(c));
    if (e != hipSuccess) return fail(MISORT_E_HIP, "merge_split_tail: %s", hipGetErrorString(e));
    return MISORT_OK;
}

// The small-bracket test of a hypercube stage: k received keys against a block
// of loc (k <= loc / tail_div, no product to overflow).
bool tail_bracket(const misort_ctx* c, int64_t k, int64_t loc) { return c->tail_div > 0 && k <= loc / c->tail_div; }

// Splitter samples of a sorted block: a[min(c*S, n-1)], c = 0..ceil(n/S).
int64_t sample_stride(int64_t n) { return std::max<int64_t>(256, (n + 32767) / 32768); }
int64_t sample_count(int64_t n) { return n <= 0 ? 0 : (n + sample_stride(n) - 1) / sample_stride(n) + 1; }

// Lower bound of the merge-path co-rank i* = #A keys among the n_a smallest
// of A U B (A first on ties), from the two sample sets alone.  For i < i_lo
// A[i] <= B[n_a-1-i] is certain, so i* >= i_lo.  Both partners evaluate this
// on the same samples, so they agree on the exchange size without another
// round trip.
template <typename T>
int64_t corank_lower(const std::vector<T>& sa, int64_t na, const std::vector<T>& sb, int64_t nb) {
    if (na == 0) return 0;
    if (nb == 0) return na;
    const int64_t Sa = sample_stride(na), Sb = sample_stride(nb);
    const int64_t Ca = (int64_t)sa.size() - 1, Cb = (int64_t)sb.size() - 1;
    auto upperA = [&](int64_t i) { return sa[std::min(i / Sa + 1, Ca)]; };
    auto lowerB = [&](int64_t j) { return sb[std::min(j / Sb, Cb)]; };
    int64_t lo = na > nb ? na - nb : 0, hi = na;  // answer in [lo, hi]
    while (lo < hi) {  // first i whose "A[i] <= B[na-1-i]" is not certain
        const int64_t mid = lo + (hi - lo) / 2;
        if (upperA(mid) <= lowerB(na - 1 - mid)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Pair exchange of one hypercube stage (partner = rank ^ 2^bit) spread over
// every xGMI link.  A stage pairs the P GPUs, so a plain send/recv drives one
// of each GPU's P-1 links.  Here each message is cut into P parts: parts 0 and
// 1 go straight to the partner (one per round), part 2+j goes through the j-th
// other GPU, which receives it in round 1 and forwards it in round 2.  Every
// directed link carries one part per round, so a stage moves in 2/P of the
// direct time (4x less at P = 8).  All ranks take part, including those whose
// own message is empty, because they relay for the others.
int relay_exchange(misort_ctx* c, size_t w, int bit, const void* sbuf, size_t sbytes, void* rbuf, size_t rbytes,
                   hipStream_t s, size_t* rbytes_out = nullptr, const std::vector<int64_t>* known = nullptr) {
    const int P = c->nranks, me = c->rank, pm = me ^ (1 << bit);
    int rc;
    std::vector<int64_t> m;  // units (w bytes) each rank sends to its partner
    const int64_t mine = (int64_t)(sbytes / w);
    if (known) m = *known;  // gathered by the caller
    else if ((rc = c->tr->allgather_i64(&mine, 1, m, s))) return rc;
    if ((int)m.size() != P || m[me] != mine) return fail(MISORT_E_INVALID, "relay: size table mismatch");
    if (rbytes_out) {  // the partner's size is learnt here; rbytes is the capacity
        if ((size_t)m[pm] * w > rbytes) return fail(MISORT_E_CAPACITY, "relay: partner message exceeds buffer");
        *rbytes_out = (size_t)m[pm] * w;
    } else if ((size_t)m[pm] * w != rbytes) {
        return fail(MISORT_E_INVALID, "relay: partner size mismatch");
    }
    auto bnd = [&](int x, int i) { return (int64_t)((__int128)i * m[x] / P); };
    auto rel = [&](int x) {  // relays of x's pair, ascending
        std::vector<int> r;
        for (int y = 0; y < P; ++y)
            if (y != x && y != (x ^ (1 << bit))) r.push_back(y);
        return r;
    };
    auto idx_in = [&](int x, int y) {
        const std::vector<int> r = rel(x);
        return (int)(std::find(r.begin(), r.end(), y) - r.begin());
    };
    // staging for the parts this rank relays: x's part 2 + idx_in(x, me)
    std::vector<int64_t> soff(P, 0), scnt(P, 0);
    int64_t tot = 0;
    for (int x = 0; x < P; ++x) {
        if (x == me || x == pm) continue;
        const int j = idx_in(x, me);
        soff[x] = tot;
        scnt[x] = bnd(x, 3 + j) - bnd(x, 2 + j);
        tot += scnt[x];
    }
    if ((rc = c->relay_buf.ensure(std::max<size_t>(16, (size_t)tot * w)))) return rc;
    char* stg = (char*)c->relay_buf.p;
    const char* sb = (const char*)sbuf;
    char* rb = (char*)rbuf;
    const std::vector<int> mine_rel = rel(me);
    std::vector<Transport::Op> r1, r2;
    r1.push_back({pm, true, sb + bnd(me, 0) * w, nullptr, (size_t)(bnd(me, 1) - bnd(me, 0)) * w});
    r1.push_back({pm, false, nullptr, rb + bnd(pm, 0) * w, (size_t)(bnd(pm, 1) - bnd(pm, 0)) * w});
    r2.push_back({pm, true, sb + bnd(me, 1) * w, nullptr, (size_t)(bnd(me, 2) - bnd(me, 1)) * w});
    r2.push_back({pm, false, nullptr, rb + bnd(pm, 1) * w, (size_t)(bnd(pm, 2) - bnd(pm, 1)) * w});
    for (size_t j = 0; j < mine_rel.size(); ++j) {
        const int y = mine_rel[j];
        r1.push_back({y, true, sb + bnd(me, 2 + (int)j) * w, nullptr,
                      (size_t)(bnd(me, 3 + (int)j) - bnd(me, 2 + (int)j)) * w});
        r2.push_back({y, false, nullptr, rb + bnd(pm, 2 + (int)j) * w,
                      (size_t)(bnd(pm, 3 + (int)j) - bnd(pm, 2 + (int)j)) * w});
    }
    for (int x = 0; x < P; ++x) {
        if (x == me || x == pm) continue;
        r1.push_back({x, false, nullptr, stg + soff[x] * w, (size_t)scnt[x] * w});
        r2.push_back({x ^ (1 << bit), true, stg + soff[x] * w, nullptr, (size_t)scnt[x] * w});
    }
    if ((rc = c->tr->group_p2p(r1, s))) return rc;
    return c->tr->group_p2p(r2, s);
}

// The message sizes of a relayed stage: every rank contributes the pair
// (coded words, raw words) from device memory (d_pair, 2 int64) and sends
// min of the two; all ranks of the stage make this same collective call,
// whatever their own message is (coded, raw or empty).  units[r] = rank r's
// message in 4-byte words.
int relay_sizes(misort_ctx* c, const int64_t* d_pair, std::vector<int64_t>& pairs, std::vector<int64_t>& units,
                hipStream_t s) {
    int rc = c->tr->allgather_i64_dev(d_pair, 2, pairs, s);
    if (rc) return rc;
    units.resize((size_t)c->nranks);
    for (int r = 0; r < c->nranks; ++r) units[r] = std::min(pairs[(size_t)2 * r], pairs[(size_t)2 * r + 1]);
    return MISORT_OK;
}

// A relayed raw (or empty) message of `bytes` (a multiple of 4): the size
// round is relay_sizes with coded = raw.
int relay_raw(misort_ctx* c, int bit, const void* sbuf, size_t bytes, void* rbuf, size_t rbytes, hipStream_t s) {
    int rc = c->small.ensure(kSmallBytes);
    if (rc) return rc;
    int64_t* d_sz = (int64_t*)c->small.p + 2;
    const int64_t w2[2] = {(int64_t)(bytes / 4), (int64_t)(bytes / 4)};
    if ((rc = h2d(c, d_sz, w2, 16, s))) return rc;
    std::vector<int64_t> pairs, units;
    if ((rc = relay_sizes(c, d_sz, pairs, units, s))) return rc;
    return relay_exchange(c, 4, bit, sbuf, bytes, rbuf, rbytes, s, nullptr, &units);
}

// One compare-split message exchange, delta-coded (codec.hip), with the
// exchange count k computed on the device: run = {send offset, k} (device,
// from exchange_count) into `base`, k <= kmax.  The encoder takes the run from
// device memory, the ranks exchange their (coded words, raw words) pairs
// straight from device memory, and one host sync serves the count, the
// coded-or-raw choice and the sizes -- the host never waits for k alone.
// *k_out = k (0: nothing crossed; the relay still ran, others may pass through
// this rank); *rkeys receives the partner's k keys (decoded into c->recv, or
// the raw message in c->enc_recv when the partner sent it uncoded).
int coded_exchange(misort_ctx* c, int dtype, int q, bool relayed, const void* base, int64_t nloc, bool keep_max,
                   const int64_t* run, int64_t kmax, int64_t* k_out, const void** rkeys, hipStream_t s,
                   const std::function<bool(int, int)>& pair_coded) {
    const size_t w = key_bytes(dtype);
    const int64_t maxw = misort::codec_max_words(kmax, (int)w), raw_max = kmax * (int64_t)w / 4;
    int rc;
    if ((rc = c->enc_send.ensure((size_t)std::max<int64_t>(maxw, 4) * 4))) return rc;
    if ((rc = c->enc_recv.ensure((size_t)std::max<int64_t>(std::max(maxw, raw_max), 4) * 4))) return rc;
    const size_t scr = misort::codec_scratch_bytes(kmax) + 64;
    if ((rc = c->codec_scr.ensure(scr))) return rc;
    int64_t* d_sz = (int64_t*)c->small.p;  // [coded words, raw words] mine, then the partner's
    hipError_t e = w == 4 ? misort::codec_encode_dev<uint32_t>((const uint32_t*)base, run, kmax,
                                                               (uint32_t*)c->enc_send.p, c->codec_scr.p, scr, d_sz, s)
                          : misort::codec_encode_dev<uint64_t>((const uint64_t*)base, run, kmax,
                                                               (uint32_t*)c->enc_send.p, c->codec_scr.p, scr, d_sz, s);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "codec_encode: %s", hipGetErrorString(e));
    // every side sends whichever of coded and raw is smaller; the receiver tells
    // them apart by the size (coded < raw)
    std::vector<int64_t> all, m;
    const int me = c->rank;
    if (relayed) {
        if ((rc = relay_sizes(c, d_sz, all, m, s))) return rc;
    } else {
        // P = 2 (or no relay): the partner's pair by sendrecv, mine by copy
        all.assign((size_t)2 * c->nranks, 0);
        if ((rc = c->tr->sendrecv(d_sz, 16, d_sz + 2, 16, q, s))) return rc;
        if ((rc = fetch(c, s, {{&all[(size_t)2 * me], d_sz, 16}, {&all[(size_t)2 * q], d_sz + 2, 16}}))) return rc;
    }
    const int64_t raw_words = all[(size_t)2 * me + 1];
    const int64_t k = raw_words * 4 / (int64_t)w;
    // Both partners derive k from the same samples.  The check is collective:
    // a relayed stage hands every rank every pair's sizes, so every rank tests
    // every pair and all of them fail together; at P = 2 the two partners see
    // the same two values.
    const int bit = ilog2(q ^ me);
    for (int r = 0; r < c->nranks; ++r) {
        if (!relayed && r != me) continue;
        const int rq = r ^ (1 << bit);
        // pairs with an empty block exchange whole blocks raw in the same
        // relayed stage (relay_raw): their sizes legitimately differ
        if (r != me && !pair_coded(r, rq)) continue;
        if (all[(size_t)2 * rq + 1] != all[(size_t)2 * r + 1] || all[(size_t)2 * r + 1] < 0)
            return fail(MISORT_E_INVALID, "exchange count mismatch between ranks %d and %d (%lld vs %lld words)", r,
                        rq, (long long)all[(size_t)2 * r + 1], (long long)all[(size_t)2 * rq + 1]);
    }
    if (k < 0 || k > kmax)
        return fail(MISORT_E_INVALID, "exchange count %lld outside [0, %lld]", (long long)k, (long long)kmax);
    *k_out = k;
    auto units = [&](int r) { return std::min(all[(size_t)2 * r], all[(size_t)2 * r + 1]); };  // 4-byte words sent
    const bool use = all[(size_t)2 * me] < raw_words;
    // the raw message is the run itself: the keep-max side's bottom k keys, the
    // keep-min side's top k (run[0] on the device)
    const int64_t off = keep_max ? 0 : nloc - k;
    const void* msg = use ? c->enc_send.p : (const char*)base + (size_t)off * w;
    const size_t mbytes = (size_t)units(me) * 4;
    if (mbytes != (use ? (size_t)all[(size_t)2 * me] * 4 : (size_t)k * w))
        return fail(MISORT_E_INVALID, "coded message size");
    size_t rb = (size_t)units(q) * 4;
    if (rb > c->enc_recv.bytes) return fail(MISORT_E_CAPACITY, "coded message size");
    if (relayed) {
        size_t rb2 = 0;
        rc = relay_exchange(c, 4, ilog2(q ^ c->rank), msg, mbytes, c->enc_recv.p, c->enc_recv.bytes, s, &rb2, &m);
        if (!rc && rb2 != rb) return fail(MISORT_E_INVALID, "relay: partner size mismatch");
    } else if (k > 0) {
        rc = c->tr->sendrecv(msg, mbytes, c->enc_recv.p, rb, q, s);
    }
    if (rc) return rc;
    if (k == 0) return MISORT_OK;
    c->xchg_bytes += (int64_t)(mbytes + rb);
    c->xchg_raw_bytes += (int64_t)(2 * k * w);
    if ((int64_t)rb >= raw_words * 4) {  // sent uncoded
        *rkeys = c->enc_recv.p;
        return MISORT_OK;
    }
    e = w == 4 ? misort::codec_decode<uint32_t>((const uint32_t*)c->enc_recv.p, k, (uint32_t*)c->recv.p, s)
               : misort::codec_decode<uint64_t>((const uint32_t*)c->enc_recv.p, k, (uint64_t*)c->recv.p, s);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "codec_decode: %s", hipGetErrorString(e));
    *rkeys = c->recv.p;
    return MISORT_OK;
}

// io: optional chunked first/last pass (host staging).  Its after_last hook is
// used only when no exchange stage follows the local sort (P = 1); it then also
// owns the f64 back-conversion of each output chunk.
int parallel_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t loc,
                  int64_t max_size, hipStream_t s, const misort::StageIO* io = nullptr) {
    if (!valid_dtype(dtype)) return fail(MISORT_E_INVALID, "bad dtype %d", dtype);
    if (loc < 0) return fail(MISORT_E_INVALID, "negative loc_size %lld", (long long)loc);
    const int p = c->nranks;
    if (p & (p - 1)) return fail(MISORT_E_NOT_POW2, "bitonic sort requires 2^d processors");
    int rc;
    // (loc, max_size) of every rank.  The capacity check is collective: every
    // rank tests every block against the smallest max_size, so all ranks fail
    // together instead of some entering the exchange alone.  max_size <= 0
    // means "the largest block" (the reference's N/P+1 bound, psort.cc:557).
    const int64_t mine[2] = {loc, max_size};
    std::vector<int64_t> lm(mine, mine + 2);
    if (p > 1 && (rc = c->tr->allgather_i64(mine, 2, lm, s))) return rc;
    std::vector<int64_t> sizes(p);
    int64_t cap = INT64_MAX, big = 0;
    for (int r = 0; r < p; ++r) {
        sizes[r] = lm[2 * r];
        big = std::max(big, sizes[r]);
        if (lm[2 * r + 1] > 0) cap = std::min(cap, lm[2 * r + 1]);
    }
    if (cap == INT64_MAX) cap = big;
    for (int r = 0; r < p; ++r)
        if (sizes[r] > cap)
            return fail(MISORT_E_CAPACITY, "rank %d holds %lld keys > max_size %lld", r,
                        (long long)sizes[r], (long long)cap);
    int partner[64], keep[64];
    const int nst = misort_bitonic_schedule(p, c->rank, partner, keep);
    const size_t w = key_bytes(dtype);
    const bool f64 = dtype == MISORT_F64;
    void* work = nullptr;
    if (nst > 0) {
        int64_t maxp = 0, maxs = 0;
        for (int st = 0; st < nst; ++st) {
            maxp = std::max(maxp, sizes[partner[st]]);
            maxs = std::max(maxs, sample_count(sizes[partner[st]]));
        }
        if ((rc = c->work.ensure(std::max<size_t>(16, (size_t)loc * w)))) return rc;
        if ((rc = c->recv.ensure(std::max<size_t>(16, (size_t)maxp * w)))) return rc;
        if ((rc = c->samp_me.ensure(std::max<size_t>(16, (size_t)sample_count(loc) * w)))) return rc;
        if ((rc = c->samp_peer.ensure(std::max<size_t>(16, (size_t)maxs * w)))) return rc;
        work = c->work.p;
    }
    // The local sort writes where the stage parity leaves the result in `out`.
    void* cur = (nst & 1) ? work : out;
    misort::StageIO lio;
    const bool chunk_out = io && io->after_last && nst == 0;
    bool chunked = false;  // the local sort's last pass handed its output over chunk by chunk
    if (io) {
        lio = *io;
        if (!chunk_out) {
            lio.after_last = nullptr;
        } else {
            const auto after = io->after_last;
            lio.after_last = [&chunked, after](int64_t k0, int64_t k1, hipStream_t st) {
                chunked = true;
                return after(k0, k1, st);
            };
        }
    }
    // no compare-split after the local sort: its last pass writes f64 bits
    bool ord_done = f64 && nst == 0 && !chunk_out;
    if ((rc = do_local_sort(c, dtype, in, cur, loc, f64, s, io ? &lio : nullptr, ord_done))) return rc;
    if (chunk_out && chunked) return MISORT_OK;  // after_last owned the f64 back-conversion
    if (chunk_out) {
        // a last pass that is not chunked (a multi-way pass): the caller copies
        // the whole block out, converted here
        if (f64) HIPCHK(misort::ord_to_f64((uint64_t*)cur, loc, s));
        return MISORT_OK;
    }
    void* other = (cur == work) ? out : work;
    misort::LaunchHook* hk = hook(c);
    struct StageMark {  // attributes profiled launches to the hypercube stage
        Profiler& pr;
        StageMark(Profiler& p_, int st) : pr(p_) { pr.stage = st; }
        ~StageMark() { pr.stage = -1; }
    };
    for (int st = 0; st < nst; ++st) {
        StageMark mark(c->prof, st);
        // the exchange leg's profiler record, closed on every way out of the
        // stage (error returns included) so later records never nest in it
        struct XgRecord {
            misort::LaunchHook* hk;
            Profiler& pr;
            hipStream_t s;
            bool open;
            XgRecord(misort::LaunchHook* h, Profiler& p_, hipStream_t s_) : hk(h), pr(p_), s(s_), open(h != nullptr) {
                if (hk) hk->before(misort::KIND_EXCHANGE, 0.0, s);
            }
            void close(double bytes) {
                if (!open) return;
                pr.cur.bytes = bytes;
                hk->after(misort::KIND_EXCHANGE, s);
                open = false;
            }
            ~XgRecord() { close(0.0); }
        } xg(hk, c->prof, s);
        auto xg_close = [&](double bytes) { xg.close(bytes); };
        const int q = partner[st];
        const int64_t nq = sizes[q];
        const bool mx = keep[st] != 0;  // this rank keeps the upper part
        // min side = "A" (keeps its n_a smallest), max side = "B"
        const int64_t na = mx ? nq : loc, nb = mx ? loc : nq;
        int64_t k;  // keys each side sends: A's top k, B's bottom k
        const bool relayed = c->relay && p > 2;
        const void* rkeys = c->recv.p;
        const int64_t moved0 = c->xchg_bytes;
        if ((rc = c->small.ensure(kSmallBytes))) return rc;
        int64_t* d_run = (int64_t*)c->small.p + 4;  // {send offset, k} on the device
        // the codec's offsets and word totals are 32-bit: messages that could
        // reach 2^32 words go raw (both sides decide from the same bound)
        const int64_t kmax = std::min(na, nb);
        // the same rule for every pair of the stage (every rank knows every block size)
        auto pair_coded = [&](int r, int rq) {
            const int64_t km = std::min(sizes[r], sizes[rq]);
            return !c->full_exchange && km > 0 && c->compress && misort::codec_max_words(km, (int)w) < ((int64_t)1 << 32);
        };
        const bool coded = pair_coded(c->rank, q);
        if (!c->full_exchange && loc > 0 && nq > 0) {
            const int64_t cm = sample_count(loc), cq = sample_count(nq);
            hipError_t e = w == 4 ? misort::gather_samples<uint32_t>((const uint32_t*)cur, loc, sample_stride(loc),
                                                                     (uint32_t*)c->samp_me.p, cm, s)
                                  : misort::gather_samples<uint64_t>((const uint64_t*)cur, loc, sample_stride(loc),
                                                                     (uint64_t*)c->samp_me.p, cm, s);
            if (e != hipSuccess) return fail(MISORT_E_HIP, "gather_samples: %s", hipGetErrorString(e));
            if ((rc = c->tr->sendrecv(c->samp_me.p, (size_t)cm * w, c->samp_peer.p, (size_t)cq * w, q, s)))
                return rc;
        }
        c->xchg_stages += 1;
        c->xchg_full_bytes += (int64_t)((loc + nq) * w);
        if (coded) {
            // k on the device; the host learns it in the stage's one size exchange
            const void* sa = mx ? c->samp_peer.p : c->samp_me.p;
            const void* sb = mx ? c->samp_me.p : c->samp_peer.p;
            hipError_t e = w == 4 ? misort::exchange_count<uint32_t>((const uint32_t*)sa, na, (const uint32_t*)sb,
                                                                     nb, mx, loc, d_run, s)
                                  : misort::exchange_count<uint64_t>((const uint64_t*)sa, na, (const uint64_t*)sb,
                                                                     nb, mx, loc, d_run, s);
            if (e != hipSuccess) return fail(MISORT_E_HIP, "exchange_count: %s", hipGetErrorString(e));
            if ((rc = coded_exchange(c, dtype, q, relayed, cur, loc, mx, d_run, kmax, &k, &rkeys, s, pair_coded))) return rc;
            if (k == 0) {  // no key crosses: both blocks stay as they are
                xg_close(0.0);
                continue;
            }
            xg_close((double)(c->xchg_bytes - moved0));
            if (tail_bracket(c, k, loc)) {
                // a small bracket: rewrite only the end of the block it reaches
                if ((rc = do_merge_split_tail(c, dtype, cur, loc, rkeys, k, other, keep[st], s))) return rc;
                continue;
            }
            // the last stage, writing `out`: f64 bits straight from the merge
            const bool oo = f64 && st == nst - 1 && other == out;
            if ((rc = do_merge_split(c, dtype, cur, loc, rkeys, k, other, keep[st], s, oo))) return rc;
            ord_done = ord_done || oo;
            std::swap(cur, other);
            continue;
        }
        if (c->full_exchange || loc == 0 || nq == 0) {
            k = -1;
        } else {
            // raw exchange: k from the samples on the host
            const int64_t cm = sample_count(loc), cq = sample_count(nq);
            int64_t ilo;
            if (w == 4) {
                std::vector<uint32_t> me(cm), pe(cq);
                if ((rc = fetch(c, s, {{me.data(), c->samp_me.p, cm * w}, {pe.data(), c->samp_peer.p, cq * w}})))
                    return rc;
                ilo = mx ? corank_lower(pe, na, me, nb) : corank_lower(me, na, pe, nb);
            } else {
                std::vector<uint64_t> me(cm), pe(cq);
                if ((rc = fetch(c, s, {{me.data(), c->samp_me.p, cm * w}, {pe.data(), c->samp_peer.p, cq * w}})))
                    return rc;
                ilo = mx ? corank_lower(pe, na, me, nb) : corank_lower(me, na, pe, nb);
            }
            k = na - ilo;
        }
        if (k == 0) {  // no key crosses: both blocks stay as they are
            // relay units are 4 bytes on every rank of the stage (coded messages are words)
            if (relayed && (rc = relay_raw(c, ilog2(q ^ c->rank), cur, 0, c->recv.p, 0, s))) return rc;
            xg_close(0.0);
            continue;
        }
        // A sends its top k = A[na-k, na); B sends its bottom k = B[0, k)
        const void* sbuf;
        size_t sbytes, rbytes;
        int64_t nrecv;
        if (k < 0) {  // whole blocks, as MPI_Sendrecv does
            sbuf = cur;
            sbytes = (size_t)loc * w;
            rbytes = (size_t)nq * w;
            nrecv = nq;
        } else {
            sbuf = mx ? cur : (const char*)cur + (size_t)(loc - k) * w;
            sbytes = rbytes = (size_t)k * w;
            nrecv = k;
        }
        if (relayed) rc = relay_raw(c, ilog2(q ^ c->rank), sbuf, sbytes, c->recv.p, rbytes, s);
        else rc = c->tr->sendrecv(sbuf, sbytes, c->recv.p, rbytes, q, s);
        if (rc) return rc;
        c->xchg_bytes += (int64_t)(sbytes + rbytes);
        c->xchg_raw_bytes += (int64_t)(sbytes + rbytes);
        xg_close((double)(c->xchg_bytes - moved0));
        if (k > 0 && tail_bracket(c, k, loc)) {
            if ((rc = do_merge_split_tail(c, dtype, cur, loc, rkeys, nrecv, other, keep[st], s))) return rc;
            continue;
        }
        const bool oo = f64 && st == nst - 1 && other == out;
        if ((rc = do_merge_split(c, dtype, cur, loc, rkeys, nrecv, other, keep[st], s, oo))) return rc;
        ord_done = ord_done || oo;
        std::swap(cur, other);
    }
    if (f64 && !ord_done && loc > 0) {
        // one sweep: copy (skipped stages left the keys in `work`) and map back together
        HIPCHK(misort::ord_to_f64_copy((const uint64_t*)cur, (uint64_t*)out, loc, s));
    } else if (cur != out && loc > 0) {
        HIPCHK(hipMemcpyAsync(out, cur, (size_t)loc * w, hipMemcpyDeviceToDevice, s));
    }
    return MISORT_OK;
}

// psort.cc:377-490 parallel_quick_sort on the GPU: d rounds over shrinking
// hypercube sub-groups; each round takes the median of medians of the group as
// pivot and swaps the part below it (low half of the group) or at/above it
// (high half) with the partner rank.  The reference re-sorts the whole buffer
// each round (std::sort); the runs stay sorted here, so a device merge of the
// kept part and the received part gives the same sequence.
int parallel_quick(misort_ctx* c, int dtype, const void* in, int64_t loc, void* out, int64_t out_cap,
                   int64_t* out_n, hipStream_t s) {
    if (!valid_dtype(dtype)) return fail(MISORT_E_INVALID, "bad dtype %d", dtype);
    if (loc < 0) return fail(MISORT_E_INVALID, "negative loc_size");
    const int p = c->nranks;
    if (p & (p - 1)) return fail(MISORT_E_NOT_POW2, "Quick sort requires 2^d processors");  // psort.cc:378-382
    const size_t w = key_bytes(dtype);
    const bool f64 = dtype == MISORT_F64;
    int rc;
    if ((rc = c->qa.ensure(std::max<size_t>(16, (size_t)loc * w)))) return rc;
    if ((rc = c->qcnt.ensure(64))) return rc;
    if ((rc = do_local_sort(c, dtype, in, c->qa.p, loc, f64, s))) return rc;  // psort.cc:398
    int64_t rs = loc;
    uint64_t stale0 = 0;  // result_buffer[0] as last written: the median of an empty rank (psort.cc:399)
    auto key_at = [&](int64_t i, uint64_t& v) -> int {  // one key of the current run, to the host
        v = 0;
        return fetch(c, s, {{&v, (const char*)c->qa.p + (size_t)i * w, w}});
    };
    const int d = ilog2(p);
    for (int i = 0; i < d; ++i) {                       // psort.cc:389
        const int g = p >> i, half = g >> 1;            // new_comm_size (psort.cc:392-403)
        const int color = c->rank / g;                  // psort.cc:393
        const bool low = (c->rank % g) < half;          // my_new_id < my_partner (psort.cc:431)
        const int partner = c->rank ^ half;             // psort.cc:424
        uint64_t med = stale0;
        if (rs > 0) {
            if ((rc = key_at(0, stale0))) return rc;
            if ((rc = key_at(rs / 2, med))) return rc;  // my_median = result_buffer[rs/2] (psort.cc:399)
        }
        std::vector<int64_t> all(1, (int64_t)med);
        const int64_t mine = (int64_t)med;
        if (p > 1 && (rc = c->tr->allgather_i64(&mine, 1, all, s))) return rc;  // psort.cc:409-410
        std::vector<uint64_t> grp(all.begin() + (size_t)color * g, all.begin() + (size_t)color * g + g);
        std::sort(grp.begin(), grp.end());                                      // psort.cc:413
        const uint64_t pivot = grp[g / 2];                                      // psort.cc:414
        int64_t* dcnt = (int64_t*)c->qcnt.p;
        hipError_t e = w == 4 ? misort::lower_bound<uint32_t>((const uint32_t*)c->qa.p, rs, (uint32_t)pivot, dcnt, s)
                              : misort::lower_bound<uint64_t>((const uint64_t*)c->qa.p, rs, pivot, dcnt, s);
        if (e != hipSuccess) return fail(MISORT_E_HIP, "lower_bound: %s", hipGetErrorString(e));
        int64_t pi = 0;                                                         // psort.cc:417
        if ((rc = fetch(c, s, {{&pi, dcnt, 8}}))) return rc;
        // low half keeps [0, pi) and sends [pi, rs); high half keeps [pi, rs), sends [0, pi)
        const int64_t keep_off = low ? 0 : pi, keep_n = low ? pi : rs - pi;
        const int64_t send_off = low ? pi : 0, send_n = low ? rs - pi : pi;
        // MPI_Send/MPI_Recv + MPI_Get_count (psort.cc:438-471): counts first, then keys
        if ((rc = h2d(c, dcnt, &send_n, 8, s))) return rc;
        if ((rc = c->tr->sendrecv(dcnt, 8, dcnt + 1, 8, partner, s))) return rc;
        int64_t recv_n = 0;
        if ((rc = fetch(c, s, {{&recv_n, dcnt + 1, 8}}))) return rc;
        if ((rc = c->recv.ensure(std::max<size_t>(16, (size_t)recv_n * w)))) return rc;
        if ((rc = c->tr->sendrecv((const char*)c->qa.p + (size_t)send_off * w, (size_t)send_n * w, c->recv.p,
                                  (size_t)recv_n * w, partner, s)))
            return rc;
        const int64_t nn = keep_n + recv_n;
        if ((rc = c->qb.ensure(std::max<size_t>(16, (size_t)nn * w)))) return rc;
        if ((rc = c->scratch.ensure((size_t)((nn + 2047) / 2048 + 2) * sizeof(int64_t)))) return rc;
        const char* kp = (const char*)c->qa.p + (size_t)keep_off * w;
        e = w == 4 ? misort::merge_full<uint32_t>((const uint32_t*)kp, keep_n, (const uint32_t*)c->recv.p, recv_n,
                                                  (uint32_t*)c->qb.p, (int64_t*)c->scratch.p, s, hook(c))
                   : misort::merge_full<uint64_t>((const uint64_t*)kp, keep_n, (const uint64_t*)c->recv.p, recv_n,
                                                  (uint64_t*)c->qb.p, (int64_t*)c->scratch.p, s, hook(c));
        if (e != hipSuccess) return fail(MISORT_E_HIP, "merge: %s", hipGetErrorString(e));
        c->qa.swap(c->qb);
        rs = nn;
        c->xchg_stages += 1;
        c->xchg_bytes += (int64_t)((send_n + recv_n) * w);
    }
    *out_n = rs;                                                                // psort.cc:486
    if (rs > out_cap)
        return fail(MISORT_E_CAPACITY, "quick sort result of %lld keys exceeds the output capacity %lld",
                    (long long)rs, (long long)out_cap);
    if (rs > 0) HIPCHK(hipMemcpyAsync(out, c->qa.p, (size_t)rs * w, hipMemcpyDeviceToDevice, s));
    if (f64) HIPCHK(misort::ord_to_f64((uint64_t*)out, rs, s));
    return MISORT_OK;
}

// Sample sort (the reference's parallel_sample_{native,bitonic}_sort,
// psort.cc:203-375, redesigned for RCCL over xGMI): local sort, regular
// samples of every rank all-gathered, P-1 splitters taken as (key, rank,
// position) tuples so that duplicate keys still split evenly, ONE all-to-all-v
// in which every GPU pair uses its own link, a merge tree over the P received
// runs, and a small second all-to-all-v that moves the keys into the
// reference block layout (psort.cc:556-562).  The result is the globally
// sorted sequence in the caller's block sizes.
constexpr int kSamplesPerRank = 1024;

int parallel_sample(misort_ctx* c, int dtype, const void* in, void* out, int64_t loc, int64_t max_size,
                    hipStream_t s) {
    if (!valid_dtype(dtype)) return fail(MISORT_E_INVALID, "bad dtype %d", dtype);
    if (loc < 0 || (max_size > 0 && max_size < loc))
        return fail(MISORT_E_INVALID, "loc_size %lld > max_size %lld", (long long)loc, (long long)max_size);
    const int p = c->nranks, me = c->rank;
    const size_t w = key_bytes(dtype);
    const bool f64 = dtype == MISORT_F64;
    int rc;
    if ((rc = c->qa.ensure(std::max<size_t>(16, (size_t)loc * w)))) return rc;
    if ((rc = do_local_sort(c, dtype, in, c->qa.p, loc, f64, s))) return rc;
    if (p == 1) {
        if (loc > 0) HIPCHK(hipMemcpyAsync(out, c->qa.p, (size_t)loc * w, hipMemcpyDeviceToDevice, s));
        if (f64) HIPCHK(misort::ord_to_f64((uint64_t*)out, loc, s));
        return MISORT_OK;
    }
    std::vector<int64_t> sizes;
    if ((rc = c->tr->allgather_i64(&loc, 1, sizes, s))) return rc;
    // regular samples a[j*S] of the sorted block, with their positions
    const int M = kSamplesPerRank;
    const int64_t S = std::max<int64_t>(1, (loc + M - 1) / M);
    const int64_t cnt = loc > 0 ? (loc + S - 1) / S : 0;
    if ((rc = c->samp_me.ensure((size_t)M * 8 + 16))) return rc;
    std::vector<int64_t> mine(2 * (size_t)M, -1);
    if (cnt > 0) {
        hipError_t e = w == 4 ? misort::gather_samples<uint32_t>((const uint32_t*)c->qa.p, loc, S,
                                                                 (uint32_t*)c->samp_me.p, cnt, s)
                              : misort::gather_samples<uint64_t>((const uint64_t*)c->qa.p, loc, S,
                                                                 (uint64_t*)c->samp_me.p, cnt, s);
        if (e != hipSuccess) return fail(MISORT_E_HIP, "gather_samples: %s", hipGetErrorString(e));
        std::vector<unsigned char> raw((size_t)cnt * w);
        if ((rc = fetch(c, s, {{raw.data(), c->samp_me.p, raw.size()}}))) return rc;
        for (int64_t j = 0; j < cnt; ++j) {
            uint64_t v = 0;
            memcpy(&v, &raw[(size_t)j * w], w);
            mine[2 * j] = (int64_t)v;
            mine[2 * j + 1] = j * S;
        }
    }
    std::vector<int64_t> all;
    if ((rc = c->tr->allgather_i64(mine.data(), 2 * M, all, s))) return rc;
    struct Tup {
        uint64_t v;
        int r;
        int64_t pos;
        bool operator<(const Tup& o) const {
            return v != o.v ? v < o.v : r != o.r ? r < o.r : pos < o.pos;
        }
    };
    std::vector<Tup> tup;
    for (int r = 0; r < p; ++r)
        for (int j = 0; j < M; ++j) {
            const int64_t pos = all[((size_t)r * M + j) * 2 + 1];
            if (pos >= 0) tup.push_back(Tup{(uint64_t)all[((size_t)r * M + j) * 2], r, pos});
        }
    std::sort(tup.begin(), tup.end());
    // split points of this block for the P-1 splitters
    std::vector<int64_t> split(p + 1, 0);
    split[p] = loc;
    const int ns = p - 1;
    if (!tup.empty() && loc > 0) {
        std::vector<Tup> sp(ns);
        std::vector<unsigned char> vals((size_t)ns * w);
        for (int j = 1; j < p; ++j) {
            sp[j - 1] = tup[(size_t)j * tup.size() / p];
            memcpy(&vals[(size_t)(j - 1) * w], &sp[j - 1].v, w);
        }
        if ((rc = c->samp_peer.ensure(vals.size() + 16))) return rc;
        if ((rc = c->qcnt.ensure((size_t)ns * 16 + 64))) return rc;
        int64_t* dlb = (int64_t*)c->qcnt.p;
        int64_t* dub = dlb + ns;
        if ((rc = h2d(c, c->samp_peer.p, vals.data(), vals.size(), s))) return rc;
        hipError_t e = w == 4 ? misort::bounds<uint32_t>((const uint32_t*)c->qa.p, loc, (const uint32_t*)c->samp_peer.p,
                                                         ns, dlb, dub, s)
                              : misort::bounds<uint64_t>((const uint64_t*)c->qa.p, loc, (const uint64_t*)c->samp_peer.p,
                                                         ns, dlb, dub, s);
        if (e != hipSuccess) return fail(MISORT_E_HIP, "bounds: %s", hipGetErrorString(e));
        std::vector<int64_t> lbub(2 * (size_t)ns);
        if ((rc = fetch(c, s, {{lbub.data(), dlb, lbub.size() * 8}}))) return rc;
        for (int j = 1; j < p; ++j) {
            const Tup& t = sp[j - 1];
            // keys of this rank below the tuple (key, rank, position) in (key, rank, position) order
            int64_t x = me < t.r ? lbub[ns + j - 1] : me > t.r ? lbub[j - 1] : t.pos;
            split[j] = std::max(split[j - 1], std::min(x, loc));
        }
    } else if (loc > 0) {
        for (int j = 1; j < p; ++j) split[j] = 0;  // no samples anywhere: everything to the last rank
    }
    std::vector<int64_t> scnt(p), soff(p), rcnt(p), roff(p), kc(p);
    for (int q = 0; q < p; ++q) {
        kc[q] = split[q + 1] - split[q];
        soff[q] = split[q] * (int64_t)w;
        scnt[q] = kc[q] * (int64_t)w;
    }
    std::vector<int64_t> mat;
    if ((rc = c->tr->allgather_i64(kc.data(), p, mat, s))) return rc;
    int64_t nrecv = 0;
    for (int q = 0; q < p; ++q) {
        rcnt[q] = mat[(size_t)q * p + me] * (int64_t)w;
        roff[q] = nrecv * (int64_t)w;
        nrecv += mat[(size_t)q * p + me];
    }
    if ((rc = c->recv.ensure(std::max<size_t>(16, (size_t)nrecv * w)))) return rc;
    if ((rc = c->qb.ensure(std::max<size_t>(16, (size_t)nrecv * w)))) return rc;
    if ((rc = c->tr->alltoallv(c->qa.p, soff.data(), scnt.data(), c->recv.p, roff.data(), rcnt.data(), s)))
        return rc;
    c->xchg_stages += 1;
    c->xchg_bytes += (int64_t)(loc * w - scnt[me] + nrecv * w - rcnt[me]);
    // merge tree over the P runs (adjacent pairs keep their place, buffers alternate)
    std::vector<int64_t> ro(p), rn(p);
    for (int q = 0; q < p; ++q) {
        ro[q] = roff[q] / (int64_t)w;
        rn[q] = rcnt[q] / (int64_t)w;
    }
    char* src = (char*)c->recv.p;
    char* dst = (char*)c->qb.p;
    if ((rc = c->scratch.ensure((size_t)((nrecv + 2047) / 2048 + p + 2) * sizeof(int64_t)))) return rc;
    while (ro.size() > 1) {
        std::vector<int64_t> no, nn;
        for (size_t i = 0; i < ro.size(); i += 2) {
            if (i + 1 == ro.size()) {
                if (rn[i]) HIPCHK(hipMemcpyAsync(dst + ro[i] * w, src + ro[i] * w, (size_t)rn[i] * w,
                                                 hipMemcpyDeviceToDevice, s));
                no.push_back(ro[i]);
                nn.push_back(rn[i]);
                continue;
            }
            hipError_t e = w == 4
                ? misort::merge_full<uint32_t>((const uint32_t*)(src + ro[i] * w), rn[i],
                                               (const uint32_t*)(src + ro[i + 1] * w), rn[i + 1],
                                               (uint32_t*)(dst + ro[i] * w), (int64_t*)c->scratch.p, s, hook(c))
                : misort::merge_full<uint64_t>((const uint64_t*)(src + ro[i] * w), rn[i],
                                               (const uint64_t*)(src + ro[i + 1] * w), rn[i + 1],
                                               (uint64_t*)(dst + ro[i] * w), (int64_t*)c->scratch.p, s, hook(c));
            if (e != hipSuccess) return fail(MISORT_E_HIP, "merge: %s", hipGetErrorString(e));
            no.push_back(ro[i]);
            nn.push_back(rn[i] + rn[i + 1]);
        }
        ro.swap(no);
        rn.swap(nn);
        std::swap(src, dst);
    }
    // the reference block layout: keys at global ranks [T_q, T_q + sizes[q]) go to rank q
    std::vector<int64_t> have;
    if ((rc = c->tr->allgather_i64(&nrecv, 1, have, s))) return rc;
    int64_t A = 0, Tme = 0;
    for (int q = 0; q < me; ++q) {
        A += have[q];
        Tme += sizes[q];
    }
    int64_t Tq = 0, Aq = 0;
    for (int q = 0; q < p; ++q) {
        const int64_t s0 = std::max(A, Tq), s1 = std::min(A + nrecv, Tq + sizes[q]);
        soff[q] = (s1 > s0 ? s0 - A : 0) * (int64_t)w;
        scnt[q] = (s1 > s0 ? s1 - s0 : 0) * (int64_t)w;
        const int64_t r0 = std::max(Aq, Tme), r1 = std::min(Aq + have[q], Tme + loc);
        roff[q] = (r1 > r0 ? r0 - Tme : 0) * (int64_t)w;
        rcnt[q] = (r1 > r0 ? r1 - r0 : 0) * (int64_t)w;
        Tq += sizes[q];
        Aq += have[q];
    }
    if ((rc = c->tr->alltoallv(src, soff.data(), scnt.data(), out, roff.data(), rcnt.data(), s))) return rc;
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
    delete c->tr;
    c->tr = nullptr;
    if (c->pinned) (void)hipHostFree(c->pinned);
    if (c->stream) {
        misort::mergek_release(c->stream);  // the merge passes' scratch for this stream
        misort::mergek_release_fg6(c->stream);
        (void)hipStreamDestroy(c->stream);
    }
    delete c;
    return MISORT_OK;
}

void* misort_stream(misort_ctx* c) { return c ? (void*)c->stream : nullptr; }

int misort_synchronize(misort_ctx* c) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    int rc = sync(c, c->stream);
    return rc ? rc : planning_check(c->stream);
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
    delete c->tr;
    c->tr = nullptr;
    c->nranks = 1;
    c->rank = 0;
    if (nranks > 1) {
        auto* t = new RcclTransport();
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        t->dog.arm("ncclCommInitRank");  // all ranks must join within the deadline
        ncclResult_t r = ncclCommInitRank(&t->comm, nranks, u, rank);
        t->dog.disarm();
        if (r != ncclSuccess) {
            delete t;
            return fail(MISORT_E_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
        }
        t->nranks = nranks;
        t->rank = rank;
        const int rc = t->connect_all(c->stream);
        if (rc) {
            delete t;
            return rc;
        }
        c->tr = t;
    }
    c->nranks = nranks;
    c->rank = rank;
    return MISORT_OK;
}

int misort_group_create(int nranks, misort_group** out) try {
    if (!out || nranks < 1) return fail(MISORT_E_INVALID, "bad group arguments");
    if (nranks & (nranks - 1)) return fail(MISORT_E_NOT_POW2, "bitonic sort requires 2^d processors");
    *out = new misort_group(nranks);
    return MISORT_OK;
} catch (const std::bad_alloc&) {
    return fail(MISORT_E_INVALID, "out of host memory");
}

int misort_group_destroy(misort_group* g) {
    delete g;
    return MISORT_OK;
}

int misort_comm_init_group(misort_ctx* c, misort_group* g, int rank) {
    if (!c || !g || rank < 0 || rank >= g->n) return fail(MISORT_E_INVALID, "bad group rank");
    HIPCHK(hipSetDevice(c->device));
    delete c->tr;
    c->tr = nullptr;
    auto* t = new LocalTransport();
    t->g = g;
    t->nranks = g->n;
    t->rank = rank;
    t->epoch.assign(g->n, 0);
    auto& slot = g->slots[rank];
    if (hipEventCreateWithFlags(&slot.ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&slot.done, hipEventDisableTiming) != hipSuccess) {
        delete t;
        return fail(MISORT_E_HIP, "hipEventCreate failed");
    }
    c->tr = t;
    c->nranks = g->n;
    c->rank = rank;
    return MISORT_OK;
}

int64_t misort_sample_stride(int64_t n) { return n < 0 ? MISORT_E_INVALID : sample_stride(n); }
int64_t misort_sample_count(int64_t n) { return n < 0 ? MISORT_E_INVALID : sample_count(n); }

int64_t misort_exchange_count(int dtype, const void* samples_min, int64_t n_min, const void* samples_max,
                              int64_t n_max) {
    if (!valid_dtype(dtype) || n_min < 0 || n_max < 0) return fail(MISORT_E_INVALID, "bad exchange args");
    if (n_min == 0 || n_max == 0) return -1;  // whole (possibly empty) blocks
    const int64_t ca = sample_count(n_min), cb = sample_count(n_max);
    int64_t ilo;
    if (dtype == MISORT_U32) {
        std::vector<uint32_t> a((const uint32_t*)samples_min, (const uint32_t*)samples_min + ca);
        std::vector<uint32_t> b((const uint32_t*)samples_max, (const uint32_t*)samples_max + cb);
        ilo = corank_lower(a, n_min, b, n_max);
    } else {
        // u64 keys, or f64 keys already mapped to order-preserving u64
        std::vector<uint64_t> a((const uint64_t*)samples_min, (const uint64_t*)samples_min + ca);
        std::vector<uint64_t> b((const uint64_t*)samples_max, (const uint64_t*)samples_max + cb);
        ilo = corank_lower(a, n_min, b, n_max);
    }
    return n_min - ilo;
}

int misort_set_relay(misort_ctx* c, int on) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    c->relay = on != 0;
    return MISORT_OK;
}

int misort_codec_probe(misort_ctx* c, int dtype, const void* keys, int64_t n, int reps, float* enc_ms,
                       float* dec_ms, int64_t* coded_bytes, void* decoded) {
    if (!c || (dtype != MISORT_U32 && dtype != MISORT_U64) || n <= 0 || !keys || reps < 1)
        return fail(MISORT_E_INVALID, "bad codec_probe arguments");
    const size_t w = key_bytes(dtype);
    int rc;
    if ((rc = c->enc_send.ensure((size_t)misort::codec_max_words(n, (int)w) * 4))) return rc;
    const size_t scr = misort::codec_scratch_bytes(n) + 64;
    if ((rc = c->codec_scr.ensure(scr))) return rc;
    if ((rc = c->small.ensure(kSmallBytes))) return rc;
    if ((rc = c->recv.ensure((size_t)n * w))) return rc;
    void* out = decoded ? decoded : c->recv.p;
    hipStream_t s = c->stream;
    hipEvent_t e0, e1, e2;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventCreate(&e2));
    hipError_t e = hipSuccess;
    auto enc = [&] {
        return w == 4 ? misort::codec_encode<uint32_t>((const uint32_t*)keys, n, (uint32_t*)c->enc_send.p,
                                                      c->codec_scr.p, scr, (int64_t*)c->small.p, s)
                      : misort::codec_encode<uint64_t>((const uint64_t*)keys, n, (uint32_t*)c->enc_send.p,
                                                      c->codec_scr.p, scr, (int64_t*)c->small.p, s);
    };
    auto dec = [&] {
        return w == 4 ? misort::codec_decode<uint32_t>((const uint32_t*)c->enc_send.p, n, (uint32_t*)out, s)
                      : misort::codec_decode<uint64_t>((const uint32_t*)c->enc_send.p, n, (uint64_t*)out, s);
    };
    e = enc();
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    for (int i = 0; i < reps && e == hipSuccess; ++i) e = enc();
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    for (int i = 0; i < reps && e == hipSuccess; ++i) e = dec();
    if (e == hipSuccess) e = hipEventRecord(e2, s);
    if (e == hipSuccess) e = hipEventSynchronize(e2);
    int64_t words = 0;
    if (e == hipSuccess) e = hipMemcpy(&words, c->small.p, 8, hipMemcpyDeviceToHost);
    if (e == hipSuccess && enc_ms) e = hipEventElapsedTime(enc_ms, e0, e1);
    if (e == hipSuccess && dec_ms) e = hipEventElapsedTime(dec_ms, e1, e2);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipEventDestroy(e2);
    HIPCHK(e);
    if (enc_ms) *enc_ms /= reps;
    if (dec_ms) *dec_ms /= reps;
    if (coded_bytes) *coded_bytes = words * 4;
    return MISORT_OK;
}

int misort_set_compress(misort_ctx* c, int on) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    c->compress = on != 0;
    return MISORT_OK;
}

int misort_exchange_raw_bytes(misort_ctx* c, int64_t* raw_bytes) {
    if (!c || !raw_bytes) return fail(MISORT_E_INVALID, "null argument");
    *raw_bytes = c->xchg_raw_bytes;
    c->xchg_raw_bytes = 0;
    return MISORT_OK;
}

int misort_set_full_exchange(misort_ctx* c, int on) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    c->full_exchange = on != 0;
    return MISORT_OK;
}

int misort_exchange_stats(misort_ctx* c, int64_t* stages, int64_t* bytes, int64_t* full_bytes) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    if (stages) *stages = c->xchg_stages;
    if (bytes) *bytes = c->xchg_bytes;
    if (full_bytes) *full_bytes = c->xchg_full_bytes;
    c->xchg_stages = c->xchg_bytes = c->xchg_full_bytes = 0;
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
    // f64: mapped to ordered u64 by the first pass, back by the last
    return do_local_sort(c, dtype, in, out, n, dtype == MISORT_F64, s, nullptr, dtype == MISORT_F64);
}

int misort_pass_probe(misort_ctx* c, int dtype, const void* in, void* out, int64_t n, int kind, int hi,
                      int r, int flip, int reps, float* ms) {
    if (!c || (dtype != MISORT_U32 && dtype != MISORT_U64) || n <= 0 || !in || !out || in == out || reps < 1 || !ms)
        return fail(MISORT_E_INVALID, "bad pass_probe arguments");
    if (kind != misort::KIND_TILE_SORT && kind != misort::KIND_RUNS && kind != misort::KIND_RUNSK)
        return fail(MISORT_E_INVALID, "bad pass kind");
    hipStream_t s = c->stream;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    hipError_t err = hipSuccess;
    auto run = [&](const void* a, void* b) {
        return dtype == MISORT_U32
                   ? misort::run_pass<uint32_t>((const uint32_t*)a, (uint32_t*)b, n, kind, hi, r, flip, s)
                   : misort::run_pass<uint64_t>((const uint64_t*)a, (uint64_t*)b, n, kind, hi, r, flip, s);
    };
    err = run(in, out);  // warm-up (and argument check)
    if (err == hipSuccess) err = hipEventRecord(e0, s);
    for (int i = 0; i < reps && err == hipSuccess; ++i) err = (i & 1) ? run(out, (void*)in) : run(in, out);
    if (err == hipSuccess) err = hipEventRecord(e1, s);
    if (err == hipSuccess) err = hipEventSynchronize(e1);
    if (err == hipSuccess) err = hipEventElapsedTime(ms, e0, e1);
    if (err == hipSuccess) *ms /= reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (err == hipErrorInvalidValue) return fail(MISORT_E_INVALID, "pass shape does not fit n");
    HIPCHK(err);
    return MISORT_OK;
}

int misort_parallel_bitonic_sort_oop(misort_ctx* c, int dtype, const void* in, void* out,
                                     int64_t loc, int64_t max_size, void* stream) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    if (c->nranks > 1 && !c->tr) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    if (loc > 0 && (!in || !out)) return fail(MISORT_E_INVALID, "null buffer");
    const uint64_t calls0 = c->tr ? c->tr->calls : 0;
    return collective_result(c, calls0, parallel_sort(c, dtype, in, out, loc, max_size, pick(c, stream)));
}

int misort_parallel_bitonic_sort(misort_ctx* c, int dtype, void* keys, int64_t loc,
                                 int64_t max_size, void* stream) {
    return misort_parallel_bitonic_sort_oop(c, dtype, keys, keys, loc, max_size, stream);
}

int misort_parallel_quick_sort(misort_ctx* c, int dtype, const void* in, int64_t loc, void* out,
                               int64_t out_capacity, int64_t* out_size, void* stream) {
    if (!c || !out_size) return fail(MISORT_E_INVALID, "null argument");
    if (c->nranks > 1 && !c->tr) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    if ((loc > 0 && !in) || (out_capacity > 0 && !out)) return fail(MISORT_E_INVALID, "null buffer");
    const uint64_t calls0 = c->tr ? c->tr->calls : 0;
    return collective_result(c, calls0, parallel_quick(c, dtype, in, loc, out, out_capacity, out_size, pick(c, stream)));
}

int misort_parallel_sample_sort(misort_ctx* c, int dtype, const void* in, void* out, int64_t loc,
                                int64_t max_size, void* stream) {
    if (!c) return fail(MISORT_E_INVALID, "null ctx");
    if (c->nranks > 1 && !c->tr) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    if (loc > 0 && (!in || !out)) return fail(MISORT_E_INVALID, "null buffer");
    if (in == out && loc > 0) return fail(MISORT_E_INVALID, "sample sort is out of place (d_in != d_out)");
    const uint64_t calls0 = c->tr ? c->tr->calls : 0;
    return collective_result(c, calls0, parallel_sample(c, dtype, in, out, loc, max_size, pick(c, stream)));
}

int misort_merge_split(misort_ctx* c, int dtype, const void* local, int64_t nloc, const void* recv,
                       int64_t nrecv, void* out, int keep_max, void* stream) {
    if (!c || !valid_dtype(dtype) || nloc < 0 || nrecv < 0)
        return fail(MISORT_E_INVALID, "bad merge_split arguments");
    hipStream_t s = pick(c, stream);
    if (dtype != MISORT_F64) return do_merge_split(c, dtype, local, nloc, recv, nrecv, out, keep_max, s);
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

int misort_merge_split_tail(misort_ctx* c, int dtype, void* block, int64_t nblock, const void* recv, int64_t nrecv,
                            int keep_max, void* stream) {
    if (!c || !valid_dtype(dtype) || nblock < 0 || nrecv < 0 || (nblock > 0 && !block) || (nrecv > 0 && !recv))
        return fail(MISORT_E_INVALID, "bad merge_split_tail arguments");
    if (nblock > 0 && nrecv > 0) {
        // the received run must not overlap the block rewritten in place
        const char *b0 = (const char*)block, *b1 = b0 + nblock * key_bytes(dtype);
        const char *r0 = (const char*)recv, *r1 = r0 + nrecv * key_bytes(dtype);
        if (r0 < b1 && b0 < r1) return fail(MISORT_E_INVALID, "merge_split_tail: recv overlaps the block");
    }
    if (nblock == 0) return MISORT_OK;
    hipStream_t s = pick(c, stream);
    int rc;
    // the staging buffer: the context's work buffer (a block's worth)
    if ((rc = c->work.ensure((size_t)nblock * key_bytes(dtype)))) return rc;
    if (dtype != MISORT_F64) return do_merge_split_tail(c, dtype, block, nblock, recv, nrecv, c->work.p, keep_max, s);
    // f64 (the ordered form the hypercube stages merge in): the block mapped
    // in place, the received keys as an ordered copy, mapped back after
    if ((rc = c->recv.ensure(std::max<size_t>(8, (size_t)nrecv * 8)))) return rc;
    HIPCHK(hipMemcpyAsync(c->recv.p, recv, (size_t)nrecv * 8, hipMemcpyDeviceToDevice, s));
    HIPCHK(misort::f64_to_ord((uint64_t*)block, nblock, s));
    HIPCHK(misort::f64_to_ord((uint64_t*)c->recv.p, nrecv, s));
    if ((rc = do_merge_split_tail(c, dtype, block, nblock, c->recv.p, nrecv, c->work.p, keep_max, s))) return rc;
    HIPCHK(misort::ord_to_f64((uint64_t*)block, nblock, s));
    return MISORT_OK;
}

int misort_check_sort(misort_ctx* c, int dtype, const void* keys, int64_t n, int64_t* errors,
                      void* stream) {
    if (!c || !valid_dtype(dtype) || n < 0 || !errors) return fail(MISORT_E_INVALID, "bad check args");
    if (c->nranks > 1 && !c->tr) return fail(MISORT_E_NO_COMM, "communicator not initialised");
    hipStream_t s = pick(c, stream);
    const int p = c->nranks;
    // Per rank: {local descents, n, first key bits, last key bits}.
    int rc = c->small.ensure(kSmallBytes);
    if (rc) return rc;
    uint64_t* mine = (uint64_t*)c->small.p;
    HIPCHK(hipMemsetAsync(mine, 0, sizeof(uint64_t) * 4, s));
    hipError_t e = hipSuccess;
    if (dtype == MISORT_U32) e = misort::count_descents<uint32_t>((const uint32_t*)keys, n, (unsigned long long*)mine, s);
    else if (dtype == MISORT_U64) e = misort::count_descents<uint64_t>((const uint64_t*)keys, n, (unsigned long long*)mine, s);
    else e = misort::count_descents<double>((const double*)keys, n, (unsigned long long*)mine, s);
    if (e != hipSuccess) return fail(MISORT_E_HIP, "count_descents: %s", hipGetErrorString(e));
    // (n itself is set on the host after the fetch: a copy from pageable
    // memory behind a pending transfer would block with no deadline)
    const size_t w = key_bytes(dtype);
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(mine + 2, keys, w, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(mine + 3, (const char*)keys + (size_t)(n - 1) * w, w, hipMemcpyDeviceToDevice, s));
    }
    // ... and a fifth word: this rank's merge passes rejected a chunk (gathered
    // with the rest, so every rank reports it together)
    int64_t four[5];
    if ((rc = fetch(c, s, {{four, mine, 4 * sizeof(int64_t)}}))) return rc;
    four[1] = n;
    const int perr = planning_check(s);
    if (perr == MISORT_E_HIP) {
        // this rank cannot take part in the gather: abort the communicator so
        // the peers fail now instead of waiting out their deadline
        if (p > 1) {
            const std::string why = g_err;
            c->tr->abort_all(why.c_str());
            g_err = why;
        }
        return perr;
    }
    four[4] = perr != MISORT_OK;
    std::vector<int64_t> alli(four, four + 5);
    if (p > 1) {
        const uint64_t calls0 = c->tr->calls;
        if ((rc = c->tr->allgather_i64(four, 5, alli, s))) return collective_result(c, calls0, rc);
    }
    for (int r = 0; r < p; ++r)
        if (alli[5 * (size_t)r + 4])
            return fail(MISORT_E_INTERNAL, "rank %d: a merge pass rejected its chunk bounds (incomplete output)", r);
    std::vector<uint64_t> all;
    for (int r = 0; r < p; ++r) all.insert(all.end(), alli.begin() + 5 * (size_t)r, alli.begin() + 5 * (size_t)r + 4);
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

// Host staging: keys travel host <-> HBM in chunks through a ring of pinned
// buffers, overlapped with the sort:
//   in:  host memcpy of chunk i into a pinned slot (several threads) | DMA of
//        chunk i-1 on the copy stream | SORT pass of chunk i-2 on the sort
//        stream (tile-local, so it starts as soon as its chunk has landed);
//   out: (P = 1) the final MERGE pass and the f64 back-conversion run chunk by
//        chunk, each chunk's D2H and host copy overlapping the next chunk;
//        (P > 1) chunked D2H after the last compare-split.
// MISORT_STAGE_CHUNK sets the chunk (keys, rounded to the tile; default 2^24).
namespace {

void par_memcpy(void* dst, const void* src, size_t bytes) {
    static const int T = [] {
        const char* e = getenv("MISORT_STAGE_THREADS");
        int t = e ? atoi(e) : 8;
        return t < 1 ? 1 : t > 64 ? 64 : t;
    }();
    const size_t MIN = (size_t)4 << 20;  // below this, one thread
    if (T == 1 || bytes < 2 * MIN) {
        memcpy(dst, src, bytes);
        return;
    }
    int t = (int)std::min<size_t>((size_t)T, bytes / MIN);
    const size_t part = (bytes / t + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (int i = 1; i < t; ++i) {
        const size_t o = (size_t)i * part;
        if (o >= bytes) break;
        th.emplace_back([=] { memcpy((char*)dst + o, (const char*)src + o, std::min(part, bytes - o)); });
    }
    memcpy(dst, src, std::min(part, bytes));
    for (auto& x : th) x.join();
}

int64_t stage_chunk(int dtype) {
    const char* e = getenv("MISORT_STAGE_CHUNK");
    int64_t ch = e ? atoll(e) : ((int64_t)1 << 24);
    const int64_t tile = (int64_t)1 << misort::tile_log2((int)key_bytes(dtype));
    if (ch < tile) ch = tile;
    return (ch + tile - 1) / tile * tile;
}

int ring_ensure(misort_ctx* c, size_t bytes) {
    if (!c->copy_stream) HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (int i = 0; i < misort_ctx::RING; ++i) {
        if (!c->ring_ev[i]) HIPCHK(hipEventCreateWithFlags(&c->ring_ev[i], hipEventDisableTiming));
        c->ring_busy[i] = false;
    }
    if (bytes <= c->ring_bytes) return MISORT_OK;
    for (int i = 0; i < misort_ctx::RING; ++i) {
        if (c->ring[i]) HIPCHK(hipHostFree(c->ring[i]));
        c->ring[i] = nullptr;
    }
    c->ring_bytes = 0;
    for (int i = 0; i < misort_ctx::RING; ++i) HIPCHK(hipHostMalloc(&c->ring[i], bytes, hipHostMallocDefault));
    c->ring_bytes = bytes;
    return MISORT_OK;
}

// Output side: chunk [k0, k1) of dev (ready in stream order on `s`) -> host.
struct OutPipe {
    misort_ctx* c;
    const char* dev;
    char* host;
    size_t w;
    int next = 0;
    int64_t pend_k0[misort_ctx::RING] = {}, pend_k1[misort_ctx::RING] = {};
    int drain(int slot) {
        if (!c->ring_busy[slot]) return MISORT_OK;
        HIPCHK(hipEventSynchronize(c->ring_ev[slot]));
        par_memcpy(host + pend_k0[slot] * w, c->ring[slot], (size_t)(pend_k1[slot] - pend_k0[slot]) * w);
        c->ring_busy[slot] = false;
        return MISORT_OK;
    }
    int push(int64_t k0, int64_t k1, hipStream_t s) {
        const int slot = next;
        next = (next + 1) % misort_ctx::RING;
        int rc = drain(slot);
        if (rc) return rc;
        HIPCHK(hipMemcpyAsync(c->ring[slot], dev + k0 * w, (size_t)(k1 - k0) * w, hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(c->ring_ev[slot], s));
        c->ring_busy[slot] = true;
        pend_k0[slot] = k0;
        pend_k1[slot] = k1;
        return MISORT_OK;
    }
    int finish() {
        for (int i = 0; i < misort_ctx::RING; ++i) {
            const int slot = (next + i) % misort_ctx::RING;
            int rc = drain(slot);
            if (rc) return rc;
        }
        return MISORT_OK;
    }
};

}  // namespace

int misort_sort_host(misort_ctx* c, int dtype, const void* h_in, void* h_out, int64_t loc,
                     int64_t max_size) {
    if (!c || !valid_dtype(dtype) || loc < 0 || (loc > 0 && (!h_in || !h_out)))
        return fail(MISORT_E_INVALID, "bad sort_host arguments");
    if (max_size > 0 && loc > max_size)
        return fail(MISORT_E_INVALID, "loc_size %lld > max_size %lld", (long long)loc, (long long)max_size);
    const size_t w = key_bytes(dtype);
    const int64_t ch = stage_chunk(dtype);
    int rc = c->host_keys.ensure(std::max<size_t>((size_t)std::max<int64_t>(loc, 1) * w, 64));
    if (rc) return rc;
    if ((rc = ring_ensure(c, (size_t)std::min<int64_t>(std::max<int64_t>(loc, 1), ch) * w))) return rc;
    char* dev = (char*)c->host_keys.p;
    hipStream_t s = c->stream, cs = c->copy_stream;
    int in_next = 0;
    misort::StageIO io;
    io.chunk = ch;
    io.before_first = [&](int64_t k0, int64_t k1, hipStream_t st) -> int {
        const int slot = in_next;
        in_next = (in_next + 1) % misort_ctx::RING;
        if (c->ring_busy[slot]) HIPCHK(hipEventSynchronize(c->ring_ev[slot]));
        const size_t bytes = (size_t)(k1 - k0) * w;
        par_memcpy(c->ring[slot], (const char*)h_in + k0 * w, bytes);
        HIPCHK(hipMemcpyAsync(dev + k0 * w, c->ring[slot], bytes, hipMemcpyHostToDevice, cs));
        HIPCHK(hipEventRecord(c->ring_ev[slot], cs));
        c->ring_busy[slot] = true;
        HIPCHK(hipStreamWaitEvent(st, c->ring_ev[slot], 0));
        return MISORT_OK;
    };
    OutPipe op{c, dev, (char*)h_out, w};
    bool staged_out = false;
    io.after_last = [&](int64_t k0, int64_t k1, hipStream_t st) -> int {
        if (!staged_out) {  // the input side is done with the ring
            for (int i = 0; i < misort_ctx::RING; ++i)
                if (c->ring_busy[i]) {
                    HIPCHK(hipEventSynchronize(c->ring_ev[i]));
                    c->ring_busy[i] = false;
                }
            staged_out = true;
        }
        if (dtype == MISORT_F64) HIPCHK(misort::ord_to_f64((uint64_t*)(dev + k0 * w), k1 - k0, st));
        return op.push(k0, k1, st);
    };
    const uint64_t calls0 = c->tr ? c->tr->calls : 0;
    if (loc == 0) return collective_result(c, calls0, parallel_sort(c, dtype, dev, dev, 0, max_size, s));
    if ((rc = parallel_sort(c, dtype, dev, dev, loc, max_size, s, &io))) return collective_result(c, calls0, rc);
    if (!staged_out) {
        // P > 1 (or a plan whose last pass is not contiguous): chunked D2H now
        for (int i = 0; i < misort_ctx::RING; ++i)
            if (c->ring_busy[i]) {
                HIPCHK(hipEventSynchronize(c->ring_ev[i]));
                c->ring_busy[i] = false;
            }
        for (int64_t k0 = 0; k0 < loc; k0 += ch)
            if ((rc = op.push(k0, std::min(loc, k0 + ch), s))) return rc;
    }
    if ((rc = op.finish())) return collective_result(c, calls0, rc);
    if ((rc = sync(c, s))) return collective_result(c, calls0, rc);
    // a merge pass that rejected its chunk bounds left the output incomplete:
    // report it here, not on a later unrelated misort_synchronize
    return collective_result(c, calls0, planning_check(s));
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

int misort_profile_stage(misort_ctx* c, int stage, int64_t* count, double* exchange_ms, double* merge_ms,
                         double* exchange_bytes) {
    if (!c || stage < 0 || stage >= Profiler::MAX_STAGES) return fail(MISORT_E_INVALID, "bad stage");
    int rc = c->prof.collect();
    if (rc) return rc;
    if (count) *count = c->prof.st_count[stage];
    if (exchange_ms) *exchange_ms = c->prof.st_ms[stage][0];
    if (merge_ms) *merge_ms = c->prof.st_ms[stage][1];
    if (exchange_bytes) *exchange_bytes = c->prof.st_bytes[stage];
    return MISORT_OK;
}

int misort_profile_trace(misort_ctx* c, int max, int* kinds, double* ms, double* bytes) {
    if (!c || max < 0 || (max > 0 && (!kinds || !ms || !bytes))) return fail(MISORT_E_INVALID, "bad trace arguments");
    int rc = c->prof.collect();
    if (rc) return rc;
    const int n = (int)std::min<size_t>(c->prof.trace.size(), (size_t)max);
    for (int i = 0; i < n; ++i) {
        kinds[i] = c->prof.trace[i].kind;
        ms[i] = c->prof.trace[i].ms;
        bytes[i] = c->prof.trace[i].bytes;
    }
    return (int)std::min<size_t>(c->prof.trace.size(), (size_t)INT32_MAX);
}

int misort_tile_log2(int key_bytes_) { return misort::tile_log2(key_bytes_); }

int misort_plan(int64_t n, int key_bytes, int* passes, int max_passes) {
    if (key_bytes != 4 && key_bytes != 8) return fail(MISORT_E_INVALID, "key_bytes must be 4 or 8");
    if (max_passes > 0 && !passes) return fail(MISORT_E_INVALID, "null passes");
    return misort::plan_passes(n, key_bytes, passes, max_passes < 0 ? 0 : max_passes);
}

}  // extern "C"
