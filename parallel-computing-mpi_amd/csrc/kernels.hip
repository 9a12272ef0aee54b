// kernels.hip -- compare-split merge, check_sort and helper kernels (gfx950),
// plus the planner knobs shared by the per-key-type sort units.
//
// Replaces the merge loop of compare_split_{max,min} (psort.cc:116-164) and the
// descent count of check_sort (psort.cc:497-520).  The bitonic tile engine
// itself lives in bitonic.h (instantiated by sort_u32.hip / sort_u64.hip).
#include "bitonic.h"

namespace misort {

PlanKnobs::PlanKnobs() {
    auto env = [](const char* k, int& v) {
        if (const char* e = getenv(k)) v = atoi(e);
    };
    env("MISORT_PERSIST", persist);
    env("MISORT_PERSIST_U64", persist_u64);
    env("MISORT_GRID_MULT", grid_mult);
    env("MISORT_MULTIWAY", multiway);
    env("MISORT_MULTIWAY_U64", multiway_u64);
    env("MISORT_SORT_TILE_U32", sort_tile_u32);
    if (grid_mult < 1) grid_mult = 1;
    if (sort_tile_u32 != 0 && sort_tile_u32 != SORT_LT_MERGE && sort_tile_u32 != SORT_LT_U32) {
        // a pin the plan cannot honour would silently measure the per-size rule
        fprintf(stderr, "misort: MISORT_SORT_TILE_U32=%d ignored (0, %d or %d); the tile is chosen per size\n",
                sort_tile_u32, SORT_LT_MERGE, SORT_LT_U32);
        sort_tile_u32 = 0;
    }
}

const PlanKnobs& plan_knobs() {
    static PlanKnobs k;
    return k;
}

int mergek_fence_log2(int64_t n, int key_bytes) {
    // MISORT_FENCE_FG6_MIN (u32) / MISORT_FENCE_FG6_MIN_U64: log2 keys from which
    // the 64-key fences pay (fuller chunks against twice the fences to merge,
    // count and search; profiles/r05/plan/fg6_ab.txt); 0 = never.  Round 6: with
    // the 12864-key u32 chunks (runsk.hip) a 128-key fence leaves the chunks full
    // enough, and 64-key fences lose at every u32 size (2^30 85.0 vs 85.8-86.3
    // Gkeys/s, 2^28/2^29 -3.6 %; profiles/r06/plan/fg6_ab.txt): u32 never, u64 from 2^29
    static const int m32 = getenv("MISORT_FENCE_FG6_MIN") ? atoi(getenv("MISORT_FENCE_FG6_MIN")) : 0;
    static const int m64 = getenv("MISORT_FENCE_FG6_MIN_U64") ? atoi(getenv("MISORT_FENCE_FG6_MIN_U64")) : 29;
    const int m = key_bytes == 8 ? m64 : m32;
    return m > 0 && m < 63 && n >= ((int64_t)1 << m) ? 6 : MERGEK_FENCE_LOG2;
}

// The largest SORT tile per key type (log2 keys): every plan's tiles divide it.
int tile_log2(int key_bytes) { return key_bytes == 4 ? KT<uint32_t>::LT : KT<uint64_t>::LT; }

int plan_passes(int64_t n, int key_bytes, int* out, int max) {
    if (n <= 0) return 0;
    const std::vector<Pass>& ps = key_bytes == 4 ? plan_for<uint32_t>(n) : plan_for<uint64_t>(n);
    const int np = (int)ps.size();
    for (int i = 0; i < np && i < max; ++i) {
        out[4 * i + 0] = ps[i].kind;
        out[4 * i + 1] = ps[i].hi;
        out[4 * i + 2] = ps[i].R;
        out[4 * i + 3] = ps[i].flip;
    }
    return np;
}

namespace {

// ----------------------------------------------------------- merge-split

constexpr int MS_NT = 256, MS_ITEMS = 8, MS_TILE = MS_NT * MS_ITEMS;

// Number of A keys among the first d keys of merge(A, B), A first on ties.
template <typename K>
__device__ int64_t corank(const K* A, int64_t na, const K* B, int64_t nb, int64_t d) {
    int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[d - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The same by a radix-R lifting search: R - 1 probes per round (their loads in
// flight together), log_R of the bisection's dependent rounds -- the partition
// of a whole-block merge-split is latency-bound (one thread per 2048-output
// tile, 27 rounds at 2^27 + 2^26 keys).
template <int R, typename K>
__device__ int64_t corank_r(const K* A, int64_t na, const K* B, int64_t nb, int64_t d) {
    const int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    if (lo >= hi) return lo;
    int64_t st = 1;
    while (st * R <= hi - lo) st *= R;
    int64_t base = lo;  // A[i] <= B[d - 1 - i] holds for every i < base
    for (; st > 0; st /= R) {
        K a[R - 1], b[R - 1];
#pragma unroll
        for (int u = 0; u < R - 1; ++u) {
            const int64_t i = base + (u + 1) * st - 1;
            const int64_t ic = i < hi ? i : hi - 1;  // clamped: never taken
            a[u] = A[ic];
            b[u] = B[d - 1 - ic];
        }
        int64_t add = 0;
#pragma unroll
        for (int u = 0; u < R - 1; ++u) add += base + (u + 1) * st - 1 < hi && a[u] <= b[u] ? st : 0;
        base += add;
    }
    return base;
}

// radix 4: merge-split 0.251 -> 0.243 ms per whole-block stage of config 4 at
// P = 8; radix 8 / 16 (more loads a round) 0.259 / 0.273
// (profiles/r06/rankwork/corank_ab.txt)
constexpr int CORANK_RADIX = 4;
template <typename K>
__global__ void k_merge_partition(const K* __restrict__ A, int64_t na, const K* __restrict__ B,
                                  int64_t nb, int64_t d0, int64_t nout, int64_t ntiles,
                                  int64_t* __restrict__ co) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const int64_t off = t * MS_TILE < nout ? t * MS_TILE : nout;
    co[t] = corank_r<CORANK_RADIX>(A, na, B, nb, d0 + off);
}

// Output keys [d0 + t*TILE, ...) of merge(A, B): each workgroup stages its A
// and B ranges in LDS, each lane merges MS_ITEMS consecutive outputs.
// ORD (u64 only): the stage is the sort's last over f64 keys; the outputs
// are stored as IEEE double bits (no separate back-conversion sweep).
template <typename K, bool ORD = false>
__global__ __launch_bounds__(MS_NT) void k_merge_tiles(const K* __restrict__ A, int64_t na,
                                                       const K* __restrict__ B, int64_t nb,
                                                       int64_t d0, int64_t nout,
                                                       const int64_t* __restrict__ co,
                                                       K* __restrict__ out) {
    __shared__ K s[MS_TILE];
    const int64_t t = blockIdx.x;
    const int64_t ds = t * MS_TILE;
    const int64_t de = (t + 1) * MS_TILE < nout ? (t + 1) * MS_TILE : nout;
    const int64_t i0 = co[t], i1 = co[t + 1];
    const int64_t j0 = d0 + ds - i0, j1 = d0 + de - i1;
    const int la = (int)(i1 - i0), lb = (int)(j1 - j0), len = la + lb;
    // all MS_ITEMS loads of a lane are issued before the first LDS write (one
    // memory latency per tile: the per-key loop waited out one per key)
    {
        K x[MS_ITEMS];
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k) {
            const int e = k * MS_NT + threadIdx.x;
            const K* q = e < la ? A + i0 + e : B + j0 + (e - la);
            x[k] = e < len ? *q : (K)0;
        }
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k)
            if (k * MS_NT + (int)threadIdx.x < len) s[k * MS_NT + threadIdx.x] = x[k];
    }
    __syncthreads();
    const int dk = threadIdx.x * MS_ITEMS < len ? threadIdx.x * MS_ITEMS : len;
    int lo = dk - lb > 0 ? dk - lb : 0, hi = dk < la ? dk : la;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] <= s[la + dk - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int ia = lo, ib = dk - lo;
    K r[MS_ITEMS];
#pragma unroll
    for (int k = 0; k < MS_ITEMS; ++k) {
        const K av = ia < la ? s[ia] : KT<K>::MAX;
        const K bv = ib < lb ? s[la + ib] : KT<K>::MAX;
        const bool takeA = ia < la && (ib >= lb || av <= bv);
        r[k] = takeA ? av : bv;
        ia += takeA;
        ib += !takeA;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MS_ITEMS; ++k)
        if (dk + k < len) s[dk + k] = r[k];
    __syncthreads();
    for (int k = threadIdx.x; k < len; k += MS_NT) {
        if constexpr (ORD) out[ds + k] = (K)f64_of_ord((uint64_t)s[k]);
        else out[ds + k] = s[k];
    }
}

// ------------------------------------------------- in-place tail merge-split
//
// When the partner's k keys touch only one end of this rank's block, the
// compare-split rewrites just that end, in place.  Keep-min (the block A
// keeps its na smallest of A U B, B = the partner's bottom k keys): A's keys
// up to and including B[0] stay where they are (A first on ties), so
// out[0, p0) = A[0, p0), p0 = #{A[i] <= B[0]}, and out[p0, na) = the first
// na - p0 of merge(A[p0, na), B).  Keep-max (B = the partner's top k): A's
// keys after B[k-1] stay, out[q0, na) = A[q0, na), q0 = #{A[i] <= B[k-1]},
// and out[0, q0) = merge positions [k, k + q0) of merge(A[0, q0), B).  The
// window of A is staged first (a tile's writes would overwrite keys a later
// tile still reads); then the window merges back into A through the usual
// partition + LDS tiles, with sizes the device computed (the host knows k,
// not the window): win = {window start in A, window length W, merge
// diagonal offset}.  O(W + k) traffic instead of O(na): a 2^27-key block
// with k = 4096 moved 0.2 ms of whole-block merge (profiles/r04 rank work).
// The window: the first i with a[i] > x by a 1024-ary search (one workgroup,
// 1024 probes per round: three rounds of loads for a 2^27-key block instead
// of 27 dependent ones).
constexpr int TW_NT = 1024;
template <typename K>
__global__ __launch_bounds__(TW_NT) void k_tail_window(const K* __restrict__ a, int64_t na, const K* __restrict__ b,
                                                       int64_t nb, int keep_max, int64_t* __restrict__ win) {
    int64_t w0 = 0, W = na;
    if (nb > 0) {
        const K x = keep_max ? b[nb - 1] : b[0];
        int64_t lo = 0, hi = na;  // a[i] <= x for i < lo; the answer is in [lo, hi]
        while (lo < hi) {
            const int64_t step = (hi - lo + TW_NT - 1) / TW_NT;
            const int64_t q = lo + (int64_t)threadIdx.x * step;
            const int c = __syncthreads_count(q < hi && a[q] <= x);  // a prefix of the probes
            if (step == 1) {
                lo += c;
                break;
            }
            const int64_t nlo = c > 0 ? lo + (int64_t)(c - 1) * step + 1 : lo;
            const int64_t qc = lo + (int64_t)c * step;
            hi = qc < hi ? qc : hi;
            lo = nlo;
        }
        if (keep_max) {
            W = lo;
        } else {
            w0 = lo;
            W = na - lo;
        }
    }
    if (threadIdx.x == 0) {
        win[0] = w0;
        win[1] = W;
        win[2] = keep_max ? nb : 0;
    }
}

template <typename K>
__global__ void k_tail_stage(const K* __restrict__ a, K* __restrict__ st, const int64_t* __restrict__ win) {
    const int64_t w0 = win[0], W = win[1];
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < W; i += stride) st[w0 + i] = a[w0 + i];
}

template <typename K>
__global__ void k_tail_partition(const K* __restrict__ st, const K* __restrict__ b, int64_t nb,
                                 const int64_t* __restrict__ win, int64_t* __restrict__ co) {
    const int64_t w0 = win[0], W = win[1], d0 = win[2];
    const int64_t ntiles = (W + MS_TILE - 1) / MS_TILE;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= ntiles; t += stride) {
        const int64_t off = t * MS_TILE < W ? t * MS_TILE : W;
        co[t] = corank(st + w0, W, b, nb, d0 + off);
    }
}

// The window's output tiles, a persistent grid walking them (the grid is
// sized for the worst case W = na; most windows are a few tiles).
template <typename K>
__global__ __launch_bounds__(MS_NT) void k_tail_merge(const K* __restrict__ st, const K* __restrict__ b, int64_t nb,
                                                      const int64_t* __restrict__ win, const int64_t* __restrict__ co,
                                                      K* __restrict__ a, int keep_max) {
    __shared__ K sh[MS_TILE];
    const int64_t w0 = win[0], W = win[1], d0 = win[2];
    const int64_t ntiles = (W + MS_TILE - 1) / MS_TILE;
    const K* A = st + w0;
    K* out = a + (keep_max ? 0 : w0);
    for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int64_t ds = t * MS_TILE;
        const int64_t de = (t + 1) * MS_TILE < W ? (t + 1) * MS_TILE : W;
        const int64_t i0 = co[t], i1 = co[t + 1];
        const int64_t j0 = d0 + ds - i0, j1 = d0 + de - i1;
        const int la = (int)(i1 - i0), lb = (int)(j1 - j0), len = la + lb;
        K x[MS_ITEMS];
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k) {
            const int e = k * MS_NT + threadIdx.x;
            const K* q = e < la ? A + i0 + e : b + j0 + (e - la);
            x[k] = e < len ? *q : (K)0;
        }
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k)
            if (k * MS_NT + (int)threadIdx.x < len) sh[k * MS_NT + threadIdx.x] = x[k];
        __syncthreads();
        const int dk = threadIdx.x * MS_ITEMS < len ? threadIdx.x * MS_ITEMS : len;
        int lo = dk - lb > 0 ? dk - lb : 0, hi = dk < la ? dk : la;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (sh[mid] <= sh[la + dk - 1 - mid]) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = dk - lo;
        K r[MS_ITEMS];
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k) {
            const K av = ia < la ? sh[ia] : KT<K>::MAX;
            const K bv = ib < lb ? sh[la + ib] : KT<K>::MAX;
            const bool takeA = ia < la && (ib >= lb || av <= bv);
            r[k] = takeA ? av : bv;
            ia += takeA;
            ib += !takeA;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < MS_ITEMS; ++k)
            if (dk + k < len) sh[dk + k] = r[k];
        __syncthreads();
        for (int k = threadIdx.x; k < len; k += MS_NT) out[ds + k] = sh[k];
        __syncthreads();
    }
}

// ---------------------------------------------------------------- helpers

template <typename T>
__global__ void k_count_desc(const T* __restrict__ a, int64_t n, unsigned long long* cnt) {
    unsigned long long c = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride)
        c += a[i] > a[i + 1] ? 1ull : 0ull;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

template <typename K>
__global__ void k_gather_samples(const K* __restrict__ a, int64_t n, int64_t stride, K* __restrict__ out,
                                 int64_t count) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= count) return;
    const int64_t x = c * stride < n - 1 ? c * stride : n - 1;
    out[c] = a[x];
}

// The compare-split bracket on the device (runtime.cpp corank_lower, same
// predicate, same answer): i_lo = the first i in [max(0, na-nb), na] whose
// "A[i] <= B[na-1-i]" is not certain from the samples (sa: samples of A's na
// keys, sb: of B's nb keys, stride max(256, ceil(n/32768)), the last sample
// index clamped).  The predicate is true then false, so one workgroup narrows
// [lo, hi] by EXN points per round instead of one bisection step per load.
// run = {send offset, k}: k = na - i_lo keys each side sends, from offset 0
// (the keep-max side sends its bottom k) or nloc - k (the keep-min side its top k).
constexpr int EXN = 1024;
inline int64_t dev_sample_stride_host(int64_t n) { return std::max<int64_t>(256, (n + 32767) / 32768); }
__device__ __forceinline__ int64_t dev_sample_stride(int64_t n) {
    const int64_t s = (n + 32767) / 32768;
    return s > 256 ? s : 256;
}
template <typename K>
__global__ __launch_bounds__(EXN) void k_exchange_count(const K* __restrict__ sa, int64_t ca, int64_t na,
                                                        const K* __restrict__ sb, int64_t cb, int64_t nb, int mx,
                                                        int64_t nloc, int64_t* __restrict__ run) {
    const int64_t Sa = dev_sample_stride(na), Sb = dev_sample_stride(nb);
    auto certain = [&](int64_t i) {  // A[i] <= B[na-1-i] from the samples
        const int64_t ia = i / Sa + 1 < ca - 1 ? i / Sa + 1 : ca - 1;
        const int64_t jb = (na - 1 - i) / Sb < cb - 1 ? (na - 1 - i) / Sb : cb - 1;
        return sa[ia] <= sb[jb];
    };
    int64_t lo = na > nb ? na - nb : 0, hi = na;
    if (na == 0) lo = hi = 0;
    else if (nb == 0) lo = hi = na;
    while (lo < hi) {
        const int64_t step = (hi - lo + EXN - 1) / EXN;
        const int64_t x = lo + (int64_t)threadIdx.x * step;
        const int c = __syncthreads_count(x < hi && certain(x));  // a prefix of the points
        if (step == 1) {
            lo += c;
            break;
        }
        const int64_t nlo = c > 0 ? lo + (int64_t)(c - 1) * step + 1 : lo;
        const int64_t xc = lo + (int64_t)c * step;
        hi = xc < hi ? xc : hi;
        lo = nlo;
    }
    if (threadIdx.x == 0) {
        const int64_t k = na - lo;
        run[0] = mx ? 0 : nloc - k;
        run[1] = k;
    }
}

// psort.cc:88-101: first index i in [0, n) with x <= a[i] (n if none), one lane.
template <typename K>
__global__ void k_lower_bound(const K* __restrict__ a, int64_t n, K x, int64_t* __restrict__ out) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (x <= a[mid]) hi = mid;
        else lo = mid + 1;
    }
    *out = lo;
}

// lower and upper bound of nv values in a sorted run, one lane per value.
template <typename K>
__global__ void k_bounds(const K* __restrict__ a, int64_t n, const K* __restrict__ vals, int nv,
                         int64_t* __restrict__ lb, int64_t* __restrict__ ub) {
    const int v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v >= nv) return;
    const K x = vals[v];
    int64_t lo = 0, hi = n;
    while (lo < hi) {  // first a[i] >= x
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    lb[v] = lo;
    hi = n;
    while (lo < hi) {  // first a[i] > x
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= x) lo = mid + 1;
        else hi = mid;
    }
    ub[v] = lo;
}

// b[i] = map(a[i]) (a == b: in place)
__global__ void k_f64_ord(const uint64_t* a, uint64_t* b, int64_t n, int to_ord) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        b[i] = to_ord ? ord_of_f64(a[i]) : f64_of_ord(a[i]);
}

__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, int64_t g) {
    uint64_t z = seed + (uint64_t)(g + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename K>
__global__ void k_fill_splitmix(K* out, int64_t n, uint64_t seed, int64_t g0) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t z = splitmix_at(seed, g0 + i);
        out[i] = sizeof(K) == 4 ? (K)(z >> 32) : (K)z;
    }
}

int stream_grid(int64_t n, int threads) {
    int64_t g = (n + threads - 1) / threads;
    if (g > 2048) g = 2048;
    return g < 1 ? 1 : (int)g;
}

}  // namespace

template <typename K>
hipError_t merge_split(const K* a, int64_t na, const K* b, int64_t nb, K* out, int keep_max,
                       int64_t* scratch, hipStream_t s, LaunchHook* hook, bool ord_out) {
    if (na <= 0) return hipSuccess;
    if (ord_out && sizeof(K) != 8) return hipErrorInvalidValue;
    const int64_t d0 = keep_max ? nb : 0;
    const int64_t ntiles = (na + MS_TILE - 1) / MS_TILE;
    HookScope hs(hook, KIND_MERGE_SPLIT, (double)(2 * na + (nb < na ? nb : na)) * sizeof(K), s);
    k_merge_partition<K><<<(unsigned)((ntiles + 1 + 255) / 256), 256, 0, s>>>(a, na, b, nb, d0, na,
                                                                              ntiles, scratch);
    if (ord_out) k_merge_tiles<K, true><<<(unsigned)ntiles, MS_NT, 0, s>>>(a, na, b, nb, d0, na, scratch, out);
    else k_merge_tiles<K><<<(unsigned)ntiles, MS_NT, 0, s>>>(a, na, b, nb, d0, na, scratch, out);
    return hipGetLastError();
}

template <typename K>
hipError_t merge_split_tail(K* a, int64_t na, const K* b, int64_t nb, int keep_max, K* stage, int64_t* scratch,
                            hipStream_t s, LaunchHook* hook) {
    if (na <= 0) return hipSuccess;
    const int64_t ntiles = (na + MS_TILE - 1) / MS_TILE;  // the worst case, W = na
    // its own kind: the window (found on the device) is usually far smaller
    // than the block, so these bytes are only an upper bound
    HookScope hs(hook, KIND_MERGE_SPLIT_TAIL, (double)(2 * na + (nb < na ? nb : na)) * sizeof(K), s);
    int64_t* win = scratch;
    int64_t* co = scratch + 4;
    k_tail_window<K><<<1, TW_NT, 0, s>>>(a, na, b, nb, keep_max, win);
    k_tail_stage<K><<<stream_grid(na, 256), 256, 0, s>>>(a, stage, win);
    const int64_t pg = (ntiles + 1 + 255) / 256;
    k_tail_partition<K><<<(unsigned)(pg < 256 ? pg : 256), 256, 0, s>>>(stage, b, nb, win, co);
    k_tail_merge<K><<<(unsigned)(ntiles < 1024 ? ntiles : 1024), MS_NT, 0, s>>>(stage, b, nb, win, co, a, keep_max);
    return hipGetLastError();
}

template <typename K>
hipError_t merge_full(const K* a, int64_t na, const K* b, int64_t nb, K* out, int64_t* scratch, hipStream_t s,
                      LaunchHook* hook) {
    const int64_t nout = na + nb;
    if (nout <= 0) return hipSuccess;
    const int64_t ntiles = (nout + MS_TILE - 1) / MS_TILE;
    HookScope hs(hook, KIND_MERGE_SPLIT, 2.0 * (double)nout * sizeof(K), s);
    k_merge_partition<K><<<(unsigned)((ntiles + 1 + 255) / 256), 256, 0, s>>>(a, na, b, nb, 0, nout, ntiles,
                                                                              scratch);
    k_merge_tiles<K><<<(unsigned)ntiles, MS_NT, 0, s>>>(a, na, b, nb, 0, nout, scratch, out);
    return hipGetLastError();
}

template <typename K>
hipError_t lower_bound(const K* a, int64_t n, K x, int64_t* d_out, hipStream_t s) {
    k_lower_bound<K><<<1, 1, 0, s>>>(a, n, x, d_out);
    return hipGetLastError();
}

template <typename K>
hipError_t bounds(const K* a, int64_t n, const K* vals, int nv, int64_t* lb, int64_t* ub, hipStream_t s) {
    if (nv <= 0) return hipSuccess;
    k_bounds<K><<<(unsigned)((nv + 63) / 64), 64, 0, s>>>(a, n, vals, nv, lb, ub);
    return hipGetLastError();
}

template <typename T>
hipError_t count_descents(const T* a, int64_t n, unsigned long long* count, hipStream_t s) {
    if (n < 2) return hipSuccess;
    k_count_desc<T><<<stream_grid(n, 256), 256, 0, s>>>(a, n, count);
    return hipGetLastError();
}

template <typename K>
hipError_t gather_samples(const K* a, int64_t n, int64_t stride, K* out, int64_t count, hipStream_t s) {
    if (n <= 0 || count <= 0) return hipSuccess;
    k_gather_samples<K><<<(unsigned)((count + 255) / 256), 256, 0, s>>>(a, n, stride, out, count);
    return hipGetLastError();
}
template hipError_t gather_samples<uint32_t>(const uint32_t*, int64_t, int64_t, uint32_t*, int64_t, hipStream_t);
template hipError_t gather_samples<uint64_t>(const uint64_t*, int64_t, int64_t, uint64_t*, int64_t, hipStream_t);

template <typename K>
hipError_t exchange_count(const K* sa, int64_t na, const K* sb, int64_t nb, int keep_max, int64_t nloc,
                          int64_t* run, hipStream_t s) {
    const int64_t ca = na > 0 ? (na + dev_sample_stride_host(na) - 1) / dev_sample_stride_host(na) + 1 : 0;
    const int64_t cb = nb > 0 ? (nb + dev_sample_stride_host(nb) - 1) / dev_sample_stride_host(nb) + 1 : 0;
    k_exchange_count<K><<<1, EXN, 0, s>>>(sa, ca, na, sb, cb, nb, keep_max, nloc, run);
    return hipGetLastError();
}
template hipError_t exchange_count<uint32_t>(const uint32_t*, int64_t, const uint32_t*, int64_t, int, int64_t,
                                             int64_t*, hipStream_t);
template hipError_t exchange_count<uint64_t>(const uint64_t*, int64_t, const uint64_t*, int64_t, int, int64_t,
                                             int64_t*, hipStream_t);

hipError_t f64_to_ord(uint64_t* a, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_f64_ord<<<stream_grid(n, 256), 256, 0, s>>>(a, a, n, 1);
    return hipGetLastError();
}

hipError_t ord_to_f64(uint64_t* a, int64_t n, hipStream_t s) { return ord_to_f64_copy(a, a, n, s); }

hipError_t ord_to_f64_copy(const uint64_t* a, uint64_t* b, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_f64_ord<<<stream_grid(n, 256), 256, 0, s>>>(a, b, n, 0);
    return hipGetLastError();
}

hipError_t fill_splitmix_u32(uint32_t* out, int64_t n, uint64_t seed, int64_t g0, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_fill_splitmix<uint32_t><<<stream_grid(n, 256), 256, 0, s>>>(out, n, seed, g0);
    return hipGetLastError();
}

hipError_t fill_splitmix_u64(uint64_t* out, int64_t n, uint64_t seed, int64_t g0, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_fill_splitmix<uint64_t><<<stream_grid(n, 256), 256, 0, s>>>(out, n, seed, g0);
    return hipGetLastError();
}

template hipError_t merge_split<uint32_t>(const uint32_t*, int64_t, const uint32_t*, int64_t,
                                          uint32_t*, int, int64_t*, hipStream_t, LaunchHook*, bool);
template hipError_t merge_split<uint64_t>(const uint64_t*, int64_t, const uint64_t*, int64_t,
                                          uint64_t*, int, int64_t*, hipStream_t, LaunchHook*, bool);
template hipError_t merge_split_tail<uint32_t>(uint32_t*, int64_t, const uint32_t*, int64_t, int, uint32_t*,
                                               int64_t*, hipStream_t, LaunchHook*);
template hipError_t merge_split_tail<uint64_t>(uint64_t*, int64_t, const uint64_t*, int64_t, int, uint64_t*,
                                               int64_t*, hipStream_t, LaunchHook*);
template hipError_t merge_full<uint32_t>(const uint32_t*, int64_t, const uint32_t*, int64_t, uint32_t*,
                                         int64_t*, hipStream_t, LaunchHook*);
template hipError_t merge_full<uint64_t>(const uint64_t*, int64_t, const uint64_t*, int64_t, uint64_t*,
                                         int64_t*, hipStream_t, LaunchHook*);
template hipError_t bounds<uint32_t>(const uint32_t*, int64_t, const uint32_t*, int, int64_t*, int64_t*,
                                     hipStream_t);
template hipError_t bounds<uint64_t>(const uint64_t*, int64_t, const uint64_t*, int, int64_t*, int64_t*,
                                     hipStream_t);
template hipError_t lower_bound<uint32_t>(const uint32_t*, int64_t, uint32_t, int64_t*, hipStream_t);
template hipError_t lower_bound<uint64_t>(const uint64_t*, int64_t, uint64_t, int64_t*, hipStream_t);
template hipError_t count_descents<uint32_t>(const uint32_t*, int64_t, unsigned long long*,
                                             hipStream_t);
template hipError_t count_descents<uint64_t>(const uint64_t*, int64_t, unsigned long long*,
                                             hipStream_t);
template hipError_t count_descents<double>(const double*, int64_t, unsigned long long*,
                                           hipStream_t);

}  // namespace misort
