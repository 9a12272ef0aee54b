// runs.hip -- merge levels of the local sort (gfx950): ascending runs of 2^lw
// keys -> ascending runs of 2^(lw+1), one HBM read + one HBM write per key.
//
// The reference's local sort is std::sort (psort.cc:175); the bitonic SORT tile
// of bitonic.h sorts 2^LT-key tiles, and every level above it is a merge of
// neighbouring runs -- most of them in the multi-way passes of runsk.hip, a
// level left over (and the fence merges of those passes) here.  Output is
// bit-identical: the keys carry no payload, so every correct sort of them
// writes the same bytes.
//
// Per level, two launches (one on levels of at most 2^20 keys, whose merge
// workgroups search their own co-ranks: MISORT_RUN_FUSE):
//   k_runs_partition  32 lanes per output tile: the merge-path co-rank of the
//                     tile's first output within its pair (a 32-ary search, A
//                     first on ties);
//   k_runs_merge      one workgroup per output tile of NT*IT keys: its A and B
//                     ranges are streamed into LDS, each lane finds its own
//                     co-rank in LDS and merges IT consecutive outputs, and the
//                     tile leaves through LDS as 16-byte non-temporal stores.
#include "kernels.h"

#include <map>
#include <mutex>

// Build-time A/B switches (tools/build_variant.sh): non-temporal tile loads / stores.

namespace misort {
namespace {

template <typename K>
struct RunKT;
template <>
struct RunKT<uint32_t> {
    static constexpr int IT = 16;
    static constexpr int NT = 512;  // 8192-key tiles, 32 KiB of LDS (NT 256: -2 %, 1024: -8 %; IT 32: 1.5x slower)
    static constexpr int V = 4;
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
};
template <>
struct RunKT<uint64_t> {
    static constexpr int IT = 8;
    static constexpr int NT = 1024;  // 8192-key tiles, 64 KiB of LDS (256 x 16: -4 %, 512 x 16: -11 %)
    static constexpr int V = 2;
    typedef uint64_t vec __attribute__((ext_vector_type(2)));
};


// fences of the u64 multi-way passes (runsk.hip): key << 64 | run/position tag
typedef unsigned __int128 u128;
template <>
struct RunKT<u128> {
    static constexpr int IT = 4;
    static constexpr int NT = 1024;  // 4096-fence tiles, 64 KiB of LDS
    static constexpr int V = 1;
    typedef u128 vec;
};

template <typename K>
constexpr K KT_MAX = (K)~(K)0;

// lane element e of a vector (a plain value when V = 1)
template <typename K>
__device__ __forceinline__ void vset(typename RunKT<K>::vec& x, int e, K v) {
    if constexpr (RunKT<K>::V == 1) x = v;
    else x[e] = v;
}

struct PairGeo {
    int64_t base, na, nb;
};

__device__ __forceinline__ PairGeo pair_geo(int64_t g, int64_t n, int lw) {
    const int64_t w = (int64_t)1 << lw;
    const int64_t base = (g >> (lw + 1)) << (lw + 1);
    const int64_t rest = n - base;
    const int64_t na = rest < w ? rest : w;
    const int64_t rb = rest - w;
    const int64_t nb = rb <= 0 ? 0 : (rb < w ? rb : w);
    return PairGeo{base, na, nb};
}

// co[i] = the number of A keys among the first d outputs of merge(A, B), A
// first on ties, for the first output d of tile t0 + i within its pair.
// One group of PART_LANES lanes per tile start: each round the lanes evaluate
// the co-rank predicate (A[x] <= B[d-1-x]: true, then false) at PART_LANES
// evenly spaced points of the bracket and keep the step around the first
// false one -- ceil(log32(range)) dependent rounds of loads instead of
// log2(range) (a 2^23-key pair: 5 instead of 23; the kernel is a chain of
// load latencies).
constexpr int PART_LANES = 32;

// The co-rank of output d of one pair (A: na keys, B: nb keys) by one group of
// PART_LANES lanes (sub: this lane's index in the group, shift: the group's
// first bit in the wave's ballot).
template <typename K>
__device__ __forceinline__ int64_t corank_group(const K* __restrict__ A, const K* __restrict__ B, int64_t d,
                                                int64_t na, int64_t nb, int sub, int shift) {
    int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const int64_t step = (hi - lo + PART_LANES - 1) / PART_LANES;
        const int64_t x = lo + sub * step;
        const bool t = x < hi && A[x] <= B[d - 1 - x];
        const int c = __popc((uint32_t)(__ballot(t) >> shift));  // the true points are a prefix
        const int64_t nhi = lo + c * step;
        lo = c > 0 ? lo + (c - 1) * step + 1 : lo;
        hi = nhi < hi ? nhi : hi;
    }
    return lo;
}

template <typename K, int NT, int IT>
__global__ __launch_bounds__(256) void k_runs_partition(const K* __restrict__ src, int64_t n, int lw, int64_t t0,
                                                        int64_t ntiles, int64_t* __restrict__ co) {
    constexpr int TILE = NT * IT;
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / PART_LANES;
    const int sub = (int)(threadIdx.x % PART_LANES), shift = (int)(threadIdx.x & 63) & ~(PART_LANES - 1);
    if (i >= ntiles) return;  // whole lane groups
    const int64_t g0 = (t0 + i) * TILE;
    const PairGeo p = pair_geo(g0, n, lw);
    const K* A = src + p.base;
    const int64_t lo = corank_group(A, A + ((int64_t)1 << lw), g0 - p.base, p.na, p.nb, sub, shift);
    if (sub == 0) co[i] = lo;
}

// FUSED: the workgroup finds its own two co-ranks (wave 0: lanes 0-31 the
// tile's first output, lanes 32-63 the one past its last) instead of reading
// k_runs_partition's -- one launch per level fewer, for levels whose few tiles
// leave the chip idle anyway.
template <typename K, int NT, int IT, bool FUSED>
__global__ __launch_bounds__(NT) void k_runs_merge(const K* __restrict__ src, K* __restrict__ dst,
                                                       int64_t n, int lw, int64_t t0,
                                                       const int64_t* __restrict__ co) {
    constexpr int V = RunKT<K>::V, TILE = NT * IT;
    typedef typename RunKT<K>::vec vec;
    __shared__ __attribute__((aligned(16))) K s[TILE];
    const int tid = threadIdx.x;
    const int64_t t = blockIdx.x;
    const int64_t g0 = (t0 + t) * TILE;
    const int64_t g1 = g0 + TILE < n ? g0 + TILE : n;
    const PairGeo p = pair_geo(g0, n, lw);
    int64_t i0, i1;
    if constexpr (FUSED) {
        static_assert(NT >= 64, "wave 0 searches both co-ranks");
        __shared__ int64_t sco[2];
        if (tid < 64) {
            // tiles never straddle pairs (2^lw >= TILE): g1 <= the pair's end,
            // where the search returns na at once
            const int h = tid >> 5;
            const K* A = src + p.base;
            const int64_t c = corank_group(A, A + ((int64_t)1 << lw), (h ? g1 : g0) - p.base, p.na, p.nb,
                                           tid & (PART_LANES - 1), h * PART_LANES);
            if ((tid & (PART_LANES - 1)) == 0) sco[h] = c;
        }
        __syncthreads();
        i0 = sco[0];
        i1 = sco[1];
    } else {
        i0 = co[t];
        i1 = g1 == p.base + p.na + p.nb ? p.na : co[t + 1];
    }
    const int64_t j0 = g0 - p.base - i0, j1 = g1 - p.base - i1;
    const int la = (int)(i1 - i0), lb = (int)(j1 - j0), len = la + lb;
    const K* __restrict__ A = src + p.base + i0;
    const K* __restrict__ B = src + p.base + ((int64_t)1 << lw) + j0;
    // s = A range ++ B range: all IT loads of a lane are issued before the
    // first LDS write (one memory latency per tile, not one per key)
    {
        K x[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int e = k * NT + tid;
            const K* q = e < la ? A + e : B + (e - la);
            x[k] = e < len ? __builtin_nontemporal_load(q) : KT_MAX<K>;
        }
#pragma unroll
        for (int k = 0; k < IT; ++k) s[k * NT + tid] = x[k];
    }
    __syncthreads();

    // this lane's outputs [dk, dk + IT) of the tile
    const int dk = tid * IT < len ? tid * IT : len;
    int lo = dk - lb > 0 ? dk - lb : 0, hi = dk < la ? dk : la;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[mid] <= s[la + dk - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    int ia = lo, ib = dk - lo;
    K av = s[ia < la ? ia : 0], bv = s[ib < lb ? la + ib : 0];
    K r[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool takeA = ia < la && (ib >= lb || av <= bv);
        r[k] = takeA ? av : bv;
        ia += takeA;
        ib += !takeA;
        const int nx = takeA ? (ia < la ? ia : 0) : (ib < lb ? la + ib : 0);
        const K v = s[nx];
        av = takeA ? v : av;
        bv = takeA ? bv : v;
    }
    __syncthreads();
    if (dk + IT <= len) {
#pragma unroll
        for (int k = 0; k < IT; k += V) {
            vec x;
#pragma unroll
            for (int e = 0; e < V; ++e) vset<K>(x, e, r[k + e]);
            *reinterpret_cast<vec*>(s + dk + k) = x;
        }
    } else {
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (dk + k < len) s[dk + k] = r[k];
    }
    __syncthreads();
    K* __restrict__ out = dst + g0;
    if (len == TILE) {
#pragma unroll
        for (int k = 0; k < IT / V; ++k) {
            const int e = (k * NT + tid) * V;
            __builtin_nontemporal_store(*reinterpret_cast<const vec*>(s + e), reinterpret_cast<vec*>(out + e));
        }
    } else {
        for (int k = tid; k < len; k += NT) out[k] = s[k];
    }
}

// Co-rank scratch: one grow-only buffer per (device, stream), so sorts on
// different streams (the in-process group drives several ranks from one
// process, possibly on one device) never share it; on one stream the launches
// are ordered.
std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, std::pair<void*, size_t>> g_scratch;

int64_t* corank_scratch(size_t bytes, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_mu);
    auto& e = g_scratch[{dev, s}];
    if (e.second < bytes) {
        // the old buffer may still be read by launches queued on s
        if (e.first && (hipStreamSynchronize(s) != hipSuccess || hipFree(e.first) != hipSuccess)) return nullptr;
        e = {nullptr, 0};
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        e = {p, bytes};
    }
    return (int64_t*)e.first;
}

template <typename K, int NT, int IT>
hipError_t merge_level_it(const K* src, K* dst, int64_t n, int lw, hipStream_t s, int64_t o0, int64_t o1,
                          bool fused = false, LaunchHook* hook = nullptr) {
    constexpr int TILE = NT * IT;
    if (o1 <= 0 || o1 > n) o1 = n;
    if (n <= 0 || o0 >= o1) return hipSuccess;
    if (lw < 12 || lw > 40 || ((int64_t)1 << lw) < TILE || src == dst || o0 < 0 || o0 % TILE ||
        (o1 != n && o1 % TILE))
        return hipErrorInvalidValue;
    const int64_t t0 = o0 / TILE, ntiles = (o1 - o0 + TILE - 1) / TILE;
    hipEvent_t ea = nullptr, eb = nullptr;
    if (hook && hook->binds()) (void)hook->bind(-1, KIND_RUNS, 2.0 * (double)n * sizeof(K), &ea, &eb);
    if (fused) {
        launch_timed(k_runs_merge<K, NT, IT, true>, dim3((unsigned)ntiles), dim3(NT), 0, s, ea, eb, src, dst, n, lw,
                     t0, (const int64_t*)nullptr);
        return hipGetLastError();
    }
    // co[i] for tiles t0 .. t0 + ntiles (the one past the range bounds the last)
    const int64_t nco = t0 + ntiles < (n + TILE - 1) / TILE ? ntiles + 1 : ntiles;
    int64_t* co = corank_scratch((size_t)(ntiles + 1) * sizeof(int64_t), s);
    if (!co) return hipErrorOutOfMemory;
    k_runs_partition<K, NT, IT><<<(unsigned)((nco * PART_LANES + 255) / 256), 256, 0, s>>>(src, n, lw, t0, nco, co);
    launch_timed(k_runs_merge<K, NT, IT, false>, dim3((unsigned)ntiles), dim3(NT), 0, s, ea, eb, src, dst, n, lw, t0,
                 (const int64_t*)co);
    return hipGetLastError();
}

// Merge levels over at most RUN_SMALL_N keys use 256-lane tiles when set.
constexpr int64_t RUN_SMALL_N = (int64_t)1 << 20;

int env_knob(const char* k) {
    const char* e = getenv(k);
    return e ? atoi(e) : 0;
}
// MISORT_RUN_IT: keys per lane of the merge tile (16, 32 on 256 lanes, or 8 on 1024 lanes);
// MISORT_RUN_NT: lanes per merge workgroup (256, 512 or 1024).
int run_it_knob() {
    static const int v = env_knob("MISORT_RUN_IT");
    return v;
}
int run_nt_knob() {
    static const int v = env_knob("MISORT_RUN_NT");
    return v;
}
// MISORT_RUN_FUSE: merge workgroups find their own co-ranks (no k_runs_partition
// launch) on levels of at most RUN_SMALL_N keys (1, the default), never (0) or
// on every level (2).
int run_fuse_knob() {
    static const int v = getenv("MISORT_RUN_FUSE") ? env_knob("MISORT_RUN_FUSE") : 1;
    return v;
}

}  // namespace

template <typename K>
hipError_t merge_level(const K* src, K* dst, int64_t n, int lw, hipStream_t s, int64_t o0, int64_t o1,
                       LaunchHook* hook) {
    constexpr int IT = RunKT<K>::IT, NT = RunKT<K>::NT;
    if (lw < 0 || lw > 40) return hipErrorInvalidValue;
    if (run_it_knob() == 2 * IT) return merge_level_it<K, 256, 2 * IT>(src, dst, n, lw, s, o0, o1, false, hook);
    if (run_it_knob() == IT / 2 && ((int64_t)1 << lw) >= 1024 * (IT / 2))
        return merge_level_it<K, 1024, IT / 2>(src, dst, n, lw, s, o0, o1, false, hook);  // same tile, half the keys per lane
    const bool fits = ((int64_t)1 << lw) >= 1024 * IT;  // runs no shorter than the largest tile
    if (run_nt_knob() == 256) return merge_level_it<K, 256, IT>(src, dst, n, lw, s, o0, o1, false, hook);
    if (run_nt_knob() == 512 && fits) return merge_level_it<K, 512, IT>(src, dst, n, lw, s, o0, o1, false, hook);
    if (run_nt_knob() == 1024 && fits) return merge_level_it<K, 1024, IT>(src, dst, n, lw, s, o0, o1, false, hook);
    // small levels (the fence merges of small sorts: 2^17 u64 fences at 2^24 u32
    // keys are 16 default tiles) take 4x smaller tiles, so more CUs share them
    const bool fuse = run_fuse_knob() == 2 || (run_fuse_knob() == 1 && n <= RUN_SMALL_N);
    if (n <= RUN_SMALL_N && NT > 256 && ((int64_t)1 << lw) >= 256 * IT)
        return merge_level_it<K, 256, IT>(src, dst, n, lw, s, o0, o1, fuse, hook);
    if (((int64_t)1 << lw) >= NT * IT) return merge_level_it<K, NT, IT>(src, dst, n, lw, s, o0, o1, fuse, hook);
    return merge_level_it<K, 256, IT>(src, dst, n, lw, s, o0, o1, fuse, hook);  // runs shorter than the default tile
}

template hipError_t merge_level<uint32_t>(const uint32_t*, uint32_t*, int64_t, int, hipStream_t, int64_t,
                                          int64_t, LaunchHook*);
template hipError_t merge_level<uint64_t>(const uint64_t*, uint64_t*, int64_t, int, hipStream_t, int64_t,
                                          int64_t, LaunchHook*);
template hipError_t merge_level<u128>(const u128*, u128*, int64_t, int, hipStream_t, int64_t, int64_t, LaunchHook*);

}  // namespace misort
