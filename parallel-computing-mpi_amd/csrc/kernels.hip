// kernels.hip -- gfx950 (CDNA4) bitonic sort kernels.
//
// Replaces the reference's local std::sort (psort.cc:175) and the merge loop of
// compare_split_{max,min} (psort.cc:116-164).  Written for wave64 / 160 KiB LDS /
// 8 TB/s HBM3E; no MFMA (sorting is not a contraction).
//
// Sorting network: bitonic sort in the "flip" formulation.  Level m (blocks of
// s = 2^m keys) starts with the flip stage, which compares i with its mirror
// i ^ (s-1), and continues with half-cleaner stages i <-> i ^ 2^j for
// j = m-2 .. 0.  Every compare-exchange puts the minimum at the lower index, so
// no direction bits exist and every block is ascending after its level.  A
// sentinel (all-ones) suffix can only move upwards, so the padding of n up to a
// power of two is VIRTUAL: indices >= n read as all-ones and are never stored.
//
// Three kernel families sweep the network:
//   k_tile_sort   levels 1..LT of one 2^LT-key tile held in LDS (64 KiB);
//   k_global_pass R (<=5) consecutive large strides of one level, fused in
//                 registers: each lane holds 2^R rows x one 16-byte vector,
//                 every row a fully coalesced 1 KiB wave access;
//   k_tile_merge  the strides < 2^LT of one level, in an LDS tile.
// Inside an LDS tile a "phase" gives each lane the 32 keys that differ only in a
// 5-bit window [b, b+5) of the index; the phase's stages run in registers and
// the XOR swizzle phys(i) = i ^ ((i >> 5) & 31) keeps every ds_read/ds_write of
// a phase bank-conflict free for all windows.
//
// A pass over 2^k keys moves 2 * 2^k * sizeof(K) algorithmic HBM bytes.
#include "kernels.h"

namespace misort {
namespace {

template <typename K>
struct KT;
template <>
struct KT<uint32_t> {
    static constexpr uint32_t MAX = 0xFFFFFFFFu;
    static constexpr int V = 4;     // keys per 16-byte vector
    static constexpr int LT = 14;   // log2 keys per LDS tile (64 KiB)
    static constexpr int NT = 512;  // tile workgroup: 32 keys per lane
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
};
template <>
struct KT<uint64_t> {
    static constexpr uint64_t MAX = ~0ull;
    static constexpr int V = 2;
    static constexpr int LT = 13;
    static constexpr int NT = 256;
    typedef uint64_t vec __attribute__((ext_vector_type(2)));
};

constexpr int RMAX = 5;         // strides fused per global pass
constexpr int GP_THREADS = 256; // global-pass workgroup

__device__ __forceinline__ uint64_t ord_of_f64(uint64_t b) {
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t f64_of_ord(uint64_t o) {
    return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
}

template <typename K>
__device__ __forceinline__ void cx(K& a, K& b) {
    const K lo = __builtin_elementwise_min(a, b);
    const K hi = __builtin_elementwise_max(a, b);
    a = lo;
    b = hi;
}

// 16-byte vector load of keys [i0, i0+V); indices >= n read as the sentinel.
template <typename K, bool ORD>
__device__ __forceinline__ void load_vec(const K* __restrict__ p, int64_t i0, int64_t n,
                                         K (&w)[KT<K>::V]) {
    constexpr int V = KT<K>::V;
    if (i0 + V <= n) {
        const typename KT<K>::vec x = *reinterpret_cast<const typename KT<K>::vec*>(p + i0);
#pragma unroll
        for (int j = 0; j < V; ++j) w[j] = x[j];
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j) w[j] = (i0 + j < n) ? p[i0 + j] : KT<K>::MAX;
    }
    if constexpr (ORD) {
#pragma unroll
        for (int j = 0; j < V; ++j)
            if (i0 + j < n) w[j] = ord_of_f64(w[j]);
    }
}

template <typename K>
__device__ __forceinline__ void store_vec(K* __restrict__ p, int64_t i0, int64_t n,
                                          const K (&w)[KT<K>::V]) {
    constexpr int V = KT<K>::V;
    if (i0 + V <= n) {
        typename KT<K>::vec x;
#pragma unroll
        for (int j = 0; j < V; ++j) x[j] = w[j];
        *reinterpret_cast<typename KT<K>::vec*>(p + i0) = x;
    } else {
#pragma unroll
        for (int j = 0; j < V; ++j)
            if (i0 + j < n) p[i0 + j] = w[j];
    }
}

__device__ __forceinline__ int phys(int i) { return i ^ ((i >> 5) & 31); }

// Stages of one phase on the 32 keys of a lane.  Relative stride bits
// top, top-1, .., top-cnt+1; the first is the flip stage when `flip`.
// top/cnt/flip are wave-uniform, so the guards are scalar branches.
template <typename K>
__device__ __forceinline__ void reg_stages(K (&v)[32], int top, int cnt, bool flip) {
#pragma unroll
    for (int r = 4; r >= 0; --r) {
        if (r > top || r <= top - cnt) continue;
        if (flip && r == top) {
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (!(c & (1 << r))) cx(v[c], v[c ^ ((2 << r) - 1)]);
        } else {
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (!(c & (1 << r))) cx(v[c], v[c | (1 << r)]);
        }
    }
}

// One LDS phase with index window [b, b+5).  The lane's other index bits are
// its thread id.  For a flip phase the keys whose window bit `top` is set take
// the mirrored low bits (below b), so each lane holds both halves of every
// mirror pair.
template <typename K>
__device__ __forceinline__ void lds_phase(K* s, int t, int b, int top, int cnt, bool flip) {
    const int lowm = (1 << b) - 1;
    const int tl = t & lowm;
    const int th = (t >> b) << (b + 5);
    const int tlm = flip ? (tl ^ lowm) : tl;
    K v[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) {
        const int l = ((c >> top) & 1) ? tlm : tl;
        v[c] = s[phys(th | (c << b) | l)];
    }
    reg_stages(v, top, cnt, flip);
#pragma unroll
    for (int c = 0; c < 32; ++c) {
        const int l = ((c >> top) & 1) ? tlm : tl;
        s[phys(th | (c << b) | l)] = v[c];
    }
}

// Half-cleaner strides hi..0 of a level (or the flip first when `flip`).
template <typename K>
__device__ __forceinline__ void lds_strides(K* s, int t, int hi, bool flip) {
    while (hi >= 0) {
        const int b = hi > 4 ? hi - 4 : 0;
        lds_phase<K>(s, t, b, hi - b, hi - b + 1, flip);
        __syncthreads();
        flip = false;
        hi = b - 1;
    }
}

template <typename K, bool ORD>
__device__ __forceinline__ void tile_load(K* s, const K* __restrict__ src, int64_t base,
                                          int64_t n, int t) {
    constexpr int LT = KT<K>::LT, NT = KT<K>::NT, V = KT<K>::V;
#pragma unroll
    for (int k = 0; k < (1 << LT) / (NT * V); ++k) {
        const int e = (k * NT + t) * V;
        K w[V];
        load_vec<K, ORD>(src, base + e, n, w);
#pragma unroll
        for (int j = 0; j < V; ++j) s[phys(e + j)] = w[j];
    }
}

template <typename K>
__device__ __forceinline__ void tile_store(const K* s, K* __restrict__ dst, int64_t base,
                                           int64_t n, int t) {
    constexpr int LT = KT<K>::LT, NT = KT<K>::NT, V = KT<K>::V;
#pragma unroll
    for (int k = 0; k < (1 << LT) / (NT * V); ++k) {
        const int e = (k * NT + t) * V;
        K w[V];
#pragma unroll
        for (int j = 0; j < V; ++j) w[j] = s[phys(e + j)];
        store_vec<K>(dst, base + e, n, w);
    }
}

// Levels 1..LT of the tile starting at blockIdx.x << LT: sorted ascending runs
// of 2^LT keys (the last run holds min(n - base, 2^LT) real keys).
template <typename K, bool ORD>
__global__ __launch_bounds__(KT<K>::NT) void k_tile_sort(const K* __restrict__ in,
                                                          K* __restrict__ out, int64_t n) {
    constexpr int LT = KT<K>::LT;
    __shared__ K s[1 << LT];
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x << LT;
    tile_load<K, ORD>(s, in, base, n, t);
    __syncthreads();
    {   // levels 1..5: window [0,5), 32 consecutive keys per lane
        K v[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) v[c] = s[phys((t << 5) | c)];
#pragma unroll
        for (int m = 1; m <= 5; ++m) reg_stages(v, m - 1, m, true);
#pragma unroll
        for (int c = 0; c < 32; ++c) s[phys((t << 5) | c)] = v[c];
    }
    __syncthreads();
    for (int m = 6; m <= LT; ++m) lds_strides<K>(s, t, m - 1, true);
    tile_store<K>(s, out, base, n, t);
}

// Strides 2^(LT-1) .. 1 of a level m > LT, in place.
template <typename K>
__global__ __launch_bounds__(KT<K>::NT) void k_tile_merge(K* __restrict__ a, int64_t n) {
    constexpr int LT = KT<K>::LT;
    __shared__ K s[1 << LT];
    const int t = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x << LT;
    if (base >= n) return;
    tile_load<K, false>(s, a, base, n, t);
    __syncthreads();
    lds_strides<K>(s, t, LT - 1, false);
    tile_store<K>(s, a, base, n, t);
}

// Wave-uniform global pointer: readfirstlane pins it in SGPRs, so a row access
// is `global_load_dwordx4 v, v_off, s[base]` with ONE 32-bit lane offset shared
// by all rows (two for a flip pass) instead of a 64-bit VGPR address per row.
typedef __attribute__((address_space(1))) char gchar;

template <typename T>
__device__ __forceinline__ gchar* uniform_ptr(T* p) {
    const uint64_t u = reinterpret_cast<uint64_t>(p);
    const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)u);
    const uint32_t h = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
    return reinterpret_cast<gchar*>(((uint64_t)h << 32) | l);
}

template <typename V>
__device__ __forceinline__ V gload(const gchar* p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) V*>(p);
}
template <typename V>
__device__ __forceinline__ void gstore(gchar* p, const V& x) {
    *reinterpret_cast<__attribute__((address_space(1))) V*>(p) = x;
}

// R consecutive strides 2^hi .. 2^(hi-R+1) (hi-R+1 >= LT) of one level, in
// place.  Lane q owns V consecutive "low" positions (index bits below lo) of
// every one of the 2^R rows (bits lo..hi); bits above hi are the batch.  With
// FLIP (first pass of a level, hi = m-1) the rows whose top bit is set take the
// mirrored low positions, i.e. a descending 16-byte vector.
//
// A workgroup's 256*V low positions lie inside one 2^lo row segment
// (lo >= LT > log2(256*V)), so its row bases are uniform.  The host launches
// the bounds-free variant (CHECK=false) for the prefix of workgroups whose rows
// all lie below n and the checked variant for the rest.
template <typename K, int R, bool FLIP, bool CHECK>
__global__ __launch_bounds__(GP_THREADS) void k_global_pass(K* __restrict__ a, int64_t n, int hi,
                                                            int64_t block0) {
    constexpr int V = KT<K>::V, ROWS = 1 << R;
    typedef typename KT<K>::vec vec;
    const int lo = hi - R + 1;
    const int64_t w0 = (block0 + blockIdx.x) * (int64_t)(GP_THREADS * V);
    const int64_t wbase = (w0 >> lo) << (hi + 1);
    const uint32_t low = (uint32_t)(w0 & (((int64_t)1 << lo) - 1)) + threadIdx.x * V;
    const uint32_t lowm = ((1u << lo) - 1u) - low - (V - 1);  // mirrored start
    if (CHECK && wbase + low >= n) return;  // every row of this lane is virtual padding
    const uint32_t boff = low * (uint32_t)sizeof(K), boffm = lowm * (uint32_t)sizeof(K);
    K v[ROWS][V];
#pragma unroll
    for (int c = 0; c < ROWS; ++c) {
        const bool mir = FLIP && ((c >> (R - 1)) & 1);
        K w[V];
        if constexpr (CHECK) {
            load_vec<K, false>(a, wbase + ((int64_t)c << lo) + (mir ? lowm : low), n, w);
        } else {
            const gchar* rowp = uniform_ptr(a + wbase + ((int64_t)c << lo));
            const vec x = gload<vec>(rowp + (mir ? boffm : boff));
#pragma unroll
            for (int j = 0; j < V; ++j) w[j] = x[j];
        }
#pragma unroll
        for (int j = 0; j < V; ++j) v[c][j] = mir ? w[V - 1 - j] : w[j];
    }
#pragma unroll
    for (int r = R - 1; r >= 0; --r) {
#pragma unroll
        for (int c = 0; c < ROWS; ++c) {
            if (c & (1 << r)) continue;
            const int p = (FLIP && r == R - 1) ? (c ^ (ROWS - 1)) : (c | (1 << r));
#pragma unroll
            for (int j = 0; j < V; ++j) cx(v[c][j], v[p][j]);
        }
    }
#pragma unroll
    for (int c = 0; c < ROWS; ++c) {
        const bool mir = FLIP && ((c >> (R - 1)) & 1);
        K w[V];
#pragma unroll
        for (int j = 0; j < V; ++j) w[j] = mir ? v[c][V - 1 - j] : v[c][j];
        if constexpr (CHECK) {
            store_vec<K>(a, wbase + ((int64_t)c << lo) + (mir ? lowm : low), n, w);
        } else {
            gchar* rowp = uniform_ptr(a + wbase + ((int64_t)c << lo));
            vec x;
#pragma unroll
            for (int j = 0; j < V; ++j) x[j] = w[j];
            gstore<vec>(rowp + (mir ? boffm : boff), x);
        }
    }
}

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

template <typename K>
__global__ void k_merge_partition(const K* __restrict__ A, int64_t na, const K* __restrict__ B,
                                  int64_t nb, int64_t d0, int64_t nout, int64_t ntiles,
                                  int64_t* __restrict__ co) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    const int64_t off = t * MS_TILE < nout ? t * MS_TILE : nout;
    co[t] = corank(A, na, B, nb, d0 + off);
}

// Output keys [d0 + t*TILE, ...) of merge(A, B): each workgroup stages its A
// and B ranges in LDS, each lane merges MS_ITEMS consecutive outputs.
template <typename K>
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
    for (int k = threadIdx.x; k < la; k += MS_NT) s[k] = A[i0 + k];
    for (int k = threadIdx.x; k < lb; k += MS_NT) s[la + k] = B[j0 + k];
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
    for (int k = threadIdx.x; k < len; k += MS_NT) out[ds + k] = s[k];
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

__global__ void k_f64_ord(uint64_t* a, int64_t n, int to_ord) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        a[i] = to_ord ? ord_of_f64(a[i]) : f64_of_ord(a[i]);
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

int ceil_log2(int64_t n) {
    int k = 0;
    while (((int64_t)1 << k) < n) ++k;
    return k;
}

int stream_grid(int64_t n, int threads) {
    int64_t g = (n + threads - 1) / threads;
    if (g > 2048) g = 2048;
    return g < 1 ? 1 : (int)g;
}

struct HookScope {
    LaunchHook* h;
    Kind k;
    hipStream_t s;
    HookScope(LaunchHook* h_, Kind k_, double bytes, hipStream_t s_) : h(h_), k(k_), s(s_) {
        if (h) h->before(k, bytes, s);
    }
    ~HookScope() {
        if (h) h->after(k, s);
    }
};

template <typename K, int R>
void launch_global(bool flip, K* a, int64_t n, int hi, int k, hipStream_t s) {
    constexpr int V = KT<K>::V;
    const int lo = hi - R + 1;
    const int64_t lanes = ((int64_t)1 << k) / ((int64_t)(1 << R) * V);
    const int64_t blocks = lanes / GP_THREADS;
    // workgroups per 2^lo segment; segments below n >> (hi+1) are entirely real
    const int64_t per_seg = ((int64_t)1 << lo) / (GP_THREADS * V);
    int64_t full = (n >> (hi + 1)) * per_seg;
    if (full > blocks) full = blocks;
    if (full > 0) {
        if (flip) k_global_pass<K, R, true, false><<<(unsigned)full, GP_THREADS, 0, s>>>(a, n, hi, 0);
        else k_global_pass<K, R, false, false><<<(unsigned)full, GP_THREADS, 0, s>>>(a, n, hi, 0);
    }
    if (blocks > full) {
        const unsigned rest = (unsigned)(blocks - full);
        if (flip) k_global_pass<K, R, true, true><<<rest, GP_THREADS, 0, s>>>(a, n, hi, full);
        else k_global_pass<K, R, false, true><<<rest, GP_THREADS, 0, s>>>(a, n, hi, full);
    }
}

template <typename K>
void launch_global_r(int r, bool flip, K* a, int64_t n, int hi, int k, hipStream_t s) {
    switch (r) {
        case 1: launch_global<K, 1>(flip, a, n, hi, k, s); break;
        case 2: launch_global<K, 2>(flip, a, n, hi, k, s); break;
        case 3: launch_global<K, 3>(flip, a, n, hi, k, s); break;
        case 4: launch_global<K, 4>(flip, a, n, hi, k, s); break;
        default: launch_global<K, 5>(flip, a, n, hi, k, s); break;
    }
}

}  // namespace

int tile_log2(int key_bytes) { return key_bytes == 4 ? KT<uint32_t>::LT : KT<uint64_t>::LT; }

template <typename K>
hipError_t local_sort(const K* in, K* out, int64_t n, bool ord_in, hipStream_t s,
                      LaunchHook* hook) {
    constexpr int LT = KT<K>::LT, NT = KT<K>::NT;
    if (n <= 0) return hipSuccess;
    const int k = ceil_log2(n);
    const unsigned tiles = (unsigned)((n + (1 << LT) - 1) >> LT);
    const double pass_bytes = 2.0 * (double)n * sizeof(K);
    {
        HookScope hs(hook, KIND_TILE_SORT, pass_bytes, s);
        if constexpr (sizeof(K) == 8) {
            if (ord_in) k_tile_sort<K, true><<<tiles, NT, 0, s>>>(in, out, n);
            else k_tile_sort<K, false><<<tiles, NT, 0, s>>>(in, out, n);
        } else {
            if (ord_in) return hipErrorInvalidValue;
            k_tile_sort<K, false><<<tiles, NT, 0, s>>>(in, out, n);
        }
    }
    for (int m = LT + 1; m <= k; ++m) {
        int hi = m - 1;
        bool first = true;
        while (hi >= LT) {
            const int r = hi - LT + 1 < RMAX ? hi - LT + 1 : RMAX;
            HookScope hs(hook, KIND_GLOBAL, pass_bytes, s);
            launch_global_r<K>(r, first, out, n, hi, k, s);
            hi -= r;
            first = false;
        }
        HookScope hs(hook, KIND_TILE_MERGE, pass_bytes, s);
        k_tile_merge<K><<<tiles, NT, 0, s>>>(out, n);
    }
    return hipGetLastError();
}

template <typename K>
hipError_t merge_split(const K* a, int64_t na, const K* b, int64_t nb, K* out, int keep_max,
                       int64_t* scratch, hipStream_t s, LaunchHook* hook) {
    if (na <= 0) return hipSuccess;
    const int64_t d0 = keep_max ? nb : 0;
    const int64_t ntiles = (na + MS_TILE - 1) / MS_TILE;
    HookScope hs(hook, KIND_MERGE_SPLIT, (double)(2 * na + (nb < na ? nb : na)) * sizeof(K), s);
    k_merge_partition<K><<<(unsigned)((ntiles + 1 + 255) / 256), 256, 0, s>>>(a, na, b, nb, d0, na,
                                                                              ntiles, scratch);
    k_merge_tiles<K><<<(unsigned)ntiles, MS_NT, 0, s>>>(a, na, b, nb, d0, na, scratch, out);
    return hipGetLastError();
}

template <typename T>
hipError_t count_descents(const T* a, int64_t n, unsigned long long* count, hipStream_t s) {
    if (n < 2) return hipSuccess;
    k_count_desc<T><<<stream_grid(n, 256), 256, 0, s>>>(a, n, count);
    return hipGetLastError();
}

hipError_t f64_to_ord(uint64_t* a, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_f64_ord<<<stream_grid(n, 256), 256, 0, s>>>(a, n, 1);
    return hipGetLastError();
}

hipError_t ord_to_f64(uint64_t* a, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    k_f64_ord<<<stream_grid(n, 256), 256, 0, s>>>(a, n, 0);
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

template hipError_t local_sort<uint32_t>(const uint32_t*, uint32_t*, int64_t, bool, hipStream_t,
                                         LaunchHook*);
template hipError_t local_sort<uint64_t>(const uint64_t*, uint64_t*, int64_t, bool, hipStream_t,
                                         LaunchHook*);
template hipError_t merge_split<uint32_t>(const uint32_t*, int64_t, const uint32_t*, int64_t,
                                          uint32_t*, int, int64_t*, hipStream_t, LaunchHook*);
template hipError_t merge_split<uint64_t>(const uint64_t*, int64_t, const uint64_t*, int64_t,
                                          uint64_t*, int, int64_t*, hipStream_t, LaunchHook*);
template hipError_t count_descents<uint32_t>(const uint32_t*, int64_t, unsigned long long*,
                                             hipStream_t);
template hipError_t count_descents<uint64_t>(const uint64_t*, int64_t, unsigned long long*,
                                             hipStream_t);
template hipError_t count_descents<double>(const double*, int64_t, unsigned long long*,
                                           hipStream_t);

}  // namespace misort
