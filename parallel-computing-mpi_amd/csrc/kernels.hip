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
// Passes over HBM (each moves every key once in and once out):
//   k_stream<SORT>   levels 1..LT of every 2^LT-key tile (LDS, 64 KiB + pad);
//   k_stream<ROWS>   up to 9 consecutive large strides of one level: a tile is
//                    2^R rows at the stride distance times 2^(LT-R) consecutive
//                    keys, so every row segment is a coalesced >= 128 B run;
//   k_stream<MERGE>  the strides < 2^LT of one level, in an LDS tile;
//   k_global_pass    (optional, MISORT_REGPASS) register-only large strides.
// All of them share one persistent, register-prefetching tile engine.
//
// A pass over 2^k keys moves 2 * 2^k * sizeof(K) algorithmic HBM bytes.
#include "kernels.h"

#include <stdlib.h>

namespace misort {
namespace {

template <typename K>
struct KT;
template <>
struct KT<uint32_t> {
    static constexpr uint32_t MAX = 0xFFFFFFFFu;
    static constexpr int V = 4;     // keys per 16-byte vector
    static constexpr int LT = 14;   // log2 keys per LDS tile (64 KiB + padding)
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
};
template <>
struct KT<uint64_t> {
    static constexpr uint64_t MAX = ~0ull;
    static constexpr int V = 2;
    static constexpr int LT = 13;
    typedef uint64_t vec __attribute__((ext_vector_type(2)));
};

constexpr int RMAX = 5;         // strides fused per register-only global pass
constexpr int RMAX_ROWS = 9;    // strides fused per ROWS (LDS) pass
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

// ------------------------------------------------- streaming tile engine
//
// Persistent workgroups walk a list of 2^LT-key tiles.  While the LDS phases of
// tile i run, the 16-byte loads of tile i+1 are already in flight into a
// register buffer, so HBM streams continuously with 2 workgroups per CU.
//
// A tile is a set of 2^LT keys that one network segment touches only among
// themselves, addressed through a "virtual" index v in [0, 2^LT):
//   CONTIG   v -> tile*2^LT + v                       (tile sort / tile merge)
//   ROWS     v = (c << logB) | j -> wbase + (c << lo) + low(c) + j
//            2^R rows c at global stride 2^lo (the R strides 2^hi..2^lo of one
//            level, R = LT - logB) times B = 2^logB consecutive keys.  For the
//            first pass of a level (flip), rows whose top bit is set start at
//            the mirrored block 2^lo - L0 - B, which turns the level's global
//            flip i <-> i ^ (2^(hi+1) - 1) into the tile's own flip v <-> ~v.
//
// Register slots: lane t loads LOADS = 32/V vectors, slot k = virtual keys
// (k*NT + t)*V .. +V-1, so the top KB = log2(LOADS) virtual bits are the slot
// index and the bottom VB = log2(V) bits the vector component.  Strides on
// those bits run in registers before the LDS write (slots) and after the LDS
// read (components); only the strides in between cost an LDS phase.  For a
// flip on the top slot bit the upper slots load the mirrored lane's vector
// reversed, so every mirror pair meets in one lane at one component.
//
// LDS layout: key v at word v + v/32.  The padding keeps every phase's
// 32-lane accesses on distinct banks, and since v + v/32 is additive over
// disjoint bit fields every access is one base VGPR plus an immediate offset.
enum TileMode : int { TM_SORT = 0, TM_MERGE = 1, TM_ROWS = 2 };

struct TileMap {
    int64_t ntiles;  // real tiles (a prefix of the tile list)
    int lo, hi, logB, flip;
};

template <typename K, int LT>
struct TileGeo {
    static constexpr int T = 1 << LT, NT = T / 32, V = KT<K>::V, LOADS = T / (NT * V);
    static constexpr int KB = LOADS == 16 ? 4 : LOADS == 8 ? 3 : LOADS == 4 ? 2 : 1;
    static constexpr int VB = V == 4 ? 2 : 1;
};

__host__ __device__ constexpr int pad(int v) { return v + (v >> 5); }

template <int LT, int MODE>
__device__ __forceinline__ int64_t tile_index(const TileMap& m, int64_t tile, int e) {
    if constexpr (MODE != TM_ROWS) {
        return (tile << LT) + e;
    } else {
        const int R = LT - m.logB;
        const int sh = m.lo - m.logB;  // log2 tiles per 2^(hi+1) segment
        const int64_t seg = tile >> sh, lb = tile & (((int64_t)1 << sh) - 1);
        const int64_t L0 = lb << m.logB;
        const int c = e >> m.logB, j = e & ((1 << m.logB) - 1);
        const bool mir = m.flip && ((c >> (R - 1)) & 1);
        const int64_t low = mir ? (((int64_t)1 << m.lo) - L0 - ((int64_t)1 << m.logB)) : L0;
        return (seg << (m.hi + 1)) + ((int64_t)c << m.lo) + low + j;
    }
}

// Every key of the tile lies below n (then no per-element bounds checks).
template <int LT, int MODE>
__device__ __forceinline__ bool tile_full(const TileMap& m, int64_t tile, int64_t n) {
    if constexpr (MODE != TM_ROWS) {
        return ((tile + 1) << LT) <= n;
    } else {
        return (((tile >> (m.lo - m.logB)) + 1) << (m.hi + 1)) <= n;
    }
}

// Slot k of lane t: virtual vector start, and whether it is held mirrored.
template <typename K, int LT, bool MIRROR>
__device__ __forceinline__ int slot_lane(int k, int t) {
    typedef TileGeo<K, LT> G;
    return (MIRROR && k >= G::LOADS / 2) ? (G::NT - 1 - t) : t;
}

template <typename K, int LT, int MODE, bool MIRROR, bool ORD>
__device__ __forceinline__ void tile_fetch(K (*pre)[KT<K>::V], const K* src, const TileMap& m,
                                           int64_t tile, int64_t n, int t) {
    typedef TileGeo<K, LT> G;
    const bool full = tile_full<LT, MODE>(m, tile, n);
#pragma unroll
    for (int k = 0; k < G::LOADS; ++k) {
        const int e = (k * G::NT + slot_lane<K, LT, MIRROR>(k, t)) * G::V;
        const int64_t gi = tile_index<LT, MODE>(m, tile, e);
        typename KT<K>::vec x;
        if (full) {
            // streamed once per pass: non-temporal (measured +10 % on this shape,
            // tools/hbm_shapes.hip)
            x = __builtin_nontemporal_load(reinterpret_cast<const typename KT<K>::vec*>(src + gi));
            if constexpr (ORD) {
#pragma unroll
                for (int j = 0; j < G::V; ++j) x[j] = ord_of_f64(x[j]);
            }
        } else {
            K w[G::V];
            load_vec<K, ORD>(src, gi, n, w);
#pragma unroll
            for (int j = 0; j < G::V; ++j) x[j] = w[j];
        }
        const bool mk = MIRROR && k >= G::LOADS / 2;
#pragma unroll
        for (int j = 0; j < G::V; ++j) pre[k][j] = mk ? x[G::V - 1 - j] : x[j];
    }
}

template <typename K, int LT, int MODE>
__device__ __forceinline__ void store_slot(K* dst, const TileMap& m, int64_t tile, int64_t n,
                                           bool full, int e, const K (&w)[KT<K>::V]) {
    const int64_t gi = tile_index<LT, MODE>(m, tile, e);
    if (full) {
        typename KT<K>::vec x;
#pragma unroll
        for (int j = 0; j < KT<K>::V; ++j) x[j] = w[j];
        __builtin_nontemporal_store(x, reinterpret_cast<typename KT<K>::vec*>(dst + gi));
    } else {
        store_vec<K>(dst, gi, n, w);
    }
}

// Compile-time stage list on 32 register keys: relative bits TOP..TOP-CNT+1.
template <typename K, int TOP, int CNT, bool FLIP>
__device__ __forceinline__ void reg_stages_c(K (&v)[32]) {
#pragma unroll
    for (int r = TOP; r > TOP - CNT; --r) {
        const bool fl = FLIP && r == TOP;
#pragma unroll
        for (int c = 0; c < 32; ++c)
            if (!(c & (1 << r))) cx(v[c], v[fl ? (c ^ ((2 << r) - 1)) : (c | (1 << r))]);
    }
}

// One LDS phase, window [B, B+5) of the virtual index, compile-time shape.
template <typename K, int B, int TOP, int CNT, bool FLIP>
__device__ __forceinline__ void phase_c(K* s, int t) {
    constexpr int lowm = (1 << B) - 1;
    const int tl = t & lowm;
    const int th = (t >> B) << (B + 5);
    const int a0 = pad(th | tl);
    const int a1 = FLIP ? pad(th | (tl ^ lowm)) : a0;
    K v[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) v[c] = s[(((c >> TOP) & 1) ? a1 : a0) + pad(c << B)];
    reg_stages_c<K, TOP, CNT, FLIP>(v);
#pragma unroll
    for (int c = 0; c < 32; ++c) s[(((c >> TOP) & 1) ? a1 : a0) + pad(c << B)] = v[c];
}

// Strides HI..STOP of the virtual index through LDS phases (flip first).
template <typename K, int HI, int STOP, bool FLIP>
__device__ __forceinline__ void lds_range(K* s, int t) {
    if constexpr (HI >= STOP) {
        constexpr int B = HI > 4 ? HI - 4 : 0;
        constexpr int LOWEST = B > STOP ? B : STOP;
        phase_c<K, B, HI - B, HI - LOWEST + 1, FLIP>(s, t);
        __syncthreads();
        lds_range<K, LOWEST - 1, STOP, false>(s, t);
    }
}

// Levels L..LT of the tile sort (level 1..5 done by the caller).
template <typename K, int L, int LT>
__device__ __forceinline__ void sort_levels(K* s, int t) {
    if constexpr (L <= LT) {
        lds_range<K, L - 1, 0, true>(s, t);
        sort_levels<K, L + 1, LT>(s, t);
    }
}

template <typename K, int LT, int MODE, int R, bool FLIP, bool ORD>
__global__ __launch_bounds__((TileGeo<K, LT>::NT), (2 * TileGeo<K, LT>::NT / 256)) void k_stream(
    const K* in, K* out, int64_t n, TileMap m) {
    typedef TileGeo<K, LT> G;
    constexpr bool MIRROR = MODE == TM_ROWS && FLIP;
    // slot-bit strides done in registers before the LDS write
    constexpr int PRE = MODE == TM_MERGE ? G::KB : MODE == TM_ROWS ? (R < G::KB ? R : G::KB) : 0;
    __shared__ K s[pad(G::T)];
    const int t = threadIdx.x;
    K pre[G::LOADS][G::V];
    int64_t tile = blockIdx.x;
    if (tile >= m.ntiles) return;
    tile_fetch<K, LT, MODE, MIRROR, ORD>(pre, in, m, tile, n, t);
    for (; tile < m.ntiles; tile += gridDim.x) {
#pragma unroll
        for (int i = 0; i < PRE; ++i) {
            const int r = G::KB - 1 - i;
            const bool fl = MIRROR && i == 0;
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                if (k & (1 << r)) continue;
                const int p = fl ? (k ^ (G::LOADS - 1)) : (k | (1 << r));
#pragma unroll
                for (int j = 0; j < G::V; ++j) cx(pre[k][j], pre[p][j]);
            }
        }
        const bool full = tile_full<LT, MODE>(m, tile, n);
        if constexpr (MODE == TM_ROWS && R <= G::KB) {
            // every stride of this pass was a slot bit: store straight from registers
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                K w[G::V];
                const bool mk = MIRROR && k >= G::LOADS / 2;
#pragma unroll
                for (int j = 0; j < G::V; ++j) w[j] = mk ? pre[k][G::V - 1 - j] : pre[k][j];
                store_slot<K, LT, MODE>(out, m, tile, n, full,
                                        (k * G::NT + slot_lane<K, LT, MIRROR>(k, t)) * G::V, w);
            }
            const int64_t nxt = tile + gridDim.x;
            if (nxt < m.ntiles) tile_fetch<K, LT, MODE, MIRROR, ORD>(pre, in, m, nxt, n, t);
        } else {
            // registers -> LDS (mirrored slots to their own virtual position)
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                const bool mk = MIRROR && k >= G::LOADS / 2;
                const int e = (k * G::NT + slot_lane<K, LT, MIRROR>(k, t)) * G::V;
#pragma unroll
                for (int j = 0; j < G::V; ++j) s[pad(e + j)] = mk ? pre[k][G::V - 1 - j] : pre[k][j];
            }
            __syncthreads();
            const int64_t nxt = tile + gridDim.x;
            if (nxt < m.ntiles) tile_fetch<K, LT, MODE, MIRROR, ORD>(pre, in, m, nxt, n, t);
            if constexpr (MODE == TM_SORT) {
                {   // levels 1..5: window [0,5), 32 consecutive keys per lane
                    K v[32];
                    const int a0 = pad(t << 5);
#pragma unroll
                    for (int c = 0; c < 32; ++c) v[c] = s[a0 + c];
                    reg_stages_c<K, 0, 1, true>(v);
                    reg_stages_c<K, 1, 2, true>(v);
                    reg_stages_c<K, 2, 3, true>(v);
                    reg_stages_c<K, 3, 4, true>(v);
                    reg_stages_c<K, 4, 5, true>(v);
#pragma unroll
                    for (int c = 0; c < 32; ++c) s[a0 + c] = v[c];
                }
                __syncthreads();
                sort_levels<K, 6, LT>(s, t);
            } else if constexpr (MODE == TM_MERGE) {
                lds_range<K, LT - G::KB - 1, G::VB, false>(s, t);
            } else {
                lds_range<K, LT - G::KB - 1, LT - R, false>(s, t);
            }
            // LDS -> registers -> HBM; in a merge the vector-component strides run here
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                const int e = (k * G::NT + t) * G::V;
                K w[G::V];
#pragma unroll
                for (int j = 0; j < G::V; ++j) w[j] = s[pad(e + j)];
                if constexpr (MODE == TM_MERGE) {
#pragma unroll
                    for (int r = G::VB - 1; r >= 0; --r)
#pragma unroll
                        for (int j = 0; j < G::V; ++j)
                            if (!(j & (1 << r))) cx(w[j], w[j | (1 << r)]);
                }
                store_slot<K, LT, MODE>(out, m, tile, n, full, e, w);
            }
            __syncthreads();
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

template <typename K>
__global__ void k_gather_samples(const K* __restrict__ a, int64_t n, int64_t stride, K* __restrict__ out,
                                 int64_t count) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= count) return;
    const int64_t x = c * stride < n - 1 ? c * stride : n - 1;
    out[c] = a[x];
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

namespace {

// Pass-planner knobs (environment, read once): MISORT_RMAX = most strides one
// ROWS pass fuses (default 9), MISORT_REGPASS = largest stride count that uses
// the register-only pass instead (default 0 = never).
struct PlanKnobs {
    int rmax = RMAX_ROWS, regpass = 0;
    int grid_mult = 0;  // MISORT_GRID_MULT: persistent grid = mult x resident capacity; 0 (default) =
                        // one tile per workgroup, measured faster than any persistent grid
    PlanKnobs() {
        if (const char* e = getenv("MISORT_GRID_MULT")) grid_mult = atoi(e) < 0 ? 0 : atoi(e);
        if (const char* e = getenv("MISORT_RMAX")) rmax = atoi(e) < 1 ? 1 : atoi(e);
        if (rmax > RMAX_ROWS) rmax = RMAX_ROWS;
        if (const char* e = getenv("MISORT_REGPASS")) regpass = atoi(e);
        if (regpass > RMAX) regpass = RMAX;
    }
};
const PlanKnobs& knobs() {
    static PlanKnobs k;
    return k;
}

template <typename K, int LT, int MODE, int R, bool FLIP, bool ORD>
void launch_stream(const K* in, K* out, int64_t n, const TileMap& m, hipStream_t s) {
    typedef TileGeo<K, LT> G;
    static int64_t cap = 0;  // resident workgroups for this instantiation
    if (cap == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_stream<K, LT, MODE, R, FLIP, ORD>,
                                                           G::NT, 0);
        cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
    }
    const int gm = knobs().grid_mult;
    const int64_t want = gm == 0 ? m.ntiles : cap * gm;
    const int64_t grid = m.ntiles < want ? m.ntiles : want;
    if (grid > 0) k_stream<K, LT, MODE, R, FLIP, ORD><<<(unsigned)grid, G::NT, 0, s>>>(in, out, n, m);
}

template <typename K, int R>
void launch_rows_r(K* a, int64_t n, const TileMap& m, hipStream_t s) {
    constexpr int LT = KT<K>::LT;
    if (m.flip) launch_stream<K, LT, TM_ROWS, R, true, false>(a, a, n, m, s);
    else launch_stream<K, LT, TM_ROWS, R, false, false>(a, a, n, m, s);
}

// One ROWS pass: strides 2^hi .. 2^(hi-R+1) of a level over 2^k (virtual) keys.
template <typename K>
void launch_rows(K* a, int64_t n, int hi, int R, bool flip, hipStream_t s) {
    constexpr int LT = KT<K>::LT;
    TileMap m{};
    m.lo = hi - R + 1;
    m.hi = hi;
    m.logB = LT - R;
    m.flip = flip;
    const int64_t per_seg = ((int64_t)1 << m.lo) >> m.logB;
    const int64_t full_segs = n >> (hi + 1);
    const int64_t rem = n - (full_segs << (hi + 1));
    int64_t part = (rem + ((int64_t)1 << m.logB) - 1) >> m.logB;
    if (part > per_seg) part = per_seg;
    m.ntiles = full_segs * per_seg + part;
    switch (R) {
        case 1: launch_rows_r<K, 1>(a, n, m, s); break;
        case 2: launch_rows_r<K, 2>(a, n, m, s); break;
        case 3: launch_rows_r<K, 3>(a, n, m, s); break;
        case 4: launch_rows_r<K, 4>(a, n, m, s); break;
        case 5: launch_rows_r<K, 5>(a, n, m, s); break;
        case 6: launch_rows_r<K, 6>(a, n, m, s); break;
        case 7: launch_rows_r<K, 7>(a, n, m, s); break;
        case 8: launch_rows_r<K, 8>(a, n, m, s); break;
        default: launch_rows_r<K, 9>(a, n, m, s); break;
    }
}

}  // namespace

template <typename K>
hipError_t local_sort(const K* in, K* out, int64_t n, bool ord_in, hipStream_t s,
                      LaunchHook* hook) {
    constexpr int LT = KT<K>::LT;
    if (n <= 0) return hipSuccess;
    const int k = ceil_log2(n);
    const double pass_bytes = 2.0 * (double)n * sizeof(K);
    TileMap tm{};
    tm.ntiles = (n + (1 << LT) - 1) >> LT;
    {
        HookScope hs(hook, KIND_TILE_SORT, pass_bytes, s);
        if constexpr (sizeof(K) == 8) {
            if (ord_in) launch_stream<K, LT, TM_SORT, 0, false, true>(in, out, n, tm, s);
            else launch_stream<K, LT, TM_SORT, 0, false, false>(in, out, n, tm, s);
        } else {
            if (ord_in) return hipErrorInvalidValue;
            launch_stream<K, LT, TM_SORT, 0, false, false>(in, out, n, tm, s);
        }
    }
    const PlanKnobs& kn = knobs();
    for (int m = LT + 1; m <= k; ++m) {
        // strides 2^(m-1) .. 2^LT split into near-equal passes of <= rmax
        const int x = m - LT;
        const int parts = (x + kn.rmax - 1) / kn.rmax;
        int hi = m - 1;
        for (int p = 0; p < parts; ++p) {
            const int R = x / parts + (p < x % parts ? 1 : 0);
            HookScope hs(hook, KIND_GLOBAL, pass_bytes, s);
            if (R <= kn.regpass) launch_global_r<K>(R, p == 0, out, n, hi, k, s);
            else launch_rows<K>(out, n, hi, R, p == 0, s);
            hi -= R;
        }
        HookScope hs(hook, KIND_TILE_MERGE, pass_bytes, s);
        launch_stream<K, LT, TM_MERGE, 0, false, false>(out, out, n, tm, s);
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

template <typename K>
hipError_t gather_samples(const K* a, int64_t n, int64_t stride, K* out, int64_t count, hipStream_t s) {
    if (n <= 0 || count <= 0) return hipSuccess;
    k_gather_samples<K><<<(unsigned)((count + 255) / 256), 256, 0, s>>>(a, n, stride, out, count);
    return hipGetLastError();
}
template hipError_t gather_samples<uint32_t>(const uint32_t*, int64_t, int64_t, uint32_t*, int64_t, hipStream_t);
template hipError_t gather_samples<uint64_t>(const uint64_t*, int64_t, int64_t, uint64_t*, int64_t, hipStream_t);

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
