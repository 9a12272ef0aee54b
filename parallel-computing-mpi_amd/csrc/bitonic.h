// bitonic.h -- the gfx950 (CDNA4) bitonic tile engine and its pass planner.
//
// Replaces the reference's local std::sort (psort.cc:175).  Written for wave64 /
// 160 KiB LDS / 8 TB/s HBM3E; no MFMA (sorting is not a contraction).  Included
// by one translation unit per key type (sort_u32.hip, sort_u64.hip), which
// instantiate local_sort<K>; kernels.hip uses only the shared device helpers.
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
//   k_stream<SORT>   levels 1..LT of every 2^LT-key tile in LDS;
//   k_stream<ROWS>   up to LT-5 consecutive large strides of one level: a tile
//                    is 2^R rows at the stride distance times 2^(LT-R)
//                    consecutive keys, so every row segment is a coalesced
//                    >= 128 B run;
//   k_stream<MERGE>  the strides < 2^LT of one level, in an LDS tile;
//   k_stream<SPAN>   the last LT-R strides of level m (2^(LT-R-1)..1) AND the
//                    first R strides of level m+1 (its flip, then
//                    2^(m-1)..2^(m-R+1)) in one ROWS-shaped tile, so the pass
//                    boundary need not fall on a level boundary (see plan()).
// All of them share one tile engine (one-shot or persistent + prefetching).
//
// A pass over n keys moves 2 * n * sizeof(K) algorithmic HBM bytes.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "kernels.h"
#include "pass_costs.h"

namespace misort {

// Pass-planner knobs (environment, read once per process, kernels.hip):
//   MISORT_TILE_LOG2       SORT/MERGE tile, log2 u32 keys: 15 (default: 128 KiB
//                          of LDS, one 1024-lane workgroup per CU) or 14 (64 KiB,
//                          two 512-lane workgroups per CU); u64 tiles are half;
//   MISORT_ROWS_TILE_LOG2  the same for ROWS passes (default 15);
//   MISORT_RMAX            most strides one ROWS pass fuses (cap LT_rows - 5);
//   MISORT_PERSIST         tile modes (bit 1 << TileMode: 1 SORT, 2 MERGE, 4 ROWS)
//                          that run a persistent grid of MISORT_GRID_MULT x the
//                          resident capacity with the next tile's loads in
//                          flight (default 3); the others launch one workgroup
//                          per tile;
//   MISORT_PINGPONG        1 (default): passes alternate between the output and
//                          a scratch buffer (copy-shaped HBM traffic); 0: in place;
//   MISORT_SPAN            1 (default): plan passes across level boundaries with
//                          SPAN passes (fewest passes); 0: one MERGE per level;
//   MISORT_ROW_BYTES_LOG2  shortest row run a ROWS/SPAN tile may use (default 8:
//                          256 B; 7 allows 128-B rows);
//   MISORT_COST_TABLE      1 (default): the planner prices passes from the
//                          measured table (pass_costs.h); 0: from the model;
//   MISORT_TILE_LOG2_U64, MISORT_ROWS_TILE_LOG2_U64, MISORT_PERSIST_U64
//                          the tile sizes (14 or 13) and persistent modes of
//                          the u64 (and f64) sort, chosen apart from u32's.
//                          Default 13/13/1: two 512-lane workgroups per CU and
//                          only the SORT pass persistent -- 8.11 -> 8.76 Gkeys/s
//                          at 2^29 u64 although the plan has 3 more passes
//                          (profiles/r01/ab/u64_tiles.txt);
//   MISORT_SORT_U32        1 (default): the u32 SORT pass runs k_sort_u32; 0: k_stream.
struct PlanKnobs {
    int tile_u32 = 15, rows_tile_u32 = 15, rmax = 10, persist = 3 | 8, grid_mult = 1, pingpong = 1;
    int span = 1, row_bytes_log2 = 8, cost_table = 1, wide = 1;
    int tile_u64 = 13, rows_tile_u64 = 13, persist_u64 = 1, sort_u32 = 1;
    // first level finished by merge passes (runs.hip) instead of the network
    // (0 = network only), per key type.  Measured at 2^30 u32 / 2^29 u64: the
    // SORT tile's level is best (profiles/r01/runs/).
    int merge_from_u32 = 15, merge_from_u64 = 13;
    // u32 sorts of at most 2^merge_min_log2 keys (cache-resident) stay on the
    // network, whose passes are shorter there.  Against the multi-way passes
    // (round 2, profiles/r02/s2f): 2^20 0.171 vs 0.183 ms, 2^22 0.255 vs
    // 0.296, but 2^24 0.580 vs 0.479 ms (three 8-way passes beat ~14 network
    // passes), so 2^24 (BASELINE config 2) now takes the merge passes.
    int merge_min_log2_u32 = 23;
    // u32 merge levels: up to this many levels per multi-way pass (runsk.hip,
    // 2^lk-way, lk <= 4); 0 or 1: one 2-way pass per level (MISORT_MULTIWAY).
    // -1 (default): 3 when the L levels past the SORT tile are a multiple of
    // 3 (then 8-way passes only), else 4 (the fewest passes) -- measured per
    // size (profiles/r02/ab_mw_u32): L = 15 (2^30) 8-way 64.1 vs 63.2 Gkeys/s
    // with 16-way, L = 12 63.5 vs 63.2; L = 10, 11, 13, 14 the fewer passes
    // win by 4 / 3 / 1.6 / 0.7 %
    int multiway = -1;
    // the same for u64 (and f64) keys (MISORT_MULTIWAY_U64): 128-bit fences,
    // 8192-key chunks at 2 workgroups per CU.  16-way passes measured faster
    // for u64 at every size (profiles/r02/ab_mw: 2^24 +8 %, 2^26 +4 %, 2^27
    // +1.5 %, 2^29 +2.5 % over 8-way): fewer passes, and u64 chains cost less
    // per byte than u32 ones
    int multiway_u64 = 4;
    PlanKnobs();
    // the cap for L levels
    int multiway_cap(int kb, int L) const {
        if (kb != 4) return multiway_u64;
        if (multiway >= 0) return multiway;
        return L % 3 == 0 ? 3 : 4;
    }
    int merge_from(int kb) const { return kb == 4 ? merge_from_u32 : merge_from_u64; }
    // per key type: the large (128 KiB) SORT/MERGE and ROWS tiles, persistent modes
    bool big(int kb) const { return kb == 4 ? tile_u32 == 15 : tile_u64 == 14; }
    bool rbig(int kb) const { return kb == 4 ? rows_tile_u32 == 15 : rows_tile_u64 == 14; }
    int persist_mask(int kb) const { return kb == 4 ? persist : persist_u64; }
};
const PlanKnobs& plan_knobs();

namespace {

template <typename K>
struct KT;
template <>
struct KT<uint32_t> {
    static constexpr uint32_t MAX = 0xFFFFFFFFu;
    static constexpr int V = 4;         // keys per 16-byte vector
    static constexpr int LT_SMALL = 14; // log2 keys per half-size LDS tile (64 KiB + padding)
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
};
template <>
struct KT<uint64_t> {
    static constexpr uint64_t MAX = ~0ull;
    static constexpr int V = 2;
    static constexpr int LT_SMALL = 13;
    typedef uint64_t vec __attribute__((ext_vector_type(2)));
};

constexpr int RMAX_ROWS = 10;   // most strides one ROWS pass fuses (LT - R >= 5: 128-B row runs)

__device__ __forceinline__ uint64_t ord_of_f64(uint64_t b) {
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t f64_of_ord(uint64_t o) {
    return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
}

// u64 compare-exchanges on one v_cmp_u64 (cx); register stages batch their
// compares ahead of the selects (reg_stages_c).
#ifndef MISORT_CX64_ONECMP
#define MISORT_CX64_ONECMP 1
#endif
#ifndef MISORT_CX64_BATCH
#define MISORT_CX64_BATCH 1
#endif
template <typename K>
__device__ __forceinline__ void cx(K& a, K& b) {
    if constexpr (sizeof(K) == 8 && MISORT_CX64_ONECMP) {
        // no 64-bit min/max: as min and max each would cost a v_cmp_u64 + 2
        // v_cndmask, the selects take one compare -- the empty asm hides that
        // the selected values are the compared ones, so they are not folded
        // back into umin/umax
        const bool lt = a < b;
        asm("" : "+v"(a), "+v"(b));
        const K lo = lt ? a : b;
        const K hi = lt ? b : a;
        a = lo;
        b = hi;
    } else {
        const K lo = __builtin_elementwise_min(a, b);
        const K hi = __builtin_elementwise_max(a, b);
        a = lo;
        b = hi;
    }
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
enum TileMode : int { TM_SORT = 0, TM_MERGE = 1, TM_ROWS = 2, TM_SPAN = 3 };

// ROWS and SPAN tiles are row-shaped; SORT and MERGE tiles are contiguous.
__host__ __device__ constexpr bool rowsy(int mode) { return mode == TM_ROWS || mode == TM_SPAN; }

struct TileMap {
    int64_t ntiles;  // real tiles (a prefix of the tile list)
    int lo, hi, logB, flip;
};

// LDS word of virtual key v (conflict-free for every 5-bit window, additive
// over disjoint bit fields).  A variant that keeps 2^10+ strides multiples of
// 64 words (ds_read2st64 pairs for the high windows) measured the same
// (51.13 vs 51.16 ms per 2^30 sort), so the simple one stays.
__host__ __device__ constexpr int pad(int v) { return v + (v >> 5); }
__host__ __device__ constexpr int lds_words(int t) { return pad(t); }

template <typename K, int LT>
struct TileGeo {
    static constexpr int T = 1 << LT, NT = T / 32, V = KT<K>::V, LOADS = T / (NT * V);
    static constexpr int KB = LOADS == 16 ? 4 : LOADS == 8 ? 3 : LOADS == 4 ? 2 : 1;
    static constexpr int VB = V == 4 ? 2 : 1;
    // LDS tile (keys + bank padding): 2 workgroups per CU up to 80 KiB, else 1
    static constexpr int LDS = lds_words(T) * (int)sizeof(K);
    static constexpr int WG_PER_CU = LDS <= 80 * 1024 ? 2 : 1;
    static constexpr int WAVES_PER_EU = WG_PER_CU * NT / 256;  // -> VGPR budget per lane
};

template <int LT, int MODE>
__device__ __forceinline__ int64_t tile_index(const TileMap& m, int64_t tile, int e) {
    if constexpr (!rowsy(MODE)) {
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
    if constexpr (!rowsy(MODE)) {
        return ((tile + 1) << LT) <= n;
    } else {
        return (((tile >> (m.lo - m.logB)) + 1) << (m.hi + 1)) <= n;
    }
}

// Slot k of lane t: the lane whose vector it holds (mirrored slots: the
// mirror lane, components reversed).
template <typename K, int LT, bool MIRROR>
__device__ __forceinline__ int slot_lane(int k, int t) {
    typedef TileGeo<K, LT> G;
    return (MIRROR && k >= G::LOADS / 2) ? (G::NT - 1 - t) : t;
}

// Virtual start of the vector of slot k, lane t, when the KB slot bits sit at
// virtual bits [SL, SL+KB): components are bits [0, VB), the lane fills the
// bits below and above the slot window.  SL = LT-KB is the plain layout
// (k*NT + t)*V.  Any SL >= VB+5 keeps 32 consecutive lanes on consecutive
// vectors (coalesced HBM access, conflict-free LDS access under pad()).
template <typename K, int LT, int SL>
__device__ __forceinline__ int place(int k, int t) {
    typedef TileGeo<K, LT> G;
    constexpr int LB = SL - G::VB;  // lane bits below the slot window
    return ((t & ((1 << LB) - 1)) << G::VB) | (k << SL) | ((t >> LB) << (SL + G::KB));
}

template <typename K, int LT, int MODE, int SL, bool MIRROR, bool ORD>
__device__ __forceinline__ void tile_fetch(K (*pre)[KT<K>::V], const K* src, const TileMap& m,
                                           int64_t tile, int64_t n, int t) {
    typedef TileGeo<K, LT> G;
    const bool full = tile_full<LT, MODE>(m, tile, n);
#pragma unroll
    for (int k = 0; k < G::LOADS; ++k) {
        const int e = place<K, LT, SL>(k, slot_lane<K, LT, MIRROR>(k, t));
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
        if constexpr (sizeof(K) == 8 && MISORT_CX64_ONECMP && MISORT_CX64_BATCH) {
            // u64: the stage's 16 compares first, then the selects (cx<u64>
            // one pair at a time waits 2 cycles between each compare and its
            // selects)
            bool lt[16];
            int q = 0;
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (!(c & (1 << r))) lt[q++] = v[c] < v[fl ? (c ^ ((2 << r) - 1)) : (c | (1 << r))];
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (!(c & (1 << r))) asm("" : "+v"(v[c]), "+v"(v[fl ? (c ^ ((2 << r) - 1)) : (c | (1 << r))]));
            q = 0;
#pragma unroll
            for (int c = 0; c < 32; ++c) {
                if (c & (1 << r)) continue;
                K& a = v[c];
                K& b = v[fl ? (c ^ ((2 << r) - 1)) : (c | (1 << r))];
                const bool l = lt[q++];
                const K lo = l ? a : b, hi = l ? b : a;
                a = lo;
                b = hi;
            }
        } else {
#pragma unroll
            for (int c = 0; c < 32; ++c)
                if (!(c & (1 << r))) cx(v[c], v[fl ? (c ^ ((2 << r) - 1)) : (c | (1 << r))]);
        }
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

// ------------------------------------------------ wave-local LDS phases
//
// With 32 consecutive keys per lane, a wave owns the 2^11 keys v>>11 == wave.
// An LDS phase whose window lies below bit 11 (B <= 6) touches only its wave's
// keys, so between two such phases the wave needs no workgroup barrier: LDS
// ops of one wave execute in order, and a compiler barrier keeps the reads
// after the writes.  Levels 9..11 then run without s_barrier and the waves
// drift apart, overlapping one wave's LDS traffic with another's min/max; a
// barrier remains around every phase whose window reaches bit 11.
constexpr int WAVE_BITS = 11;
#ifndef MISORT_SORT_WAVE_SYNC
#define MISORT_SORT_WAVE_SYNC 1
#endif
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

// Strides HI..STOP (flip first); NEXT_HI: top bit of the phase after the range
// (-1: what follows reads across waves).
template <typename K, int HI, int STOP, bool FLIP, int NEXT_HI>
__device__ __forceinline__ void lds_range_w(K* s, int t) {
    if constexpr (HI >= STOP) {
        constexpr int B = HI > 4 ? HI - 4 : 0;
        constexpr int LOWEST = B > STOP ? B : STOP;
        phase_c<K, B, HI - B, HI - LOWEST + 1, FLIP>(s, t);
        constexpr int NXT = LOWEST - 1 >= STOP ? LOWEST - 1 : NEXT_HI;
        if constexpr (!MISORT_SORT_WAVE_SYNC || HI >= WAVE_BITS || NXT >= WAVE_BITS || NXT < 0) __syncthreads();
        else wave_sync();
        lds_range_w<K, LOWEST - 1, STOP, false, NEXT_HI>(s, t);
    }
}

template <typename K, int L, int LT>
__device__ __forceinline__ void sort_levels_w(K* s, int t) {
    if constexpr (L <= LT) {
        lds_range_w<K, L - 1, 0, true, (L < LT ? L : -1)>(s, t);
        sort_levels_w<K, L + 1, LT>(s, t);
    }
}

// ------------------------------------------------ in-wave tile sort (u32)
//
// The SORT pass for u32 keys keeps each wave's 2^11 keys in registers for
// levels 1..11: lane l of wave w holds the 32 consecutive keys
// v = (w << 11) | (l << 5) | c, c = register.  Stages on c run in registers;
// stages on the lane bits (virtual bits 5..10) exchange between lanes without
// LDS -- DPP (quad_perm, row_shl/shr with bank masks, row_mirror,
// row_half_mirror) within a 16-lane row, v_permlane16/32_swap across rows --
// and the element whose top compared bit is 0 keeps the minimum through one
// v_med3_u32 (med3(x, p, 0) = min, med3(x, p, ~0) = max).  With
// MISORT_WAVE_LEVELS = 11, levels 12..15 do their wave-bit strides
// (2^14..2^11) in one LDS phase each and return to the register layout (10 LDS
// round trips per tile instead of 27) -- but the cross-lane ops are VALU-heavy
// (DPP hazards, two DPPs for xor 4/8, permlane swaps): measured per 2^30 SORT
// pass 6.9 ms (in the wave up to level 11), 5.23 (7), 5.16 (8), 5.21 (9),
// 5.57 ms (all LDS; profiles/r01/ab/wave_levels.txt).  Default: levels 6..8 in
// the wave (quad_perm / row_half_mirror only), 9..15 in LDS phases.
// (Semantics of every cross-lane op: tools/dpp_probe.hip.)
// Probe-only (tools/build_variant.sh): last level the u32 SORT pass's LDS
// phases run (15 = the whole tile; smaller values time the tile's lower levels
// and do not sort).
// Build-time variant: first level of the u32 SORT tile done as an LDS merge
// (0: the bitonic network for every level; see tile_merge_levels).
#ifndef MISORT_SORT_MERGE_FROM
#define MISORT_SORT_MERGE_FROM 0
#endif
#ifndef MISORT_SORT_TOP
#define MISORT_SORT_TOP 15
#endif
// Probe-only (tools/build_variant.sh): last level the u64 SORT tile's LDS phases run.
#ifndef MISORT_SORT_TOP_U64
#define MISORT_SORT_TOP_U64 99
#endif
#ifndef MISORT_WAVE_SORT
#define MISORT_WAVE_SORT 1
#endif
// highest level run in the wave (6..11); the levels above go through LDS phases
#ifndef MISORT_WAVE_LEVELS
#define MISORT_WAVE_LEVELS 8
#endif

__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
    return max(min(a, b), min(max(a, b), c));  // v_med3_u32
}

template <int CTRL, int BANK>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, 0xF, BANK, false);
}
// all lanes written: no `old` operand to materialise
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_all(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

// Value of v in lane (lane ^ X), X in {1,2,3,4,7,8,15,16,31,32,63}.
template <int X>
__device__ __forceinline__ uint32_t lane_xor(uint32_t v, int lane) {
    if constexpr (X == 1) return dpp_all<0xB1>(v);        // quad_perm [1,0,3,2]
    else if constexpr (X == 2) return dpp_all<0x4E>(v);   // quad_perm [2,3,0,1]
    else if constexpr (X == 3) return dpp_all<0x1B>(v);   // quad_perm [3,2,1,0]
    else if constexpr (X == 7) return dpp_all<0x141>(v);  // row_half_mirror
    else if constexpr (X == 15) return dpp_all<0x140>(v); // row_mirror
    else if constexpr (X == 4) return dpp<0x114, 0xA>(dpp<0x104, 0x5>(v, v), v);  // row_shl/shr:4
    else if constexpr (X == 8) return dpp<0x118, 0xC>(dpp<0x108, 0x3>(v, v), v);  // row_shl/shr:8
    else if constexpr (X == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane & 16) ? r[0] : r[1];
    } else if constexpr (X == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane & 32) ? r[0] : r[1];
    } else if constexpr (X == 31) return lane_xor<16>(lane_xor<15>(v, lane), lane);
    else return lane_xor<32>(lane_xor<31>(v, lane), lane);  // X == 63
}

// Flip of level m (6..11): v <-> v ^ (2^m - 1) = register c <-> 31-c, lane ^ (2^(m-5)-1).
template <int M>
__device__ __forceinline__ void wave_flip(uint32_t (&x)[32], int lane) {
    constexpr int X = (1 << (M - 5)) - 1;
    const uint32_t bnd = ((lane >> (M - 6)) & 1) ? 0xFFFFFFFFu : 0u;
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        const uint32_t pa = lane_xor<X>(x[31 - c], lane), pb = lane_xor<X>(x[c], lane);
        x[c] = med3u(x[c], pa, bnd);
        x[31 - c] = med3u(x[31 - c], pb, bnd);
    }
}

// Half-cleaner on lane bit J (virtual bit 5+J).
template <int J>
__device__ __forceinline__ void wave_half(uint32_t (&x)[32], int lane) {
    if constexpr (J >= 4) {
        // rows apart: v_permlane{16,32}_swap pairs registers (c, c+16) so that
        // every lane holds (lower, upper) of one pair; compare; swap back
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            auto r = J == 4 ? __builtin_amdgcn_permlane16_swap(x[c], x[c + 16], false, false)
                            : __builtin_amdgcn_permlane32_swap(x[c], x[c + 16], false, false);
            uint32_t lo = min(r[0], r[1]), hi = max(r[0], r[1]);
            auto b = J == 4 ? __builtin_amdgcn_permlane16_swap(lo, hi, false, false)
                            : __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
            x[c] = b[0];
            x[c + 16] = b[1];
        }
    } else {
        const uint32_t bnd = ((lane >> J) & 1) ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int c = 0; c < 32; ++c) x[c] = med3u(x[c], lane_xor<(1 << J)>(x[c], lane), bnd);
    }
}

// Half-cleaners on lane bits J..0, then the register bits 4..0.
template <int J>
__device__ __forceinline__ void wave_halves(uint32_t (&x)[32], int lane) {
    if constexpr (J >= 0) {
        wave_half<J>(x, lane);
        wave_halves<J - 1>(x, lane);
    } else {
        reg_stages_c<uint32_t, 4, 5, false>(x);
    }
}

// Levels M..TOP (<= 11) entirely in the wave.
template <int M, int TOP>
__device__ __forceinline__ void wave_levels(uint32_t (&x)[32], int lane) {
    if constexpr (M <= TOP) {
        wave_flip<M>(x, lane);
        wave_halves<M - 7>(x, lane);
        wave_levels<M + 1, TOP>(x, lane);
    }
}

// Levels M..LT: wave-bit strides in one LDS phase (window [10,15)), the rest in the wave.
template <int M, int LT>
__device__ __forceinline__ void wave_big_levels(uint32_t* s, uint32_t (&x)[32], int t) {
    if constexpr (M <= LT) {
        const int a0 = pad(t << 5);
#pragma unroll
        for (int c = 0; c < 32; ++c) s[a0 + c] = x[c];
        __syncthreads();
        phase_c<uint32_t, 10, M - 11, M - 11, true>(s, t);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < 32; ++c) x[c] = s[a0 + c];
        wave_halves<5>(x, t & 63);
        wave_big_levels<M + 1, LT>(s, x, t);
    }
}

// Stages on the slot bits of register-held vectors: relative slot bits
// TOP..TOP-CNT+1, the first one a flip if FLIP (the flip complements every
// slot bit; mirrored upper slots complete it to the tile's own v <-> ~v).
template <typename K, int LOADS, int TOP, int CNT, bool FLIP>
__device__ __forceinline__ void slot_stages(K (*w)[KT<K>::V]) {
#pragma unroll
    for (int i = 0; i < CNT; ++i) {
        const int r = TOP - i;
        const bool fl = FLIP && i == 0;
#pragma unroll
        for (int k = 0; k < LOADS; ++k) {
            if (k & (1 << r)) continue;
            const int p = fl ? (k ^ ((2 << r) - 1)) : (k | (1 << r));
#pragma unroll
            for (int j = 0; j < KT<K>::V; ++j) cx(w[k][j], w[p][j]);
        }
    }
}

// Compile-time schedule of one non-SORT pass (host and device).  A pass runs a
// stage sequence on virtual bits; stages on slot bits run in registers, the
// rest in 5-bit LDS phases.  Two free choices cut LDS phases:
//   * the load slot window SL: a SPAN pass puts it on the top KB bits of its
//     tail, so those stages run before the LDS write;
//   * the final-read slot window SF: the LAST stages of the pass (the low head
//     bits of a SPAN or ROWS pass) run in registers after the LDS read; a
//     head of <= KB stages runs there entirely, its flip through mirrored
//     upper slots.
// Sequences: ROWS  LT-1 .. LT-R (flip first if FLIP);
//            MERGE LT-1 .. 0;
//            SPAN  LT-R-1 .. 0, then flip(LT-1), LT-2 .. LT-R.
struct ProgGeo {
    int LT, KB, VB, MODE, R;
    bool FLIP;
    int POSTCAP;  // most final-read register stages (register budget: 2 when a
                  // persistent grid keeps the next tile's 32 keys in flight)
};
struct ProgPlan {
    int SL;            // load slot window
    bool MLOAD;        // mirrored upper slots at load (flip on slot bits)
    int PRE, PRE_TOP;  // register stages after the load (relative top, count)
    bool PRE_FLIP;
    bool DIRECT;       // every stage in registers: no LDS at all
    int T_HI, T_LO;    // first LDS range (no flip); empty when T_HI < T_LO
    int H_HI, H_LO;    // second LDS range, flip first (SPAN head); empty when H_HI < H_LO
    int SF;            // final-read slot window
    bool MFIN;         // mirrored upper slots at the final read
    int POST, POST_TOP;
    bool POST_FLIP;
    bool COMP;         // component-bit stages after the final read (MERGE)
    int phases;        // LDS phases (5-bit windows)
};
__host__ __device__ constexpr int windows(int hi, int lo) { return hi < lo ? 0 : (hi - lo + 5) / 5; }
// Build-time switches of the schedule choices (A/B probes: tools/build_variant.sh).
// Measured (profiles/r01/ab/prog_variants.txt): the register tail/head tricks
// make SPAN passes slower (shorter load runs; spills beside the persistent
// prefetch), the final-read window makes ROWS R=4..8 passes faster (R=6: no
// LDS phase at all) -- so SPAN keeps its LDS-only schedule by default.
#ifndef MISORT_SPAN_PRE
#define MISORT_SPAN_PRE 0
#endif
#ifndef MISORT_SPAN_POST
#define MISORT_SPAN_POST 0
#endif
#ifndef MISORT_ROWS_POST
#define MISORT_ROWS_POST 1
#endif
__host__ __device__ constexpr ProgPlan prog_plan(ProgGeo g) {
    ProgPlan p{};
    const int TOPS = g.LT - g.KB, MINW = g.VB + 5;
    const int cap = g.POSTCAP < g.KB ? g.POSTCAP : g.KB;
    p.SL = TOPS;
    p.SF = TOPS;
    p.T_HI = -1; p.T_LO = 0; p.H_HI = -1; p.H_LO = 0;
    if (g.MODE == TM_MERGE) {
        p.PRE = g.KB; p.PRE_TOP = g.KB - 1;
        p.T_HI = TOPS - 1; p.T_LO = g.VB;
        p.COMP = true;
    } else if (g.MODE == TM_ROWS) {
        p.MLOAD = g.FLIP;
        p.PRE = g.R < g.KB ? g.R : g.KB; p.PRE_TOP = g.KB - 1; p.PRE_FLIP = g.FLIP;
        if (g.R <= g.KB) {
            p.DIRECT = true;
        } else {
            // stages after the load: TOPS-1 .. last; the final window starts at last
            const int last = g.LT - g.R;
            const int rest = TOPS - last;
            const int q = rest < cap ? rest : cap;
            if (MISORT_ROWS_POST && last >= MINW && q > 0) {
                p.SF = last;
                p.POST = q; p.POST_TOP = q - 1;
                p.T_HI = TOPS - 1; p.T_LO = last + q;
            } else {
                p.T_HI = TOPS - 1; p.T_LO = last;
            }
        }
    } else if (g.MODE == TM_SPAN) {
        const int TA = g.LT - g.R;
        if (MISORT_SPAN_PRE && TA - g.KB >= MINW) {
            p.SL = TA - g.KB;
            p.PRE = g.KB; p.PRE_TOP = g.KB - 1;
            p.T_HI = TA - g.KB - 1;
        } else {
            p.T_HI = TA - 1;
        }
        p.T_LO = 0;
        if (!MISORT_SPAN_POST) {
            p.H_HI = g.LT - 1; p.H_LO = TA;
        } else if (g.R <= cap) {
            // the whole head (flip first) on the top slot bits, mirrored read
            p.MFIN = true;
            p.POST = g.R; p.POST_TOP = g.KB - 1; p.POST_FLIP = true;
        } else if (TA >= MINW && cap > 0) {
            // the head's last `cap` stages in registers, the rest in LDS
            p.SF = TA;
            p.POST = cap; p.POST_TOP = cap - 1;
            p.H_HI = g.LT - 1; p.H_LO = TA + cap;
        } else {
            p.H_HI = g.LT - 1; p.H_LO = TA;
        }
    }
    p.phases = windows(p.T_HI, p.T_LO) + windows(p.H_HI, p.H_LO);
    return p;
}

// Slot-pairing masks of a register stage list: stage i of TOP..TOP-CNT+1 pairs
// slot k with k ^ pmask(i) (a flip complements every slot bit up to TOP).
__host__ __device__ constexpr int pmask(int i, int top, bool flip) {
    return (flip && i == 0) ? ((2 << top) - 1) : (1 << (top - i));
}
__host__ __device__ constexpr int psub(int S, int cnt, int top, bool flip) {
    int x = 0;
    for (int i = 0; i < cnt; ++i)
        if ((S >> i) & 1) x ^= pmask(i, top, flip);
    return x;
}
// k is the smallest slot of its group (the slots the stage list connects).
__host__ __device__ constexpr bool pgroup_rep(int k, int cnt, int top, bool flip) {
    for (int S = 1; S < (1 << cnt); ++S)
        if ((k ^ psub(S, cnt, top, flip)) < k) return false;
    return true;
}

// LDS -> registers (final slot window SF, mirrored upper slots if MF) -> the
// pass's last register stages -> HBM.  Slots are handled one stage-connected
// group at a time, so only 2^CNT vectors are live.
// fence (SORT tiles only, may be null): the first multi-way merge pass's
// fences, written here instead of gathered from HBM by k_fence_gather -- the
// key at every 2^MERGEK_FENCE_LOG2-th position of the sorted tile, packed as
// runsk.hip's fpack does for runs of 2^LT keys in groups of 2^flk (u32 keys:
// 64-bit fences, u64 keys: 128-bit).
template <typename K, int LT, int MODE, int SF, bool MF, int TOP, int CNT, bool FLIP, bool COMP>
__device__ __forceinline__ void final_store(const K* s, K* out, const TileMap& m, int64_t tile, int64_t n,
                                            bool full, int t, void* fence = nullptr, int flk = 0) {
    typedef TileGeo<K, LT> G;
    constexpr int NG = 1 << CNT;
#pragma unroll
    for (int k0 = 0; k0 < G::LOADS; ++k0) {
        if (!pgroup_rep(k0, CNT, TOP, FLIP)) continue;
        K w[NG][G::V];
#pragma unroll
        for (int S = 0; S < NG; ++S) {
            const int k = k0 ^ psub(S, CNT, TOP, FLIP);
            const bool mk = MF && k >= G::LOADS / 2;
            const int e = place<K, LT, SF>(k, slot_lane<K, LT, MF>(k, t));
#pragma unroll
            for (int j = 0; j < G::V; ++j) w[S][j] = s[pad(e + (mk ? G::V - 1 - j : j))];
        }
#pragma unroll
        for (int i = 0; i < CNT; ++i) {
            const int r = TOP - i;
#pragma unroll
            for (int S = 0; S < NG; ++S) {
                if ((S >> i) & 1) continue;
                const int kA = k0 ^ psub(S, CNT, TOP, FLIP);
                const bool a_low = !((kA >> r) & 1);  // the lower virtual index takes the minimum
                const int lo = a_low ? S : (S | (1 << i)), hi = a_low ? (S | (1 << i)) : S;
#pragma unroll
                for (int j = 0; j < G::V; ++j) cx(w[lo][j], w[hi][j]);
            }
        }
#pragma unroll
        for (int S = 0; S < NG; ++S) {
            if constexpr (COMP) {
#pragma unroll
                for (int r = G::VB - 1; r >= 0; --r)
#pragma unroll
                    for (int j = 0; j < G::V; ++j)
                        if (!(j & (1 << r))) cx(w[S][j], w[S][j | (1 << r)]);
            }
            const int k = k0 ^ psub(S, CNT, TOP, FLIP);
            const bool mk = MF && k >= G::LOADS / 2;
            K x[G::V];
#pragma unroll
            for (int j = 0; j < G::V; ++j) x[j] = mk ? w[S][G::V - 1 - j] : w[S][j];
            const int e = place<K, LT, SF>(k, slot_lane<K, LT, MF>(k, t));
            store_slot<K, LT, MODE>(out, m, tile, n, full, e, x);
            if constexpr (MODE == TM_SORT) {
                constexpr int FGM = (1 << MERGEK_FENCE_LOG2) - 1;
                const int64_t gi = (tile << LT) + e;
                if (fence && (e & FGM) == 0 && gi < n) {
                    const uint32_t tag = ((uint32_t)((gi >> LT) & ((1 << flk) - 1)) << (32 - flk)) |
                                         (uint32_t)((e & ((1 << LT) - 1)) >> MERGEK_FENCE_LOG2);
                    if constexpr (sizeof(K) == 4)
                        ((uint64_t*)fence)[gi >> MERGEK_FENCE_LOG2] = ((uint64_t)x[0] << 32) | tag;
                    else
                        ((unsigned __int128*)fence)[gi >> MERGEK_FENCE_LOG2] =
                            ((unsigned __int128)x[0] << 64) | tag;
                }
            }
        }
    }
}

// PERSIST: the grid is smaller than the tile list and every workgroup walks
// tiles with the next tile's loads in flight; otherwise one tile per workgroup
// (no prefetch registers live across the LDS phases).
template <typename K, int LT, int MODE, int R, bool FLIP, bool ORD, bool PERSIST>
__global__ __launch_bounds__((TileGeo<K, LT>::NT), (TileGeo<K, LT>::WAVES_PER_EU)) void k_stream(
    const K* in, K* out, int64_t n, TileMap m, void* fence, int flk) {
    typedef TileGeo<K, LT> G;
    constexpr ProgPlan P = prog_plan(ProgGeo{LT, G::KB, G::VB, MODE, R, FLIP, PERSIST ? 2 : G::KB});
    constexpr int SL = MODE == TM_SORT ? LT - G::KB : P.SL;
    __shared__ K s[lds_words(G::T)];
    const int t = threadIdx.x;
    K pre[G::LOADS][G::V];
    int64_t tile = blockIdx.x;
    if (tile >= m.ntiles) return;
    tile_fetch<K, LT, MODE, SL, P.MLOAD, ORD>(pre, in, m, tile, n, t);
    for (; tile < m.ntiles; tile += gridDim.x) {
        slot_stages<K, G::LOADS, P.PRE_TOP, P.PRE, P.PRE_FLIP>(pre);
        const bool full = tile_full<LT, MODE>(m, tile, n);
        if constexpr (P.DIRECT) {
            // every stride of this pass was a slot bit: store straight from registers
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                K w[G::V];
                const bool mk = P.MLOAD && k >= G::LOADS / 2;
#pragma unroll
                for (int j = 0; j < G::V; ++j) w[j] = mk ? pre[k][G::V - 1 - j] : pre[k][j];
                store_slot<K, LT, MODE>(out, m, tile, n, full, place<K, LT, SL>(k, slot_lane<K, LT, P.MLOAD>(k, t)), w);
            }
            const int64_t nxt = tile + gridDim.x;
            if (PERSIST && nxt < m.ntiles) tile_fetch<K, LT, MODE, SL, P.MLOAD, ORD>(pre, in, m, nxt, n, t);
        } else {
            // registers -> LDS (mirrored slots to their own virtual position)
#pragma unroll
            for (int k = 0; k < G::LOADS; ++k) {
                const bool mk = P.MLOAD && k >= G::LOADS / 2;
                const int e = place<K, LT, SL>(k, slot_lane<K, LT, P.MLOAD>(k, t));
#pragma unroll
                for (int j = 0; j < G::V; ++j) s[pad(e + j)] = mk ? pre[k][G::V - 1 - j] : pre[k][j];
            }
            __syncthreads();
            const int64_t nxt = tile + gridDim.x;
            if (PERSIST && nxt < m.ntiles) tile_fetch<K, LT, MODE, SL, P.MLOAD, ORD>(pre, in, m, nxt, n, t);
            if constexpr (MODE == TM_SORT && MISORT_WAVE_SORT && sizeof(K) == 4 && LT == 15) {
                // levels 1..11 in the wave, 12..15 with one LDS phase each
                uint32_t x[32];
                const int a0 = pad(t << 5);
#pragma unroll
                for (int c = 0; c < 32; ++c) x[c] = s[a0 + c];
                reg_stages_c<uint32_t, 0, 1, true>(x);
                reg_stages_c<uint32_t, 1, 2, true>(x);
                reg_stages_c<uint32_t, 2, 3, true>(x);
                reg_stages_c<uint32_t, 3, 4, true>(x);
                reg_stages_c<uint32_t, 4, 5, true>(x);
                constexpr int WL = MISORT_WAVE_LEVELS;
                wave_levels<6, WL>(x, t & 63);
                if constexpr (WL >= 11) {
                    __syncthreads();  // every wave has read its keys: the LDS tile is free
                    wave_big_levels<12, LT>((uint32_t*)s, x, t);
#pragma unroll
                    for (int c = 0; c < 32; ++c) s[a0 + c] = x[c];
                    __syncthreads();
                } else {
                    // each lane rewrites only the keys it read: no barrier before
#pragma unroll
                    for (int c = 0; c < 32; ++c) s[a0 + c] = x[c];
                    __syncthreads();
                    sort_levels<K, WL + 1, LT>(s, t);
                }
            } else if constexpr (MODE == TM_SORT) {
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
                if constexpr (MISORT_SORT_WAVE_SYNC) wave_sync();  // level 6 stays inside the wave
                else __syncthreads();
                sort_levels_w<K, 6, (sizeof(K) == 8 && MISORT_SORT_TOP_U64 < LT ? MISORT_SORT_TOP_U64 : LT)>(s, t);
            } else {
                lds_range_w<K, P.T_HI, P.T_LO, false, (P.H_HI >= P.H_LO ? P.H_HI : -1)>(s, t);
                lds_range_w<K, P.H_HI, P.H_LO, true, -1>(s, t);
            }
            // LDS -> registers (final slot window) -> last stages -> HBM
            constexpr int SF = MODE == TM_SORT ? LT - G::KB : P.SF;
            final_store<K, LT, MODE, SF, P.MFIN, P.POST_TOP, P.POST, P.POST_FLIP, P.COMP>(s, out, m, tile, n,
                                                                                        full, t, fence, flk);
            __syncthreads();
        }
        if constexpr (!PERSIST) break;
    }
}


[[maybe_unused]] int ceil_log2(int64_t n) {
    int k = 0;
    while (((int64_t)1 << k) < n) ++k;
    return k;
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


// fence/flk: SORT passes only, see final_store (null: no fences).
template <typename K, int LT, int MODE, int R, bool FLIP, bool ORD>
void launch_stream(const K* in, K* out, int64_t n, const TileMap& m, hipStream_t s, void* fence = nullptr,
                   int flk = 0) {
    typedef TileGeo<K, LT> G;
    static int64_t cap = 0;  // resident workgroups for this instantiation
    const bool persist = (plan_knobs().persist_mask((int)sizeof(K)) >> MODE) & 1;
    if (persist && cap == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_stream<K, LT, MODE, R, FLIP, ORD, true>,
                                                           G::NT, 0);
        cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
    }
    const int64_t want = persist ? cap * plan_knobs().grid_mult : m.ntiles;
    const int64_t grid = m.ntiles < want ? m.ntiles : want;
    if (grid <= 0) return;
    if (persist) k_stream<K, LT, MODE, R, FLIP, ORD, true><<<(unsigned)grid, G::NT, 0, s>>>(in, out, n, m, fence, flk);
    else k_stream<K, LT, MODE, R, FLIP, ORD, false><<<(unsigned)grid, G::NT, 0, s>>>(in, out, n, m, fence, flk);
}

template <typename K, int LT, int MODE, int R>
void launch_rows_r(const K* in, K* out, int64_t n, const TileMap& m, hipStream_t s) {
    if constexpr (R <= LT - 5) {
        if constexpr (MODE == TM_SPAN) launch_stream<K, LT, MODE, R, true, false>(in, out, n, m, s);
        else if (m.flip) launch_stream<K, LT, MODE, R, true, false>(in, out, n, m, s);
        else launch_stream<K, LT, MODE, R, false, false>(in, out, n, m, s);
    }
}

// One ROWS pass (strides 2^hi .. 2^(hi-R+1) of a level) or SPAN pass (the
// strides 2^(LT-R-1)..1 of level hi, then level hi+1's flip and strides
// 2^(hi-1)..2^(hi-R+1)) over n (virtual) keys.  Both use the tile of 2^R rows
// at stride 2^(hi-R+1) times 2^(LT-R) consecutive keys.
template <typename K, int LT, int MODE>
void launch_rows(const K* in, K* out, int64_t n, int hi, int R, bool flip, hipStream_t s) {
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
        case 1: launch_rows_r<K, LT, MODE, 1>(in, out, n, m, s); break;
        case 2: launch_rows_r<K, LT, MODE, 2>(in, out, n, m, s); break;
        case 3: launch_rows_r<K, LT, MODE, 3>(in, out, n, m, s); break;
        case 4: launch_rows_r<K, LT, MODE, 4>(in, out, n, m, s); break;
        case 5: launch_rows_r<K, LT, MODE, 5>(in, out, n, m, s); break;
        case 6: launch_rows_r<K, LT, MODE, 6>(in, out, n, m, s); break;
        case 7: launch_rows_r<K, LT, MODE, 7>(in, out, n, m, s); break;
        case 8: launch_rows_r<K, LT, MODE, 8>(in, out, n, m, s); break;
        case 9: launch_rows_r<K, LT, MODE, 9>(in, out, n, m, s); break;
        default: launch_rows_r<K, LT, MODE, 10>(in, out, n, m, s); break;
    }
}

// ------------------------------------------------ u32 SORT pass kernel
//
// k_stream<SORT>'s body for u32 keys (in-wave levels 1..MISORT_WAVE_LEVELS,
// LDS phases above), with the full/partial tile split made at compile time:
// the persistent grid walks only full tiles, and a one-workgroup launch sorts
// the partial last tile.  Inside k_stream the bounds-checked load/store paths
// pushed the persistent SORT kernel to 128 VGPRs with spills, and one spill
// reload right after the next tile's prefetch issued an s_waitcnt vmcnt(0)
// that waited for the whole prefetch (vmcnt is in order), so the prefetch hid
// nothing.  The tile base is uniform (SGPRs); lanes add 32-bit offsets.
template <bool FULL>
__device__ __forceinline__ void sort_fetch(uint32_t (*pre)[4], const uint32_t* in, int64_t tile, int64_t n, int t) {
    const uint32_t* tb = in + (tile << 15);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int e = place<uint32_t, 15, 12>(k, t);
        if constexpr (FULL) {
            const KT<uint32_t>::vec x = __builtin_nontemporal_load(reinterpret_cast<const KT<uint32_t>::vec*>(tb + e));
#pragma unroll
            for (int j = 0; j < 4; ++j) pre[k][j] = x[j];
        } else {
            load_vec<uint32_t, false>(in, (tile << 15) + e, n, pre[k]);
        }
    }
}

// Levels L0..LT of the u32 SORT tile as merges in LDS (build-time variant,
// MISORT_SORT_MERGE_FROM = L0): before level L the tile holds ascending runs of
// 2^(L-1) keys at s[pad(v)]; lane t writes outputs [32t, 32t + 32) of its pair's
// merge -- a co-rank search, 32 serial LDS reads, then (after a barrier) 32
// LDS writes.  The final store's register stages then act on sorted data, where
// a half-cleaner changes nothing.
template <int L, int LT>
__device__ __forceinline__ void tile_merge_levels(uint32_t* s, int t) {
    if constexpr (L <= LT) {
        constexpr int W = 1 << (L - 1);
        const int v0 = t << 5;
        const int base = (v0 >> L) << L, d = v0 - base;
        const int bb = base + W;
        int lo = d > W ? d - W : 0, hi = d < W ? d : W;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s[pad(base + mid)] <= s[pad(bb + d - 1 - mid)]) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = d - lo;
        uint32_t av = s[pad(base + (ia < W ? ia : 0))], bv = s[pad(bb + (ib < W ? ib : 0))];
        uint32_t r[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) {
            const bool takeA = ia < W && (ib >= W || av <= bv);
            r[c] = takeA ? av : bv;
            ia += takeA;
            ib += !takeA;
            const int nx = takeA ? base + (ia < W ? ia : 0) : bb + (ib < W ? ib : 0);
            const uint32_t x = s[pad(nx)];
            av = takeA ? x : av;
            bv = takeA ? bv : x;
        }
        __syncthreads();
        const int a0 = pad(v0);
#pragma unroll
        for (int c = 0; c < 32; ++c) s[a0 + c] = r[c];
        __syncthreads();
        tile_merge_levels<L + 1, LT>(s, t);
    }
}

template <bool PERSIST, bool FULL>
__global__ __launch_bounds__(1024, 1) void k_sort_u32(const uint32_t* in, uint32_t* out, int64_t n, TileMap m,
                                                      int64_t tile0, uint64_t* fence, int flk) {
    typedef uint32_t K;
    constexpr int LT = 15;
    typedef TileGeo<K, LT> G;
    constexpr ProgPlan P = prog_plan(ProgGeo{LT, G::KB, G::VB, TM_SORT, 0, false, PERSIST ? 2 : G::KB});
    constexpr int SL = LT - G::KB, WL = MISORT_WAVE_LEVELS;
    static_assert(G::LOADS == 8 && G::NT == 1024 && WL >= 5 && WL <= 10, "u32 SORT tile shape");
    __shared__ K s[lds_words(G::T)];
    int64_t tile = tile0 + blockIdx.x;
    if (tile >= m.ntiles) return;
    K pre[G::LOADS][G::V];
    sort_fetch<FULL>(pre, in, tile, n, (int)threadIdx.x);
    for (; tile < m.ntiles; tile += gridDim.x) {
        // lane id through an opaque copy: the per-lane LDS/HBM addresses are
        // recomputed every tile instead of being hoisted into ~16 loop-invariant
        // VGPRs (which pushed the kernel into spills)
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        const int a0 = pad(t << 5);
        slot_stages<K, G::LOADS, P.PRE_TOP, P.PRE, P.PRE_FLIP>(pre);
#pragma unroll
        for (int k = 0; k < G::LOADS; ++k) {
            const int e = place<K, LT, SL>(k, t);
#pragma unroll
            for (int j = 0; j < G::V; ++j) s[pad(e + j)] = pre[k][j];
        }
        __syncthreads();
        uint32_t x[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) x[c] = s[a0 + c];
        reg_stages_c<uint32_t, 0, 1, true>(x);
        reg_stages_c<uint32_t, 1, 2, true>(x);
        reg_stages_c<uint32_t, 2, 3, true>(x);
        reg_stages_c<uint32_t, 3, 4, true>(x);
        reg_stages_c<uint32_t, 4, 5, true>(x);
        wave_levels<6, WL>(x, t & 63);
        // each lane rewrites only the keys it read: no barrier before, and the
        // next phase (level WL+1 <= 11) stays inside the wave
#pragma unroll
        for (int c = 0; c < 32; ++c) s[a0 + c] = x[c];
        if constexpr (WL + 1 <= WAVE_BITS && MISORT_SORT_WAVE_SYNC) wave_sync();
        else __syncthreads();
        // the next tile's loads fly during the LDS phases (issued here, not
        // before the wave levels, so their registers and the cross-lane
        // temporaries are never live together)
        const int64_t nxt = tile + gridDim.x;
        if (PERSIST && nxt < m.ntiles) sort_fetch<FULL>(pre, in, nxt, n, t);
        if constexpr (MISORT_SORT_MERGE_FROM > WL) {
            sort_levels_w<K, WL + 1, MISORT_SORT_MERGE_FROM - 1>(s, t);
            tile_merge_levels<MISORT_SORT_MERGE_FROM, LT>(s, t);
        } else {
            sort_levels_w<K, WL + 1, MISORT_SORT_TOP>(s, t);
        }
        final_store<K, LT, TM_SORT, SL, P.MFIN, P.POST_TOP, P.POST, P.POST_FLIP, P.COMP>(s, out, m, tile, n, FULL,
                                                                                         t, fence, flk);
        if constexpr (!PERSIST) break;
        __syncthreads();
    }
}

// fence/flk: see final_store (null: no fences).
inline void launch_sort_u32(const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s, uint64_t* fence = nullptr,
                            int flk = 0) {
    static int64_t cap = 0;
    TileMap m{};
    const int64_t nfull = n >> 15;
    const bool persist = plan_knobs().persist & 1;
    if (persist && cap == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_u32<true, true>, 1024, 0);
        cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
    }
    if (nfull > 0) {
        m.ntiles = nfull;
        const int64_t want = persist ? cap * plan_knobs().grid_mult : nfull;
        const int64_t grid = nfull < want ? nfull : want;
        if (persist) k_sort_u32<true, true><<<(unsigned)grid, 1024, 0, s>>>(in, out, n, m, 0, fence, flk);
        else k_sort_u32<false, true><<<(unsigned)grid, 1024, 0, s>>>(in, out, n, m, 0, fence, flk);
    }
    if ((nfull << 15) < n) {
        m.ntiles = nfull + 1;
        k_sort_u32<false, false><<<1, 1024, 0, s>>>(in, out, n, m, nfull, fence, flk);
    }
}

// ------------------------------------------------ wide ROWS pass (u32)
//
// A ROWS pass over a 2^16-key tile (256 KiB) that lives in registers: 1024
// lanes x 64 keys, twice the LDS tile.  The tile is 2^R rows at stride 2^lo
// times 2^(16-R) consecutive keys, so R = 10 strides still read 256-B row runs
// (the LDS-tile ROWS pass needs 128-B runs for R = 10, which HBM serves ~35 %
// slower).  Two register layouts, one LDS transpose between them:
//   load   v = (k << 12) | (t << 2) | q   slot k = the top 4 row bits, whose
//          stages (flip first: mirrored upper slots, as in k_stream) run in
//          registers right after the loads; 16 lanes per 256-B row run;
//   store  v = (t & 63) | (r << 6) | ((t >> 6) << 12)   register r = virtual
//          bits 6..11, where the other R-4 row stages run; a wave's dword
//          store covers 64 consecutive keys (one 256-B row run).
// The transpose moves the tile through the 2^15-key LDS array in two rounds
// (virtual bit 15 = load slot bit 3 = store lane bit 9), so the pass costs one
// LDS round trip per key whatever R is (the LDS-tile pass needs two at R >= 9).
// The DP planner prices it from the measured table like every other shape.
constexpr int WIDE_LT = 16, WIDE_NT = 1024, WIDE_RMIN = 4, WIDE_RMAX = 10;

// FULL: every key of the tile lies below n (no bounds checks; a separate body
// so the partial-tile checks do not raise the common path's register use).
template <int R, bool FLIP, bool FULL>
__device__ __forceinline__ void rows_wide_tile(const uint32_t* in, uint32_t* out, int64_t n, const TileMap& m,
                                               int64_t tile, uint32_t* s, int t) {
    constexpr int LT = WIDE_LT, NT = WIDE_NT, LOADS = 16, V = 4;
    constexpr bool full = FULL;
    uint32_t w[LOADS][V];
    // slot k is row bit group k << (12 - logB): gi(k) = gi(first slot of its half) + (k % 8) << ks
    const int ks = 12 - (LT - R) + m.lo;
    const int64_t g0 = tile_index<LT, TM_ROWS>(m, tile, t << 2);
    const int64_t g8 = FLIP ? tile_index<LT, TM_ROWS>(m, tile, (8 << 12) | ((NT - 1 - t) << 2)) : g0 + ((int64_t)8 << ks);
#pragma unroll
    for (int k = 0; k < LOADS; ++k) {
        const bool mk = FLIP && k >= LOADS / 2;
        const int64_t gi = (k < 8 ? g0 : g8) + ((int64_t)(k & 7) << ks);
        uint32_t x[V];
        if (full) {
            const KT<uint32_t>::vec y =
                __builtin_nontemporal_load(reinterpret_cast<const KT<uint32_t>::vec*>(in + gi));
#pragma unroll
            for (int j = 0; j < V; ++j) x[j] = y[j];
        } else {
            load_vec<uint32_t, false>(in, gi, n, x);
        }
#pragma unroll
        for (int j = 0; j < V; ++j) w[k][j] = mk ? x[V - 1 - j] : x[j];
    }
    // row bits 15..12 (slot bits 3..0), the level's flip first
    slot_stages<uint32_t, LOADS, 3, 4, FLIP>(w);
    // transpose, one half of the tile (virtual bit 15 = h) per round
    uint32_t x[64];
    const int sb = (t & 63) | (((t >> 6) & 7) << 12);  // store-layout lane bits below bit 15
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h) __syncthreads();  // round 0's readers are done with the array
#pragma unroll
        for (int k = 8 * h; k < 8 * h + 8; ++k) {
            const bool mk = FLIP && k >= LOADS / 2;
            const int e = ((k & 7) << 12) | ((mk ? NT - 1 - t : t) << 2);
#pragma unroll
            for (int j = 0; j < V; ++j) s[pad(e + j)] = mk ? w[k][V - 1 - j] : w[k][j];
        }
        __syncthreads();
        if ((t >> 9) == h) {
#pragma unroll
            for (int r = 0; r < 64; ++r) x[r] = s[pad(sb) + pad(r << 6)];
        }
    }
    // row bits 11..16-R (register bits 5..10-R)
#pragma unroll
    for (int r = 5; r > 5 - (R - 4); --r)
#pragma unroll
        for (int c = 0; c < 64; ++c)
            if (!(c & (1 << r))) cx(x[c], x[c | (1 << r)]);
    // register r: its low CB bits are column bits 6.., the rest row bits
    constexpr int CB = (LT - R) - 6;
    const int64_t gs = tile_index<LT, TM_ROWS>(m, tile, (t & 63) | ((t >> 6) << 12));
#pragma unroll
    for (int r = 63; r >= 0; --r) {
        const int64_t gi = gs + ((r & ((1 << CB) - 1)) << 6) + ((int64_t)(r >> CB) << m.lo);
        if (full) __builtin_nontemporal_store(x[r], out + gi);
        else if (gi < n) out[gi] = x[r];
    }
}

// Full tiles (every key below n) come first in the tile list; the partial ones
// (the last 2^(hi+1) segment of a non-power-of-two n) run in a second launch.
template <int R, bool FLIP, bool FULL>
__global__ __launch_bounds__(WIDE_NT, 1) void k_rows_wide(const uint32_t* in, uint32_t* out, int64_t n,
                                                          TileMap m, int64_t tile0) {
    static_assert(R >= WIDE_RMIN && R <= WIDE_RMAX, "wide ROWS: 4 <= R <= 10");
    __shared__ uint32_t s[lds_words(1 << (WIDE_LT - 1))];
    rows_wide_tile<R, FLIP, FULL>(in, out, n, m, tile0 + blockIdx.x, s, threadIdx.x);
}

template <int R, bool FLIP>
void launch_wide_rf(const uint32_t* in, uint32_t* out, int64_t n, const TileMap& m, int64_t nfull,
                    hipStream_t s) {
    if (nfull > 0) k_rows_wide<R, FLIP, true><<<(unsigned)nfull, WIDE_NT, 0, s>>>(in, out, n, m, 0);
    if (m.ntiles > nfull)
        k_rows_wide<R, FLIP, false><<<(unsigned)(m.ntiles - nfull), WIDE_NT, 0, s>>>(in, out, n, m, nfull);
}

template <int R>
void launch_wide_r(const uint32_t* in, uint32_t* out, int64_t n, const TileMap& m, int64_t nfull, hipStream_t s) {
    if (m.flip) launch_wide_rf<R, true>(in, out, n, m, nfull, s);
    else launch_wide_rf<R, false>(in, out, n, m, nfull, s);
}

// One wide ROWS pass: strides 2^hi .. 2^(hi-R+1) of a level, 4 <= R <= 10, hi >= 15.
inline void launch_rows_wide(const uint32_t* in, uint32_t* out, int64_t n, int hi, int R, bool flip,
                             hipStream_t s) {
    TileMap m{};
    m.lo = hi - R + 1;
    m.hi = hi;
    m.logB = WIDE_LT - R;
    m.flip = flip;
    const int64_t per_seg = ((int64_t)1 << m.lo) >> m.logB;
    const int64_t full_segs = n >> (hi + 1);
    const int64_t rem = n - (full_segs << (hi + 1));
    int64_t part = (rem + ((int64_t)1 << m.logB) - 1) >> m.logB;
    if (part > per_seg) part = per_seg;
    m.ntiles = full_segs * per_seg + part;
    const int64_t nf = full_segs * per_seg;
    switch (R) {
        case 4: launch_wide_r<4>(in, out, n, m, nf, s); break;
        case 5: launch_wide_r<5>(in, out, n, m, nf, s); break;
        case 6: launch_wide_r<6>(in, out, n, m, nf, s); break;
        case 7: launch_wide_r<7>(in, out, n, m, nf, s); break;
        case 8: launch_wide_r<8>(in, out, n, m, nf, s); break;
        case 9: launch_wide_r<9>(in, out, n, m, nf, s); break;
        default: launch_wide_r<10>(in, out, n, m, nf, s); break;
    }
}

// One HBM pass of the plan.
struct Pass {
    Kind kind;  // KIND_TILE_SORT, KIND_GLOBAL (ROWS), KIND_SPAN, KIND_TILE_MERGE
    int hi, R;  // ROWS: strides 2^hi..2^(hi-R+1); SPAN: level hi+1's head of R strides
    bool flip;
};

// Level-by-level plan (MISORT_SPAN=0): one SORT pass (levels 1..LT of each
// 2^LT tile), then per level m > LT the strides 2^(m-1)..2^LT in near-equal
// ROWS passes of <= rmax strides each, and one MERGE pass for the strides < 2^LT.
inline std::vector<Pass> plan_levels(int k, int LT, int rmax) {
    std::vector<Pass> ps;
    ps.push_back(Pass{KIND_TILE_SORT, LT - 1, 0, false});
    for (int m = LT + 1; m <= k; ++m) {
        const int x = m - LT;
        const int parts = (x + rmax - 1) / rmax;
        int hi = m - 1;
        for (int p = 0; p < parts; ++p) {
            const int R = x / parts + (p < x % parts ? 1 : 0);
            ps.push_back(Pass{KIND_GLOBAL, hi, R, p == 0});
            hi -= R;
        }
        ps.push_back(Pass{KIND_TILE_MERGE, LT - 1, 0, false});
    }
    return ps;
}

// Cheapest plan (default).  After the SORT pass, the stages of levels LT+1..k
// form one sequence of (level m, stride bit b) for b = m-1..0.  A pass takes a
// consecutive run of it whose bits fit one LT-bit tile:
//   ROWS  bits hi..hi-R+1 of one level (flip iff hi = m-1), R <= rmax, whose
//         tile keeps >= 2^cmin consecutive keys per row (coalescing);
//   MERGE bits LT-1..0 of one level;
//   SPAN  bits LT-R-1..0 of level m, then bits m..m-R+1 of level m+1 (the
//         flip first): a ROWS tile of R row bits whose 2^(LT-R)-key rows hold
//         the tail's bits.
// Dynamic programming over the sequence minimises the modelled time: one HBM
// sweep per pass, plus a little per LDS phase of the pass's schedule
// (prog_plan) and for the shortest (2^cmin-key) rows.  For 2^30 u32 keys this
// is 1 + 29 passes instead of the level-by-level plan's 1 + 35.
inline double model_cost(int LT, int KB, int VB, int mode, int R, bool flip, int cmin, int kb) {
    const bool persist = (plan_knobs().persist_mask(kb) >> mode) & 1;
    const ProgPlan pp = prog_plan(ProgGeo{LT, KB, VB, mode, R, flip, persist ? 2 : KB});
    const bool short_rows = (mode == TM_ROWS || mode == TM_SPAN) && LT - R <= cmin;
    return 1.0 + 0.035 * pp.phases + (short_rows ? 0.03 : 0.0);
}

// Cost of one pass in "median pass" units: the measured table (pass_costs.h,
// tools/pass_costs.py: every shape timed alone on an MI355X at 2^logn keys;
// the closest logn to this sort's 2^k is used) where it has the shape, else
// the model above.  The table captures what the model cannot: rows at some
// power-of-two strides run up to 40 % slower than at others (HBM channel
// aliasing), so the planner steers around them.
inline double table_cost(int kind, int kb, int lt, int R, bool flip, int hi, int k) {
    if (!plan_knobs().cost_table) return -1.0;
    int best = -1, bd = 1 << 30;
    for (int i = 0; i < kNumPassCosts; ++i) {
        const PassCost& e = kPassCosts[i];
        if (e.key_bytes != kb || e.lt != lt || e.kind != kind || e.R != R || (e.flip != 0) != flip || e.hi != hi)
            continue;
        const int d = e.logn > k ? e.logn - k : k - e.logn;
        if (d < bd) { bd = d; best = i; }
    }
    if (best < 0) return -1.0;
    // unit: the median of the table's passes at that size and tile
    const int ln = kPassCosts[best].logn;
    std::vector<float> v;
    for (int i = 0; i < kNumPassCosts; ++i)
        if (kPassCosts[i].key_bytes == kb && kPassCosts[i].lt == lt && kPassCosts[i].logn == ln)
            v.push_back(kPassCosts[i].us);
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    return kPassCosts[best].us / v[v.size() / 2];
}

inline double pass_cost(int LT, int KB, int VB, int mode, int R, bool flip, int cmin, int kb, int hi, int k) {
    const int kind = mode == TM_ROWS ? KIND_GLOBAL : mode == TM_SPAN ? KIND_SPAN : KIND_TILE_MERGE;
    const double c = table_cost(kind, kb, LT, R, flip, hi, k);
    return c >= 0 ? c : model_cost(LT, KB, VB, mode, R, flip, cmin, kb);
}

// Wide ROWS pass (k_rows_wide): one LDS round trip, rows of 2^(16-R) keys.
inline double wide_cost(int R, bool flip, int cmin, int hi, int k) {
    const double c = table_cost(KIND_WIDE, 4, WIDE_LT - 1, R, flip, hi, k);  // measured beside the 2^15 tiles
    return c >= 0 ? c : 1.0 + 0.035 + (WIDE_LT - R <= cmin ? 0.03 : 0.0);
}

inline std::vector<Pass> plan_span(int k, int LT, int rmax, int cmin, int KB, int VB, int kb, bool wide) {
    struct St { int m, b; };
    std::vector<St> seq;
    for (int m = LT + 1; m <= k; ++m)
        for (int b = m - 1; b >= 0; --b) seq.push_back(St{m, b});
    const int N = (int)seq.size();
    const double INF = 1e30;
    std::vector<double> best(N + 1, INF);
    std::vector<Pass> how(N + 1);
    std::vector<int> nxt(N + 1, N);
    best[N] = 0;
    for (int p = N - 1; p >= 0; --p) {
        const int m = seq[p].m, b = seq[p].b;
        auto take = [&](int q, double c, Pass ps) {
            if (q <= N && best[q] + c < best[p]) {
                best[p] = best[q] + c;
                how[p] = ps;
                nxt[p] = q;
            }
        };
        if (b >= LT) {
            for (int R = 1; R <= rmax && LT - R >= cmin; ++R) {
                const int lo = b - R + 1;
                if (lo < LT - R) break;
                take(p + R, pass_cost(LT, KB, VB, TM_ROWS, R, b == m - 1, cmin, kb, b, k),
                     Pass{KIND_GLOBAL, b, R, b == m - 1});
            }
            // the wide (2^16-key register) tile: R <= 10 with >= 2^cmin-key rows
            for (int R = WIDE_RMIN; wide && R <= WIDE_RMAX && WIDE_LT - R >= cmin && b - R + 1 >= 0; ++R) {
                if (b - R + 1 < WIDE_LT - R) break;
                take(p + R, wide_cost(R, b == m - 1, cmin, b, k), Pass{KIND_WIDE, b, R, b == m - 1});
            }
        } else if (b == LT - 1) {
            take(p + LT, pass_cost(LT, KB, VB, TM_MERGE, 0, false, cmin, kb, LT - 1, k),
                 Pass{KIND_TILE_MERGE, LT - 1, 0, false});
        }
        if (b < LT && m < k) {
            const int R = LT - (b + 1);
            if (R >= 1 && R <= rmax && LT - R >= cmin)
                take(p + (b + 1) + R, pass_cost(LT, KB, VB, TM_SPAN, R, true, cmin, kb, m, k),
                     Pass{KIND_SPAN, m, R, true});
        }
    }
    std::vector<Pass> ps;
    ps.push_back(Pass{KIND_TILE_SORT, LT - 1, 0, false});
    if (N > 0 && best[0] >= INF) return plan_levels(k, LT, rmax);
    for (int p = 0; p < N; p = nxt[p]) ps.push_back(how[p]);
    return ps;
}

inline std::vector<Pass> plan(int k, int LT, int rmax, int cmin, bool span, int KB, int VB, int kb, bool wide) {
    return span ? plan_span(k, LT, rmax, cmin, KB, VB, kb, wide) : plan_levels(k, LT, rmax);
}

// The plan local_sort_lt runs for n keys (shared with plan_passes()).  It
// depends only on ceil_log2(n) (the knobs are read once), and the DP over the
// measured cost table takes milliseconds of host time, so each size is
// planned once per process: without the cache a 2^20-key sort spent ~0.5 ms
// per call on the host planning it (profiles/r01/size_sweep_v9.jsonl; 2^24 u32 went 1.47 -> 0.60 ms).
//
// runs: the sort has a scratch buffer to ping-pong with, so levels from
// merge_from on may run as merge passes (KIND_RUNS, hi = log2 of the input
// run length), one HBM pass per level instead of about two network passes.
template <typename K, int LT, int LTR>
std::vector<Pass> plan_uncached(int k, bool runs);

template <typename K, int LT, int LTR>
const std::vector<Pass>& plan_for(int64_t n, bool runs = true) {
    static std::mutex mu;
    static std::vector<Pass> cache[2][64];
    const int k = ceil_log2(n);
    std::lock_guard<std::mutex> g(mu);
    if (cache[runs][k].empty()) cache[runs][k] = plan_uncached<K, LT, LTR>(k, runs);
    return cache[runs][k];
}

template <typename K, int LT, int LTR>
std::vector<Pass> plan_uncached(int k, bool runs) {
    const PlanKnobs& kn = plan_knobs();
    const int m0 = kn.merge_from((int)sizeof(K));
    if (runs && m0 > 0 && k > m0 && !(sizeof(K) == 4 && k <= kn.merge_min_log2_u32)) {
        std::vector<Pass> ps = plan_uncached<K, LT, LTR>(m0 < LT ? LT : m0, false);
        int lw = m0 < LT ? LT : m0;
        // the levels in as few multi-way passes as the cap allows (a pass of
        // lk levels is one HBM sweep; runsk.hip needs lw >= 15 and lw + lk <=
        // 30 for u32, 13 and 29 for u64), the larger ones first; a single
        // level left over runs as a 2-way pass (which keeps host staging's
        // chunked final pass)
        const int lwk_max = merge_levelk_lwk_max((int)sizeof(K));
        const int L = (k < lwk_max ? k : lwk_max) - lw;  // levels the multi-way passes can take
        const int mw = kn.multiway_cap((int)sizeof(K), L);
        if (mw >= 2 && lw >= merge_levelk_lw_min((int)sizeof(K))) {
            const int cap = mw < 4 ? mw : 4;
            if (L >= 2) {
                const int np = (L + cap - 1) / cap;  // fewest passes
                for (int i = 0; i < np; ++i) {
                    // spread the levels: the first L % np passes take one more
                    const int lk = L / np + (i < L % np ? 1 : 0);
                    ps.push_back(Pass{KIND_RUNSK, lw, lk, false});
                    lw += lk;
                }
            }
        }
        for (; lw < k; ++lw) ps.push_back(Pass{KIND_RUNS, lw, 0, false});
        return ps;
    }
    const int rmax = kn.rmax < LTR - 5 ? kn.rmax : LTR - 5;
    int cmin = kn.row_bytes_log2 - (sizeof(K) == 4 ? 2 : 3);
    if (cmin < 5) cmin = 5;
    typedef TileGeo<K, LT> G;
    // wide ROWS passes: u32 keys with the 2^15-key LDS tiles (hi >= 15)
    const bool wide = kn.wide && sizeof(K) == 4 && LTR == WIDE_LT - 1;
    return plan(k, LT, rmax, cmin, kn.span && LT == LTR, G::KB, G::VB, (int)sizeof(K), wide);
}

// The u32 SORT pass runs k_sort_u32 (launch_pass's condition).
inline bool sort_u32_path() { return MISORT_WAVE_SORT && MISORT_WAVE_LEVELS <= 10 && plan_knobs().sort_u32; }

// One pass of a plan over n keys, src -> dst.
template <typename K, int LT, int LTR>
void launch_pass(const K* src, K* dst, int64_t n, const Pass& p, bool ord_in, hipStream_t s,
                 void* fence = nullptr, int flk = 0) {
    TileMap tm{};
    tm.ntiles = (n + (1 << LT) - 1) >> LT;
    if (p.kind == KIND_TILE_SORT) {
        if constexpr (sizeof(K) == 8) {
            if (ord_in) {
                launch_stream<K, LT, TM_SORT, 0, false, true>(src, dst, n, tm, s, fence, flk);
            } else {
                launch_stream<K, LT, TM_SORT, 0, false, false>(src, dst, n, tm, s, fence, flk);
            }
        } else if (LT == 15 && MISORT_WAVE_SORT && MISORT_WAVE_LEVELS <= 10 && plan_knobs().sort_u32) {
            launch_sort_u32(src, dst, n, s, (uint64_t*)fence, flk);
        } else {
            launch_stream<K, LT, TM_SORT, 0, false, false>(src, dst, n, tm, s);
        }
    } else if (p.kind == KIND_GLOBAL) {
        launch_rows<K, LTR, TM_ROWS>(src, dst, n, p.hi, p.R, p.flip, s);
    } else if (p.kind == KIND_SPAN) {
        launch_rows<K, LTR, TM_SPAN>(src, dst, n, p.hi, p.R, true, s);
    } else if (p.kind == KIND_WIDE) {
        if constexpr (sizeof(K) == 4) launch_rows_wide(src, dst, n, p.hi, p.R, p.flip, s);
    } else {
        launch_stream<K, LT, TM_MERGE, 0, false, false>(src, dst, n, tm, s);
    }
}

// LT: SORT/MERGE tile; LTR: ROWS tile.
template <typename K, int LT, int LTR>
hipError_t local_sort_lt(const K* in, K* out, int64_t n, bool ord_in, K* scratch, hipStream_t s,
                         LaunchHook* hook, const StageIO* io) {
    const PlanKnobs& kn = plan_knobs();
    const bool pp = kn.pingpong && scratch != nullptr && scratch != out && scratch != in;
    const std::vector<Pass>& ps = plan_for<K, LT, LTR>(n, pp);  // merge passes need two buffers
    const int np = (int)ps.size();
    const double bytes = 2.0 * (double)n * sizeof(K);
    const K* src = in;
    int fence_phase = 0;  // multi-way passes: fence buffer holding the next pass's fences
    // the u32 SORT pass writes the first multi-way pass's fences (no gather pass)
    // (u32: k_sort_u32 with the 2^15 tile; u64: the k_stream SORT tile)
    const bool sort_fences = np > 1 && ps[0].kind == KIND_TILE_SORT && ps[1].kind == KIND_RUNSK &&
                             ps[1].hi == LT && !(io && io->before_first) &&
                             (sizeof(K) == 8 || (LT == 15 && sort_u32_path()));
    for (int i = 0; i < np; ++i) {
        // ping-pong: pass i writes `out` iff an even number of passes follow it
        K* dst = (!pp || ((np - 1 - i) & 1) == 0) ? out : scratch;
        const Pass& p = ps[i];
        HookScope hs(hook, p.kind, bytes, s);
        if (p.kind == KIND_RUNSK) {
            const bool prevk = i > 0 && (ps[i - 1].kind == KIND_RUNSK || (i == 1 && sort_fences));
            const int lk_next = i + 1 < np && ps[i + 1].kind == KIND_RUNSK ? ps[i + 1].R : 0;
            const hipError_t e = merge_levelk(src, dst, n, p.hi, p.R, s, fence_phase, !prevk, lk_next, hook);
            if (e != hipSuccess) return e;
            fence_phase ^= 1;
            src = dst;
            continue;
        }
        const bool runs = p.kind == KIND_RUNS;
        const bool contig = p.kind == KIND_TILE_SORT || p.kind == KIND_TILE_MERGE || runs;
        const bool cin = io && io->before_first && i == 0;
        const bool cout = io && io->after_last && i == np - 1 && contig;
        if (cin || cout) {
            // chunk by chunk (contiguous tiles only: offsets keep the tile grid)
            const int64_t ch = io->chunk;
            if (ch <= 0 || (ch & ((1 << LT) - 1)) || !contig) return hipErrorInvalidValue;
            for (int64_t k0 = 0; k0 < n; k0 += ch) {
                const int64_t k1 = n - k0 < ch ? n : k0 + ch;
                if (cin && io->before_first(k0, k1, s)) return hipErrorUnknown;
                if (runs) {
                    // a merge level reads across chunks: whole input, output range [k0, k1)
                    if (merge_level<K>(src, dst, n, p.hi, s, k0, k1) != hipSuccess) return hipErrorInvalidValue;
                } else {
                    launch_pass<K, LT, LTR>(src + k0, dst + k0, k1 - k0, p, ord_in, s);
                }
                if (cout && io->after_last(k0, k1, s)) return hipErrorUnknown;
            }
        } else if (runs) {
            const hipError_t e = merge_level<K>(src, dst, n, p.hi, s);
            if (e != hipSuccess) return e;
        } else if (i == 0 && sort_fences) {
            void* f = mergek_fence_buffer(n, (int)sizeof(K), 0, s);
            if (!f) return hipErrorOutOfMemory;
            launch_pass<K, LT, LTR>(src, dst, n, p, ord_in, s, f, ps[1].R);
        } else {
            launch_pass<K, LT, LTR>(src, dst, n, p, ord_in, s);
        }
        src = dst;
    }
    return hipGetLastError();
}

}  // namespace

// Definition shared by sort_u32.hip / sort_u64.hip (one explicit instantiation each).
template <typename K>
hipError_t local_sort(const K* in, K* out, int64_t n, bool ord_in, K* scratch, hipStream_t s,
                      LaunchHook* hook, const StageIO* io) {
    if (n <= 0) return hipSuccess;
    if (sizeof(K) == 4 && ord_in) return hipErrorInvalidValue;
    constexpr int S = KT<K>::LT_SMALL;  // 14 (u32) / 13 (u64): the 64 KiB tile
    const PlanKnobs& kn = plan_knobs();
    const bool big = kn.big((int)sizeof(K)), rbig = kn.rbig((int)sizeof(K));
    if (big && rbig) return local_sort_lt<K, S + 1, S + 1>(in, out, n, ord_in, scratch, s, hook, io);
    if (big) return local_sort_lt<K, S + 1, S>(in, out, n, ord_in, scratch, s, hook, io);
    return local_sort_lt<K, S, S>(in, out, n, ord_in, scratch, s, hook, io);
}

// One pass of any shape (pass-cost probes, tools/pass_costs.py), with the key
// type's current tiles (both large or both small).
template <typename K>
hipError_t run_pass(const K* in, K* out, int64_t n, int kind, int hi, int R, int flip, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    constexpr int S = KT<K>::LT_SMALL;
    const PlanKnobs& kn = plan_knobs();
    const bool big = kn.big((int)sizeof(K)), rbig = kn.rbig((int)sizeof(K));
    if (big != rbig) return hipErrorInvalidValue;
    const int LT = big ? S + 1 : S;
    const Pass p{(Kind)kind, hi, R, flip != 0};
    if (kind == KIND_RUNS) return merge_level<K>(in, out, n, hi, s);  // runs of 2^hi -> 2^(hi+1)
    if (kind == KIND_RUNSK)  // runs of 2^hi -> 2^(hi+R), R = 1..4 (0: 2)
        return merge_levelk(in, out, n, hi, R > 0 ? R : 2, s, 0, true, 0);
    if (kind < 0 || kind >= KIND_COUNT || kind == KIND_MERGE_SPLIT || kind == KIND_OTHER ||
        kind == KIND_EXCHANGE)
        return hipErrorInvalidValue;
    if (kind == KIND_GLOBAL || kind == KIND_SPAN) {
        if (R < 1 || R > LT - 5 || hi - R + 1 < LT - R || ((int64_t)1 << (hi + 1)) > ((int64_t)1 << ceil_log2(n)))
            return hipErrorInvalidValue;
    }
    if (kind == KIND_WIDE) {
        if (sizeof(K) != 4 || !big || R < WIDE_RMIN || R > WIDE_RMAX || hi - R + 1 < WIDE_LT - R ||
            ((int64_t)1 << (hi + 1)) > ((int64_t)1 << ceil_log2(n)))
            return hipErrorInvalidValue;
    }
    if (big) launch_pass<K, S + 1, S + 1>(in, out, n, p, false, s);
    else launch_pass<K, S, S>(in, out, n, p, false, s);
    return hipGetLastError();
}

}  // namespace misort
