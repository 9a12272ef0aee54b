// bitonic.h -- the gfx950 (CDNA4) bitonic SORT tile and the local-sort plan.
//
// Replaces the reference's local std::sort (psort.cc:175).  Written for wave64 /
// 160 KiB LDS / 8 TB/s HBM3E; no MFMA (sorting is not a contraction).  Included
// by one translation unit per key type (sort_u32.hip, sort_u64.hip), which
// instantiate local_sort<K>; kernels.hip uses only the shared device helpers.
//
// A local sort of n keys is ONE pass of SORT tiles followed by merge passes:
//   SORT     every 2^LT-key tile (u32: 2^15 = 128 KiB of LDS, one 1024-lane
//            workgroup per CU; u64: 2^13, two 256-lane workgroups per CU) is
//            sorted by the bitonic network in LDS and registers -- levels 1..LT
//            in one HBM read and one HBM write per key;
//   RUNSK    2^lk-way merge passes (runsk.hip): lk merge levels per HBM sweep
//            (u32, 2^30 keys past the tile: three 16-way passes and one 8-way);
//   RUNS     a single level left over (or every level, MISORT_MULTIWAY=0):
//            2-way merge passes (runs.hip).
// The keys carry no payload, so any correct sort writes the same bytes as the
// reference's std::sort.  Rounds 1-2 also carried a network engine for the
// levels past the tile (ROWS / SPAN / MERGE passes of the bitonic network,
// planned by a dynamic program over a measured cost table); from round 3 the
// merge passes beat it at every size (profiles/r03/small_u32: 2^16 1.00 vs
// 0.89 Gkeys/s, 2^20 6.77 vs 6.21, 2^23 30.4 vs 25.0), so it is retired.
//
// Sorting network of the tile: bitonic sort in the "flip" formulation.  Level m
// (blocks of s = 2^m keys) starts with the flip stage, which compares i with its
// mirror i ^ (s-1), and continues with half-cleaner stages i <-> i ^ 2^j for
// j = m-2 .. 0.  Every compare-exchange puts the minimum at the lower index, so
// no direction bits exist and every block is ascending after its level.  A
// sentinel (all-ones) suffix can only move upwards, so the padding of a partial
// last tile up to 2^LT is VIRTUAL: indices >= n read as all-ones and are never
// stored.
//
// A pass over n keys moves 2 * n * sizeof(K) algorithmic HBM bytes.
#pragma once
#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "kernels.h"
#include "lds_merge.h"

namespace misort {

// Planner knobs (environment, read once per process, kernels.hip):
//   MISORT_PERSIST         bit 0: the u32 SORT pass runs a persistent grid of
//                          MISORT_GRID_MULT x the resident capacity with the
//                          next tile's loads in flight (default 1); 0: one
//                          workgroup per tile;
//   MISORT_PERSIST_U64     the same for the u64 (and f64) SORT pass (default 1);
//   MISORT_MULTIWAY        u32 merge levels per multi-way pass (runsk.hip,
//                          2^lk-way, lk <= 4); 0 or 1: one 2-way pass per level;
//                          -1 (default): 4 (see multiway_cap);
//   MISORT_MULTIWAY_U64    the same for u64 (and f64) keys (default 4).
struct PlanKnobs {
    int persist = 1, persist_u64 = 1, grid_mult = 1;
    // -1 (default): 4, the fewest passes (up to 16-way) at every size.  Round
    // 2 had kept 8-way passes where the levels split into threes (L = 12, 15:
    // 2^27, 2^30); with the two-keys-per-read merge chain the fewest passes win
    // everywhere (profiles/r04/mw, one box, 2 x 10 sorts each): 2^26 +2.0 %,
    // 2^27 +1.3 %, 2^28 +3.8 %, 2^29 +2.2 %, 2^30 +0.9 %, 2^31 +0.6 %
    int multiway = -1;
    // u64 (and f64): 128-bit fences, 8192-key chunks at 2 workgroups per CU.
    // 16-way passes measured faster for u64 at every size (profiles/r02/ab_mw:
    // 2^24 +8 %, 2^26 +4 %, 2^27 +1.5 %, 2^29 +2.5 % over 8-way): fewer
    // passes, and u64 chains cost less per byte than u32 ones
    int multiway_u64 = 4;
    // u32 SORT tile (log2 keys): 0 (default) = per size (sort_tile_u32), 14 or 15 = always
    int sort_tile_u32 = 0;
    PlanKnobs();
    // the cap for L levels
    int multiway_cap(int kb, int L) const {
        if (kb != 4) return multiway_u64;
        if (multiway >= 0) return multiway;
        (void)L;
        return 4;
    }
    bool persist_sort(int kb) const { return (kb == 4 ? persist : persist_u64) & 1; }
};
const PlanKnobs& plan_knobs();

namespace {

template <typename K>
struct KT;
template <>
struct KT<uint32_t> {
    static constexpr uint32_t MAX = 0xFFFFFFFFu;
    static constexpr int V = 4;   // keys per 16-byte vector
    static constexpr int LT = SORT_LT_U32;  // log2 keys of the larger SORT tile (kernels.h)
    typedef uint32_t vec __attribute__((ext_vector_type(4)));
};
template <>
struct KT<uint64_t> {
    static constexpr uint64_t MAX = ~0ull;
    static constexpr int V = 2;
    static constexpr int LT = 13; // 64 KiB + padding: two workgroups per CU
    typedef uint64_t vec __attribute__((ext_vector_type(2)));
};


// u64 compare-exchanges on one v_cmp_u64 (cx); register stages batch their
// compares ahead of the selects (reg_stages_c): u64 SORT tile at 2^29 6.71 ->
// 5.78 ms (one compare, profiles/r03/ab2) -> 5.58 ms (batched, profiles/r03/ab4).
template <typename K>
__device__ __forceinline__ void cx(K& a, K& b) {
    if constexpr (sizeof(K) == 8) {
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

// ------------------------------------------------- SORT tile engine
//
// Persistent workgroups walk the list of 2^LT-key tiles.  While the LDS phases
// of tile i run, the 16-byte loads of tile i+1 are already in flight into a
// register buffer, so HBM streams through the LDS work.  Key v of a tile is
// tile*2^LT + v.
//
// Register slots: lane t loads LOADS = 32/V vectors, slot k = virtual keys
// (k*NT + t)*V .. +V-1 (coalesced 16-byte loads and stores).
//
// LDS layout: key v at word v + v/32.  The padding keeps every phase's
// 32-lane accesses on distinct banks, and since v + v/32 is additive over
// disjoint bit fields every access is one base VGPR plus an immediate offset.
struct TileMap {
    int64_t ntiles;  // tiles (the last may be partial)
};

// LDS word of virtual key v (conflict-free for every 5-bit window, additive
// over disjoint bit fields).
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

// Virtual start of the vector of slot k, lane t: (k*NT + t)*V.
template <typename K, int LT>
__device__ __forceinline__ int place(int k, int t) {
    typedef TileGeo<K, LT> G;
    return (k * G::NT + t) * G::V;
}

template <typename K, int LT, bool ORD>
__device__ __forceinline__ void tile_fetch(K (*pre)[KT<K>::V], const K* src, int64_t tile, int64_t n, int t) {
    typedef TileGeo<K, LT> G;
    const bool full = ((tile + 1) << LT) <= n;
#pragma unroll
    for (int k = 0; k < G::LOADS; ++k) {
        const int64_t gi = (tile << LT) + place<K, LT>(k, t);
        if (full) {
            // streamed once per pass: non-temporal (measured +10 % on this shape,
            // tools/hbm_shapes.hip)
            typename KT<K>::vec x = __builtin_nontemporal_load(reinterpret_cast<const typename KT<K>::vec*>(src + gi));
#pragma unroll
            for (int j = 0; j < G::V; ++j) pre[k][j] = ORD ? ord_of_f64(x[j]) : x[j];
        } else {
            load_vec<K, ORD>(src, gi, n, pre[k]);
        }
    }
}

template <typename K, int LT>
__device__ __forceinline__ void store_slot(K* dst, int64_t tile, int64_t n, bool full, int e,
                                           const K (&w)[KT<K>::V]) {
    const int64_t gi = (tile << LT) + e;
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
        if constexpr (sizeof(K) == 8) {
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

// Levels 1..5 of the tile: the 32 register keys of a lane into ascending
// order: Batcher's odd-even merge sort (191 compare-exchanges in the same 15
// steps) instead of the bitonic stages (240); the steps after it only need
// each lane's 32 keys ascending (u32 tile 3.36 -> 3.33 ms at 2^30, u64 -2.4 %,
// profiles/r05/tile/oem_ab.txt).
// One step (P, D) of the odd-even merge sort: the pairs (i, i + D) inside
// one 2P-block, in runs of D starting at D mod P.
template <typename K, int P, int D>
__device__ __forceinline__ void oem_step(K (&v)[32]) {
    if constexpr (sizeof(K) == 8) {
        // u64: the step's compares first, then the selects (as reg_stages_c)
        bool lt[16];
        int q = 0;
#pragma unroll
        for (int j = D % P; j + D < 32; j += 2 * D)
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (i + j + D < 32 && (i + j) / (2 * P) == (i + j + D) / (2 * P)) lt[q++] = v[i + j] < v[i + j + D];
#pragma unroll
        for (int j = D % P; j + D < 32; j += 2 * D)
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (i + j + D < 32 && (i + j) / (2 * P) == (i + j + D) / (2 * P))
                    asm("" : "+v"(v[i + j]), "+v"(v[i + j + D]));
        q = 0;
#pragma unroll
        for (int j = D % P; j + D < 32; j += 2 * D)
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (i + j + D < 32 && (i + j) / (2 * P) == (i + j + D) / (2 * P)) {
                    K& a = v[i + j];
                    K& b = v[i + j + D];
                    const bool l = lt[q++];
                    const K lo = l ? a : b, hi = l ? b : a;
                    a = lo;
                    b = hi;
                }
    } else {
#pragma unroll
        for (int j = D % P; j + D < 32; j += 2 * D)
#pragma unroll
            for (int i = 0; i < D; ++i)
                if (i + j + D < 32 && (i + j) / (2 * P) == (i + j + D) / (2 * P)) cx(v[i + j], v[i + j + D]);
    }
}
template <typename K>
__device__ __forceinline__ void sort32_regs(K (&v)[32]) {
    {
        oem_step<K, 1, 1>(v);
        oem_step<K, 2, 2>(v);
        oem_step<K, 2, 1>(v);
        oem_step<K, 4, 4>(v);
        oem_step<K, 4, 2>(v);
        oem_step<K, 4, 1>(v);
        oem_step<K, 8, 8>(v);
        oem_step<K, 8, 4>(v);
        oem_step<K, 8, 2>(v);
        oem_step<K, 8, 1>(v);
        oem_step<K, 16, 16>(v);
        oem_step<K, 16, 8>(v);
        oem_step<K, 16, 4>(v);
        oem_step<K, 16, 2>(v);
        oem_step<K, 16, 1>(v);
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
        if constexpr (HI >= WAVE_BITS || NXT >= WAVE_BITS || NXT < 0) __syncthreads();
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
// v_med3_u32 (med3(x, p, 0) = min, med3(x, p, ~0) = max).  The
// cross-lane ops are VALU-heavy (DPP hazards, two DPPs for xor 4/8, permlane
// swaps): measured per 2^30 SORT pass 6.9 ms (in the wave up to level 11),
// 5.23 (7), 5.16 (8), 5.21 (9), 5.57 ms (all LDS; profiles/r01/ab/wave_levels.txt).  Default: levels 6..8 in
// the wave (quad_perm / row_half_mirror only), 9..15 in LDS phases.
// (Semantics of every cross-lane op: tools/dpp_probe.hip.)
// highest level run in the wave (6..11); the levels above go through LDS
// phases (7 / 9 measured equal or slower, profiles/r03/ab_wl)
constexpr int WAVE_LEVELS = 8;

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

// LDS -> 16-byte vectors -> HBM.  fence (may be null): the first multi-way
// merge pass's fences, written here instead of gathered from HBM by
// k_fence_gather -- the key at every 2^MERGEK_FENCE_LOG2-th position of the
// sorted tile, packed as runsk.hip's fpack does for runs of 2^LT keys in
// groups of 2^flk (u32 keys: 64-bit fences, u64 keys: 128-bit).
template <typename K, int LT>
__device__ __forceinline__ void final_store(const K* s, K* out, int64_t tile, int64_t n, bool full, int t,
                                            void* fence = nullptr, int flk = 0) {
    typedef TileGeo<K, LT> G;
#pragma unroll
    for (int k = 0; k < G::LOADS; ++k) {
        const int e = place<K, LT>(k, t);
        K x[G::V];
#pragma unroll
        for (int j = 0; j < G::V; ++j) x[j] = s[pad(e + j)];
        store_slot<K, LT>(out, tile, n, full, e, x);
        // flk = the first pass's lk | its fence stride (log2) << 8 (0: MERGEK_FENCE_LOG2)
        const int fgl = (flk >> 8) ? (flk >> 8) : MERGEK_FENCE_LOG2, lkf = flk & 0xFF;
        const int64_t gi = (tile << LT) + e;
        if (fence && (e & ((1 << fgl) - 1)) == 0 && gi < n) {
            const uint32_t tag = ((uint32_t)((gi >> LT) & ((1 << lkf) - 1)) << (32 - lkf)) | (uint32_t)(e >> fgl);
            if constexpr (sizeof(K) == 4)
                ((uint64_t*)fence)[gi >> fgl] = ((uint64_t)x[0] << 32) | tag;
            else
                ((unsigned __int128*)fence)[gi >> fgl] = ((unsigned __int128)x[0] << 64) | tag;
        }
    }
}

// The SORT tile's top levels as merge levels.  SORT_MERGE_F (u32) /
// SORT_MERGE_F_U64 = F: levels 1..F-1 run as the bitonic network
// (registers, DPP, wave-local LDS phases), leaving sorted runs of 2^(F-1) keys
// (F <= 12: a run lies inside one wave's 2^11 keys); the runs are laid out
// plainly in LDS with sentinels after each and merged pairwise in levels
// F..LT by the multi-way pass's in-LDS machinery (lds_merge.h: phased co-rank
// searches, merge chains), IT outputs per lane -- instead of barrier-separated
// LDS phases with LT - F + 1 .. LT stages each.  Measured on one box each (profiles/r04/sortmerge, sortmerge64):
//   u32 2^14 tile (the default tile from 2^25, see sort_tile_u32): the 2^30
//   SORT pass 4.31 ms as a network -> 3.61 (F = 12) -> 3.42 (F = 11) ->
//   3.60 (F = 10); the 2^15 tile with F = 12: 5.80 (one workgroup per CU).
//   u64 2^13 tile at 2^29: 5.57 ms -> 5.05 (F = 12) -> 4.74 (11) -> 4.73 (10)
//   on the persistent grid, 4.43 (12) / 4.32 (10) / 4.31 (9) one tile per
//   workgroup, 8.4 (8: 88 KiB of LDS, one workgroup per CU).
// The merge-level tiles run one tile per workgroup: the merge keeps IT more
// keys per lane live than the network, and the persistent grid's prefetch
// measured slower.
constexpr int SORT_MERGE_F = 11, SORT_MERGE_F_U64 = 10;
// The u32 merge-level tile's smallest outputs per lane (even: aligned pair
// writes; 34 = the odd-half layout: IT / 2 = 17 keeps the lanes' chain
// pointers on distinct banks; 33, the odd layout, measured first,
// profiles/r04/sorteven).  The merge levels use the multi-way passes' zero
// words (lds_merge.h, profiles/r05/zwpt) and the uniform pair geometry: all
// the tile's runs have one length, so a lane's pair is its position over the
// level's constant pair stride (u32 tile 3346 -> 3314 us at 2^30; u64 +14 us,
// kept off; profiles/r05/tile/unigeo_ab.txt).  u64 merges one key per LDS read
// (two-key chains measured equal, profiles/r05/mergek/u64_chain_ab.txt).
constexpr int SORT_IT0 = 34;
template <typename KEY, int LT, int F>
struct SortMergeShape {
    static_assert(F >= 7 && F <= 12 && F <= LT, "merge levels from runs of 64 .. 2^11 keys");
    static constexpr int NT = 1 << (LT - 5);  // 32 keys per lane
    static constexpr int K = 1 << (LT - F + 1), LKS = LT - F + 1, RUN = 1 << (F - 1);
    // two-key chains for u32, one key per read for u64
    static constexpr int CH = sizeof(KEY) == 4 ? 1 : 0;
    // outputs per lane: the smallest count from IT0 up (step 2) whose level
    // layouts fit: 2^LT keys + per pair G + QA gap.  u32: even (IT0 = 34),
    // so every level writes aligned pairs; u64: odd (33: lanes' diagonals on
    // distinct banks; a pair of u64 keys is a 16-byte write, no cheaper than two)
    static constexpr int IT0 = CH == 1 ? SORT_IT0 : 33;
    static constexpr int fit(int it) { return (1 << LT) + (K / 2) * (it + 1 + it) <= NT * it ? it : fit(it + 2); }
    static constexpr int IT = fit(IT0);
    static_assert(CH == 0 || IT % 2 == 0, "the two-key chain merges an even count");
    static constexpr int G = IT + 1;                   // sentinels after each sequence (a chain reads <= IT past it)
    static constexpr int QA = IT;                      // pairs start at lane boundaries
    static constexpr int MAXR = 1 << (LT - 1);         // a last-level pair: two runs of 2^(LT-1)
    static constexpr int GS = G;
    static constexpr int WORDS = NT * IT + G + 8;  // the level layouts (>= K runs of RUN + GS)
    static_assert(K * (RUN + GS) <= WORDS && (1 << LT) + (K / 2) * (G + QA) <= NT * IT, "SORT merge layout");
    // zero words below the A sequences (two-key chains) and, u32, the
    // uniform geometry (K runs of RUN keys at a stride of RUN + GS;
    // lds_merge.h shape_uni)
    static constexpr bool ZW = CH == 1;
    static constexpr bool UNI = sizeof(KEY) == 4;
    static constexpr int ALL_WORDS = WORDS;
};

// Levels F..LT of a tile whose runs of 2^(F-1) keys are sorted in the padded
// layout (pad(v)): lane l of wave w moves keys w * 2^11 + 64c + l to the plain
// layout (run q at q * (RUN + GS), GS sentinels after it; consecutive lanes,
// consecutive words), the runs merge in LDS, and lane t's outputs [t * IT,
// t * IT + IT) go back to LDS in plain order.  Ends with a barrier.
template <typename KEY, int LT, int F>
__device__ __forceinline__ void tile_merge_top(KEY* s, int t) {
    typedef SortMergeShape<KEY, LT, F> MS;
    const int w = t >> 6, l = t & 63;
    KEY y[32];
#pragma unroll
    for (int c = 0; c < 32; ++c) y[c] = s[pad((w << 11) + (c << 6) + l)];
    lds_barrier();  // LDS-only hand-offs: a persistent tile's prefetch stays in flight
#pragma unroll
    for (int c = 0; c < 32; ++c) {
        const int v = (w << 11) + (c << 6) + l;
        s[(v >> (F - 1)) * (MS::RUN + MS::GS) + (v & (MS::RUN - 1))] = y[c];
    }
    for (int e = t; e < MS::K * MS::GS; e += MS::NT) {
        const int q = e / MS::GS;
        // ZW: the last of the GS words is the zero word below run q + 1
        s[q * (MS::RUN + MS::GS) + MS::RUN + (e - q * MS::GS)] =
            MS::ZW && e - q * MS::GS == MS::GS - 1 ? (KEY)0 : KMAX<KEY>;
    }
    int st[MS::K], ln[MS::K];
#pragma unroll
    for (int q = 0; q < MS::K; ++q) {
        st[q] = q * (MS::RUN + MS::GS);
        ln[q] = MS::RUN;
    }
    lds_merge_prologue<KEY, MS>(s, st, t);
    lds_barrier();
    KEY r[MS::IT];
    lds_merge_levels<KEY, MS, 0>(s, st, ln, r, t, MS::WORDS - 1);
    if (t * MS::IT < (1 << LT)) {
        if constexpr (MS::CH == 1 && MS::IT % 2 == 0) {
#pragma unroll
            for (int j = 0; j < MS::IT; j += 2) *reinterpret_cast<kvec2<KEY>*>(s + t * MS::IT + j) = kvec2<KEY>{r[j], r[j + 1]};
        } else {
#pragma unroll
            for (int j = 0; j < MS::IT; ++j) s[t * MS::IT + j] = r[j];
        }
    }
    lds_barrier();
}

// LDS (plain layout) -> 16-byte vectors -> HBM, and the first multi-way
// pass's fences (final_store for the merge-level tile).
template <typename K, int LT>
__device__ __forceinline__ void final_store_plain(const K* s, K* out, int64_t tile, int64_t n, bool full, int t,
                                                  void* fence, int flk) {
    typedef TileGeo<K, LT> G;
#pragma unroll
    for (int k = 0; k < G::LOADS; ++k) {
        const int e = place<K, LT>(k, t);
        const typename KT<K>::vec v = *reinterpret_cast<const typename KT<K>::vec*>(s + e);
        K x[G::V];
#pragma unroll
        for (int j = 0; j < G::V; ++j) x[j] = v[j];
        store_slot<K, LT>(out, tile, n, full, e, x);
        // flk = the first pass's lk | its fence stride (log2) << 8 (0: MERGEK_FENCE_LOG2)
        const int fgl = (flk >> 8) ? (flk >> 8) : MERGEK_FENCE_LOG2, lkf = flk & 0xFF;
        const int64_t gi = (tile << LT) + e;
        if (fence && (e & ((1 << fgl) - 1)) == 0 && gi < n) {
            const uint32_t tag = ((uint32_t)((gi >> LT) & ((1 << lkf) - 1)) << (32 - lkf)) | (uint32_t)(e >> fgl);
            if constexpr (sizeof(K) == 4)
                ((uint64_t*)fence)[gi >> fgl] = ((uint64_t)x[0] << 32) | tag;
            else
                ((unsigned __int128*)fence)[gi >> fgl] = ((unsigned __int128)x[0] << 64) | tag;
        }
    }
}

// The SORT tile for u64 (and f64, ORD: mapped to ordered u64 on load) keys:
// levels 1..5 on 32 consecutive keys per lane in registers, 6..LT in 5-bit LDS
// phases (wave-local ones without a workgroup barrier).  PERSIST: the grid is
// smaller than the tile list and every workgroup walks tiles with the next
// tile's loads in flight; otherwise one tile per workgroup.
// The first level the u64 SORT tile merges in LDS (0: the whole tile is the
// network): one condition for the kernel and its launcher, so a probe build
// keeps the persistent grid of the network tile.
template <typename K, int LT>
constexpr int sort_tile_mf() {
    return sizeof(K) == 8 && SORT_MERGE_F_U64 <= LT ? SORT_MERGE_F_U64 : 0;
}

template <typename K, int LT, bool ORD, bool PERSIST>
__global__ __launch_bounds__((TileGeo<K, LT>::NT), (TileGeo<K, LT>::WAVES_PER_EU)) void k_sort_tile(
    const K* in, K* out, int64_t n, int64_t ntiles, void* fence, int flk) {
    typedef TileGeo<K, LT> G;
    // SORT_MERGE_F_U64 = F: levels F..LT as in-LDS merge levels
    constexpr int MF = sort_tile_mf<K, LT>();
    typedef SortMergeShape<K, LT, MF ? MF : 12> MS;
    // MERGE: 2 keys below the tile (a co-rank probe may read index -1; 16-byte alignment)
    constexpr int WORDS = MF && MS::ALL_WORDS > lds_words(G::T) ? MS::ALL_WORDS : lds_words(G::T);
    __shared__ __attribute__((aligned(16))) K sbuf[WORDS + (MF ? 2 : 0)];
    K* s = MF ? sbuf + 2 : sbuf;
    const int t = threadIdx.x;
    K pre[G::LOADS][G::V];
    int64_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    // ORD (f64 keys): mapped to ordered u64 once each lane holds its 32
    // consecutive keys, not on load (converting each loaded vector made every
    // LDS write wait for its own load: 4.27 -> 4.74 ms per 2^29 SORT pass)
    tile_fetch<K, LT, false>(pre, in, tile, n, t);
    for (; tile < ntiles; tile += gridDim.x) {
        const bool full = ((tile + 1) << LT) <= n;
        // registers -> LDS
#pragma unroll
        for (int k = 0; k < G::LOADS; ++k) {
            const int e = place<K, LT>(k, t);
#pragma unroll
            for (int j = 0; j < G::V; ++j) s[pad(e + j)] = pre[k][j];
        }
        __syncthreads();
        const int64_t nxt = tile + gridDim.x;
        if (PERSIST && nxt < ntiles) tile_fetch<K, LT, false>(pre, in, nxt, n, t);
        {   // levels 1..5: window [0,5), 32 consecutive keys per lane
            K v[32];
            const int a0 = pad(t << 5);
#pragma unroll
            for (int c = 0; c < 32; ++c) v[c] = s[a0 + c];
            if constexpr (ORD) {
                // the virtual keys past n stay MAX (sentinels, never stored)
                const int64_t v0 = (tile << LT) + (t << 5);
#pragma unroll
                for (int c = 0; c < 32; ++c)
                    if (full || v0 + c < n) v[c] = (K)ord_of_f64((uint64_t)v[c]);
            }
            sort32_regs<K>(v);
#pragma unroll
            for (int c = 0; c < 32; ++c) s[a0 + c] = v[c];
        }
        wave_sync();  // level 6 stays inside the wave
        if constexpr (MF > 0) {
            sort_levels_w<K, 6, MF - 1>(s, t);
            tile_merge_top<K, LT, MF>(s, t);
            final_store_plain<K, LT>(s, out, tile, n, full, t, fence, flk);
        } else {
            sort_levels_w<K, 6, LT>(s, t);
            final_store<K, LT>(s, out, tile, n, full, t, fence, flk);
        }
        __syncthreads();
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

// fence/flk: see final_store (null: no fences).
template <typename K, int LT, bool ORD>
void launch_sort_tile(const K* in, K* out, int64_t n, hipStream_t s, void* fence = nullptr, int flk = 0,
                      hipEvent_t ea = nullptr, hipEvent_t eb = nullptr) {
    typedef TileGeo<K, LT> G;
    static int64_t cap = 0;  // resident workgroups
    const int64_t ntiles = (n + G::T - 1) >> LT;
    // the merge-level tile runs one tile per workgroup (see SORT_MERGE_F)
    const bool persist = sort_tile_mf<K, LT>() == 0 && plan_knobs().persist_sort((int)sizeof(K));
    if (persist && cap == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_tile<K, LT, ORD, true>, G::NT, 0);
        cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
    }
    const int64_t want = persist ? cap * plan_knobs().grid_mult : ntiles;
    const int64_t grid = ntiles < want ? ntiles : want;
    if (grid <= 0) return;
    if (persist)
        launch_timed(k_sort_tile<K, LT, ORD, true>, dim3((unsigned)grid), dim3(G::NT), 0, s, ea, eb, in, out, n, ntiles,
                     fence, flk);
    else
        launch_timed(k_sort_tile<K, LT, ORD, false>, dim3((unsigned)grid), dim3(G::NT), 0, s, ea, eb, in, out, n,
                     ntiles, fence, flk);
}

// ------------------------------------------------ u32 SORT pass kernel
//
// The u32 SORT tile (in-wave levels 1..WAVE_LEVELS, LDS phases above),
// with the full/partial tile split made at compile time: the persistent grid
// walks only full tiles, and a one-workgroup launch sorts the partial last
// tile.  With bounds-checked load/store paths inside the persistent loop the
// kernel reached 128 VGPRs with spills, and one spill reload right after the
// next tile's prefetch issued an s_waitcnt vmcnt(0) that waited for the whole
// prefetch (vmcnt is in order), so the prefetch hid nothing.  The tile base is
// uniform (SGPRs); lanes add 32-bit offsets.
template <int LT, bool FULL>
__device__ __forceinline__ void sort_fetch(uint32_t (*pre)[4], const uint32_t* in, int64_t tile, int64_t n, int t) {
    const uint32_t* tb = in + (tile << LT);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int e = place<uint32_t, LT>(k, t);
        if constexpr (FULL) {
            const KT<uint32_t>::vec x = __builtin_nontemporal_load(reinterpret_cast<const KT<uint32_t>::vec*>(tb + e));
#pragma unroll
            for (int j = 0; j < 4; ++j) pre[k][j] = x[j];
        } else {
            load_vec<uint32_t, false>(in, (tile << LT) + e, n, pre[k]);
        }
    }
}

// 2^15 tile: 1024 lanes, one workgroup per CU; 2^14: 512 lanes, two
// workgroups per CU (4 waves per SIMD: 128 VGPRs per lane)
template <int LT, bool PERSIST, bool FULL>
__global__ __launch_bounds__(1 << (LT - 5), LT == 14 ? 4 : 1) void k_sort_u32(
    const uint32_t* in, uint32_t* out, int64_t n, int64_t ntiles, int64_t tile0, uint64_t* fence, int flk) {
    typedef uint32_t K;
    typedef TileGeo<K, LT> G;
    static_assert(LT == 14 || LT == 15, "u32 SORT tiles");
    constexpr int WL = WAVE_LEVELS;
    static_assert(G::LOADS == 8 && (G::NT == 1024 || G::NT == 512) && WL >= 5 && WL <= 10, "u32 SORT tile shape");
    constexpr int MF = SORT_MERGE_F;  // first merged level
    constexpr bool MERGE = LT == SORT_LT_MERGE;
    typedef SortMergeShape<K, LT, MERGE ? MF : 12> MS;
    // MERGE: 4 words below the tile (a co-rank probe may read index -1)
    __shared__ __attribute__((aligned(16))) K sbuf[(MERGE ? (MS::ALL_WORDS > lds_words(G::T) ? MS::ALL_WORDS
                                                                                               : lds_words(G::T)) + 4
                                                          : lds_words(G::T))];
    K* s = MERGE ? sbuf + 4 : sbuf;
    int64_t tile = tile0 + blockIdx.x;
    if (tile >= ntiles) return;
    K pre[G::LOADS][G::V];
    sort_fetch<LT, FULL>(pre, in, tile, n, (int)threadIdx.x);
    for (; tile < ntiles; tile += gridDim.x) {
        // lane id through an opaque copy: the per-lane LDS/HBM addresses are
        // recomputed every tile instead of being hoisted into ~16 loop-invariant
        // VGPRs (which pushed the kernel into spills)
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        const int a0 = pad(t << 5);
#pragma unroll
        for (int k = 0; k < G::LOADS; ++k) {
            const int e = place<K, LT>(k, t);
#pragma unroll
            for (int j = 0; j < G::V; ++j) s[pad(e + j)] = pre[k][j];
        }
        if constexpr (MERGE) lds_barrier();  // no wait for the previous tile's stores
        else __syncthreads();
        {
            uint32_t x[32];
#pragma unroll
            for (int c = 0; c < 32; ++c) x[c] = s[a0 + c];
            sort32_regs<uint32_t>(x);
            wave_levels<6, WL>(x, t & 63);
            // each lane rewrites only the keys it read: no barrier before, and the
            // next phase (level WL+1 <= 11) stays inside the wave
#pragma unroll
            for (int c = 0; c < 32; ++c) s[a0 + c] = x[c];
            if constexpr (WL + 1 <= WAVE_BITS) wave_sync();
            else __syncthreads();
        }
        // the next tile's loads fly during the LDS phases (issued here, not
        // before the wave levels, so their registers and the cross-lane
        // temporaries are never live together)
        const int64_t nxt = tile + gridDim.x;
        if (PERSIST && nxt < ntiles) sort_fetch<LT, FULL>(pre, in, nxt, n, t);
        if constexpr (MERGE) {
            sort_levels_w<K, WL + 1, MF - 1>(s, t);
            tile_merge_top<K, LT, MF>(s, t);
            final_store_plain<K, LT>(s, out, tile, n, FULL, t, fence, flk);
        } else {
            sort_levels_w<K, WL + 1, LT>(s, t);
            final_store<K, LT>(s, out, tile, n, FULL, t, fence, flk);
        }
        if constexpr (!PERSIST) break;
        // LDS reuse only: the merge tile keeps the next tile's loads in flight
        if constexpr (MERGE) lds_barrier();
        else __syncthreads();
    }
}

// fence/flk: see final_store (null: no fences).
// ea/eb: timing events carried by the first / last launch (null: none).
template <int LT>
void launch_sort_u32(const uint32_t* in, uint32_t* out, int64_t n, hipStream_t s, uint64_t* fence = nullptr,
                     int flk = 0, hipEvent_t ea = nullptr, hipEvent_t eb = nullptr) {
    constexpr int NT = TileGeo<uint32_t, LT>::NT;
    // the merge-level tile runs one workgroup per tile (see SORT_MERGE_F)
    constexpr bool MERGE = LT == SORT_LT_MERGE;
    static int64_t cap = 0;
    const int64_t nfull = n >> LT;
    // (on the persistent grid with the next tile's loads in flight it spills
    // 16 VGPRs and ran 3.45 -> 4.15 ms at 2^30; profiles/r04/sortwave)
    const bool persist = !MERGE && plan_knobs().persist_sort(4);
    const bool tail = (nfull << LT) < n;
    if (nfull > 0) {
        hipEvent_t b = tail ? nullptr : eb;
        if constexpr (!MERGE) {
            if (persist) {
                if (cap == 0) {
                    int per_cu = 0, cus = 0, dev = 0;
                    (void)hipGetDevice(&dev);
                    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
                    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_u32<LT, true, true>, NT, 0);
                    cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
                }
                const int64_t want = cap * plan_knobs().grid_mult;
                launch_timed(k_sort_u32<LT, true, true>, dim3((unsigned)(nfull < want ? nfull : want)), dim3(NT), 0, s,
                             ea, b, in, out, n, nfull, (int64_t)0, fence, flk);
            }
        }
        if (!persist)
            launch_timed(k_sort_u32<LT, false, true>, dim3((unsigned)nfull), dim3(NT), 0, s, ea, b, in, out, n, nfull,
                         (int64_t)0, fence, flk);
    }
    if (tail)
        launch_timed(k_sort_u32<LT, false, false>, dim3(1), dim3(NT), 0, s, nfull > 0 ? nullptr : ea, eb, in, out, n,
                     nfull + 1, nfull, fence, flk);
}

// ------------------------------------------------ the local-sort plan

// One HBM pass of the plan.
struct Pass {
    Kind kind;  // KIND_TILE_SORT, KIND_RUNSK (R levels from runs of 2^hi), KIND_RUNS (one level from 2^hi)
    int hi, R;
    bool flip;  // unused (kept in misort_plan's 4-int records)
};

// The passes for 2^k-key blocks (n <= 2^k): the SORT tile, then the levels
// LT+1..k in as few multi-way passes as the cap allows (a pass of lk levels
// is one HBM sweep; runsk.hip needs lw >= LT and lw + lk <= 30 for u32, 29
// for u64), the larger ones first; a single level left over, and levels past
// the multi-way limit, run as 2-way passes.
inline std::vector<Pass> plan_uncached(int k, int key_bytes, int LT) {
    std::vector<Pass> ps;
    ps.push_back(Pass{KIND_TILE_SORT, LT - 1, 0, false});
    int lw = LT;
    const int lwk_max = merge_levelk_lwk_max(key_bytes);
    const int L = (k < lwk_max ? k : lwk_max) - lw;  // levels the multi-way passes can take
    const int mw = plan_knobs().multiway_cap(key_bytes, L);
    if (mw >= 2 && L >= 2) {
        const int cap = mw < 4 ? mw : 4;
        const int np = (L + cap - 1) / cap;  // fewest passes
        for (int i = 0; i < np; ++i) {
            // spread the levels: the first L % np passes take one more
            const int lk = L / np + (i < L % np ? 1 : 0);
            ps.push_back(Pass{KIND_RUNSK, lw, lk, false});
            lw += lk;
        }
    }
    for (; lw < k; ++lw) ps.push_back(Pass{KIND_RUNS, lw, 0, false});
    return ps;
}

// The u32 SORT tile for 2^k-key blocks: the 2^14 merge-level tile, except
// for tiny sorts (k <= 15) and below 2^25 where only its plan has a 16-way
// pass (a 16-way pass over a small sort costs more than the faster tile
// saves).  Measured at HEAD, one box, 30 sorts per point (profiles/r04/tile):
// 2^14 vs 2^15 tiles 2^20 +11 %, 2^22 +2 %, 2^23 +4 %, 2^24 -4 % (4,3,3 vs
// 3,3,3 levels), 2^25 +1 %, 2^26 +3 %, 2^27 +4 % (four passes against three),
// 2^29 +5 %; 2^18 and 2^21 equal.
inline int sort_tile_u32(int k) {
    const int knob = plan_knobs().sort_tile_u32;
    if (knob == SORT_LT_MERGE || knob == SORT_LT_U32) return knob;
    if (k <= SORT_LT_U32) return SORT_LT_U32;
    if (k >= 25) return SORT_LT_MERGE;
    auto has16 = [k](int lt) {
        for (const Pass& p : plan_uncached(k, 4, lt))
            if (p.kind == KIND_RUNSK && p.R == 4) return true;
        return false;
    };
    return has16(SORT_LT_MERGE) && !has16(SORT_LT_U32) ? SORT_LT_U32 : SORT_LT_MERGE;
}

// Cached per (key type, ceil_log2(n)): the knobs are read once per process.
template <typename K>
const std::vector<Pass>& plan_for(int64_t n) {
    static std::mutex mu;
    static std::vector<Pass> cache[64];
    const int k = ceil_log2(n);
    std::lock_guard<std::mutex> g(mu);
    if (cache[k].empty()) cache[k] = plan_uncached(k, (int)sizeof(K), sizeof(K) == 4 ? sort_tile_u32(k) : KT<K>::LT);
    return cache[k];
}

// lt: the u32 tile (a plan's SORT record: hi + 1); u64 has one tile.
template <typename K>
void launch_sort(const K* src, K* dst, int64_t n, bool ord_in, hipStream_t s, int lt, void* fence = nullptr,
                 int flk = 0, hipEvent_t ea = nullptr, hipEvent_t eb = nullptr) {
    constexpr int LT = KT<K>::LT;
    if constexpr (sizeof(K) == 8) {
        (void)lt;
        if (ord_in) launch_sort_tile<K, LT, true>(src, dst, n, s, fence, flk, ea, eb);
        else launch_sort_tile<K, LT, false>(src, dst, n, s, fence, flk, ea, eb);
    } else if (lt == SORT_LT_MERGE) {
        launch_sort_u32<SORT_LT_MERGE>(src, dst, n, s, (uint64_t*)fence, flk, ea, eb);
    } else {
        launch_sort_u32<SORT_LT_U32>(src, dst, n, s, (uint64_t*)fence, flk, ea, eb);
    }
}

template <typename K>
hipError_t local_sort_impl(const K* in, K* out, int64_t n, bool ord_in, K* scratch, hipStream_t s,
                           LaunchHook* hook, const StageIO* io, bool ord_out) {
    // merge passes ping-pong between out and scratch
    if (scratch == nullptr || scratch == out || scratch == in) return hipErrorInvalidValue;
    const std::vector<Pass>& ps = plan_for<K>(n);
    const int LT = ps[0].hi + 1;  // this plan's SORT tile
    const int np = (int)ps.size();
    const double bytes = 2.0 * (double)n * sizeof(K);
    const K* src = in;
    int fence_phase = 0;  // multi-way passes: fence buffer holding the next pass's fences
    // the multi-way passes' fence stride: 64-key fences (runsk_fg6.hip) for
    // large sorts, every pass of one sort the same build
    const bool fg6 = mergek_fence_log2(n, (int)sizeof(K)) == 6;
    // the SORT pass writes the first multi-way pass's fences (no gather pass)
    // unless it runs chunk by chunk (host staging)
    const bool sort_fences = np > 1 && ps[1].kind == KIND_RUNSK && ps[1].hi == LT && !(io && io->before_first);
    // a binding hook times the passes by events their kernels carry (host
    // staging's chunked passes keep marker events)
    const bool bind = hook && hook->binds() && !(io && (io->before_first || io->after_last));
    if (bind) hook->bind_reset();
    for (int i = 0; i < np; ++i) {
        // pass i writes `out` iff an even number of passes follow it
        K* dst = ((np - 1 - i) & 1) == 0 ? out : scratch;
        const Pass& p = ps[i];
        HookScope hs(bind ? nullptr : hook, p.kind, bytes, s);
        if (p.kind == KIND_RUNSK) {
            const bool prevk = i > 0 && (ps[i - 1].kind == KIND_RUNSK || (i == 1 && sort_fences));
            const int lk_next = i + 1 < np && ps[i + 1].kind == KIND_RUNSK ? ps[i + 1].R : 0;
            // a binding hook only while binding (host staging records the pass
            // by the HookScope marker above; binding there too would record it
            // twice, from a stale start); a marker hook nests k_mergek's record
            LaunchHook* kh = bind || !(hook && hook->binds()) ? hook : nullptr;
            hipError_t e;
            if constexpr (sizeof(K) == 8) {
                // the last pass stores IEEE double bits itself
                const bool oo = ord_out && i == np - 1;
                e = fg6 ? merge_levelk_fg6(src, dst, n, p.hi, p.R, s, fence_phase, !prevk, lk_next, kh, oo)
                        : merge_levelk(src, dst, n, p.hi, p.R, s, fence_phase, !prevk, lk_next, kh, oo);
                if (oo && e == hipSuccess) ord_out = false;
            } else {
                e = fg6 ? merge_levelk_fg6(src, dst, n, p.hi, p.R, s, fence_phase, !prevk, lk_next, kh)
                        : merge_levelk(src, dst, n, p.hi, p.R, s, fence_phase, !prevk, lk_next, kh);
            }
            if (e != hipSuccess) return e;
            fence_phase ^= 1;
            src = dst;
            continue;
        }
        const bool runs = p.kind == KIND_RUNS;
        const bool cin = io && io->before_first && i == 0;
        const bool cout = io && io->after_last && i == np - 1;
        if (cin || cout) {
            // chunk by chunk (tile-aligned offsets keep the tile grid)
            const int64_t ch = io->chunk;
            if (ch <= 0 || (ch & ((1 << LT) - 1))) return hipErrorInvalidValue;
            for (int64_t k0 = 0; k0 < n; k0 += ch) {
                const int64_t k1 = n - k0 < ch ? n : k0 + ch;
                if (cin && io->before_first(k0, k1, s)) return hipErrorUnknown;
                if (runs) {
                    // a merge level reads across chunks: whole input, output range [k0, k1)
                    if (merge_level<K>(src, dst, n, p.hi, s, k0, k1) != hipSuccess) return hipErrorInvalidValue;
                } else {
                    launch_sort<K>(src + k0, dst + k0, k1 - k0, ord_in, s, LT);
                }
                if (cout && io->after_last(k0, k1, s)) return hipErrorUnknown;
            }
        } else if (runs) {
            const hipError_t e = merge_level<K>(src, dst, n, p.hi, s, 0, 0, bind ? hook : nullptr);
            if (e != hipSuccess) return e;
        } else {
            hipEvent_t ea = nullptr, eb = nullptr;
            if (bind) (void)hook->bind(KIND_TILE_SORT, -1, bytes, &ea, &eb);
            void* f = nullptr;
            if (i == 0 && sort_fences) {
                f = fg6 ? mergek_fence_buffer_fg6(n, (int)sizeof(K), 0, s) : mergek_fence_buffer(n, (int)sizeof(K), 0, s);
                if (!f) return hipErrorOutOfMemory;
            }
            // flk: the first pass's lk and, above bit 8, the fence stride
            launch_sort<K>(src, dst, n, ord_in, s, LT, f, f ? ps[1].R | ((fg6 ? 6 : MERGEK_FENCE_LOG2) << 8) : 0, ea, eb);
        }
        src = dst;
    }
    // a last pass that could not map the keys back (a SORT or 2-way pass:
    // small sorts, u64 levels past 2^29): one more sweep
    if constexpr (sizeof(K) == 8) {
        if (ord_out) {
            const hipError_t e = ord_to_f64((uint64_t*)out, n, s);
            if (e != hipSuccess) return e;
        }
    }
    return hipGetLastError();
}

}  // namespace

// Definition shared by sort_u32.hip / sort_u64.hip (one explicit instantiation each).
template <typename K>
hipError_t local_sort(const K* in, K* out, int64_t n, bool ord_in, K* scratch, hipStream_t s,
                      LaunchHook* hook, const StageIO* io, bool ord_out) {
    if (n <= 0) return hipSuccess;
    if (sizeof(K) == 4 && (ord_in || ord_out)) return hipErrorInvalidValue;
    // chunked output hands every chunk to after_last, which maps it itself
    if (ord_out && io && io->after_last) return hipErrorInvalidValue;
    return local_sort_impl<K>(in, out, n, ord_in, scratch, s, hook, io, ord_out);
}

// One pass of a plan's shape (probes and tests): the SORT tile pass over n keys
// (kind KIND_TILE_SORT; u32: hi = 13 the 2^14 tile, else 2^15), one merge level of runs of 2^hi (KIND_RUNS), or R
// multi-way levels from runs of 2^hi (KIND_RUNSK, R = 1..4; 0: 2).
template <typename K>
hipError_t run_pass(const K* in, K* out, int64_t n, int kind, int hi, int R, int flip, hipStream_t s) {
    (void)flip;
    if (n <= 0) return hipSuccess;
    if (kind == KIND_RUNS) return merge_level<K>(in, out, n, hi, s);
    if (kind == KIND_RUNSK) return merge_levelk(in, out, n, hi, R > 0 ? R : 2, s, 0, true, 0);
    if (kind != KIND_TILE_SORT) return hipErrorInvalidValue;
    launch_sort<K>(in, out, n, false, s, hi + 1 == SORT_LT_MERGE ? SORT_LT_MERGE : KT<K>::LT);
    return hipGetLastError();
}

}  // namespace misort
