// runsk.hip -- K-way merge passes of the local sort (gfx950, u32 and u64 keys):
// ascending runs of W = 2^lw keys, in groups of K = 2^lk (lk = 1..4), ->
// ascending runs of K*W.  One HBM read + one HBM write per key for lk merge
// levels (runs.hip does one level per pass): 2^30 keys past the 2^15-key SORT
// tile take five 8-way passes instead of fifteen 2-way ones (16-way passes are
// built too: MISORT_MULTIWAY=4).
//
// The reference's local sort is std::sort (psort.cc:175); any correct sort of
// payload-free keys writes the same bytes, so the levels past the bitonic SORT
// tile are merges.  A K-way merge needs, for each output chunk, its start in
// all K runs.  Exact fixed-size tiles would need a K-way merge-path co-rank
// per tile (nested searches); instead the chunks are cut at FENCES:
//
//   fence   = the key at every FG-th position of a run, packed with its place
//             as (key << B | run-in-group << (32 - lk) | position / FG), B =
//             the key's bits, so that the fence's unsigned order (u64 for u32
//             keys, u128 for u64 keys) is the total order (key, run,
//             position) -- ties between equal keys go to the lower run, then
//             the lower position;
//   chunks  = the fences of a group merged into that total order (k_fence_lds
//             or lk fence merge levels), every FM-th one starting a chunk;
//   bounds  = for a chunk-start fence f of run r0 at position j0*FG, run r0
//             starts at j0*FG and every other run r at its count of keys
//             before f, found by a binary search confined to the FG positions
//             between two of run r's own fences (k_bounds, one thread per
//             chunk start and run);
//   rows    = each chunk's loads as rows of RW keys inside one segment: a
//             byte offset and an LDS word per row (k_chunk_desc), so a load is
//             a scalar base plus the lane;
//   merge   = one workgroup per chunk (k_mergek): the K segments are streamed
//             into LDS, merged pairwise in lk levels in LDS, and stored through
//             LDS as 16-byte non-temporal stores; the keys at every FG-th
//             output position are written as the next pass's fences.
//
// Between two consecutive chunk starts lie FM fences; run r contributes at
// most (its fences there + 1) * FG keys, so a chunk holds at most
// (FM + K) * FG = CAP keys and FM * FG on average.  The first multi-way pass
// after the SORT tile gathers its fences from the runs (k_fence_gather);
// later passes read the fences the previous pass wrote.
#include "kernels.h"
#include "lds_merge.h"

#include <map>
#include <mutex>

namespace misort {
namespace {

// The fence stride: MERGEK_FENCE_LOG2 (kernels.h), or MISORT_RUNSK_FGL in the
// second build of this file (runsk_fg6.hip: 64-key fences, its entry points
// suffixed by MISORT_RUNSK_FN).
#ifndef MISORT_RUNSK_FGL
#define MISORT_RUNSK_FGL MERGEK_FENCE_LOG2
#endif
#ifndef MISORT_RUNSK_FN
#define MISORT_RUNSK_FN(x) x
#endif
constexpr int FG_LOG2 = MISORT_RUNSK_FGL;
constexpr int64_t FG = (int64_t)1 << FG_LOG2;  // fence stride (keys)
typedef unsigned __int128 u128;

// The first fence merge levels of a pass as LDS merge levels (k_fence_merge)
// when the pass has at least FENCE_MERGE_MIN_BLOCKS sub-groups; else ranks by
// binary searches (k_fence_lds), which can split a sub-group over several
// blocks.  Measured (profiles/r03/ab3): 2^30 u32 66.5 -> 67.0 Gkeys/s, 2^26
// 61.5 -> 62.1; at 2^24 (64 and 16 sub-groups) the merge was slower.
constexpr int64_t FENCE_MERGE_MIN_BLOCKS = 128;
// bytes of the aligned window k_bounds reads around its interpolated guess
// (64: u32 passes -1..-10 us, u64 +2 us, profiles/r05/plan/bl64_ab.txt)
constexpr int BOUNDS_LINE = 128;
// k_bounds loads the scanned fence counts beside the chunk-start fence (one
// dependent round less) and divides chunk indices in 32 bits: 2^30 pass -2 to
// -8 us, 2^28 and u64 equal (profiles/r05/plan/bearly_ab.txt).
// u32 k_mergek loads its rows straight into LDS (global_load_lds_dword: no
// VGPR staging, no ds_write per key): 2^30 k_mergek 2.034 -> 1.997 ms per pass
// (profiles/r03/ab1).  The in-LDS levels read two keys per LDS read for u32
// (merge_chain_blk; 1999 -> 1969 us, profiles/r04/ab_chain) and one for u64
// (merge_chain: the two-key chain measured equal in the tile, -6 % in the
// passes, profiles/r05/mergek/u64_chain_ab.txt); zero words below the A
// sequences for the two-key chain (profiles/r05/zwpt).

// Per key type: the fence type (key bits above 32 bits of run and position),
// the chunk workgroup (NT lanes x IT keys: CAP keys a chunk at most), the
// workgroups per CU the LDS tile allows, and the largest fence sub-group
// merged in LDS (64 KiB).
template <typename KEY>
struct KTr;
// u32, 2..8-way passes: 512 lanes x 18 outputs, 8960-key chunks (the largest
// the 18-output level layout fits: CAP + 4 (G + QA) <= 9216; 8192 before: 2^24
// +1.5 %, 2^28 +0.8 %, profiles/r04/chunk32), four workgroups per CU; 22
// outputs per lane at three per CU measured slower (profiles/r06/plan/fg6_ab.txt).
// 16-way passes: larger chunks.  A chunk holds FM * FG = CAP - K * FG keys on
// average, so at K = 16 a quarter of an 8192-key chunk's lanes idle.  Round
// 4: 22 outputs per lane (CAP 10752, three workgroups per CU) measured 2^30
// 68.9 -> 69.8 Gkeys/s; 20 or 24 per lane were slower -- an EVEN half (IT / 2
// = 10 or 12) puts the lanes' chain pointers, IT / 2 apart, on a few banks.
// Round 6: 26 outputs per lane (IT / 2 = 13, odd) and the LDS sized by the
// larger of the segments and the level outputs (not their sum): CAP 12864,
// the largest the 26-output level layout holds (CAP + 8 (G + QA) <= 512 * 26),
// still three workgroups per CU (53.4 KB); 2^30 k_mergek 2154 -> 2049 us,
// 81.6 -> 84.4 Gkeys/s, 2^28 82.2 -> 84.6 (profiles/r06/mergek/it26_ab.txt);
// 768 or 640 lanes at two workgroups per CU were slower (nt_ab.txt).  Load rows
// of 128 keys (the descriptor holds 8 bytes per row; 64 -> 128 halved it:
// 2^30 pass 2569 -> 2547 us, profiles/r05/plan/rw_ab.txt).
template <>
struct KTr<uint32_t> {
    typedef uint64_t F;
    static constexpr int NT = 512, IT = 18, CAP = 8960, WG_PER_CU = 4;
    static constexpr int IT16 = 26, CAP16 = 12864, WG16 = 3;
    // the chunk shape of a pass of lk levels
    static constexpr bool big(int lk) { return lk == 4; }
    static constexpr int it(int lk) { return big(lk) ? IT16 : IT; }
    // (k_fence_counts keeps 8-bit per-chunk counts: at most 255 + K fences of FG
    // keys a chunk, a bound only the 64-key build can reach)
    static constexpr int cap16() { return CAP16 < (255 + 16) * FG ? CAP16 : (255 + 16) * (int)FG; }
    static constexpr int cap(int lk) { return big(lk) ? cap16() : CAP; }
    static constexpr int wg(int lk) { return big(lk) ? WG16 : WG_PER_CU; }
    static constexpr int FL_LDS = 13;                       // 8192 fences = 64 KiB
    static constexpr int LW_MIN = SORT_LT_MERGE, LWK_MAX = 30;  // runs >= the smaller SORT tile; 32-bit row offsets
};
// The u64 chunk shape: 18 outputs per lane and the largest capacity whose
// level layout fits 512 x 18 slots (CAP + 8 (G + QA) <= 9216): 8832 keys
// (69 fences of 128) instead of 8192 measured 2^29 u64 35.4 -> 36.5-36.7
// Gkeys/s, k_mergek 2.46 -> 2.33 ms per pass, 2^26 +2.2 %; 9216 keys at 20 per
// lane was slower (profiles/r04/chunk64).  The 64-key build (runsk_fg6.hip)
// takes 8896 (139 fences of 64): k_mergek -5 us per 2^29 pass
// (profiles/r05/mergek/cap_ab.txt).
template <>
struct KTr<uint64_t> {
    typedef u128 F;
    static constexpr int NT = 512, IT = 18, WG_PER_CU = 2;
    static constexpr int CAP = FG_LOG2 == 6 ? 8896 : 8832;  // ~69 KiB of keys: two tiles per CU, 4 waves per SIMD
    static constexpr int FL_LDS = 12;    // 4096 fences = 64 KiB
    static constexpr int LW_MIN = 13, LWK_MAX = 29;  // runs >= the u64 SORT tile; 32-bit row offsets
    static constexpr int it(int) { return IT; }
    static constexpr int cap(int) { return CAP; }
    static constexpr int wg(int) { return WG_PER_CU; }
};

// Every sequence an in-LDS merge reads is followed by G words of MAX
// (sentinels), so a merge chain needs no end checks: it reads at most IT words
// past an exhausted sequence.  Each level places its pairs' outputs at lane
// boundaries past the previous pair's sentinels (no lane straddles two pairs).
constexpr int PAD = 4;  // keys below the tile: a co-rank probe may read index -1

constexpr int SCAN_NT_MAX = 256;  // chunks per fence-count block (SCAN_NT below)

template <typename KEY, int LK>
struct Shape {
    typedef KTr<KEY> T;
    // the merge chain of the in-LDS levels: two keys per read (u32), one (u64)
    static constexpr int CH = sizeof(KEY) == 4 ? 1 : 0;
    static constexpr int NT = T::NT, IT = T::it(LK), CAP = T::cap(LK);
    static constexpr int MAXR = CAP / 2;  // co-rank range bound: min(LA, LB) <= CAP / 2
    // zero words below the A sequences (co_rank without its i == lo test; the
    // two-key chain): the last of the G words after a sequence holds the next
    // one's, so G exceeds the keys a chain reads past a sequence (IT for the
    // two-key chain, IT + 1 for the one-key chain)
    static constexpr bool ZW = CH == 1;
    static constexpr int G = IT + 1;
    static constexpr int QA = IT;  // level outputs start at lane boundaries
    static_assert(IT % 2 == 0, "outputs stored as aligned pairs");
    // LDS slot of segment q (o = its first chunk position)
    __device__ __host__ static int seg(int o, int q) { return o + q * G; }
    static constexpr int K = 1 << LK, LKS = LK;
    static constexpr int FM = CAP / (int)FG - K;   // fences per chunk, worst case (merge_pass cuts at more)
    static constexpr int RW = LK == 4 ? 128 : (LK == 3 || NT % 256) ? 128 : 256;  // load row: RW keys of one segment
    static constexpr int NR = NT / RW;             // row parts: waves [p*RW/64, (p+1)*RW/64) load part p
    // load slots per lane: enough rows for CAP keys in K segments
    static constexpr int LS_ROWS = ((CAP + RW - 1) / RW + K + NR - 1) / NR;
    static constexpr int LS = ((IT + 1) & ~1) <= LS_ROWS ? LS_ROWS : ((IT + 1) & ~1);
    static constexpr int NROWS = LS * NR;           // lane slot j of part p holds row j * NR + p
    // the tile holds the chunk's segments with their sentinels (CAP + K G) and
    // every level's outputs (<= NT IT slots by the level layout, + G sentinels)
    static constexpr int NB_EXT = CAP + K * G > NT * IT + G ? CAP + K * G : NT * IT + G;
    static constexpr int LDS_KEYS = PAD + NB_EXT + 16;
    static_assert(FM > 0 && FM < 256 && SCAN_NT_MAX * FM < 65536,
                  "fence stride vs chunk (k_fence_counts keeps 8-bit counts and 16-bit block prefixes)");
    static_assert(CAP <= (NROWS - K) * RW, "segment rows: ceil(l_r / RW) summed over K segments");
    static_assert(CAP + (K / 2) * (G + QA) <= NT * IT, "level layout: pairs at lane boundaries");
    static_assert(LDS_KEYS < 65536, "LDS key index of a row fits 16 bits");
};

// fence <-> (key, tag): tag = run << (32 - lk) | position / FG, the low 32 bits
template <typename KEY>
__device__ __host__ __forceinline__ typename KTr<KEY>::F fpack(KEY key, int64_t gp, int lw, int lk) {
    typedef typename KTr<KEY>::F F;
    const uint32_t r = (uint32_t)(gp >> lw) & ((1u << lk) - 1);
    const uint32_t j = (uint32_t)((gp & (((int64_t)1 << lw) - 1)) >> FG_LOG2);
    return ((F)key << (8 * sizeof(KEY))) | (F)((r << (32 - lk)) | j);
}
template <typename F>
__device__ __forceinline__ auto fkey(F f) {
    if constexpr (sizeof(F) == 8) return (uint32_t)(f >> 32);
    else return (uint64_t)(f >> 64);
}
template <typename F>
__device__ __forceinline__ uint32_t ftag(F f) {
    return (uint32_t)f;
}

// Group geometry of the pass: groups of K runs of W keys; run r of group g
// starts at g*KW + r*W and holds clamp(n - start, 0, W) keys.
struct Geo {
    int64_t n;
    int lw, lk, fm;
    int64_t nfull;  // full groups
    int64_t kf;     // chunks per full group
    __device__ __host__ int K() const { return 1 << lk; }
    __device__ __host__ int64_t W() const { return (int64_t)1 << lw; }
    __device__ __host__ int64_t base(int64_t g) const { return g << (lw + lk); }
    __device__ __host__ int64_t run_len(int64_t g, int r) const {
        const int64_t rest = n - (base(g) + r * W());
        return rest <= 0 ? 0 : (rest < W() ? rest : W());
    }
    __device__ __host__ int64_t nfences(int64_t g) const {
        const int64_t glen = (n - base(g)) < K() * W() ? n - base(g) : K() * W();
        return (glen + FG - 1) >> FG_LOG2;
    }
    // a group's fences and chunks are < 2^31: a 32-bit division
    __device__ __host__ int64_t nchunks(int64_t g) const {
        return g < nfull ? kf : (int64_t)((uint32_t)(nfences(g) + fm - 1) / (uint32_t)fm);
    }
    // bounds slot of chunk t of group g (each group has nchunks + 1 slots)
    __device__ __host__ int64_t slot(int64_t g, int64_t t) const {
        return g < nfull ? g * (kf + 1) + t : nfull * (kf + 1) + t;
    }
};

// fm = 0: the worst-case bound, (fm + K) * FG <= CAP
template <typename KEY>
Geo make_geo(int64_t n, int lw, int lk, int fm = 0) {
    Geo geo{n, lw, lk, fm > 0 ? fm : KTr<KEY>::cap(lk) / (int)FG - (1 << lk), 0, 0};
    geo.nfull = n >> (lw + lk);
    geo.kf = ((((int64_t)1 << (lw + lk)) >> FG_LOG2) + geo.fm - 1) / geo.fm;
    return geo;
}

// The capacity split's fences per chunk above the worst-case bound (merge_pass).
// A chunk's size is FM * FG plus 2K window offsets of up to FG each, which
// nearly cancel on spread keys (sigma ~ FG sqrt(2K / 12), 1.6 FG at K = 16):
// 9 fences more at K = 16 (4.6 sigma of headroom with 128-key fences) and 3 at
// K = 8 (4.3 sigma) keep splits to about one per few 2^30 passes on spread
// keys -- a split's serial latency (k_split_desc) and its halves' merge sit on
// the pass's critical path, so rarer splits beat fuller chunks here: 12 fences
// more (2.8 sigma, ~0.3 % of chunks) measured slower than none at 2^28
// (profiles/r06/mergek/split_ab.txt).  (env MISORT_MK_FM_ADD: one value
// for every unfused pass, 0 = off), clamped so a half chunk still fits --
// ceil(fm / 2) + K fences of FG keys <= CAP -- and fm <= 255 (k_fence_counts'
// 8-bit counts).
template <typename KEY, int LK>
int split_fm_add() {
    static const int env = getenv("MISORT_MK_FM_ADD") ? atoi(getenv("MISORT_MK_FM_ADD")) : -1;
    // u64: equal kernel time, +25 us of split overhead per 2^29 pass (split_ab.txt): off
    const int want = env >= 0 ? env : sizeof(KEY) == 8 ? 0 : LK == 4 ? 9 : LK == 3 ? 3 : 0;
    const int K = 1 << LK, cap = KTr<KEY>::cap(LK), fm0 = cap / (int)FG - K;
    int fm = fm0 + (want > 0 ? want : 0);
    while (fm > fm0 && ((fm + 1) / 2 + K) * (int)FG > cap) --fm;
    if (fm > 255) fm = 255;
    return fm > fm0 ? fm - fm0 : 0;
}

// A group whose fence count lies just above a multiple of fm ends in a nearly
// empty chunk (2^30 u32 pass 1: 2048 fences a group, fm 93 -> 23 chunks, the
// last of 2 fences): up to FM_BALANCE fences more per chunk when that saves
// the group a chunk, within the split's bound (halves fit, 8-bit counts), and
// only where that chunk is >= 1/BAL_NC_MAX of the group's: 2^30 +0.35 %; on
// every pass (+1 fence a chunk, more splits for 1 chunk in 250) 2^27 -1 %
// (profiles/r06/mergek/balance_ab.txt).
constexpr int FM_BALANCE = 3, BAL_NC_MAX = 32;
template <typename KEY, int LK>
int balance_fm(int fm, int64_t gf) {
    const int K = 1 << LK, cap = KTr<KEY>::cap(LK);
    const int64_t nc = gf / fm;
    if (nc < 1 || nc > BAL_NC_MAX || nc * fm == gf) return fm;
    const int fm2 = (int)((gf + nc - 1) / nc);
    return fm2 <= fm + FM_BALANCE && fm2 <= 255 && ((fm2 + 1) / 2 + K) * (int)FG <= cap ? fm2 : fm;
}

// F[i] = fence of position i*FG (the first multi-way pass after the SORT tile).
template <typename KEY>
__global__ void k_fence_gather(const KEY* __restrict__ src, int64_t n, int lw, int lk,
                               typename KTr<KEY>::F* __restrict__ F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    if (i >= nf) return;
    const int64_t gp = i << FG_LOG2;
    F[i] = fpack<KEY>(src[gp], gp, lw, lk);
}

// Runs of 2^wf fences merged 2^a at a time (<= 64 KiB of fences) into total
// order in LDS: blocks b*split .. b*split + split - 1 take fences
// [b << (wf + a), ...), each ranking a 1/split slice of them (small sorts: more
// blocks than sub-groups); each fence's rank = its index in its run's list +
// its lower bound in the sub-group's other runs.
template <typename FT>
__global__ __launch_bounds__(1024) void k_fence_lds(const FT* __restrict__ F, FT* __restrict__ M, int64_t nf,
                                                    int wf_log2, int a, int split) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sraw[];
    FT* sf = reinterpret_cast<FT*>(sraw);
    const int64_t f0 = (int64_t)(blockIdx.x / split) << (wf_log2 + a);
    const int nfg = (int)((nf - f0) < ((int64_t)1 << (wf_log2 + a)) ? nf - f0 : ((int64_t)1 << (wf_log2 + a)));
    const int wf = 1 << wf_log2;
    const int K = 1 << a;
    for (int e = threadIdx.x; e < nfg; e += blockDim.x) sf[e] = F[f0 + e];
    __syncthreads();
    const int sl = (nfg + split - 1) / split, e0 = (int)(blockIdx.x % split) * sl;
    const int e1 = e0 + sl < nfg ? e0 + sl : nfg;
    for (int e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const FT v = sf[e];
        const int r = e / wf;
        int rank = e - r * wf;
        for (int q = 0; q < K; ++q) {
            if (q == r) continue;
            int lo = q * wf, hi = (q + 1) * wf < nfg ? (q + 1) * wf : nfg;
            if (lo >= hi) continue;
            const int l0 = lo;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (sf[mid] < v) lo = mid + 1;
                else hi = mid;
            }
            rank += lo - l0;
        }
        if (rank < nfg) M[f0 + rank] = v;  // always true for well-formed fences
    }
}

// The same result by merge levels in LDS: one block per sub-group of S =
// 2^(wf_log2 + a) fences (the tail padded with all-ones fences, which sort
// last and are never stored), a levels of pairwise merges, each lane taking
// FIT consecutive outputs of its pair: a co-rank search, then a chain with
// end checks.  k_fence_lds ranks every fence by K - 1 binary searches (56
// dependent LDS reads per fence at K = 8, runs of 256); a merge level costs a
// lane about 2 log2(S) reads for FIT outputs.
constexpr int FIT = 8;  // 16: 2^30 pass +11..23 us (profiles/r05/plan/fit_ab.txt)
template <typename FT>
__global__ __launch_bounds__(1024) void k_fence_merge(const FT* __restrict__ F, FT* __restrict__ M, int64_t nf,
                                                      int wf_log2, int a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sraw[];
    FT* sf = reinterpret_cast<FT*>(sraw);
    const int S = 1 << (wf_log2 + a);
    const int64_t f0 = (int64_t)blockIdx.x << (wf_log2 + a);
    const int nfg = (int)((nf - f0) < (int64_t)S ? nf - f0 : (int64_t)S);
    const int tid = threadIdx.x, NT = blockDim.x;  // NT * FIT == S
    for (int e = tid; e < S; e += NT) sf[e] = e < nfg ? F[f0 + e] : ~(FT)0;
    __syncthreads();
    const int d0 = tid * FIT;
    FT r[FIT];
    for (int l = 1; l <= a; ++l) {
        const int hl = wf_log2 + l - 1;  // log2 of each side of a pair
        const int base = (d0 >> (hl + 1)) << (hl + 1), W = 1 << hl, d = d0 - base;
        const FT* A = sf + base;
        const FT* B = A + W;
        int lo = d > W ? d - W : 0, hi = d < W ? d : W;
        while (lo < hi) {  // first i with A[i] > B[d - 1 - i] (A first on ties; fences are distinct)
            const int mid = (lo + hi) >> 1;
            if (A[mid] < B[d - 1 - mid]) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = d - lo;
        FT av = A[ia < W ? ia : W - 1], bv = B[ib < W ? ib : W - 1];
#pragma unroll
        for (int k = 0; k < FIT; ++k) {
            const bool ta = ia < W && (ib >= W || av < bv);
            r[k] = ta ? av : bv;
            ia += ta;
            ib += !ta;
            const FT x = ta ? A[ia < W ? ia : W - 1] : B[ib < W ? ib : W - 1];
            av = ta ? x : av;
            bv = ta ? bv : x;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < FIT; ++k) sf[d0 + k] = r[k];
        __syncthreads();
    }
    for (int e = tid; e < nfg; e += NT) M[f0 + e] = sf[e];  // coalesced
}

// Chunk index -> (group, chunk within the group), and the group's first chunk.
// Chunk and bounds-slot indices are < 2^31 (merge_pass checks), so the
// divisions are 32-bit.
__device__ __forceinline__ void chunk_place(const Geo& geo, int64_t c, int64_t& g, int64_t& t) {
    if (c < geo.nfull * geo.kf) {
        g = (uint32_t)c / (uint32_t)geo.kf;
        t = c - g * geo.kf;
    } else {
        g = geo.nfull;
        t = c - geo.nfull * geo.kf;
    }
}

constexpr int SCAN_NT = SCAN_NT_MAX;  // chunks per block of the fence-count scan

// Inclusive scan of a u64 over the block (all its lanes; sw holds one entry
// per wave), for packed fields.
__device__ __forceinline__ uint64_t block_scan_u64(uint64_t v, uint64_t* sw) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t u = __shfl_up(v, o, 64);
        v += lane >= o ? u : 0ull;
    }
    if (lane == 63) sw[w] = v;
    __syncthreads();
    for (int q = 0; q < w; ++q) v += sw[q];
    __syncthreads();
    return v;
}

// Fence counts per chunk and run (the chunk's FM fences of the merged order,
// by their run bits), exclusive-scanned over chunks: blocks of SCAN_NT
// chunks, P = the scan within the block, bsum = the block totals.  A run's
// fences before a chunk-start fence = P(c) - P(group's first chunk), with the
// block totals scanned in (k_scan_totals) -- this replaces a binary search of
// each run's fence list.  The block's chunks own one contiguous range of M;
// its lanes read that range coalesced and add each fence to its chunk's
// counters in LDS (8-bit fields, runs 0..7 and 8..15 in two u64 words;
// one lane per chunk reading its own FM fences ran 49 us at 2^30).
// Two ways to count, chosen by size: SLICES (few blocks, small sorts): each
// of COUNT_NT lanes counts a contiguous slice of the block's fences in
// registers and adds to a chunk's LDS counters when its slice crosses into
// the next chunk -- 2^24: 32 -> 13 us per pass, where 10 blocks had walked 56
// fences per lane; else (many blocks) the block's SCAN_NT lanes read the fence
// range coalesced and add each fence to its chunk's counters with an LDS
// atomic -- 2^30: 41.5 us, the slices' strided loads 107 us.
// One u32 LDS counter per (chunk, run): the coalesced path's atomics collide
// only between lanes of one chunk and run (the runs' 8-bit fields packed in two
// u64 words per chunk made a wave's lanes, mostly in one chunk, all add to
// one word; profiles/r03/ab_fc).  The coalesced form keeps FC_BATCH fences per
// lane in flight (their loads issued together; 2^30 pass -7 us, u64 2^29 -10
// us, profiles/r05/plan/fcb_ab.txt) and counts with FC_NT lanes (it scans with
// the first SCAN_NT): 512 instead of 256 measured 2^30 pass -6 us, u64 2^29
// -5 us (profiles/r05/plan/fcnt_ab.txt).  Reading the whole fence window in
// k_bounds instead of its interpolated line measured slower at every size
// (2^30 pass +36 us; profiles/r05/plan/win_ab.txt).
constexpr int FC_BATCH = 8;
constexpr int COUNT_NT = 1024, FC_NT = 512;
static_assert(FC_NT >= SCAN_NT && FC_NT <= COUNT_NT && FC_NT % 64 == 0, "fence-count block");
template <typename FT, bool SLICES>
__global__ __launch_bounds__(COUNT_NT) void k_fence_counts(const FT* __restrict__ M, Geo geo, int64_t nchunks,
                                                           int cpb, int* __restrict__ P, int* __restrict__ bsum,
                                                           int* __restrict__ ovf) {
    __shared__ uint64_t sws[COUNT_NT / 64];
    __shared__ uint32_t sc[SCAN_NT][16];
    const int tid = threadIdx.x;
    if (ovf && blockIdx.x == 0 && tid == 0) *ovf = 0;  // the capacity split's list, empty (k_chunk_desc fills it)
    const int64_t c0 = (int64_t)blockIdx.x * cpb, c = c0 + tid;  // cpb <= SCAN_NT chunks per block
    const int64_t c1 = c0 + cpb < nchunks ? c0 + cpb : nchunks;
    const int K = geo.K();
    const int gl = geo.lw + geo.lk;
    for (int i = tid; i < SCAN_NT * 16; i += (int)blockDim.x) (&sc[0][0])[i] = 0u;  // SCAN_NT or COUNT_NT lanes
    __syncthreads();
    int64_t g, t;
    chunk_place(geo, c0, g, t);
    const int64_t f0 = (geo.base(g) >> FG_LOG2) + t * geo.fm;
    chunk_place(geo, c1 - 1, g, t);
    const int64_t gf = geo.base(g) >> FG_LOG2, nfg = geo.nfences(g);
    const int64_t f1 = t * geo.fm + geo.fm < nfg ? gf + t * geo.fm + geo.fm : gf + nfg;
    // block-local chunk of fence e (the tail group starts at nfull); a fence's
    // index within its group (< 2^(LWK_MAX - FG_LOG2)) and FM fit 32 bits, and a
    // 32-bit division is a few VALU ops where a 64-bit one is ~100 (it bounded
    // the kernel: one division per fence)
    const uint32_t fm = (uint32_t)geo.fm;
    auto chunk_of = [&](int64_t e) {
        int64_t ge = (e << FG_LOG2) >> gl;
        ge = ge < geo.nfull ? ge : geo.nfull;
        return ge * geo.kf + (int64_t)((uint32_t)(e - (geo.base(ge) >> FG_LOG2)) / fm) - c0;
    };
    // a lane's per-run counts of one chunk (8-bit fields of lo8 / hi8) into its LDS counters
    auto flush = [&](int64_t ch, uint64_t lo8, uint64_t hi8) {
        for (int r = 0; r < K; ++r) {
            const uint32_t v = (uint32_t)(((r < 8 ? lo8 : hi8) >> (8 * (r & 7))) & 0xFF);
            if (v) atomicAdd(&sc[ch][r], v);
        }
    };
    if constexpr (SLICES) {
        const int64_t per = (f1 - f0 + COUNT_NT - 1) / COUNT_NT;
        const int64_t e0 = f0 + tid * per, e1 = e0 + per < f1 ? e0 + per : f1;
        int64_t cur = -1;  // the chunk being counted
        uint64_t lo8 = 0, hi8 = 0;
        for (int64_t e = e0; e < e1; ++e) {
            const int64_t ce = chunk_of(e);
            if (ce != cur) {
                if (cur >= 0) flush(cur, lo8, hi8);
                cur = ce;
                lo8 = hi8 = 0;
            }
            const int r = (int)((ftag(M[e]) >> (32 - geo.lk)) & (K - 1));
            const uint64_t one = 1ull << (8 * (r & 7));
            if (r < 8) lo8 += one;
            else hi8 += one;
        }
        if (cur >= 0) flush(cur, lo8, hi8);
    } else {
        // FCB fences per lane in flight: their loads first, then their counts
        constexpr int FCB = FC_BATCH;
        for (int64_t e0 = f0 + tid; e0 < f1; e0 += FCB * FC_NT) {
            uint32_t tg[FCB];
#pragma unroll
            for (int u = 0; u < FCB; ++u) {
                const int64_t e = e0 + (int64_t)u * FC_NT;
                tg[u] = e < f1 ? ftag(M[e]) : 0u;
            }
#pragma unroll
            for (int u = 0; u < FCB; ++u) {
                const int64_t e = e0 + (int64_t)u * FC_NT;
                if (e >= f1) break;
                const int r = (int)((tg[u] >> (32 - geo.lk)) & (K - 1));
                atomicAdd(&sc[chunk_of(e)][r], 1u);
            }
        }
    }
    __syncthreads();
    // scan 4 runs at a time as 16-bit fields of one u64 (block prefixes <=
    // SCAN_NT * FM < 2^16): K/4 block scans instead of K
    auto count_of = [&](int q) { return tid < cpb ? (uint64_t)sc[tid][q] : 0ull; };
    for (int q0 = 0; q0 < K; q0 += 4) {
        uint64_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = q0 + j;
            v |= (q < K ? count_of(q) : 0ull) << (16 * j);
        }
        const uint64_t inc = block_scan_u64(v, sws);
        const int nq = K - q0 < 4 ? K - q0 : 4;
        for (int j = 0; j < nq; ++j) {
            const int q = q0 + j;
            const int vi = (int)((inc >> (16 * j)) & 0xFFFF), vq = (int)((v >> (16 * j)) & 0xFFFF);
            if (tid < cpb && c < nchunks) P[c * K + q] = vi - vq;
            if (threadIdx.x == SCAN_NT - 1) bsum[(int64_t)blockIdx.x * K + q] = vi;
        }
    }
}

// Exclusive scan of the block totals: one wave per two runs (their totals as
// the 32-bit fields of one u64; totals < 2^31), in rounds of 64 x TOT_B
// blocks: a lane loads TOT_B consecutive totals at once, scans them in
// registers, and a wave scan of the lane sums places them (one round of load
// latency per 64 * TOT_B blocks; a 256-lane block scan per 256 blocks and run
// pair took 4 dependent rounds per pair at 2^30).
constexpr int TOT_B = 16;
__global__ __launch_bounds__(512) void k_scan_totals(int* __restrict__ bsum, int64_t nb, int K) {
    const int lane = threadIdx.x & 63, q = 2 * (int)(threadIdx.x >> 6);
    if (q >= K) return;
    const bool two = q + 1 < K;
    uint64_t carry = 0;
    for (int64_t r0 = 0; r0 < nb; r0 += 64 * TOT_B) {
        const int64_t b0 = r0 + (int64_t)lane * TOT_B;
        uint64_t v[TOT_B], sum = 0;
#pragma unroll
        for (int j = 0; j < TOT_B; ++j) {
            const int64_t b = b0 + j;
            v[j] = b < nb ? (uint64_t)(uint32_t)bsum[b * K + q] |
                                (two ? (uint64_t)(uint32_t)bsum[b * K + q + 1] << 32 : 0ull)
                          : 0ull;
            sum += v[j];
        }
        uint64_t inc = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t u = __shfl_up(inc, o, 64);
            inc += lane >= o ? u : 0ull;
        }
        uint64_t ex = carry + inc - sum;
#pragma unroll
        for (int j = 0; j < TOT_B; ++j) {
            const int64_t b = b0 + j;
            if (b < nb) {
                bsum[b * K + q] = (int)(uint32_t)ex;
                if (two) bsum[b * K + q + 1] = (int)(uint32_t)(ex >> 32);
            }
            ex += v[j];
        }
        carry += __shfl(inc, 63, 64);
    }
}

// Small sorts (fused planning, runs of <= 2^MISORT_FENCE_RANK_MAX fences): the
// group's fences into total order AND the per-chunk fence counts in ONE launch,
// in place of the fence merge levels (k_fence_lds / k_fence_merge and global
// merge levels) and k_fence_counts -- at these sizes each of those launches is
// latency-bound.  A thread per fence: its rank in the group = its index in its
// run + its lower bound in each other run (K - 1 power-of-two searches over
// the run's fence list, stepping together so their loads overlap; lanes of a
// wave hold neighbouring fences of one run, so they probe the same or
// adjacent lines).  Counts: chunk t starts at merged fence t * fm, and run q's
// fences before it are the i with rank(q, i) < t * fm, so fence i of run q
// (rank p, its predecessor's rank p') writes i for every t with p' < t * fm <=
// p, and the run's last fence writes i + 1 for the chunks after it -- every
// (chunk, run) entry once, as absolute counts (the block totals bsum are
// zeroed: no scan).  Block b owns fences [b (RANK_NT - 1), (b + 1) (RANK_NT -
// 1)); its thread 0 ranks the fence before them (the predecessor of thread 1's).
constexpr int RANK_NT = 256;
template <typename FT, int LK>
__global__ __launch_bounds__(RANK_NT) void k_fence_rank(const FT* __restrict__ F, FT* __restrict__ M, Geo geo,
                                                        int64_t nf, int wf_log2, int* __restrict__ P,
                                                        int* __restrict__ bsum, int64_t nbsum) {
    constexpr int K = 1 << LK;
    __shared__ int sp[RANK_NT];
    const int tid = threadIdx.x;
    for (int64_t j = (int64_t)blockIdx.x * RANK_NT + tid; j < nbsum; j += (int64_t)gridDim.x * RANK_NT) bsum[j] = 0;
    const int64_t e = (int64_t)blockIdx.x * (RANK_NT - 1) - 1 + tid;
    const bool valid = e >= 0 && e < nf;
    const int gl = wf_log2 + LK, wf = 1 << wf_log2;
    int64_t g = 0, gbase = 0;
    int nfg = 0, q = 0, i = 0, p = -1;
    if (valid) {
        g = e >> gl;
        gbase = g << gl;
        nfg = nf - gbase < ((int64_t)1 << gl) ? (int)(nf - gbase) : 1 << gl;
        const int gi = (int)(e - gbase);
        q = gi >> wf_log2;
        i = gi & (wf - 1);
        const FT v = F[e];
        int pos[K], len[K];
        const FT* fr[K];  // run r's fences (a run with none, or q itself: fence e, never taken)
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int l = nfg - r * wf;
            len[r] = r == q ? 0 : (l <= 0 ? 0 : (l < wf ? l : wf));
            pos[r] = 0;
            fr[r] = len[r] > 0 ? F + gbase + ((int64_t)r << wf_log2) : F + e;
        }
        // unconditional loads at clamped probes (a guarded load per run made
        // each wait for the last), then the steps taken.  The searches are
        // bound by load issue: a radix-4 search (3x the loads in half the
        // rounds) ran 1.6x slower, and loads of the key halves only over the
        // K - 1 other runs 1.25x slower (profiles/r06/plan/rank_ab.txt)
        for (int st = wf; st > 0; st >>= 1) {
            FT x[K];
#pragma unroll
            for (int r = 0; r < K; ++r) {
                const int j = pos[r] + st < len[r] ? pos[r] + st : len[r];
                x[r] = fr[r][j > 0 ? j - 1 : 0];
            }
#pragma unroll
            for (int r = 0; r < K; ++r) pos[r] += pos[r] + st <= len[r] && x[r] < v ? st : 0;
        }
        p = i;
#pragma unroll
        for (int r = 0; r < K; ++r) p += pos[r];
        M[gbase + p] = v;
    }
    sp[tid] = p;
    __syncthreads();
    if (!valid || tid == 0) return;
    const uint32_t fm = (uint32_t)geo.fm;
    const int64_t c0 = g * geo.kf;  // the group's first chunk (the tail group's too)
    const int nch = (int)geo.nchunks(g);
    const int lq = nfg - q * wf < wf ? nfg - q * wf : wf;  // run q's fences in the group
    const int t0 = i == 0 ? 0 : (int)((uint32_t)sp[tid - 1] / fm) + 1;  // thread tid - 1 holds fence e - 1
    const int t1 = (int)((uint32_t)p / fm);
    for (int t = t0; t <= t1; ++t) P[(c0 + t) * K + q] = i;
    if (i == lq - 1)
        for (int t = t1 + 1; t < nch; ++t) P[(c0 + t) * K + q] = i + 1;
    // runs with no fences in this group (a tail group): zero counts
    const int gi = (int)(e - gbase), nruns = (nfg + wf - 1) >> wf_log2;
    if (gi < nch)
        for (int r = nruns; r < K; ++r) P[(c0 + gi) * K + r] = 0;
}

// Interpolated guess of where v falls between positions a and b whose keys
// are ka < kb.
template <typename KEY>
__device__ __forceinline__ int64_t interp(KEY v, KEY ka, KEY kb, int64_t a, int64_t b) {
    if constexpr (sizeof(KEY) == 4) {
        return a + (int64_t)(((uint64_t)(v - ka) * (uint64_t)(b - a)) / (uint64_t)(kb - ka));
    } else {
        return a + (int64_t)((double)(v - ka) / (double)(kb - ka) * (double)(b - a));
    }
}

// Run r's position of the first key after fence f in the total order (key,
// run, position) -- f's own position for r = f's run -- given lo = run r's
// fences before f: the keys before f lie among the FG positions after the
// last of them (-1: more fences than the run has, malformed input fences;
// k_chunk_desc then rejects the chunk, no read outside the run).
template <typename KEY>
__device__ int64_t window_bound(const KEY* __restrict__ src, const typename KTr<KEY>::F* __restrict__ F,
                                const Geo& geo, int64_t g, int r, typename KTr<KEY>::F f, int64_t lo, bool line) {
    typedef typename KTr<KEY>::F FT;
    const int64_t base = geo.base(g), W = geo.W(), len = geo.run_len(g, r);
    const KEY v = (KEY)fkey(f);
    const int r0 = (int)((ftag(f) >> (32 - geo.lk)) & (geo.K() - 1));
    if (r == r0) return (int64_t)(ftag(f) & ((1u << (32 - geo.lk)) - 1)) << FG_LOG2;
    if (len == 0) return 0;
    if (lo <= 0) return 0;  // run r's first key comes after f
    if (lo > (len + FG - 1) >> FG_LOG2) return -1;
    // keys before f: all of positions <= (lo-1)*FG, none from lo*FG on.  The
    // first position after f (key > v if r < r0, key >= v if r > r0) lies in
    // [a, b]; it is guessed by interpolating v between the window's two
    // fence keys, bracketed by galloping from the guess, then binary-searched:
    // on spread keys the probes stay within a line or two of the answer
    // (a plain binary search touches ~5 lines of the 1 KiB window; the kernel
    // is bound by those probe lines).
    const KEY* kr = src + base + r * W;
    const FT* fr = F + ((base + r * W) >> FG_LOG2);
    const int64_t a = ((lo - 1) << FG_LOG2) + 1, b = (lo << FG_LOG2) < len ? (lo << FG_LOG2) : len;
    const bool le = r < r0;
    auto before = [&](int64_t q) {
        const KEY k = kr[q];
        return le ? k <= v : k < v;
    };
    const KEY ka = (KEY)fkey(fr[lo - 1]);
    int64_t p = a + ((b - a) >> 1);
    if ((lo << FG_LOG2) < len) {
        const KEY kb = (KEY)fkey(fr[lo]);
        if (kb > ka) p = interp<KEY>(v, ka, kb, a, b);
    }
    p = p < a ? a : (p > b ? b : p);
    int64_t lo_b, hi_b;  // the answer lies in [lo_b, hi_b]
    // line: first the guess's aligned 128-byte line in one round of vector
    // loads: on spread keys it usually holds the answer (a count of the keys
    // before it); otherwise it narrows the range to one side.  It cuts the
    // dependent probe rounds, which pays when many searches share the memory
    // system; a few thousand latency-bound ones run faster without it.
    constexpr int BW = BOUNDS_LINE / (int)sizeof(KEY);
    const int64_t blk = (p < b ? p : b - 1) & ~(int64_t)(BW - 1);
    bool fwd;
    if (line && a < b && blk + BW <= len && ((uintptr_t)kr & 15) == 0) {
        kvec<KEY> q[BW * (int)sizeof(KEY) / 16];
#pragma unroll
        for (int i = 0; i < BW * (int)sizeof(KEY) / 16; ++i) q[i] = reinterpret_cast<const kvec<KEY>*>(kr + blk)[i];
        const int64_t l0 = blk > a ? blk : a, l1 = blk + BW < b ? blk + BW : b;
        int c = 0;
#pragma unroll
        for (int i = 0; i < BW; ++i) {
            const KEY k = q[i / (16 / (int)sizeof(KEY))][i % (16 / (int)sizeof(KEY))];
            c += (blk + i >= l0 && blk + i < l1 && (le ? k <= v : k < v)) ? 1 : 0;
        }
        if (c > 0 && c < l1 - l0) return l0 + c;
        if (c == 0) {  // the answer is at or before l0
            lo_b = a;
            hi_b = l0;
            fwd = false;
        } else {  // after all of the line's keys in [a, b)
            lo_b = l1;
            hi_b = b;
            fwd = true;
        }
    } else if (p < b && before(p)) {
        lo_b = p + 1;
        hi_b = b;
        fwd = true;
    } else {
        lo_b = a;
        hi_b = p;
        fwd = false;
    }
    if (fwd) {
        for (int64_t step = 4;; step <<= 1) {
            const int64_t x = lo_b + step - 1;
            if (x >= hi_b) break;
            if (before(x)) {
                lo_b = x + 1;
            } else {
                hi_b = x;
                break;
            }
        }
    } else {
        for (int64_t step = 4;; step <<= 1) {
            const int64_t x = hi_b - step;
            if (x < lo_b) break;
            if (!before(x)) {
                hi_b = x;
            } else {
                lo_b = x + 1;
                break;
            }
        }
    }
    while (lo_b < hi_b) {
        const int64_t mid = (lo_b + hi_b) >> 1;
        if (before(mid)) lo_b = mid + 1;
        else hi_b = mid;
    }
    return lo_b;
}


// The start of chunk t of group g in run r (a position within the run), or
// the run's length for the group's end slot (t = the group's chunk count).
// Run r's fences before the chunk-start fence f come from the scanned counts
// (loaded beside f: one dependent round less; chunk indices are < 2^31).
template <typename KEY>
__device__ int64_t chunk_bound(const KEY* __restrict__ src, const typename KTr<KEY>::F* __restrict__ F,
                               const typename KTr<KEY>::F* __restrict__ M, const int* __restrict__ P,
                               const int* __restrict__ bsum, int cpb, const Geo& geo, int64_t g, int64_t t, int r,
                               bool line) {
    if (t == geo.nchunks(g)) return geo.run_len(g, r);
    const int K = geo.K();
    const uint32_t c = (uint32_t)(g * geo.kf + t), c0 = (uint32_t)(g * geo.kf);  // the tail group starts at nfull * kf too
    const int pc = P[(int64_t)c * K + r] + bsum[(int64_t)(c / (uint32_t)cpb) * K + r];
    const int pc0 = P[(int64_t)c0 * K + r] + bsum[(int64_t)(c0 / (uint32_t)cpb) * K + r];
    const typename KTr<KEY>::F f = M[(geo.base(g) >> FG_LOG2) + t * geo.fm];
    return window_bound<KEY>(src, F, geo, g, r, f, (int64_t)pc - pc0, line);
}

// One thread per (bounds slot, run).
template <typename KEY>
__global__ void k_bounds(const KEY* __restrict__ src, const typename KTr<KEY>::F* __restrict__ F,
                         const typename KTr<KEY>::F* __restrict__ M, const int* __restrict__ P,
                         const int* __restrict__ bsum, int cpb, Geo geo, int64_t nslots,
                         int64_t* __restrict__ bounds, bool line) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= (nslots << geo.lk)) return;
    const int64_t s = id >> geo.lk;
    const int r = (int)(id & (geo.K() - 1));
    int64_t g, t;
    if (s < geo.nfull * (geo.kf + 1)) {
        g = (uint32_t)s / (uint32_t)(geo.kf + 1);
        t = s - g * (geo.kf + 1);
    } else {
        g = geo.nfull;
        t = s - geo.nfull * (geo.kf + 1);
    }
    bounds[id] = chunk_bound<KEY>(src, F, M, P, bsum, cpb, geo, g, t, r, line);
}

// Chunk descriptors: for chunk c, its group's base, its output offset, the
// chunk positions where its K segments start, and its LOAD ROWS.  A chunk is
// loaded in NROWS rows of RW consecutive keys, each row inside one segment
// (segment r takes ceil(l_r / RW) rows; the K take <= CAP/RW + K = NROWS):
// row j = byte offset of its first key from the group base, and how many of
// its RW keys are real plus the LDS slot the first goes to (segment r's keys
// start at LDS slot o_r + r*G, leaving G slots for sentinels after each).
// The tables are stored by part: entry p*LS + j is row j*NR + p, so a wave
// reads its LS entries as a few wide scalar loads.
// Validated so that no chunk can address memory outside its group's runs:
// a bad chunk gets no rows and is left unwritten (the sort then fails its
// checks).
template <typename KEY, int LK>
struct alignas(128) Desc {  // whole 128-byte lines: a chunk's entries never share a line with another's
    int64_t gbase, out0;
    int o[Shape<KEY, LK>::K + 1];           // chunk position of segment r; o[K] = chunk length
    uint32_t off[Shape<KEY, LK>::NROWS];  // byte offset of the row's first key from the group base
    uint32_t la[Shape<KEY, LK>::NROWS];   // real keys of the row (0..RW) | LDS slot of its first key << 16
};

// DC chunks per one-wave workgroup (16; 4 for small sorts, which then still
// spread over many waves), in two phases.  Lane = chunk: read its 2K
// bounds (one contiguous row), check them and prefix the segment lengths and
// row counts into an LDS header, plus a row -> segment map.  Lane = table
// entry: each (chunk, row) entry is computed from the header and stored, so
// consecutive lanes write consecutive words of a descriptor.  (One lane per
// chunk and entry keeps the instruction count at a few dozen per chunk; a wave
// per chunk spent ~500, k_chunk_desc being bound by them.)
constexpr int DC_NT = 64;

template <typename KEY, int LK>
struct DescHdr {
    static constexpr int K = Shape<KEY, LK>::K;
    int64_t gbase, out0;
    int so[K + 1], srow[K + 1], sln[K];
    uint32_t sb[K];
};

// A chunk's descriptor header from its bounds st / en in the K runs of group g
// (ok = false: an empty chunk): the segments' chunk positions, load-row
// counts and byte offsets, the row -> segment map, and the output offset.
template <typename KEY, int LK, bool UNROLL = true>
__device__ void desc_header(DescHdr<KEY, LK>& h, uint8_t* seg, const Geo& geo, int64_t g, const int64_t* st,
                            const int64_t* en, bool ok) {
    typedef Shape<KEY, LK> S;
    constexpr int K = S::K;
    int R = 0, o = 0;
    int64_t out = geo.base(g);
#pragma unroll(UNROLL ? K : 1)
    for (int r = 0; r < K; ++r) {
        const int ln = ok ? (int)(en[r] - st[r]) : 0, s0 = ok ? (int)st[r] : 0;
        h.srow[r] = R;
        h.so[r] = o;
        h.sln[r] = ln;
        // byte offset of segment r's first key from the group base (< KW*sizeof(KEY) <= 2^32)
        h.sb[r] = (((uint32_t)r << geo.lw) + (uint32_t)s0) * (uint32_t)sizeof(KEY);
        const int nr = (ln + S::RW - 1) / S::RW;
        for (int q = 0; q < nr; ++q) seg[R + q] = (uint8_t)r;
        R += nr;
        o += ln;
        out += s0;
    }
    h.srow[K] = R;
    h.so[K] = o;
    h.gbase = geo.base(g);
    h.out0 = out;
}

// Table entry j of a descriptor from its header (entry j is row (j % LS) * NR
// + j / LS: stored by part).
template <typename KEY, int LK>
__device__ __forceinline__ void desc_entry(Desc<KEY, LK>* d, const DescHdr<KEY, LK>& h, const uint8_t* seg, int j) {
    typedef Shape<KEY, LK> S;
    constexpr int K = S::K;
    const int row = (j % S::LS) * S::NR + j / S::LS;
    uint32_t off = 0, la = 0;
    if (row < h.srow[K]) {  // rows past the chunk: no keys
        const int rr = seg[row];
        const int k = row - h.srow[rr], rem = h.sln[rr] - k * S::RW;
        off = h.sb[rr] + (uint32_t)(k * S::RW * (int)sizeof(KEY));
        la = (uint32_t)(rem < S::RW ? rem : S::RW) | ((uint32_t)(S::seg(h.so[rr], rr) + k * S::RW) << 16);
    }
    d->off[j] = off;
    d->la[j] = la;
}

// The capacity split (merge_pass): chunk (g, t), whose exact size exceeds CAP,
// cut at its middle merged fence into two descriptors d[0], d[1] by the 64
// lanes of one wave.  Each half holds at most ceil(fm / 2) + K fences' worth
// of keys <= CAP (merge_pass bounds fm so).  Lane r < K finds run r's bound at
// the middle fence: its fences before the chunk start (the scanned counts)
// plus those among the chunk's first fences, then the window search of
// k_bounds; lanes 0 and 1 build the halves' headers.  hdr / seg / sm: LDS
// scratch for two headers and K bounds.
template <typename KEY, int LK>
__device__ __forceinline__ void split_chunk(const KEY* __restrict__ src, const typename KTr<KEY>::F* __restrict__ F,
                            const typename KTr<KEY>::F* __restrict__ M, const int* __restrict__ P,
                            const int* __restrict__ bsum, int cpb, const Geo& geo, int64_t g, int64_t t,
                            const int64_t* b0, Desc<KEY, LK>* d, int* err, bool line, DescHdr<KEY, LK>* hdr,
                            uint8_t (*seg)[Shape<KEY, LK>::NROWS], int64_t* sm, int lane) {
    typedef Shape<KEY, LK> S;
    constexpr int K = S::K, NROWS = S::NROWS;
    const int64_t gf = geo.base(g) >> FG_LOG2, nfg = geo.nfences(g), f0 = t * geo.fm;
    const int mid = (int)((f0 + geo.fm < nfg ? geo.fm : nfg - f0) / 2);
    if (lane < K) {
        const int r = lane;
        const uint32_t c = (uint32_t)(g * geo.kf + t), c0 = (uint32_t)(g * geo.kf);
        int64_t lo = (int64_t)(P[(int64_t)c * K + r] + bsum[(int64_t)(c / (uint32_t)cpb) * K + r]) -
                     (P[(int64_t)c0 * K + r] + bsum[(int64_t)(c0 / (uint32_t)cpb) * K + r]);
        for (int e = 0; e < mid; ++e) lo += (int)((ftag(M[gf + f0 + e]) >> (32 - geo.lk)) & (K - 1)) == r ? 1 : 0;
        sm[r] = mid > 0 ? window_bound<KEY>(src, F, geo, g, r, M[gf + f0 + mid], lo, line) : -1;
    }
    __syncthreads();
    if (lane < 2) {
        // half 0: [b0, sm), half 1: [sm, b0 + K) (generic pointers: few registers)
        const int64_t* st = lane ? sm : b0;
        const int64_t* en = lane ? b0 + K : sm;
        bool ok = mid > 0;
        int64_t tot = 0;
        for (int r = 0; r < K; ++r) {
            ok = ok && st[r] >= 0 && en[r] >= st[r] && en[r] <= geo.run_len(g, r);
            tot += en[r] - st[r];
        }
        ok = ok && tot <= S::CAP;
        if (!ok) atomicOr(err, 1);
        desc_header<KEY, LK, false>(hdr[lane], seg[lane], geo, g, st, en, ok);
    }
    __syncthreads();
    for (int e = lane; e < 2 * NROWS; e += 64) {
        const int h = e / NROWS;
        desc_entry<KEY, LK>(d + h, hdr[h], seg[h], e - h * NROWS);
    }
    for (int e = lane; e < 2 * (K + 1); e += 64) {
        const int h = e / (K + 1), r = e - h * (K + 1);
        d[h].o[r] = hdr[h].so[r];
    }
    if (lane < 2) {
        d[lane].gbase = hdr[lane].gbase;
        d[lane].out0 = hdr[lane].out0;
    }
    __syncthreads();
}

// PLAN (small sorts, MISORT_PLAN_FUSE): the workgroup computes its chunks'
// bounds itself (chunk_bound: the DC chunk starts and the end of the last one,
// lane = (chunk, run)) into LDS, in place of a k_bounds launch.  nbs > 0: bsum
// holds the RAW block totals of the nbs fence-count blocks (nbs * K <=
// PLAN_SCAN_MAX) and every workgroup scans them in LDS, in place of a
// k_scan_totals launch (a few KB of L2 reads per workgroup).
constexpr int PLAN_SCAN_MAX = 2048;
template <typename KEY, int LK, int DC, bool PLAN>
__global__ __launch_bounds__(DC_NT) void k_chunk_desc(const int64_t* __restrict__ bounds, Geo geo, int64_t nchunks,
                                                   Desc<KEY, LK>* __restrict__ desc, int* __restrict__ err,
                                                   const KEY* __restrict__ src = nullptr,
                                                   const typename KTr<KEY>::F* __restrict__ F = nullptr,
                                                   const typename KTr<KEY>::F* __restrict__ M = nullptr,
                                                   const int* __restrict__ P = nullptr,
                                                   const int* __restrict__ bsum = nullptr, int cpb = 0,
                                                   bool line = false, int nbs = 0, int* __restrict__ ovf = nullptr,
                                                   Desc<KEY, LK>* __restrict__ dov = nullptr) {
    typedef Shape<KEY, LK> S;
    constexpr int K = S::K, NROWS = S::NROWS;
    __shared__ DescHdr<KEY, LK> hdr[DC];
    __shared__ uint8_t seg[DC][NROWS];  // row -> its segment
    __shared__ int64_t sbd[PLAN ? DC + 1 : 1][K];  // PLAN: item j = the start of chunk cb + j (j = nc: the
                                                   // slot after chunk cb + nc - 1)
    __shared__ int sbs[PLAN ? PLAN_SCAN_MAX : 1];  // PLAN, nbs > 0: the scanned block totals
    const int lane = threadIdx.x;
    const int64_t cb = (int64_t)blockIdx.x * DC;
    const int nc = nchunks - cb < DC ? (int)(nchunks - cb) : DC;
    if constexpr (PLAN) {
        const int* bs = bsum;
        if (nbs > 0) {
            // exclusive scan over blocks, per run: lane = (segment, run), NSEG
            // segments of consecutive blocks per run, a shuffle scan of the
            // segment sums across the lanes of one run
            static_assert(DC_NT % K == 0, "whole runs per wave");
            constexpr int NSEG = DC_NT / K;
            for (int e = lane; e < nbs * K; e += DC_NT) sbs[e] = bsum[e];
            __syncthreads();
            const int r = lane % K, sg = lane / K, rps = (nbs + NSEG - 1) / NSEG;
            const int b0 = sg * rps < nbs ? sg * rps : nbs, b1 = b0 + rps < nbs ? b0 + rps : nbs;
            int sum = 0;
            for (int b = b0; b < b1; ++b) sum += sbs[b * K + r];
            int inc = sum;
#pragma unroll
            for (int o = 1; o < NSEG; o <<= 1) {
                const int u = __shfl_up(inc, o * K, DC_NT);
                inc += sg >= o ? u : 0;
            }
            int ex = inc - sum;
            for (int b = b0; b < b1; ++b) {
                const int v = sbs[b * K + r];
                sbs[b * K + r] = ex;
                ex += v;
            }
            __syncthreads();
            bs = sbs;
        }
        for (int e = lane; e < (nc + 1) * K; e += DC_NT) {
            const int j = e / K, r = e - j * K;
            int64_t g, t;
            chunk_place(geo, cb + (j < nc ? j : nc - 1), g, t);
            sbd[j][r] = chunk_bound<KEY>(src, F, M, P, bs, cpb, geo, g, j < nc ? t : t + 1, r, line);
        }
        __syncthreads();
    }
    if (lane < nc) {
        int64_t g, t;
        chunk_place(geo, cb + lane, g, t);
        int64_t st[K], en[K];
        if constexpr (PLAN) {
            // the chunk's end: the runs' ends for the group's last chunk, else
            // the next item (the next chunk's start, or the slot after the block's last)
            const bool last = t + 1 == geo.nchunks(g);
#pragma unroll
            for (int r = 0; r < K; ++r) {
                st[r] = sbd[lane][r];
                en[r] = last ? geo.run_len(g, r) : sbd[lane + 1][r];
            }
        } else {
            const int64_t* b0 = bounds + K * geo.slot(g, t);
#pragma unroll
            for (int r = 0; r < K; ++r) {
                st[r] = b0[r];
                en[r] = b0[K + r];
            }
        }
        // bounds outside the runs would be a logic error: never let them address memory
        bool ok = true;
        int64_t tot = 0;
#pragma unroll
        for (int r = 0; r < K; ++r) {
            const int64_t ln = en[r] - st[r];
            ok = ok && st[r] >= 0 && ln >= 0 && en[r] <= geo.run_len(g, r);
            tot += ln;
        }
        // ovf (fm above the worst-case bound, see merge_pass): a chunk larger
        // than CAP keys gets an empty descriptor here and is listed in ovf for
        // k_split_desc
        const bool big = ok && tot > S::CAP;
        if (big && ovf) ovf[1 + atomicAdd(ovf, 1)] = (int)(cb + lane);
        else if (!ok || big) atomicOr(err, 1);  // a planning bug: the chunk stays unwritten, the host is told
        desc_header<KEY, LK>(hdr[lane], seg[lane], geo, g, st, en, ok && !big);
    }
    __syncthreads();
    Desc<KEY, LK>* d = desc + cb;
    for (int e = lane; e < nc * NROWS; e += DC_NT) {
        const int cl = e / NROWS;
        desc_entry<KEY, LK>(d + cl, hdr[cl], seg[cl], e - cl * NROWS);
    }
    for (int e = lane; e < nc * (K + 1); e += DC_NT) {
        const int cl = e / (K + 1), r = e - cl * (K + 1);
        d[cl].o[r] = hdr[cl].so[r];
    }
    if (lane < nc) {
        d[lane].gbase = hdr[lane].gbase;
        d[lane].out0 = hdr[lane].out0;
    }
}

// The chunks k_chunk_desc listed (ovf[1 .. ovf[0]]), each cut in two into
// dov[2i], dov[2i + 1] (split_chunk): one wave per listed chunk (the list is
// usually empty: every wave exits at once).  1024 waves, so that a long list --
// inputs whose window offsets do not cancel -- is cut in parallel: with 64 a
// 2^30 pass at a margin of 11 fences spent 260 us here
// (profiles/r06/mergek/fm_add_ab.txt).
constexpr int SPLIT_WG = 1024;
template <typename KEY, int LK>
__global__ __launch_bounds__(64) void k_split_desc(const KEY* __restrict__ src, const typename KTr<KEY>::F* __restrict__ F,
                                                  const typename KTr<KEY>::F* __restrict__ M, const int* __restrict__ P,
                                                  const int* __restrict__ bsum, int cpb, Geo geo,
                                                  const int64_t* __restrict__ bounds, const int* __restrict__ ovf,
                                                  Desc<KEY, LK>* __restrict__ dov, int* __restrict__ err, bool line) {
    typedef Shape<KEY, LK> S;
    __shared__ DescHdr<KEY, LK> hdr[2];
    __shared__ uint8_t seg[2][S::NROWS];
    __shared__ int64_t sm[S::K];
    const int cnt = ovf[0];
    for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
        int64_t g, t;
        chunk_place(geo, ovf[1 + i], g, t);
        split_chunk<KEY, LK>(src, F, M, P, bsum, cpb, geo, g, t, bounds + S::K * geo.slot(g, t), dov + 2 * (int64_t)i,
                             err, line, hdr, seg, sm, (int)threadIdx.x);
    }
}

// The wave's row part (uniform) and the lane's place in its row.
template <typename KEY, int LK>
__device__ __forceinline__ int row_part(int tid) {
    return __builtin_amdgcn_readfirstlane(tid) / Shape<KEY, LK>::RW;
}

// The chunk's in-LDS work after its keys and sentinels are in LDS: the merge
// levels, the outputs back to LDS (shifted so every 16-byte global vector is
// one aligned LDS vector), out to HBM, and the next pass's fences.
// The key as stored: ORD (u64, the sort's last pass over f64 keys) maps the
// ordered form back to IEEE double bits.
template <bool ORD, typename KEY>
__device__ __forceinline__ KEY out_key(KEY k) {
    if constexpr (ORD) return (KEY)f64_of_ord((uint64_t)k);
    else return k;
}
template <bool ORD, typename V>
__device__ __forceinline__ V out_vec(V v) {
    if constexpr (ORD) {
        V o;
#pragma unroll
        for (int j = 0; j < (int)(sizeof(V) / sizeof(uint64_t)); ++j) o[j] = f64_of_ord(v[j]);
        return o;
    } else {
        return v;
    }
}

template <typename KEY, int LK, bool FENCES, int MODE, bool ORD = false>
__device__ __forceinline__ void mergek_chunk(KEY* s, const Desc<KEY, LK>* d, KEY* __restrict__ dst,
                                             typename KTr<KEY>::F* __restrict__ fout, int lwn, int lkn, int tid) {
    typedef Shape<KEY, LK> S;
    constexpr int K = S::K, NT = S::NT, IT = S::IT;
    constexpr int VK = 16 / (int)sizeof(KEY);  // keys per 16-byte vector
    constexpr int LAST = S::LDS_KEYS - PAD - 1;
    const int len = d->o[K];
    KEY r[IT];  // the lane's outputs [pos, pos + IT)
    const int pos = tid * IT;
    // the first level's input sequences: the chunk's segments
    int st[K], ln[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        st[q] = S::seg(d->o[q], q);
        ln[q] = d->o[q + 1] - d->o[q];
    }
    lds_merge_levels<KEY, S, MODE>(s, st, ln, r, tid, LAST);
    const int64_t out0 = d->out0;
    // the chunk goes to LDS shifted by out0 mod VK, so every global 16-byte
    // vector is one aligned LDS vector (a lane's outputs past len are MAX and
    // land past the chunk)
    const int sh = (int)(out0 & (VK - 1));
    if (pos < len) {
        KEY* q = s + sh + pos;
        if ((sh & 1) == 0) {
            // even shift (uniform per chunk): aligned pairs, one 8-byte (u64:
            // 16-byte) write per two keys instead of one write per key
            // (2277-2282 us per 2^30 pass instead of 2282-2291, profiles/r04/pairstage)
#pragma unroll
            for (int j = 0; j < IT; j += 2) *reinterpret_cast<kvec2<KEY>*>(q + j) = kvec2<KEY>{r[j], r[j + 1]};
        } else {
#pragma unroll
            for (int k = 0; k < IT; ++k) q[k] = r[k];
        }
    }
    lds_barrier();
    const int nv = (sh + len + VK - 1) / VK;
    KEY* __restrict__ o = dst + (out0 - sh);
    for (int v = tid; v < nv; v += NT) {
        const int e = VK * v;
        if (e >= sh && e + VK <= sh + len) {
            __builtin_nontemporal_store(out_vec<ORD>(*reinterpret_cast<const kvec<KEY>*>(s + e)),
                                        reinterpret_cast<kvec<KEY>*>(o + e));
        } else {
#pragma unroll
            for (int j = 0; j < VK; ++j)
                if (e + j >= sh && e + j < sh + len) o[e + j] = out_key<ORD>(s[e + j]);
        }
    }
    if constexpr (FENCES) {
        // the chunk's fences are consecutive entries of fout: one coalesced
        // store per fence from consecutive lanes
        const int64_t first = (out0 + FG - 1) & ~(FG - 1);
        const int nf = first < out0 + len ? (int)((out0 + len - first + FG - 1) >> FG_LOG2) : 0;
        if (tid < nf) {
            const int64_t gp = first + ((int64_t)tid << FG_LOG2);
            fout[gp >> FG_LOG2] = fpack<KEY>(s[(int)(gp - (out0 - sh))], gp, lwn, lkn);
        }
    }
}

// The sentinels after every segment of the chunk (ZW: G - 1 of them and a
// zero word, the word below the next segment), the zero word below the first
// and the first level's pair table (pt).
template <typename KEY, int LK>
__device__ __forceinline__ void mergek_sentinels(KEY* s, const Desc<KEY, LK>* d, int tid) {
    typedef Shape<KEY, LK> S;
    // a wave per segment (uniform segment index: the descriptor's offsets come
    // by scalar loads), G <= 64 lanes each
    static_assert(S::G <= 64, "sentinels: one wave per segment");
    const int lane = tid & 63;
    for (int q = __builtin_amdgcn_readfirstlane(tid >> 6); q < S::K; q += S::NT / 64)
        if (lane < S::G)
            s[S::seg(d->o[q], q) + (d->o[q + 1] - d->o[q]) + lane] = S::ZW && lane == S::G - 1 ? (KEY)0 : KMAX<KEY>;
    if constexpr (S::ZW) {
        if (tid == 0) s[S::seg(d->o[0], 0) - 1] = (KEY)0;  // the zero word below the first segment
    }
}

// k_mergek: one workgroup per chunk.  (A persistent grid that loads the next
// chunk into registers during the merge levels ran 2.28 -> 2.82 ms per 2^30
// pass even with LDS-only barriers: gfx950 counts loads and stores in one
// in-order vmcnt, so waiting for the prefetch also waits for the previous
// chunk's stores; profiles/r04/persist.)  MODE (probes only, MISORT_MK_PROBE):
// 0 = the pass; 1 = no merge (the access pattern's floor); 2 = level 1 only;
// 3 = the co-rank searches of every level without the chains (for SQ
// attribution: 3 - 1 = the searches, 0 - 3 = the chains).
// Waves whose lanes all lie past a level's outputs skip its merge (a chunk
// averages FM*FG of CAP keys).
// One chunk: its rows into LDS, the sentinels, then mergek_chunk.
template <typename KEY, int LK, bool FENCES, int MODE, bool ORD>
__device__ __forceinline__ void mergek_run(KEY* tile, const KEY* __restrict__ src, KEY* __restrict__ dst,
                                           const Desc<KEY, LK>* __restrict__ d, typename KTr<KEY>::F* __restrict__ fout,
                                           int lwn, int lkn) {
    typedef Shape<KEY, LK> S;
    KEY* s = tile + PAD;
    const int tid = threadIdx.x;
    {
        // loads: lane slot j = row j * NR + part, lane offset lt; the wave's
        // table entries first (scalar registers), then all its loads
        const char* gsrc = (const char*)(src + d->gbase);
        const int part = row_part<KEY, LK>(tid), lt = tid & (S::RW - 1);
        constexpr int LS = S::LS;
        const uint32_t* offp = d->off + part * LS;
        const uint32_t* lap = d->la + part * LS;
        uint32_t off[LS], la[LS];
#pragma unroll
        for (int j = 0; j < LS; ++j) {
            off[j] = offp[j];
            la[j] = lap[j];
        }
        if constexpr (sizeof(KEY) == 4) {
            // straight into LDS: a wave's part of a row is 64 consecutive LDS
            // words from a wave-uniform base (global_load_lds_dword writes
            // base + 4 * lane), so the row's slot plus the wave's first lane
            const int wl0 = __builtin_amdgcn_readfirstlane(lt & ~63);
#pragma unroll
            for (int j = 0; j < LS; ++j)
                if (lt < (int)(la[j] & 0xFFFF))
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)((const KEY*)(gsrc + off[j]) + (uint32_t)lt),
                        (__attribute__((address_space(3))) void*)(lds_t<KEY>*)(s + (la[j] >> 16) + wl0), 4, 0, 0);
        } else {
            KEY x[LS];
#pragma unroll
            for (int j = 0; j < LS; ++j)
                if (lt < (int)(la[j] & 0xFFFF))
                    x[j] = __builtin_nontemporal_load((const KEY*)(gsrc + off[j]) + (uint32_t)lt);
#pragma unroll
            for (int j = 0; j < LS; ++j)
                if (lt < (int)(la[j] & 0xFFFF)) s[(la[j] >> 16) + lt] = x[j];
        }
        mergek_sentinels<KEY, LK>(s, d, tid);
    }
    __syncthreads();
    mergek_chunk<KEY, LK, FENCES, MODE, ORD>(s, d, dst, fout, lwn, lkn, tid);
}

// The grid: (capacity split) first ovf_wg() workgroups that walk the halves of
// the chunks k_split_desc cut (2 * ovf[0] descriptors in dov; usually none:
// they exit at once; dispatched first, so a half never trails the pass), then
// one workgroup per chunk.  One per resident slot of the chip (256 CUs x the
// workgroups per CU), so the halves of a long list run in the first round.
template <typename KEY, int LK>
constexpr int ovf_wg() { return 256 * KTr<KEY>::wg(LK); }
template <typename KEY, int LK, bool FENCES, int MODE = 0, bool ORD = false>
__global__ __launch_bounds__(KTr<KEY>::NT, KTr<KEY>::wg(LK)* KTr<KEY>::NT / 256) void k_mergek(
    const KEY* __restrict__ src, KEY* __restrict__ dst, const Desc<KEY, LK>* __restrict__ desc,
    typename KTr<KEY>::F* __restrict__ fout, int lwn, int lkn, uint32_t nprimary,
    const Desc<KEY, LK>* __restrict__ dov = nullptr, const int* __restrict__ ovf = nullptr) {
    typedef Shape<KEY, LK> S;
    __shared__ __attribute__((aligned(16))) KEY tile[S::LDS_KEYS];
    const uint32_t nov = gridDim.x - nprimary;  // the split's workgroups (0 without it)
    if (blockIdx.x >= nov) {
        mergek_run<KEY, LK, FENCES, MODE, ORD>(tile, src, dst, desc + (blockIdx.x - nov), fout, lwn, lkn);
        return;
    }
    const int cnt = 2 * ovf[0];
    for (int i = (int)blockIdx.x; i < cnt; i += (int)nov) {
        mergek_run<KEY, LK, FENCES, MODE, ORD>(tile, src, dst, dov + i, fout, lwn, lkn);
        __syncthreads();  // the tile is reused
    }
}

// Fence buffers, bounds and descriptors: one grow-only set per (device, stream).
struct Scratch {
    void* p = nullptr;
    size_t bytes = 0;
};
std::mutex g_mu;
std::map<std::pair<int, hipStream_t>, Scratch> g_scr[4];

// which = 0: the two fence buffers (a pass's input fences are the previous
// pass's output: sized by n alone, so they never move between the passes of
// one sort); which = 1: per-pass planning data (free to grow at any pass);
// 2 and 3: the same for a pass nested in a pass's fence merge (depth 1).  The
// depth-1 sets are sized by the nested pass's n (the outer pass's fence count)
// and may grow once, on the first nested pass of a new larger sort -- partway
// through that sort, after the outer pass's first planning launches are
// queued: growth synchronises the stream before it frees (a latency cost, the
// queued work never sees a freed buffer), and the depth-1 fence buffers are
// only ever read by the nested pass that wrote them.
void* scratch(int which, size_t bytes, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_mu);
    auto& e = g_scr[which][{dev, s}];
    if (e.bytes < bytes) {
        if (e.p && (hipStreamSynchronize(s) != hipSuccess || hipFree(e.p) != hipSuccess)) return nullptr;
        e = Scratch{};
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        e = Scratch{p, bytes};
    }
    return e.p;
}

// One error word per (device, stream): k_chunk_desc sets it when it rejects
// a chunk's bounds (mergek_take_error reads and clears it).
std::map<std::pair<int, hipStream_t>, int*> g_errw;
int* error_word(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_mu);
    int*& w = g_errw[{dev, s}];
    if (!w) {
        if (hipMalloc(&w, sizeof(int)) != hipSuccess) {
            w = nullptr;
            return nullptr;
        }
        if (hipMemsetAsync(w, 0, sizeof(int), s) != hipSuccess) return nullptr;
    }
    return w;
}

int64_t chunks_of(const Geo& geo) {
    const bool tail = (geo.nfull << (geo.lw + geo.lk)) < geo.n;
    return geo.nfull * geo.kf + (tail ? geo.nchunks(geo.nfull) : 0);
}

// The fence merge levels of a u32 pass as one multi-way merge pass over the
// fences themselves (u64 keys, depth 1) once at least FENCE_NEST_LEVELS of
// them would run as global 2-way merge levels and the pass has at least
// 2^MISORT_FENCE_NEST_MIN fences (env; 0 = never): one HBM sweep of the fence
// array instead of one per level.  Measured (profiles/r05/plan/nest_ab.txt):
// 2^30 u32 passes 3 and 4 (2^23 fences) -30 us each, +0.6 %; at 2^22 fences
// (2^29 keys) the nested pass's ~600 chunks underfilled the chip: +5 us, so the
// threshold was 2^23.  Round 6: with the nested pass's own planning in one
// k_fence_rank launch, 2^21 measured 2^28 +0.5 %, 2^29 +0.6 %, 2^30 equal
// (profiles/r06/plan/nest_ab.txt).
constexpr int FENCE_NEST_LEVELS = 3;

template <typename KEY, int LK>
hipError_t merge_pass(const KEY* src, KEY* dst, int64_t n, int lw, hipStream_t s, int phase, bool gather,
                      int lk_next, LaunchHook* hook, bool ord_out, int depth = 0) {
    typedef Shape<KEY, LK> S;
    typedef typename KTr<KEY>::F FT;
    // MISORT_PLAN_FUSE: 1 (default) = bounds inside k_chunk_desc below 4096
    // chunks, 2 = at every size, 0 = never (profiles/r03/ab_plan: 2^24 u32 43.1
    // -> 43.9 Gkeys/s; at 2^26, 9362 chunks, 65.2 -> 65.0)
    // MISORT_PLAN_SCAN: 1 (default) = a fused descriptor kernel scans the
    // fence-count block totals itself when they fit PLAN_SCAN_MAX, 0 = never
    static const int plan_fuse = getenv("MISORT_PLAN_FUSE") ? atoi(getenv("MISORT_PLAN_FUSE")) : 1;
    static const int plan_scan = getenv("MISORT_PLAN_SCAN") ? atoi(getenv("MISORT_PLAN_SCAN")) : 1;
    Geo geo = make_geo<KEY>(n, lw, LK);
    const bool fuse = plan_fuse == 2 || (plan_fuse == 1 && chunks_of(geo) < 4096);
    // Capacity split (unfused passes): chunks cut every fm merged fences, fm
    // above the worst-case bound by split_fm_add -- sized for a typical chunk,
    // whose K window offsets nearly cancel -- and the rare chunk that exceeds
    // CAP cut in two at its middle fence (k_chunk_desc cuts it, k_mergek's
    // extra workgroups run the halves).  A half holds at most ceil(fm / 2) + K fences'
    // worth of keys, so fm stays within 2 (CAP / FG - K) (and 8-bit counts).
    const int fma = fuse ? 0 : split_fm_add<KEY, LK>();
    if (fma > 0) geo = make_geo<KEY>(n, lw, LK, balance_fm<KEY, LK>(geo.fm + fma, ((int64_t)1 << (lw + LK)) >> FG_LOG2));
    const bool split = fma > 0;
    const bool tail = (geo.nfull << (lw + LK)) < n;
    const int64_t nchunks = chunks_of(geo);
    const int64_t nslots = geo.nfull * (geo.kf + 1) + (tail ? geo.nchunks(geo.nfull) + 1 : 0);
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    if (nchunks >= ((int64_t)1 << 31) || nslots >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    // fence buffers 0 and 1 (kept across passes); per pass: merged fences,
    // fence merge temp, bounds, fence counts and their block totals, descriptors
    // chunks per fence-count block: SCAN_NT, or fewer (down to 32) while that
    // leaves under 128 blocks -- a small sort's few blocks walked long slices
    int cpb = SCAN_NT;
    while (cpb > 32 && (nchunks + cpb - 1) / cpb < 128) cpb /= 2;
    const int64_t nbk = (nchunks + cpb - 1) / cpb;
    const size_t fb = ((size_t)nf * sizeof(FT) + 255) & ~(size_t)255;
    const size_t bb = ((size_t)nslots * S::K * 8 + 255) & ~(size_t)255;
    const size_t cb = ((size_t)nbk * cpb * S::K * 4 + 255) & ~(size_t)255;
    const size_t sb = ((size_t)nbk * S::K * 4 + 255) & ~(size_t)255;
    char* fbase = (char*)scratch(2 * depth, 2 * fb, s);
    // descriptors: one per chunk, and with the split two per listed chunk
    // (at most every chunk) plus the list
    const size_t db = (size_t)nchunks * sizeof(Desc<KEY, LK>) * (split ? 3 : 1);
    const size_t ob = split ? ((size_t)(nchunks + 1) * 4 + 255) & ~(size_t)255 : 0;
    char* base = (char*)scratch(2 * depth + 1, 2 * fb + bb + cb + sb + db + ob + 256, s);
    int* ew = error_word(s);
    if (!base || !fbase || !ew) return hipErrorOutOfMemory;
    FT* F = (FT*)(fbase + (phase & 1) * fb);
    FT* Fn = (FT*)(fbase + ((phase & 1) ^ 1) * fb);
    FT* M = (FT*)base;
    FT* T = (FT*)(base + fb);
    int64_t* bounds = (int64_t*)(base + 2 * fb);
    int* cnt = (int*)(base + 2 * fb + bb);
    int* bsum = (int*)(base + 2 * fb + bb + cb);
    Desc<KEY, LK>* desc = (Desc<KEY, LK>*)(base + 2 * fb + bb + cb + sb);
    Desc<KEY, LK>* dov = split ? desc + nchunks : nullptr;  // the halves of listed chunks
    int* ovf = split ? (int*)(base + 2 * fb + bb + cb + sb + db) : nullptr;  // [count, chunks...]
    if (gather) k_fence_gather<KEY><<<(unsigned)((nf + 255) / 256), 256, 0, s>>>(src, n, lw, LK, F);
    const int wf_log2 = lw - FG_LOG2;  // fences per run = 2^wf_log2
    // MISORT_FENCE_RANK_MAX: fused passes whose runs hold <= 2^this fences rank
    // them and count them in one launch (k_fence_rank); 0 = never
    static const int rank_max = getenv("MISORT_FENCE_RANK_MAX") ? atoi(getenv("MISORT_FENCE_RANK_MAX")) : 14;
    const bool rank = fuse && wf_log2 <= rank_max;
    if (rank) {
        k_fence_rank<FT, LK><<<(unsigned)((nf + RANK_NT - 2) / (RANK_NT - 1)), RANK_NT, 0, s>>>(
            F, M, geo, nf, wf_log2, cnt, bsum, nbk * S::K);
    } else {
        // the group's fences into total order, landing in M: the first a levels
        // in LDS (sub-groups of 2^a runs, <= 64 KiB of fences), the other
        // LK - a as fence merge levels (runs of >= 2^FL fences), ping-ponging
        // through T
        constexpr int FL = KTr<KEY>::FL_LDS;
        const int a = wf_log2 >= FL ? 0 : (FL - wf_log2 < LK ? FL - wf_log2 : LK);
        const FT* x = F;
        int left = LK - a;
        bool nest = false;
        if constexpr (sizeof(KEY) == 4) {
            static const int nest_min =
                getenv("MISORT_FENCE_NEST_MIN") ? atoi(getenv("MISORT_FENCE_NEST_MIN")) : 21;
            nest = depth == 0 && nest_min > 0 && left >= FENCE_NEST_LEVELS && nf >= ((int64_t)1 << nest_min) &&
                   wf_log2 + a >= KTr<uint64_t>::LW_MIN && wf_log2 + a + left <= KTr<uint64_t>::LWK_MAX;
        }
        if (a > 0) {
            FT* y = nest || (left & 1) ? T : M;
            const size_t lds = ((size_t)1 << (wf_log2 + a)) * sizeof(FT);
            const int64_t nb0 = (nf + ((int64_t)1 << (wf_log2 + a)) - 1) >> (wf_log2 + a);
            // >= 512 blocks where the sub-groups are few (each loads its whole sub-group)
            if (nb0 >= FENCE_MERGE_MIN_BLOCKS) {
                k_fence_merge<FT><<<(unsigned)nb0, (unsigned)(((int64_t)1 << (wf_log2 + a)) / FIT), lds, s>>>(
                    F, y, nf, wf_log2, a);
            } else {
                int split = 1;
                while (split < 8 && nb0 * split < 512 && ((int64_t)1 << (wf_log2 + a)) / (split * 2) >= 1024)
                    split *= 2;
                k_fence_lds<FT><<<(unsigned)(nb0 * split), 1024, lds, s>>>(F, y, nf, wf_log2, a, split);
            }
            x = y;
        }
        if constexpr (sizeof(KEY) == 4) {
            if (nest) {
                // the fences' runs of 2^(wf_log2 + a) into M in one pass (it
                // reads x -- F or T -- and leaves F to k_bounds)
                const uint64_t* xf = (const uint64_t*)x;
                const hipError_t e =
                    left == 4 ? merge_pass<uint64_t, 4>(xf, (uint64_t*)M, nf, wf_log2 + a, s, 0, true, 0, nullptr, false, 1)
                              : merge_pass<uint64_t, 3>(xf, (uint64_t*)M, nf, wf_log2 + a, s, 0, true, 0, nullptr, false, 1);
                if (e != hipSuccess) return e;
                left = 0;
            }
        }
        for (int l = LK - left; l < LK; ++l, --left) {
            FT* y = ((left - 1) & 1) ? T : M;
            const hipError_t e = merge_level<FT>(x, y, nf, wf_log2 + l, s);
            if (e != hipSuccess) return e;
            x = y;
        }
    }
    const int64_t nb = nbk;
    // few blocks: per-lane slices; many: coalesced atomics (k_fence_counts)
    // MISORT_FC_SLICES_MAX (tests): the block count from which the coalesced form counts
    static const int64_t slices_max = getenv("MISORT_FC_SLICES_MAX") ? atoll(getenv("MISORT_FC_SLICES_MAX")) : 256;
    if (rank) {
    } else if (nb < slices_max) {
        k_fence_counts<FT, true><<<(unsigned)nb, COUNT_NT, 0, s>>>(M, geo, nchunks, cpb, cnt, bsum, ovf);
    } else {
        k_fence_counts<FT, false><<<(unsigned)nb, FC_NT, 0, s>>>(M, geo, nchunks, cpb, cnt, bsum, ovf);
    }
    // planning kernel shapes by size (measured crossovers, profiles/r02/s3b-s3i):
    // k_bounds' line probe from 2^17 searches, 16 descriptors per workgroup from 2^14 chunks
    constexpr int64_t line_min = 1 << 17, dc16_min = 1 << 14;
    const bool line = (nslots << LK) >= line_min;
    const int nbs = !rank && fuse && plan_scan && nb * S::K <= PLAN_SCAN_MAX ? (int)nb : 0;
    if (nbs == 0 && !rank) k_scan_totals<<<1, 64 * ((S::K + 1) / 2), 0, s>>>(bsum, nb, S::K);
    if (!fuse)
        k_bounds<KEY><<<(unsigned)(((nslots << LK) + 255) / 256), 256, 0, s>>>(src, F, M, cnt, bsum, cpb, geo,
                                                                              nslots, bounds, line);
    // the launch before k_mergek: a binding hook's tick (its end starts k_mergek's record)
    hipEvent_t ta = nullptr, tb = nullptr;
    if (hook && hook->binds()) (void)hook->bind(-1, -1, 0.0, &ta, &tb);
    hipEvent_t da = ta, dbe = tb;
    const dim3 g16((unsigned)((nchunks + 15) / 16)), g4((unsigned)((nchunks + 3) / 4));
    const int* P0 = cnt;
    const FT* F0 = F;
    const FT* M0 = M;
    if (fuse) {
        if (nchunks >= dc16_min)
            launch_timed(k_chunk_desc<KEY, LK, 16, true>, g16, dim3(DC_NT), 0, s, da, dbe, (const int64_t*)nullptr, geo,
                         nchunks, desc, ew, src, F0, M0, P0, (const int*)bsum, cpb, line, nbs, (int*)nullptr,
                         (Desc<KEY, LK>*)nullptr);
        else
            launch_timed(k_chunk_desc<KEY, LK, 4, true>, g4, dim3(DC_NT), 0, s, da, dbe, (const int64_t*)nullptr, geo,
                         nchunks, desc, ew, src, F0, M0, P0, (const int*)bsum, cpb, line, nbs, (int*)nullptr,
                         (Desc<KEY, LK>*)nullptr);
    } else {
        if (nchunks >= dc16_min)
            launch_timed(k_chunk_desc<KEY, LK, 16, false>, g16, dim3(DC_NT), 0, s, da, dbe, (const int64_t*)bounds,
                         geo, nchunks, desc, ew, (const KEY*)nullptr, (const FT*)nullptr, (const FT*)nullptr,
                         (const int*)nullptr, (const int*)nullptr, 0, false, 0, ovf, (Desc<KEY, LK>*)nullptr);
        else
            launch_timed(k_chunk_desc<KEY, LK, 4, false>, g4, dim3(DC_NT), 0, s, da, dbe, (const int64_t*)bounds, geo,
                         nchunks, desc, ew, (const KEY*)nullptr, (const FT*)nullptr, (const FT*)nullptr,
                         (const int*)nullptr, (const int*)nullptr, 0, false, 0, ovf, (Desc<KEY, LK>*)nullptr);
    }
    // the listed chunks' halves (k_mergek's extra workgroups merge them)
    if (split)
        k_split_desc<KEY, LK><<<SPLIT_WG, 64, 0, s>>>(src, F0, M0, P0, (const int*)bsum, cpb, geo,
                                                      (const int64_t*)bounds, ovf, dov, ew, line);
    // the capacity split: ovf_wg more workgroups walk the cut chunks' halves
    const unsigned grid = (unsigned)nchunks + (split ? ovf_wg<KEY, LK>() : 0);
    const uint32_t np = (uint32_t)nchunks;
    const Desc<KEY, LK>* dv = dov;
    const int* ov = ovf;
    // a binding hook: the launch carries its own events and ends the pass's
    // record; else marker events around it (nested in the pass's)
    const double kb = 2.0 * (double)n * sizeof(KEY);
    hipEvent_t ea = nullptr, eb = nullptr;
    const bool bound = hook && hook->binds();
    if (bound) (void)hook->bind(KIND_RUNSK_KERNEL, KIND_RUNSK, kb, &ea, &eb);
    else if (hook) hook->before(KIND_RUNSK_KERNEL, kb, s);
    if (lk_next > 0) {
        launch_timed(k_mergek<KEY, LK, true>, dim3(grid), dim3(S::NT), 0, s, ea, eb, src, dst,
                     (const Desc<KEY, LK>*)desc, Fn, lw + LK, lk_next, np, dv, ov);
    } else if (ord_out) {
        if constexpr (sizeof(KEY) == 8)
            launch_timed(k_mergek<KEY, LK, false, 0, true>, dim3(grid), dim3(S::NT), 0, s, ea, eb, src, dst,
                         (const Desc<KEY, LK>*)desc, (FT*)nullptr, 0, 0, np, dv, ov);
    } else {
        launch_timed(k_mergek<KEY, LK, false>, dim3(grid), dim3(S::NT), 0, s, ea, eb, src, dst,
                     (const Desc<KEY, LK>*)desc, (FT*)nullptr, 0, 0, np, dv, ov);
    }
    if (hook && !bound) hook->after(KIND_RUNSK_KERNEL, s);
    static const bool probe = getenv("MISORT_MK_PROBE") && atoi(getenv("MISORT_MK_PROBE")) != 0;
    if (probe && depth == 0) {
        // same chunks, outputs to a scratch buffer (the sort is untouched)
        static KEY* junk = nullptr;
        static size_t junk_n = 0;
        if (junk_n < (size_t)n) {
            if (junk) (void)hipFree(junk);
            junk = nullptr;
            if (hipMalloc(&junk, (size_t)n * sizeof(KEY)) != hipSuccess) return hipErrorOutOfMemory;
            junk_n = (size_t)n;
        }
        k_mergek<KEY, LK, false, 1><<<np, S::NT, 0, s>>>(src, junk, desc, nullptr, 0, 0, np, dv, ov);
        k_mergek<KEY, LK, false, 2><<<np, S::NT, 0, s>>>(src, junk, desc, nullptr, 0, 0, np, dv, ov);
        k_mergek<KEY, LK, false, 3><<<np, S::NT, 0, s>>>(src, junk, desc, nullptr, 0, 0, np, dv, ov);
    }
    return hipGetLastError();
}

template <typename KEY>
hipError_t merge_levelk_t(const KEY* src, KEY* dst, int64_t n, int lw, int lk, hipStream_t s, int phase, bool gather,
                          int lk_next, LaunchHook* hook, bool ord_out = false) {
    if (n <= 0) return hipSuccess;
    // load rows address a group with 32-bit byte offsets (KW * sizeof(KEY) <=
    // 2^32); runs at least a SORT tile long
    if (lk < 1 || lk > 4 || lw < KTr<KEY>::LW_MIN || lw + lk > KTr<KEY>::LWK_MAX || src == dst || lk_next < 0 ||
        lk_next > 4 || (ord_out && (sizeof(KEY) != 8 || lk_next > 0)))
        return hipErrorInvalidValue;
    if (lk == 1) return merge_pass<KEY, 1>(src, dst, n, lw, s, phase, gather, lk_next, hook, ord_out);
    if (lk == 2) return merge_pass<KEY, 2>(src, dst, n, lw, s, phase, gather, lk_next, hook, ord_out);
    if (lk == 3) return merge_pass<KEY, 3>(src, dst, n, lw, s, phase, gather, lk_next, hook, ord_out);
    return merge_pass<KEY, 4>(src, dst, n, lw, s, phase, gather, lk_next, hook, ord_out);
}

}  // namespace

int64_t MISORT_RUNSK_FN(mergek_chunks)(int64_t n, int lw, int lk, int key_bytes) {
    return key_bytes == 8 ? chunks_of(make_geo<uint64_t>(n, lw, lk)) : chunks_of(make_geo<uint32_t>(n, lw, lk));
}

// phase: which of the two fence buffers holds this pass's input fences
// (gather: build them from src first); lk_next > 0: write the next multi-way
// pass's fences (runs of 2^(lw+lk) in groups of 2^lk_next) into the other
// buffer.
hipError_t MISORT_RUNSK_FN(merge_levelk)(const uint32_t* src, uint32_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                        bool gather, int lk_next, LaunchHook* hook) {
    return merge_levelk_t<uint32_t>(src, dst, n, lw, lk, s, phase, gather, lk_next, hook);
}
hipError_t MISORT_RUNSK_FN(merge_levelk)(const uint64_t* src, uint64_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                        bool gather, int lk_next, LaunchHook* hook, bool ord_out) {
    return merge_levelk_t<uint64_t>(src, dst, n, lw, lk, s, phase, gather, lk_next, hook, ord_out);
}
void* MISORT_RUNSK_FN(mergek_fence_buffer)(int64_t n, int key_bytes, int phase, hipStream_t s) {
    // the sizes merge_pass computes, so the buffer never moves between the two
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    const size_t fb = ((size_t)nf * (key_bytes == 8 ? sizeof(u128) : sizeof(uint64_t)) + 255) & ~(size_t)255;
    char* fbase = (char*)scratch(0, 2 * fb, s);
    return fbase ? fbase + (phase & 1) * fb : nullptr;
}
// 1 if a merge pass on stream s rejected a chunk since the last call (the
// stream is synchronised), else 0; negative on a HIP error.
int MISORT_RUNSK_FN(mergek_take_error)(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    int* w = nullptr;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_errw.find({dev, s});
        if (it == g_errw.end()) return 0;
        w = it->second;
    }
    int v = 0;
    if (hipMemcpyAsync(&v, w, sizeof v, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    if (v && (hipMemsetAsync(w, 0, sizeof(int), s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)) return -1;
    return v ? 1 : 0;
}

// Frees the fence and planning scratch kept for stream s on the current
// device (misort_destroy, for the context's own stream).
void MISORT_RUNSK_FN(mergek_release)(hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> g(g_mu);
    auto ew = g_errw.find({dev, s});
    if (ew != g_errw.end()) {
        (void)hipStreamSynchronize(s);
        (void)hipFree(ew->second);
        g_errw.erase(ew);
    }
    for (auto& m : g_scr) {
        auto it = m.find({dev, s});
        if (it == m.end()) continue;
        if (it->second.p) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(it->second.p);
        }
        m.erase(it);
    }
}
#ifndef MISORT_RUNSK_SECOND
int merge_levelk_lw_min(int key_bytes) { return key_bytes == 8 ? KTr<uint64_t>::LW_MIN : KTr<uint32_t>::LW_MIN; }
int merge_levelk_lwk_max(int key_bytes) { return key_bytes == 8 ? KTr<uint64_t>::LWK_MAX : KTr<uint32_t>::LWK_MAX; }
#endif

}  // namespace misort
