// lds_merge.h -- the in-LDS merge machinery shared by the multi-way merge
// passes (runsk.hip, k_mergek) and the u32 SORT tile's merge levels
// (bitonic.h): merge-path co-rank searches, the per-lane merge chains, and the
// level loop that merges K sorted sequences already in LDS pairwise in LK
// levels.  Every sequence is followed by G words of MAX (sentinels), so the
// chains need no end checks.
#pragma once
#include "kernels.h"

namespace misort {
namespace {

template <typename KEY>
constexpr KEY KMAX = (KEY)~(KEY)0;

// A workgroup barrier for hand-offs through LDS only: waits for this wave's
// LDS operations, not for its global loads and stores.  __syncthreads() is a
// workgroup fence as well, s_waitcnt vmcnt(0) before the s_barrier, which
// would drain a prefetch of the next chunk at every merge level.  The memory
// clobber keeps the compiler from moving memory operations across it.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <typename KEY>
using kvec = KEY __attribute__((ext_vector_type(16 / sizeof(KEY))));  // 16 bytes of keys
template <typename KEY>
using kvec2 = KEY __attribute__((ext_vector_type(2)));

template <typename KEY>
using lds_t = __attribute__((address_space(3))) KEY;

template <typename KEY>
__device__ __forceinline__ uint32_t lds_addr(const KEY* p) {
    return (uint32_t)(uintptr_t)(const lds_t<KEY>*)p;
}
template <typename KEY>
__device__ __forceinline__ KEY lds_ld(uint32_t a) {
    return *(const lds_t<KEY>*)(uintptr_t)a;
}

// Merge-path co-rank: a valid split of the first d outputs of merge(A, B)
// (every A key before it <= every B key after it and vice versa; any such
// split gives the same output values -- the keys carry no payload).  The
// largest base in [lo, hi] with A[i - 1] <= B[d - i] for every i <= base, by
// power-of-two steps with clamped probes, no data-dependent branches: the
// steps 2^j <= maxr + PH, a uniform bound on hi - lo (<= min(LA, LB)) plus the
// phase, sum to >= hi - lo + PH.  Probe addresses stay inside [A0 - 1, A0 + LA)
// and [B0, B0 + LB].
//
// Phase: lane l of each 32-lane LDS group starts its search at lo - (l %
// 32) (positions <= lo count as true: the answer is >= lo).  With a common
// start, lanes whose bases differ at a coarse step differ by a multiple of 2 *
// step, so their A probes land in ONE bank (step >= 16): the searches were
// k_mergek's largest LDS cost (SQ probe modes, profiles/r04/sq_attr: 5
// conflict cycles per probe instruction).  The phases put those probes on
// distinct banks, and the B probes at (IT + 1) * l on distinct banks too:
// u32 k_mergek 2524 -> 2435 us per 2^30 pass (profiles/r04/phase); u64
// (two-bank keys, 4 waves per SIMD) measured 2667 -> 2739 us, so u64 keeps a
// common start.  Every probe is clamped into [lo, hi] and both loads are
// unconditional, one compare per step, no exec-mask branches (2274 -> 2144 us,
// profiles/r04/cor2).
// ZW (zero word): the word before every A sequence holds 0, a key <= every
// key (and B[LB] is a sentinel), so the probe at lo holds through the data:
// no i == lo test.  The probes then run on byte addresses of A (j = &A[i-1]; B's
// probe at C - j), five VALU and two LDS reads per step instead of seven VALU,
// an SALU or and two reads.
template <typename KEY, int MAXR, bool ZW = false>
__device__ __forceinline__ int co_rank(const KEY* s, int A0, int LA, int B0, int LB, int d, int maxr) {
    // first co-rank step: the largest power of two <= MAXR + PH (MAXR: a
    // compile-time bound on hi - lo, the steps must be powers of two for the
    // lifting search); steps above maxr + PH (uniform) are skipped
    constexpr int PH = sizeof(KEY) == 4 ? 31 : 0;
    constexpr int CO_STEP0 = 1 << (31 - __builtin_clz((unsigned)(MAXR + PH)));
    static_assert(MAXR + PH <= 2 * CO_STEP0 - 1, "co-rank steps cover the range");
    const int lo = d - LB > 0 ? d - LB : 0;
    const int hi = d < LA ? d : LA;
    const KEY* a = s + A0 - 1;
    const KEY* b = s + B0 + d;
    int base = lo - (PH ? (int)(__lane_id() & 31) : 0);
    if constexpr (ZW) {
        constexpr int W = (int)sizeof(KEY), WL = W == 4 ? 2 : 3;
        const int ab = (int)lds_addr<KEY>(a);
        const int C = ab + (int)lds_addr<KEY>(b);  // b[-i] at C - &a[i]
        const int jlo = ab + (lo << WL), jhi = ab + (hi << WL);
        int jb = ab + (base << WL);
#pragma unroll
        for (int step = CO_STEP0; step >= 1; step >>= 1) {
            if (step > maxr + PH) continue;  // uniform
            const int t = jb + (step << WL);
            int j;
            asm("v_med3_i32 %0, %1, %2, %3" : "=v"(j) : "v"(t), "v"(jlo), "v"(jhi));
            const bool ok = lds_ld<KEY>((uint32_t)j) <= lds_ld<KEY>((uint32_t)(C - j));
            jb = ok ? j : jb;
        }
        base = (jb - ab) >> WL;
        return base > lo ? base : lo;
    } else {
        // a probe at hi that holds makes hi the answer (later probes repeat
        // it); a step that ends below lo tests lo, which holds by definition
        // (the answer is >= lo) and moves base up to lo, within the steps
        // left; with a common start (PH = 0) no step ends below lo
#pragma unroll
        for (int step = CO_STEP0; step >= 1; step >>= 1) {
            if (step > maxr + PH) continue;  // uniform
            const int t = base + step;
            int i;  // clamp(t, lo, hi)
            asm("v_med3_i32 %0, %1, %2, %3" : "=v"(i) : "v"(t), "v"(lo), "v"(hi));
            const bool ok = (PH != 0 && i == lo) | (a[i] <= b[-i]);
            base = ok ? i : base;
        }
        return base > lo ? base : lo;
    }
}

// IT consecutive outputs from diagonal d of merge(s[A0, A0+LA), s[B0, B0+LB)),
// both followed by sentinels.  A chain holds h, the head of the side it took
// last, and g, the other side's head: each step outputs min(h, g), keeps
// max(h, g) as the other head and reads the next key of the side it took
// (swapping the two read pointers when that side changes) -- six VALU ops and
// one LDS read per output (u32).  Ties may go either way: equal keys are
// identical.  Past the end of both sequences a chain outputs MAX (their
// sentinels).
template <typename KEY, int IT, int MAXR, bool ZW = false>
__device__ __forceinline__ void merge_chain(const KEY* s, int A0, int LA, int B0, int LB, int d, int maxr,
                                            KEY (&r)[IT]) {
    const int tot = LA + LB;
    const int dc = d < tot ? d : tot;  // lanes past the end: MAX outputs, in-bounds reads
    const int ia = co_rank<KEY, MAXR, ZW>(s, A0, LA, B0, LB, dc, maxr);
    // byte addresses of the two heads (LDS pointers are 32-bit)
    uint32_t px = lds_addr<KEY>(s + A0 + ia), py = lds_addr<KEY>(s + B0 + dc - ia);
    KEY h = lds_ld<KEY>(px), g = lds_ld<KEY>(py);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool keep = h <= g;
        KEY o;
        if constexpr (sizeof(KEY) == 4) {
            r[k] = min(h, g);
            o = max(h, g);
        } else {  // no 64-bit min/max: selects on the compare (the compiler
                  // emits umin + umax, two v_cmp_u64; hiding the compared values
                  // from it, as cx<u64> does, measured 5 % slower here:
                  // 2.52 -> 2.64 ms per 16-way pass at 2^29, profiles/r03/ab2)
            r[k] = keep ? h : g;
            o = keep ? g : h;
        }
        const uint32_t nx = keep ? px : py;
        py = keep ? py : px;
        px = nx + (uint32_t)sizeof(KEY);
        h = lds_ld<KEY>(px);
        g = o;
    }
}

// Two consecutive keys at LDS byte address a (key-aligned: ds_read2_b32 /
// ds_read2_b64).  One wide read at the pair's alignment measured far slower
// (unaligned: 4.3 ms per 2^30 pass; the aligned-pair chain with its early-key
// handling: 2.26 -> 2.56 ms; profiles/r04/ab_chain, r05/zwpt).
template <typename KEY>
__device__ __forceinline__ kvec2<KEY> lds_ld2(uint32_t a) {
    typedef KEY v2 __attribute__((ext_vector_type(2), aligned(sizeof(KEY))));
    const v2 v = *(const __attribute__((address_space(3))) v2*)(uintptr_t)a;
    return kvec2<KEY>{v.x, v.y};
}

// The four keys of two ascending pairs (v0 <= v1, n0 <= n1) in order:
// s0 = min(v0, n0), s3 = max(v1, n1), and with a = max(v0, n0) <= max(v1, n1)
// the middle two are min(a, min(v1, n1)) and max(a, min(v1, n1)) -- for u32
// a v_min_u32, v_max_u32, v_min3_u32, v_med3_u32 and v_max_u32; for u64 three
// compares, each selecting both of its outputs.
[[maybe_unused]] __device__ __forceinline__ void merge4(uint32_t v0, uint32_t v1, uint32_t n0, uint32_t n1, uint32_t& s0, uint32_t& s1,
                                       uint32_t& s2, uint32_t& s3) {
    s0 = min(v0, n0);
    const uint32_t a = max(v0, n0);
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(s1) : "v"(a), "v"(v1), "v"(n1));  // (not formed from min(min()))
    s2 = max(min(a, v1), min(max(a, v1), n1));  // v_med3_u32
    s3 = max(v1, n1);
}
[[maybe_unused]] __device__ __forceinline__ void merge4(uint64_t v0, uint64_t v1, uint64_t n0, uint64_t n1, uint64_t& s0, uint64_t& s1,
                                       uint64_t& s2, uint64_t& s3) {
    const bool c0 = v0 < n0, c1 = v1 < n1;
    s0 = c0 ? v0 : n0;
    const uint64_t a = c0 ? n0 : v0, m = c1 ? v1 : n1;
    s3 = c1 ? n1 : v1;
    const bool c2 = a < m;
    s1 = c2 ? a : m;
    s2 = c2 ? m : a;
}

// The same IT outputs as merge_chain, two per step from blocks of two keys
// (a vector merge, as in Inoue et al.'s AA-sort).  The lane holds v0 <= v1,
// the two largest keys it has read and not yet output; v1, the largest key
// read, is the last key read from one side (L), so every unread key of L is
// >= v1, and the next two outputs are the lowest two of v and the next two
// keys of the other side (S).  A step reads those two keys (one LDS read),
// outputs the lowest two of the four and keeps the upper two; when the block's
// second key exceeds v1 the sides swap roles (the block's side now holds the
// largest key read).  Five VALU ops of merging and four of pointers per two
// outputs (u32) -- the one-key chain spends six VALU and an LDS read per
// output.  A side gives at most IT keys, so the G >= IT sentinels after each
// sequence cover every read.
template <typename KEY, int IT, int MAXR, bool ZW = false>
__device__ __forceinline__ void merge_chain_blk(const KEY* s, int A0, int LA, int B0, int LB, int d, int maxr,
                                                KEY (&r)[IT]) {
    static_assert(IT % 2 == 0, "two outputs per step");
    const int tot = LA + LB;
    const int dc = d < tot ? d : tot;
    const int ia = co_rank<KEY, MAXR, ZW>(s, A0, LA, B0, LB, dc, maxr);
    constexpr uint32_t B2 = 2 * sizeof(KEY);
    const uint32_t pa = lds_addr<KEY>(s + A0 + ia), pb = lds_addr<KEY>(s + B0 + dc - ia);
    const kvec2<KEY> a = lds_ld2<KEY>(pa), b = lds_ld2<KEY>(pb);
    // S: the side whose last read key is the smaller (ties: either)
    const bool as = a.y <= b.y;
    uint32_t ps = (as ? pa : pb) + B2, pl = (as ? pb : pa) + B2;
    KEY v0, v1;
    merge4(a.x, a.y, b.x, b.y, r[0], r[1], v0, v1);
#pragma unroll
    for (int k = 1; k < IT / 2; ++k) {
        const kvec2<KEY> n = lds_ld2<KEY>(ps);
        ps += B2;
        const bool sw = n.y > v1;
        merge4(v0, v1, n.x, n.y, r[2 * k], r[2 * k + 1], v0, v1);
        const uint32_t t = sw ? pl : ps;
        pl = sw ? ps : pl;
        ps = t;
    }
}

// Shape traits the level loop reads with defaults: ZW (a zero word before
// every A sequence, co_rank without its i == lo test; G > the keys a chain
// reads past a sequence).
template <typename S, typename = void>
struct shape_zw {
    static constexpr bool v = false;
};
template <typename S>
struct shape_zw<S, decltype((void)S::ZW)> {
    static constexpr bool v = S::ZW;
};
// UNI (the SORT tile's merge levels): all K sequences are S::RUN keys long and
// sequence q starts at q * (S::RUN + S::GS), so every level's pairs sit at a
// constant stride and a lane's pair is its position over that stride -- in
// place of per-pair selects on constants (a v_mov and a v_cndmask each).
template <typename S, typename = void>
struct shape_uni {
    static constexpr bool v = false;
};
template <typename S>
struct shape_uni<S, decltype((void)S::UNI)> {
    static constexpr bool v = S::UNI;
};
// A uniform shape's level lv: its input sequences' length and stride and its
// pairs' stride (level_geometry's rounding of each output + G up to QA).
template <typename S>
constexpr int uni_len(int lv) { return S::RUN << (lv - 1); }
template <typename S>
constexpr int uni_stride(int lv) {  // the stride of level lv's outputs (lv >= 1)
    return (2 * uni_len<S>(lv) + S::G + S::QA - 1) / S::QA * S::QA;
}
template <typename S>
constexpr int uni_in_stride(int lv) { return lv == 1 ? S::RUN + S::GS : uni_stride<S>(lv - 1); }

// The pair geometry of a level of P pairs over sequences of lengths ln[]:
// pair p's output starts at qp[p] (a multiple of QA past the previous pair's G
// sentinels) and holds lp[p] keys; maxr bounds its co-rank range (uniform).
template <typename S>
__device__ __forceinline__ void level_geometry(const int* ln, int P, int (&qp)[S::K / 2], int (&lp)[S::K / 2],
                                               int& maxr) {
    int qa = 0;
    maxr = 0;
#pragma unroll
    for (int p = 0; p < S::K / 2; ++p) {
        if (p >= P) break;
        const int mr = ln[2 * p] < ln[2 * p + 1] ? ln[2 * p] : ln[2 * p + 1];
        maxr = mr > maxr ? mr : maxr;
        lp[p] = ln[2 * p] + ln[2 * p + 1];
        qp[p] = qa;
        qa = (qa + lp[p] + S::G + S::QA - 1) / S::QA * S::QA;
    }
}

// Before the first level (the caller's barrier follows): for a ZW shape the
// zero word below the first sequence (those between sequences are the
// caller's: the last of the G words after each).
template <typename KEY, typename S>
__device__ __forceinline__ void lds_merge_prologue(KEY* s, const int (&st)[S::K], int tid) {
    if constexpr (shape_zw<S>::v) {
        if (tid == 0) s[st[0] - 1] = (KEY)0;
    }
}

// The in-LDS levels: K sequences at st[q] (length ln[q], each followed by G
// sentinels) merged pairwise in LK levels by NT lanes of IT outputs each.
// Level lv writes pair p's output at qp[p] (a multiple of QA past the
// previous pair's sentinels) with G sentinels after it; the last level's
// outputs stay in registers: lane tid holds outputs [tid * IT, tid * IT + IT)
// of the merged sequence as r[0, IT).  S (a shape): K, LKS, NT, IT, G, QA,
// CH (chain: 0 one key per read, 1 two), MAXR (bound on a pair's shorter
// sequence), optionally ZW (shape_zw: G - 1 MAX sentinels and a zero word
// after each sequence) and UNI (shape_uni).  MODE (probes,
// MISORT_MK_PROBE): 1 = no merging, 2 = first level only, 3 = co-rank searches
// without chains.  The pair of a lane: per-pair selects ((K/2 - 1) x 6 per
// lane; an LDS pair table measured slower, profiles/r05/zwpt) or, UNI, its
// position over the level's constant pair stride.  Ends with a barrier after
// the last level's reads (the caller may then overwrite the LDS).
template <typename KEY, typename S, int MODE>
__device__ __forceinline__ void lds_merge_levels(KEY* s, int (&st)[S::K], int (&ln)[S::K], KEY (&r)[S::IT], int tid,
                                                 int LAST) {
    constexpr int K = S::K, LK = S::LKS, NT = S::NT, IT = S::IT, G = S::G, CH = S::CH;
    constexpr bool ZW = shape_zw<S>::v;
    static_assert(CH == 0 || CH == 1, "one- or two-key chains");
    // a two-key chain reads at most IT keys past a sequence (the one-key chain
    // IT + 1), so the G-th word after it is free for the next sequence's zero word
    static_assert(!ZW || (CH == 1 && G > IT) || (CH == 0 && G > IT + 1),
                  "zero words: a sentinel word past the chain's reads");
    constexpr KEY MAXK = KMAX<KEY>;
    const int pos = tid * IT;
    const int wpos = __builtin_amdgcn_readfirstlane(tid & ~63) * IT;  // the wave's first lane
#pragma unroll
    for (int lv = 1; lv <= LK; ++lv) {
        const int P = K >> lv;  // pairs merged at this level
        // pair p's output: [qp[p], qp[p] + lp[p]), then G sentinels; the next
        // pair starts at the first lane boundary past them
        int qp[K / 2], lp[K / 2];
        int maxr;  // the longest co-rank range of the level's pairs (uniform)
        level_geometry<S>(ln, P, qp, lp, maxr);
        // uniform: the co-rank searches skip their long steps by scalar
        // branches (a maxr the compiler left in a VGPR costs every step a
        // compare and an exec-mask save / restore)
        maxr = __builtin_amdgcn_readfirstlane(maxr);
        // the lane's pair: the last one starting at or before pos
        int A0 = st[0], LA = ln[0], B0 = st[1], LB = ln[1], Q = 0, LP = lp[0];
        if (P > 1) {
            if constexpr (shape_uni<S>::v) {
                const int SL = uni_stride<S>(lv), SI = uni_in_stride<S>(lv), L0 = uni_len<S>(lv);
                int pi = pos / SL;
                pi = pi < P - 1 ? pi : P - 1;
                A0 = 2 * pi * SI;
                LA = L0;
                B0 = A0 + SI;
                LB = L0;
                Q = pi * SL;
                LP = 2 * L0;
            } else {
#pragma unroll
                for (int p = 1; p < K / 2; ++p) {
                    if (p >= P) break;
                    const bool in = pos >= qp[p];
                    A0 = in ? st[2 * p] : A0;
                    LA = in ? ln[2 * p] : LA;
                    B0 = in ? st[2 * p + 1] : B0;
                    LB = in ? ln[2 * p + 1] : LB;
                    Q = in ? qp[p] : Q;
                    LP = in ? lp[p] : LP;
                }
            }
        }
        const int end = qp[P - 1] + lp[P - 1];
        if (MODE == 1 || (MODE == 2 && lv > 1) || MODE == 3) {
#pragma unroll
            for (int j = 0; j < IT; ++j) r[j] = s[pos + j < LAST ? pos + j : LAST];
            if (MODE == 3 && wpos < end) {  // the search alone, its result kept alive
                const int dc = pos - Q < LA + LB ? pos - Q : LA + LB;
                r[0] ^= (KEY)(co_rank<KEY, S::MAXR, ZW>(s, A0, LA, B0, LB, dc, maxr) & 1);
            }
        } else if (wpos < end) {
            if constexpr (CH == 0)
                merge_chain<KEY, IT, S::MAXR, ZW>(s, A0, LA, B0, LB, pos - Q, maxr, r);
            else
                merge_chain_blk<KEY, IT, S::MAXR, ZW>(s, A0, LA, B0, LB, pos - Q, maxr, r);
        }
        lds_barrier();
        if (lv < LK) {
            // a lane's outputs past its pair's end are MAX (the chain ran into
            // the sentinels), the value the sentinel stores write there too
            if (pos < Q + LP) {
                if constexpr (IT % 2) {
#pragma unroll
                    for (int k = 0; k < IT; ++k) s[pos + k] = r[k];
                } else {
#pragma unroll
                    for (int j = 0; j < IT; j += 2)
                        *reinterpret_cast<kvec2<KEY>*>(s + pos + j) = kvec2<KEY>{r[j], r[j + 1]};
                }
            }
            // ZW: G - 1 MAX words after each output and a zero word below each
            // pair's output but the first (the next level's A sequences start
            // there; the one below the first was written once)
            constexpr int GW = ZW ? G - 1 : G;
            for (int x = tid; x < P * GW; x += NT) {
                const int p = x / GW;
                int e = 0;
#pragma unroll
                for (int q = 0; q < K / 2; ++q)
                    if (q < P) e = p == q ? qp[q] + lp[q] : e;
                s[e + (x - p * GW)] = MAXK;
            }
            if constexpr (ZW) {
                // the last wave's lanes 1 .. P-1 (its lanes past the sentinel loop's)
                const int zl = tid - (NT - 64);
                if (zl >= 1 && zl < P) {
                    int e = 0;
#pragma unroll
                    for (int q = 1; q < K / 2; ++q)
                        if (q < P) e = zl == q ? qp[q] : e;
                    s[e - 1] = (KEY)0;
                }
            }
            lds_barrier();
#pragma unroll
            for (int p = 0; p < K / 2; ++p) {
                if (p >= P) break;
                st[p] = qp[p];
                ln[p] = lp[p];
            }
        }
    }
}

}  // namespace
}  // namespace misort
