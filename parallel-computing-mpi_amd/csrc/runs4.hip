// runs4.hip -- 4-way merge passes of the local sort (gfx950, u32 keys):
// ascending runs of W = 2^lw keys, in groups of four, -> ascending runs of 4W.
// One HBM read + one HBM write per key for TWO merge levels (runs.hip does one
// level per pass).
//
// The reference's local sort is std::sort (psort.cc:175); any correct sort of
// payload-free keys writes the same bytes, so the levels past the bitonic SORT
// tile are merges.  A 4-way merge needs, for each output chunk, its start in
// all four runs.  Exact fixed-size tiles would need a 4-way merge-path
// co-rank per tile (nested searches); instead the chunks are cut at FENCES:
//
//   fence   = the key at every FG-th position of a run, packed with its place
//             as (key << 32 | run-in-group << 30 | position / FG), so that u64
//             order is the total order (key, run, position) -- ties between
//             equal keys go to the lower run, then the lower position;
//   chunks  = the fences of a group merged into that total order (k_fence_lds
//             or two u64 merge levels), every FM-th one starting a chunk;
//   bounds  = for a chunk-start fence f of run r0 at position j0*FG, run r0
//             starts at j0*FG and every other run r at its count of keys
//             before f, found by a binary search confined to the FG positions
//             between two of run r's own fences (k_bounds4);
//   merge   = one workgroup per chunk (k_merge4): the four segments are
//             streamed into LDS, merged pairwise then once more in LDS, and
//             stored through LDS as 16-byte non-temporal stores; the keys at
//             every FG-th output position are written as the next pass's
//             fences.
//
// Between two consecutive chunk starts lie FM fences; run r contributes at
// most (its fences there + 1) * FG keys, so a chunk holds at most
// (FM + 4) * FG = CAP keys and FM * FG on average.  The first 4-way pass after
// the SORT tile gathers its fences from the runs (k_fence_gather); later
// passes read the fences the previous pass wrote.
#include "kernels.h"

#include <map>
#include <mutex>

namespace misort {
namespace {

constexpr int FG_LOG2 = 8;
constexpr int64_t FG = (int64_t)1 << FG_LOG2;  // fence stride (keys)
constexpr int FM = 28;                          // fences per chunk
constexpr int CAP = (FM + 4) * (int)FG;         // most keys of a chunk (8192; 7168 on average)
#ifndef MISORT_M4_NT
#define MISORT_M4_NT 512
#endif
constexpr int NT = MISORT_M4_NT;                // lanes per chunk workgroup
constexpr int IT = NT == 256 ? 36 : 18;         // keys per lane
// persistent grid: workgroups per CU the register budget is sized for (the
// LDS tile allows 4)
constexpr int WG_PER_CU = 4;
// load rows: RW consecutive keys of one segment; a lane's load slot j holds
// row j * (NT / RW) + tid / RW -- one row per wave and slot
constexpr int RW = 256;
constexpr int NROWS = IT * NT / RW;
// Every sequence an in-LDS merge reads is followed by G words of MAX
// (sentinels), so a merge chain needs no end checks: it reads at most IT words
// past an exhausted sequence.  Level 1 places the second pair's output at a
// lane boundary past the first pair's sentinels (no lane straddles two
// pairs); that layout needs 4 lanes' worth of room beyond CAP.  A chunk is
// loaded in rows of NT keys, each row within one segment, so the four
// segments take at most CAP/NT + 4 rows of the lanes' IT load slots.
constexpr int G = IT + 1;
static_assert(CAP <= (NT - 4) * IT, "chunk tile shape (level-1 layout)");
static_assert(CAP <= (NROWS - 4) * RW, "chunk tile shape (segment rows)");
constexpr int PAD = 4;  // words below the tile: a co-rank probe may read index -1
constexpr int LDS_WORDS = PAD + CAP + 4 * G + 2 * IT + 16;
constexpr uint64_t J_MASK = ((uint64_t)1 << 30) - 1;

typedef uint32_t vec4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) { return (uint32_t)(uintptr_t)(const lds_u32*)p; }
__device__ __forceinline__ uint32_t lds_ld(uint32_t a) { return *(const lds_u32*)(uintptr_t)a; }

__device__ __forceinline__ uint64_t fpack(uint32_t key, int64_t gp, int lw) {
    const uint64_t r = (uint64_t)(gp >> lw) & 3;
    const uint64_t j = (uint64_t)(gp & (((int64_t)1 << lw) - 1)) >> FG_LOG2;
    return ((uint64_t)key << 32) | (r << 30) | j;
}

// Group geometry of the pass: groups of 4 runs of W keys; run r of group g
// starts at g*4W + r*W and holds clamp(n - start, 0, W) keys.
struct Geo4 {
    int64_t n;
    int lw;
    int64_t nfull;  // full groups
    int64_t kf;     // chunks per full group
    __device__ __host__ int64_t W() const { return (int64_t)1 << lw; }
    __device__ __host__ int64_t base(int64_t g) const { return g << (lw + 2); }
    __device__ __host__ int64_t run_len(int64_t g, int r) const {
        const int64_t st = base(g) + r * W();
        const int64_t rest = n - st;
        return rest <= 0 ? 0 : (rest < W() ? rest : W());
    }
    __device__ __host__ int64_t nfences(int64_t g) const {
        const int64_t glen = (n - base(g)) < 4 * W() ? n - base(g) : 4 * W();
        return (glen + FG - 1) >> FG_LOG2;
    }
    __device__ __host__ int64_t nchunks(int64_t g) const { return (nfences(g) + FM - 1) / FM; }
    // bounds slot of chunk t of group g (each group has nchunks + 1 slots)
    __device__ __host__ int64_t slot(int64_t g, int64_t t) const {
        return g < nfull ? g * (kf + 1) + t : nfull * (kf + 1) + t;
    }
};

// F[i] = fence of position i*FG (the first 4-way pass after the SORT tile).
__global__ void k_fence_gather(const uint32_t* __restrict__ src, int64_t n, int lw, uint64_t* __restrict__ F) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    if (i >= nf) return;
    const int64_t gp = i << FG_LOG2;
    F[i] = fpack(src[gp], gp, lw);
}

// The fences of one group (<= 4 * 2048) merged into total order in LDS: each
// fence's rank = its index in its run's list + its lower bound in the others.
__global__ __launch_bounds__(1024) void k_fence_lds(const uint64_t* __restrict__ F, uint64_t* __restrict__ M,
                                                    Geo4 geo) {
    extern __shared__ uint64_t sf[];
    const int64_t g = blockIdx.x;
    const int64_t f0 = geo.base(g) >> FG_LOG2;
    const int nfg = (int)geo.nfences(g);
    const int wf = (int)(geo.W() >> FG_LOG2);  // fences per full run
    for (int e = threadIdx.x; e < nfg; e += blockDim.x) sf[e] = F[f0 + e];
    __syncthreads();
    for (int e = threadIdx.x; e < nfg; e += blockDim.x) {
        const uint64_t v = sf[e];
        const int r = e / wf;
        int rank = e - r * wf;
        for (int q = 0; q < 4; ++q) {
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

// One thread per bounds slot: the start of chunk t of group g in each of the
// group's four runs (positions within the runs), or the runs' lengths for the
// group's end slot.
__global__ void k_bounds4(const uint32_t* __restrict__ src, const uint64_t* __restrict__ F,
                          const uint64_t* __restrict__ M, Geo4 geo, int64_t nslots,
                          int64_t* __restrict__ bounds) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    int64_t g, t;
    if (s < geo.nfull * (geo.kf + 1)) {
        g = s / (geo.kf + 1);
        t = s - g * (geo.kf + 1);
    } else {
        g = geo.nfull;
        t = s - geo.nfull * (geo.kf + 1);
    }
    int64_t* out = bounds + 4 * s;
    const int64_t base = geo.base(g), W = geo.W();
    if (t == geo.nchunks(g)) {
        for (int r = 0; r < 4; ++r) out[r] = geo.run_len(g, r);
        return;
    }
    const uint64_t f = M[(base >> FG_LOG2) + t * FM];
    const uint32_t v = (uint32_t)(f >> 32);
    const int r0 = (int)((f >> 30) & 3);
    for (int r = 0; r < 4; ++r) {
        const int64_t len = geo.run_len(g, r);
        if (r == r0) {
            out[r] = (int64_t)(f & J_MASK) << FG_LOG2;
            continue;
        }
        if (len == 0) {
            out[r] = 0;
            continue;
        }
        // fences of run r before f (packed u64 compare = total order)
        const uint64_t* fr = F + ((base + r * W) >> FG_LOG2);
        int64_t lo = 0, hi = (len + FG - 1) >> FG_LOG2;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (fr[mid] < f) lo = mid + 1;
            else hi = mid;
        }
        if (lo == 0) {  // run r's first key comes after f
            out[r] = 0;
            continue;
        }
        // keys before f: all of positions <= (lo-1)*FG, none from lo*FG on
        const uint32_t* kr = src + base + r * W;
        int64_t a = ((lo - 1) << FG_LOG2) + 1, b = (lo << FG_LOG2) < len ? (lo << FG_LOG2) : len;
        while (a < b) {  // first position after f: key > v (r < r0) or key >= v (r > r0)
            const int64_t mid = (a + b) >> 1;
            const uint32_t k = kr[mid];
            if (r < r0 ? k <= v : k < v) a = mid + 1;
            else b = mid;
        }
        out[r] = a;
    }
}

// Merge-path co-rank: a valid split of the first d outputs of merge(A, B)
// (every A key before it <= every B key after it and vice versa; any such
// split gives the same output values -- the keys carry no payload).  The
// largest base in [lo, hi] with A[i - 1] <= B[d - i] for every i <= base, by
// 13 power-of-two steps (hi - lo <= min(LA, LB) <= CAP/2 = 2^12) with clamped
// probes: no loop control, no branches.  Probe addresses stay inside
// [A0 - 1, A0 + LA) and [B0, B0 + LB].
__device__ __forceinline__ int co_rank(const uint32_t* s, int A0, int LA, int B0, int LB, int d) {
    static_assert(CAP / 2 <= 4096 * 2 - 1, "co-rank steps");
    const int lo = d - LB > 0 ? d - LB : 0;
    const int hi = d < LA ? d : LA;
    const uint32_t* a = s + A0 - 1;
    const uint32_t* b = s + B0 + d;
    int base = lo;
#pragma unroll
    for (int step = 4096; step >= 1; step >>= 1) {
        const int i = base + step;
        const int ic = i < hi ? i : hi;
        const bool ok = i <= hi && a[ic] <= b[-ic];
        base = ok ? i : base;
    }
    return base;
}

// IT consecutive outputs from diagonal d of merge(s[A0, A0+LA), s[B0, B0+LB)),
// both followed by sentinels.  A chain holds h, the head of the side it took
// last, and g, the other side's head: each step outputs min(h, g), keeps
// max(h, g) as the other head and reads the next key of the side it took
// (swapping the two read pointers when that side changes) -- six VALU ops and
// one LDS read per output.  Ties may go either way: equal keys are identical.
// Past the end of both sequences a chain outputs MAX (their sentinels).
__device__ __forceinline__ void merge_chain(const uint32_t* s, int A0, int LA, int B0, int LB, int d,
                                            uint32_t (&r)[IT]) {
    const int tot = LA + LB;
    const int dc = d < tot ? d : tot;  // lanes past the end: MAX outputs, in-bounds reads
    const int ia = co_rank(s, A0, LA, B0, LB, dc);
    // byte addresses of the two heads (LDS pointers are 32-bit)
    uint32_t px = lds_addr(s + A0 + ia), py = lds_addr(s + B0 + dc - ia);
    uint32_t h = lds_ld(px), g = lds_ld(py);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const bool keep = h <= g;
        r[k] = min(h, g);
        const uint32_t o = max(h, g);
        const uint32_t nx = keep ? px : py;
        py = keep ? py : px;
        px = nx + 4;
        h = lds_ld(px);
        g = o;
    }
}

// Chunk descriptors: for chunk c, its group's base, its output offset, the
// chunk positions where its four segments start, and its LOAD ROWS.  A chunk
// is loaded in NROWS rows of RW consecutive keys, each row inside one segment
// (segment r takes ceil(l_r / RW) rows; the four take <= CAP/RW + 4 = NROWS):
// row j = byte offset of its first key from the group base, and how many of
// its NT keys are real plus the LDS word the first goes to (segment r's keys
// start at LDS word o_r + r*G, leaving G words for sentinels after each).
// Validated so that no chunk can address memory outside its group's runs:
// a bad chunk gets no rows and is left unwritten (the sort then fails its
// checks).
struct Desc {
    int64_t gbase, out0;
    int o1, o2, o3, len;
    uint32_t off[NROWS];  // row j: byte offset of its first key from the group base
    uint32_t la[NROWS];   // row j: real keys (0..RW) | LDS word of its first key << 16
};
static_assert(CAP + 4 * (IT + 1) < 65536, "LDS word fits 16 bits");

// One thread per (chunk, row); row slot NROWS writes the header.
__global__ void k_chunk_desc(const int64_t* __restrict__ bounds, Geo4 geo, int64_t nchunks, Desc* __restrict__ desc) {
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= nchunks * (NROWS + 1)) return;
    const int64_t c = id / (NROWS + 1);
    const int j = (int)(id - c * (NROWS + 1));
    int64_t g, t;
    if (c < geo.nfull * geo.kf) {
        g = c / geo.kf;
        t = c - g * geo.kf;
    } else {
        g = geo.nfull;
        t = c - geo.nfull * geo.kf;
    }
    const int64_t* b0 = bounds + 4 * geo.slot(g, t);
    int64_t st[4], ln[4], tot = 0;
    bool ok = true;
    for (int r = 0; r < 4; ++r) {
        st[r] = b0[r];
        ln[r] = b0[4 + r] - st[r];
        ok = ok && st[r] >= 0 && ln[r] >= 0 && st[r] + ln[r] <= geo.run_len(g, r);
        tot += ok ? ln[r] : 0;
    }
    ok = ok && tot <= CAP;
    // bounds outside the runs would be a logic error: never let them address memory
    if (!ok)
        for (int r = 0; r < 4; ++r) st[r] = ln[r] = 0;
    Desc& d = desc[c];
    if (j == NROWS) {
        d.gbase = geo.base(g);
        d.out0 = geo.base(g) + st[0] + st[1] + st[2] + st[3];
        d.o1 = (int)ln[0];
        d.o2 = (int)(ln[0] + ln[1]);
        d.o3 = (int)(ln[0] + ln[1] + ln[2]);
        d.len = (int)(ln[0] + ln[1] + ln[2] + ln[3]);
        return;
    }
    int R = 0, o = 0;
    uint32_t off = 0, la = 0;
    for (int r = 0; r < 4; ++r) {
        const int rows = (int)((ln[r] + RW - 1) / RW);
        if (j >= R && j < R + rows) {
            const int k = j - R;
            const int64_t rem = ln[r] - (int64_t)k * RW;
            off = (uint32_t)((((int64_t)r << geo.lw) + st[r] + (int64_t)k * RW) * 4);  // < 4W*4 <= 2^32 (lw <= 28)
            la = (uint32_t)(rem < RW ? rem : RW) | ((uint32_t)(o + r * G + k * RW) << 16);
        }
        R += rows;
        o += (int)ln[r];
    }
    d.off[j] = off;
    d.la[j] = la;  // rows past the chunk: no keys
}

// The wave's row half (uniform) and the lane's place in its row.
__device__ __forceinline__ int row_half(int tid) { return __builtin_amdgcn_readfirstlane(tid) / RW; }

__device__ __forceinline__ void chunk_loads(const uint32_t* src, const Desc* d, int tid, uint32_t (&x)[IT]) {
    const char* gsrc = (const char*)(src + d->gbase);
    const int h = row_half(tid), lt = tid & (RW - 1);
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const int row = j * (NT / RW) + h;
        const int lim = (int)(d->la[row] & 0xFFFF);
        if (lt < lim) x[j] = __builtin_nontemporal_load((const uint32_t*)(gsrc + d->off[row]) + (uint32_t)lt);
    }
}

// Row j's real keys go to their LDS words; then the G sentinel words after
// every segment.
__device__ __forceinline__ void chunk_to_lds(uint32_t* s, const Desc* d, int tid, const uint32_t (&x)[IT]) {
    const int h = row_half(tid), lt = tid & (RW - 1);
#pragma unroll
    for (int j = 0; j < IT; ++j) {
        const uint32_t la = d->la[j * (NT / RW) + h];
        if (lt < (int)(la & 0xFFFF)) s[(la >> 16) + lt] = x[j];
    }
    if (tid < 4 * G) {
        const int r = tid / G, i = tid - r * G;
        const int end = r == 0 ? d->o1 : r == 1 ? d->o2 : r == 2 ? d->o3 : d->len;
        s[end + r * G + i] = 0xFFFFFFFFu;
    }
}

// The two in-LDS merge levels of a chunk, its stores and fences.  MODE
// (probes only, MISORT_M4_PROBE): 0 = the pass; 1 = no merge (the access
// pattern's floor); 2 = level 1 only.  Waves whose lanes all lie past a
// level's outputs skip its merge (a chunk averages 7168 of 9216 lane slots).
template <bool FENCES, int MODE>
__device__ __forceinline__ void chunk_merge(uint32_t* s, const Desc* dc, int tid, uint32_t* __restrict__ dst,
                                            uint64_t* __restrict__ fout, int lwn) {
    const int o1 = dc->o1, o2 = dc->o2, o3 = dc->o3, len = dc->len;
    const int l0 = o1, l1 = o2 - o1, l2 = o3 - o2, l3 = len - o3;
    constexpr int LAST = LDS_WORDS - PAD - 1;
    uint32_t r[IT];
    const int pos = tid * IT;
    const int wpos = __builtin_amdgcn_readfirstlane(tid & ~63) * IT;  // the wave's first lane
    // level 1: segments at e + r*G (chunk_to_lds).  A ++ B -> [0, o2) and
    // C ++ D -> [q2, q2 + l2 + l3), q2 = the first lane boundary past A ++ B's
    // sentinels [o2, o2 + G); sentinels follow C ++ D too
    const int q2 = (o2 + G + IT - 1) / IT * IT, end1 = q2 + (len - o2);
    const bool p1 = pos < o2;
    const bool act = p1 || (pos >= q2 && pos < end1);
    if constexpr (MODE == 1) {
#pragma unroll
        for (int j = 0; j < IT; ++j) r[j] = s[pos + j < LAST ? pos + j : LAST];
    } else if (wpos < end1) {
        const int d = p1 ? pos : (pos > q2 ? pos - q2 : 0);
        merge_chain(s, p1 ? 0 : o2 + 2 * G, p1 ? l0 : l2, p1 ? o1 + G : o3 + 3 * G, p1 ? l1 : l3, d, r);
    }
    __syncthreads();
    // a lane's outputs past its pair's end are MAX (the chain ran into the
    // sentinels), the same value the sentinel stores write there
    if (act) {
        typedef uint32_t vec2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int j = 0; j < IT; j += 2) *reinterpret_cast<vec2*>(s + pos + j) = vec2{r[j], r[j + 1]};
    }
    if (tid < 2 * G) s[tid < G ? o2 + tid : end1 + tid - G] = 0xFFFFFFFFu;
    __syncthreads();
    // level 2: [0, o2) ++ [q2, end1) -> the chunk
    if constexpr (MODE != 0) {
#pragma unroll
        for (int j = 0; j < IT; ++j) r[j] = s[pos + j < LAST ? pos + j : LAST];
    } else if (wpos < len) {
        merge_chain(s, 0, o2, q2, len - o2, pos, r);
    }
    __syncthreads();
    // the chunk goes to LDS shifted by out0 mod 4, so every global 16-byte
    // vector is one aligned LDS vector (a lane's outputs past len are MAX and
    // land past the chunk)
    const int64_t out0 = dc->out0;
    const int sh = (int)(out0 & 3);
    if (pos < len) {
        uint32_t* q = s + sh + pos;
#pragma unroll
        for (int j = 0; j < IT; ++j) q[j] = r[j];
    }
    __syncthreads();
    const int nv = (sh + len + 3) >> 2;
    uint32_t* __restrict__ o = dst + (out0 - sh);
    for (int v = tid; v < nv; v += NT) {
        const int e = 4 * v;
        if (e >= sh && e + 4 <= sh + len) {
            __builtin_nontemporal_store(*reinterpret_cast<const vec4*>(s + e), reinterpret_cast<vec4*>(o + e));
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (e + j >= sh && e + j < sh + len) o[e + j] = s[e + j];
        }
    }
    if constexpr (FENCES) {
        // the chunk's fences are consecutive entries of fout: one coalesced
        // 8-byte store per fence from consecutive lanes
        const int64_t first = (out0 + FG - 1) & ~(FG - 1);
        const int nf = first < out0 + len ? (int)((out0 + len - first + FG - 1) >> FG_LOG2) : 0;
        if (tid < nf) {
            const int64_t gp = first + ((int64_t)tid << FG_LOG2);
            fout[gp >> FG_LOG2] = fpack(s[(int)(gp - (out0 - sh))], gp, lwn);
        }
    }
}

// Persistent workgroups walk the chunks; the next chunk's 36 loads per lane
// are in flight (registers) while the current chunk merges, so the HBM
// stream does not stop during the LDS phases.
template <bool FENCES, int MODE = 0>
__global__ __launch_bounds__(NT, WG_PER_CU * NT / 256) void k_merge4(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                               Geo4 geo, const Desc* __restrict__ desc,
                                               uint64_t* __restrict__ fout, int64_t nchunks) {
    __shared__ __attribute__((aligned(16))) uint32_t s_tile[LDS_WORDS];
    uint32_t* s = s_tile + PAD;
    const int tid = threadIdx.x;
    int64_t c = blockIdx.x;
    if (c >= nchunks) return;
    uint32_t x[IT];
    chunk_loads(src, desc + c, tid, x);
    for (;;) {
        // lane id through an opaque copy: lane-derived addresses are recomputed
        // every chunk instead of being hoisted into loop-invariant VGPRs, which
        // spilled -- and a spill reload waits (in-order vmcnt) for the whole
        // prefetch issued before it
        int t = threadIdx.x;
        asm volatile("" : "+v"(t));
        chunk_to_lds(s, desc + c, t, x);
        __syncthreads();
        const int64_t cn = c + gridDim.x;
        if (cn < nchunks) chunk_loads(src, desc + cn, t, x);
        chunk_merge<FENCES, MODE>(s, desc + c, t, dst, fout, geo.lw + 2);
        if (cn >= nchunks) break;
        __syncthreads();  // the next chunk overwrites the tile
        c = cn;
    }
}

// Fence buffers and bounds: one grow-only set per (device, stream).
struct Scratch4 {
    void* p = nullptr;
    size_t bytes = 0;
};
std::mutex g_mu4;
std::map<std::pair<int, hipStream_t>, Scratch4> g_scr4;

void* scratch4(size_t bytes, hipStream_t s) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(g_mu4);
    auto& e = g_scr4[{dev, s}];
    if (e.bytes < bytes) {
        if (e.p && (hipStreamSynchronize(s) != hipSuccess || hipFree(e.p) != hipSuccess)) return nullptr;
        e = Scratch4{};
        void* p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
        e = Scratch4{p, bytes};
    }
    return e.p;
}

}  // namespace

int64_t merge4_chunks(int64_t n, int lw) {
    Geo4 geo{n, lw, 0, 0};
    geo.nfull = n >> (lw + 2);
    geo.kf = ((((int64_t)4 << lw) >> FG_LOG2) + FM - 1) / FM;  // chunks of a full group
    const int64_t tail = geo.nfull << (lw + 2) < n ? geo.nchunks(geo.nfull) : 0;
    return geo.nfull * geo.kf + tail;
}

// phase: which of the two fence buffers holds this pass's input fences
// (gather: build them from src first); write_next: write the next 4-way
// pass's fences into the other buffer.
hipError_t merge_level4(const uint32_t* src, uint32_t* dst, int64_t n, int lw, hipStream_t s, int phase,
                        bool gather, bool write_next) {
    if (n <= 0) return hipSuccess;
    // load rows address a group with 32-bit byte offsets (4W*4 <= 2^32); runs at least CAP long
    if (lw < 15 || lw > 28 || src == dst) return hipErrorInvalidValue;
    Geo4 geo{n, lw, 0, 0};
    geo.nfull = n >> (lw + 2);
    geo.kf = ((((int64_t)4 << lw) >> FG_LOG2) + FM - 1) / FM;  // chunks of a full group
    const bool tail = (geo.nfull << (lw + 2)) < n;
    const int64_t nchunks = geo.nfull * geo.kf + (tail ? geo.nchunks(geo.nfull) : 0);
    const int64_t nslots = geo.nfull * (geo.kf + 1) + (tail ? geo.nchunks(geo.nfull) + 1 : 0);
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    // layout: fence buffers 0 and 1, merged fences, u64 merge temp, bounds
    const size_t fb = ((size_t)nf * 8 + 255) & ~(size_t)255;
    const size_t bb = ((size_t)nslots * 32 + 255) & ~(size_t)255;
    char* base = (char*)scratch4(4 * fb + bb + (size_t)nchunks * sizeof(Desc) + 256, s);
    if (!base) return hipErrorOutOfMemory;
    uint64_t* F = (uint64_t*)(base + (phase & 1) * fb);
    uint64_t* Fn = (uint64_t*)(base + ((phase & 1) ^ 1) * fb);
    uint64_t* M = (uint64_t*)(base + 2 * fb);
    uint64_t* T = (uint64_t*)(base + 3 * fb);
    int64_t* bounds = (int64_t*)(base + 4 * fb);
    Desc* desc = (Desc*)(base + 4 * fb + bb);
    if (gather) k_fence_gather<<<(unsigned)((nf + 255) / 256), 256, 0, s>>>(src, n, lw, F);
    const int wf_log2 = lw - FG_LOG2;  // fences per run = 2^wf_log2
    if (wf_log2 <= 11) {  // group fences <= 8192: 64 KiB of LDS
        const int ngroups = (int)(geo.nfull + (tail ? 1 : 0));
        const size_t lds = ((size_t)4 << wf_log2) * 8;
        k_fence_lds<<<ngroups, 1024, lds, s>>>(F, M, geo);
    } else {
        hipError_t e = merge_level<uint64_t>(F, T, nf, wf_log2, s);
        if (e == hipSuccess) e = merge_level<uint64_t>(T, M, nf, wf_log2 + 1, s);
        if (e != hipSuccess) return e;
    }
    k_bounds4<<<(unsigned)((nslots + 255) / 256), 256, 0, s>>>(src, F, M, geo, nslots, bounds);
    k_chunk_desc<<<(unsigned)((nchunks * (NROWS + 1) + 255) / 256), 256, 0, s>>>(bounds, geo, nchunks, desc);
    static int64_t cap = 0;  // resident workgroups (the persistent grid)
    if (cap == 0) {
        int per_cu = 0, cus = 0, dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_merge4<true>, NT, 0);
        cap = (int64_t)(per_cu < 1 ? 1 : per_cu) * (cus < 1 ? 1 : cus);
    }
    const unsigned grid = (unsigned)(nchunks < cap ? nchunks : cap);
    if (write_next) k_merge4<true><<<grid, NT, 0, s>>>(src, dst, geo, desc, Fn, nchunks);
    else k_merge4<false><<<grid, NT, 0, s>>>(src, dst, geo, desc, nullptr, nchunks);
    static const bool probe = getenv("MISORT_M4_PROBE") && atoi(getenv("MISORT_M4_PROBE")) != 0;
    if (probe) {
        // same chunks and bounds, outputs to a scratch buffer (the sort is untouched)
        static uint32_t* junk = nullptr;
        static size_t junk_n = 0;
        if (junk_n < (size_t)n) {
            if (junk) (void)hipFree(junk);
            junk = nullptr;
            if (hipMalloc(&junk, (size_t)n * 4) != hipSuccess) return hipErrorOutOfMemory;
            junk_n = (size_t)n;
        }
        k_merge4<false, 1><<<grid, NT, 0, s>>>(src, junk, geo, desc, nullptr, nchunks);
        k_merge4<false, 2><<<grid, NT, 0, s>>>(src, junk, geo, desc, nullptr, nchunks);
    }
    return hipGetLastError();
}

}  // namespace misort
