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
constexpr int FM = 31;                          // fences per chunk
constexpr int CAP = (FM + 4) * (int)FG;         // most keys of a chunk (8960; 7936 on average)
constexpr int NT = 256;
constexpr int IT = 36;                          // keys per lane (one merge chain)
// level 1 puts the second pair's output at the next multiple of IT (no lane
// straddles two pairs), which needs one spare lane's worth of room
static_assert(CAP <= (NT - 1) * IT, "chunk tile shape");
constexpr int LDS_WORDS = NT * IT + IT + 8;
constexpr int DUMP = LDS_WORDS - 1;  // target of masked-off LDS writes (no branches)
constexpr uint64_t J_MASK = ((uint64_t)1 << 30) - 1;

typedef uint32_t vec4 __attribute__((ext_vector_type(4)));

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

// Merge-path co-rank: A keys among the first d outputs of merge(A, B).
__device__ __forceinline__ int co_rank(const uint32_t* s, int A0, int LA, int B0, int LB, int d) {
    int lo = d - LB > 0 ? d - LB : 0, hi = d < LA ? d : LA;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s[A0 + mid] <= s[B0 + d - 1 - mid]) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

#ifndef MISORT_M4_CHAINS
#define MISORT_M4_CHAINS 2
#endif
constexpr int CH = MISORT_M4_CHAINS;  // independent merge chains per lane (interleaved)
constexpr int IC = IT / CH;
static_assert(IT % CH == 0, "chains split the lane's outputs");

// IT consecutive outputs from diagonal d of merge(s[A0, A0+LA), s[B0, B0+LB))
// (A first on ties), as CH chains of IC outputs whose dependent LDS reads
// interleave.  An exhausted side reads as MAX: when it ties a real MAX key of
// the other side every remaining output is MAX whichever side "wins", so the
// values stay exact without bounds on the chosen index.  A chain tracks only
// pa: after step k it has taken d_c + k + 1 keys, so pb = SUM + k - pa.
__device__ __forceinline__ void merge_chain(const uint32_t* s, int A0, int LA, int B0, int LB, int d,
                                            uint32_t (&r)[IT]) {
    const int tot = LA + LB;
    const int ea = A0 + LA, eb = B0 + LB;
    int pa[CH], sum[CH];
    uint32_t av[CH], bv[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int dc = d + c * IC < tot ? d + c * IC : tot;  // lanes past the end: garbage, in-bounds
        const int lo = co_rank(s, A0, LA, B0, LB, dc);
        pa[c] = A0 + lo;
        const int pb = B0 + dc - lo;
        sum[c] = pa[c] + pb + 1;
        const uint32_t a0 = s[pa[c]], b0 = s[pb];  // in-bounds: pa <= ea, pb <= eb
        av[c] = pa[c] < ea ? a0 : 0xFFFFFFFFu;
        bv[c] = pb < eb ? b0 : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < IC; ++k) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            const bool takeA = av[c] <= bv[c];
            r[c * IC + k] = min(av[c], bv[c]);
            pa[c] += takeA;
            const int pb = sum[c] + k - pa[c];
            const int p = takeA ? pa[c] : pb;
            const uint32_t v = s[p];
            const uint32_t w = p < (takeA ? ea : eb) ? v : 0xFFFFFFFFu;
            av[c] = takeA ? w : av[c];
            bv[c] = takeA ? bv[c] : w;
        }
    }
}

// MODE (probes only, MISORT_M4_PROBE): 0 = the pass; 1 = loads -> LDS ->
// stores with no merge (the access pattern's floor); 2 = level 1 only.
template <bool FENCES, int MODE = 0>
__global__ __launch_bounds__(NT) void k_merge4(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                               Geo4 geo, const int64_t* __restrict__ bounds,
                                               uint64_t* __restrict__ fout) {
    __shared__ __attribute__((aligned(16))) uint32_t s[LDS_WORDS];
    const int tid = threadIdx.x;
    const int64_t c = blockIdx.x;
    int64_t g, t;
    if (c < geo.nfull * geo.kf) {
        g = c / geo.kf;
        t = c - g * geo.kf;
    } else {
        g = geo.nfull;
        t = c - geo.nfull * geo.kf;
    }
    const int64_t* b0 = bounds + 4 * geo.slot(g, t);
    const int64_t base = geo.base(g);
    const int64_t W = (int64_t)1 << geo.lw;
    int s0 = (int)b0[0], s1 = (int)b0[1], s2 = (int)b0[2], s3 = (int)b0[3];
    int l0 = (int)b0[4] - s0, l1 = (int)b0[5] - s1, l2 = (int)b0[6] - s2, l3 = (int)b0[7] - s3;
    // bounds outside the runs would be a logic error: never let them address
    // memory (the chunk is then left unwritten and the sort fails its checks)
    if (s0 < 0 || l0 < 0 || s0 + l0 > geo.run_len(g, 0) || s1 < 0 || l1 < 0 || s1 + l1 > geo.run_len(g, 1) ||
        s2 < 0 || l2 < 0 || s2 + l2 > geo.run_len(g, 2) || s3 < 0 || l3 < 0 || s3 + l3 > geo.run_len(g, 3) ||
        l0 + l1 + l2 + l3 > CAP)
        s0 = s1 = s2 = s3 = l0 = l1 = l2 = l3 = 0;
    const int o1 = l0, o2 = o1 + l1, o3 = o2 + l2;
    const int len = o3 + l3 < CAP ? o3 + l3 : CAP;  // <= CAP by construction; never past the LDS tile
    const int64_t out0 = base + s0 + s1 + s2 + s3;
    // segment r occupies chunk positions [o_r, o_r + l_r); its key at chunk
    // position e is gsrc[d_r + e] (32-bit offsets within the group: 4W <= 2^32;
    // d_r >= 0 as W >= CAP)
    const uint32_t* __restrict__ gsrc = src + base;
    const uint32_t dA = (uint32_t)s0, dB = (uint32_t)W + s1 - o1, dC = 2u * (uint32_t)W + s2 - o2,
                   dD = 3u * (uint32_t)W + s3 - o3;
    {
        uint32_t x[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int e = k * NT + tid;
            const uint32_t d = e < o1 ? dA : e < o2 ? dB : e < o3 ? dC : dD;
            x[k] = e < len ? __builtin_nontemporal_load(gsrc + (d + (uint32_t)e)) : 0xFFFFFFFFu;
        }
#pragma unroll
        for (int k = 0; k < IT; ++k) s[k * NT + tid] = x[k];
    }
    __syncthreads();
    uint32_t r[IT];
    const int pos = tid * IT;
    // level 1: A ++ B -> [0, o2); C ++ D -> [q2, q2 + l2 + l3), q2 = o2 rounded
    // up to a lane boundary, so each lane merges inside one pair
    const int q2 = (o2 + IT - 1) / IT * IT, end1 = q2 + (len - o2);
    const bool p1 = pos < o2;
    if constexpr (MODE == 1) {
#pragma unroll
        for (int k = 0; k < IT; ++k) r[k] = s[pos + k];
    } else {
        merge_chain(s, p1 ? 0 : o2, p1 ? l0 : l2, p1 ? o1 : o3, p1 ? l1 : l3, p1 ? pos : pos - q2, r);
    }
    __syncthreads();
    {
        const int lim = p1 ? o2 : end1;
        if (pos + IT <= lim) {
            typedef uint32_t vec2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int k = 0; k < IT; k += 2) *reinterpret_cast<vec2*>(s + pos + k) = vec2{r[k], r[k + 1]};
        } else {
#pragma unroll
            for (int k = 0; k < IT; ++k) s[pos + k < lim ? pos + k : DUMP] = r[k];
        }
    }
    __syncthreads();
    // level 2: [0, o2) ++ [q2, end1) -> the chunk
    if constexpr (MODE != 0) {
#pragma unroll
        for (int k = 0; k < IT; ++k) r[k] = s[pos + k];
    } else {
        merge_chain(s, 0, o2, q2, len - o2, pos, r);
    }
    __syncthreads();
    // the chunk goes to LDS shifted by out0 mod 4, so every global 16-byte
    // vector is one aligned LDS vector
    const int sh = (int)(out0 & 3);
#pragma unroll
    for (int k = 0; k < IT; ++k) s[pos + k < len ? sh + pos + k : DUMP] = r[k];
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
            fout[gp >> FG_LOG2] = fpack(s[(int)(gp - (out0 - sh))], gp, geo.lw + 2);
        }
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
    // chunks index a group with 32-bit offsets (4W <= 2^32); runs at least CAP long
    if (lw < 15 || lw > 30 || src == dst) return hipErrorInvalidValue;
    Geo4 geo{n, lw, 0, 0};
    geo.nfull = n >> (lw + 2);
    geo.kf = ((((int64_t)4 << lw) >> FG_LOG2) + FM - 1) / FM;  // chunks of a full group
    const bool tail = (geo.nfull << (lw + 2)) < n;
    const int64_t nchunks = geo.nfull * geo.kf + (tail ? geo.nchunks(geo.nfull) : 0);
    const int64_t nslots = geo.nfull * (geo.kf + 1) + (tail ? geo.nchunks(geo.nfull) + 1 : 0);
    const int64_t nf = (n + FG - 1) >> FG_LOG2;
    // layout: fence buffers 0 and 1, merged fences, u64 merge temp, bounds
    const size_t fb = ((size_t)nf * 8 + 255) & ~(size_t)255;
    char* base = (char*)scratch4(4 * fb + (size_t)nslots * 32 + 256, s);
    if (!base) return hipErrorOutOfMemory;
    uint64_t* F = (uint64_t*)(base + (phase & 1) * fb);
    uint64_t* Fn = (uint64_t*)(base + ((phase & 1) ^ 1) * fb);
    uint64_t* M = (uint64_t*)(base + 2 * fb);
    uint64_t* T = (uint64_t*)(base + 3 * fb);
    int64_t* bounds = (int64_t*)(base + 4 * fb);
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
    if (write_next) k_merge4<true><<<(unsigned)nchunks, NT, 0, s>>>(src, dst, geo, bounds, Fn);
    else k_merge4<false><<<(unsigned)nchunks, NT, 0, s>>>(src, dst, geo, bounds, nullptr);
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
        k_merge4<false, 1><<<(unsigned)nchunks, NT, 0, s>>>(src, junk, geo, bounds, nullptr);
        k_merge4<false, 2><<<(unsigned)nchunks, NT, 0, s>>>(src, junk, geo, bounds, nullptr);
    }
    return hipGetLastError();
}

}  // namespace misort
