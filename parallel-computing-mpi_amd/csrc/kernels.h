// kernels.h -- internal launch interface of the gfx950 bitonic kernels
// (kernels.hip).  Not part of the public C-ABI (include/misort.h).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <functional>

namespace misort {

// IEEE double bits <-> order-preserving u64 (negative: all bits flipped; else
// the sign bit set), so every kernel compares unsigned integers.
__device__ __forceinline__ uint64_t ord_of_f64(uint64_t b) {
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t f64_of_ord(uint64_t o) {
    return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFull) : ~o;
}

// Kernel families, used for per-launch profiling (HIP events) and reporting.
enum Kind : int {
    KIND_TILE_SORT = 0,   // levels 1..LT inside one LDS tile
    KIND_GLOBAL = 1,      // retired (round 3): network ROWS pass
    KIND_TILE_MERGE = 2,  // retired (round 3): network in-tile merge pass
    KIND_MERGE_SPLIT = 3, // compare-split merge (keep lowest/highest n)
    KIND_OTHER = 4,       // f64 transform, fills, checks
    KIND_SPAN = 5,        // retired (round 3): network SPAN pass
    KIND_WIDE = 6,        // retired (round 3): network wide ROWS pass
    KIND_RUNS = 7,        // one merge level: runs of 2^hi keys -> runs of 2^(hi+1)
    KIND_EXCHANGE = 8,    // compare-split exchange leg (samples, RCCL send/recv, codec); not a kernel
    KIND_RUNSK = 9,       // R merge levels in one pass: runs of 2^hi -> 2^(hi+R), 2^R-way (runsk.hip)
    KIND_RUNSK_KERNEL = 10,  // the k_mergek launch of a KIND_RUNSK pass alone (nested in it)
    KIND_MERGE_SPLIT_TAIL = 11,  // in-place compare-split of a small bracket; bytes: an UPPER bound
                                 // (2 na + min(na, nb) keys: the device finds the window it rewrites)
    KIND_COUNT = 12
};

// Per-launch hook: called before and after every kernel launch of a sort with
// the kernel kind and its algorithmic HBM bytes (each key read once and
// written once).  nullptr = no profiling.
//
// A hook that binds() times the local sort's passes by events the kernels
// carry themselves (hipExtLaunchKernelGGL start/stop: the dispatch's own
// timestamps, no marker packets between the kernels): bind() hands out the
// events for the next launch (either may be null); kernel_kind >= 0 records
// that launch, pass_kind >= 0 the pass it ends (from the end of this sort's
// previous pass; bind_reset() starts a sort), both -1 binds a tick (the stop
// of the launch before a recorded one, where the hook times a launch from the
// previous one's end).
struct LaunchHook {
    virtual void before(Kind k, double bytes, hipStream_t s) = 0;
    virtual void after(Kind k, hipStream_t s) = 0;
    virtual bool binds() const { return false; }
    virtual void bind_reset() {}
    virtual bool bind(int kernel_kind, int pass_kind, double bytes, hipEvent_t* start, hipEvent_t* stop) {
        (void)kernel_kind, (void)pass_kind, (void)bytes;
        *start = *stop = nullptr;
        return false;
    }
    virtual ~LaunchHook() = default;
};

// A kernel launch carrying timing events (either may be null), or a plain one.
template <typename F, typename... Args>
inline void launch_timed(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, hipEvent_t start,
                         hipEvent_t stop, Args... args) {
    if (start || stop) hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, start, stop, 0u, args...);
    else kernel<<<grid, block, shmem, s>>>(args...);
}

// Chunked first/last pass of a local sort, for host staging that overlaps the
// PCIe copies with the sort (misort_sort_host).  The SORT pass runs chunk by
// chunk; before chunk [k0, k1) is read, before_first(k0, k1, s) makes stream s
// wait for those input keys.  If after_last is set, the final pass (a
// contiguous-tile MERGE or SORT pass) also runs chunk by chunk and
// after_last(k0, k1, s) is called once output keys [k0, k1) are enqueued.
// `chunk` is a multiple of the SORT tile.
struct StageIO {
    int64_t chunk = 0;
    std::function<int(int64_t, int64_t, hipStream_t)> before_first;
    std::function<int(int64_t, int64_t, hipStream_t)> after_last;
};

// Local ascending sort of n keys: in -> out (in == out allowed).
// K = uint32_t or uint64_t.  ord_in: the input holds IEEE doubles that are
// mapped to order-preserving u64 on load (K must be uint64_t); the output
// then stays in that ordered form.  scratch (n keys, distinct from in and out,
// or nullptr) lets the passes ping-pong between two buffers instead of
// rewriting `out` in place (copy-shaped HBM traffic).
// ord_out (K = uint64_t): the output is mapped back to IEEE double bits --
// by the last pass's stores when it is a multi-way pass, else by one more
// sweep (small sorts).
template <typename K>
hipError_t local_sort(const K* in, K* out, int64_t n, bool ord_in, K* scratch, hipStream_t s,
                      LaunchHook* hook, const StageIO* io = nullptr, bool ord_out = false);

// One HBM pass of a plan's shape over n keys (kind KIND_TILE_SORT, KIND_RUNS
// or KIND_RUNSK; hi, R as in the plan): probes and tests.
template <typename K>
hipError_t run_pass(const K* in, K* out, int64_t n, int kind, int hi, int R, int flip, hipStream_t s);

// Compare-split merge (device half of psort.cc:116-164): out[0..na) = the na
// smallest (keep_max=0) or largest (keep_max=1) keys of A U B, ascending.
// scratch must hold ceil(na/2048)+1 int64 co-ranks.
// ord_out (K = uint64_t): out gets IEEE double bits (the sort's last stage over f64 keys).
template <typename K>
hipError_t merge_split(const K* a, int64_t na, const K* b, int64_t nb, K* out,
                       int keep_max, int64_t* scratch, hipStream_t s, LaunchHook* hook, bool ord_out = false);

// The same compare-split IN PLACE when b touches one end of a: only the
// affected window of a (found on the device: keep-min, a's keys after b[0];
// keep-max, a's keys up to b[nb-1]) is staged into `stage` (same offsets) and
// merged back; O(window + nb) instead of O(na).  scratch holds
// ceil(na/2048) + 6 int64.
template <typename K>
hipError_t merge_split_tail(K* a, int64_t na, const K* b, int64_t nb, int keep_max, K* stage, int64_t* scratch,
                            hipStream_t s, LaunchHook* hook);

// Full merge of two ascending runs: out[0..na+nb) (A first on ties; for pure
// keys the result equals std::sort of the concatenation).  scratch holds
// ceil((na+nb)/2048)+1 int64 co-ranks.
template <typename K>
hipError_t merge_full(const K* a, int64_t na, const K* b, int64_t nb, K* out, int64_t* scratch, hipStream_t s,
                      LaunchHook* hook);

// One merge level of the local sort (runs.hip): src holds ascending runs of
// 2^lw keys (the last may be short), dst gets the ascending runs of 2^(lw+1).
// Only output keys [o0, o1) are written (o0 a multiple of 4096, o1 of 4096 or
// n; o1 <= 0 means n): the chunked last pass of host staging.  src != dst.
// hook: a binding hook times the level's merge launch as a KIND_RUNS pass.
template <typename K>
hipError_t merge_level(const K* src, K* dst, int64_t n, int lw, hipStream_t s, int64_t o0 = 0, int64_t o1 = 0,
                       LaunchHook* hook = nullptr);

// lk merge levels in one HBM pass (runsk.hip, u32 and u64, lk = 1..4): src holds
// ascending runs of 2^lw keys, dst gets ascending runs of 2^(lw+lk) (2^lk-way
// merge of each group of runs; the last group may be short).  Chunks are cut
// at fences (every 128th key of a run): `phase` selects which of two
// per-stream fence buffers holds this pass's fences; gather = build them from
// src first (the pass after a non-multi-way pass); lk_next > 0 = write the
// fences of the next multi-way pass (runs of 2^(lw+lk), groups of 2^lk_next)
// into the other buffer.  SORT_LT_MERGE <= lw, lw + lk <= 30; src != dst; buffers 16-byte
// aligned.
hipError_t merge_levelk(const uint32_t* src, uint32_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                        bool gather, int lk_next, LaunchHook* hook = nullptr);
// u64 keys: the same with 128-bit fences (key << 64 | run/position tag);
// 13 <= lw, lw + lk <= 29.
// ord_out: the pass is the sort's last (lk_next = 0) and writes IEEE double
// bits (f64_of_ord in its stores: no separate back-conversion sweep).
hipError_t merge_levelk(const uint64_t* src, uint64_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                        bool gather, int lk_next, LaunchHook* hook = nullptr, bool ord_out = false);
int64_t mergek_chunks(int64_t n, int lw, int lk, int key_bytes);
// Fence stride of the multi-way passes (log2 keys).
constexpr int MERGEK_FENCE_LOG2 = 7;  // runsk_fg6.hip: 6 (fence stride 256 measured equal to 128, profiles/r02)
// log2 keys of the u32 SORT tiles (bitonic.h).  15: 1024 lanes, one
// workgroup per CU, all 15 levels as the bitonic network.  14: 512 lanes, two
// workgroups per CU, levels 11..14 as in-LDS merge levels (SORT_MERGE_F).
// The plan picks per size (sort_tile_u32); u32 multi-way passes take runs of
// 2^14 and up.
constexpr int SORT_LT_U32 = 15, SORT_LT_MERGE = 14;
// The per-stream fence buffer `phase` of a multi-way pass over n keys (the
// one merge_levelk reads with that phase), for a SORT pass that writes the
// first pass's fences itself; null on allocation failure.
void* mergek_fence_buffer(int64_t n, int key_bytes, int phase, hipStream_t s);
void mergek_release(hipStream_t s);
int mergek_take_error(hipStream_t s);
// The same entry points of the 64-key-fence build (runsk_fg6.hip).
hipError_t merge_levelk_fg6(const uint32_t* src, uint32_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                            bool gather, int lk_next, LaunchHook* hook = nullptr);
hipError_t merge_levelk_fg6(const uint64_t* src, uint64_t* dst, int64_t n, int lw, int lk, hipStream_t s, int phase,
                            bool gather, int lk_next, LaunchHook* hook = nullptr, bool ord_out = false);
int64_t mergek_chunks_fg6(int64_t n, int lw, int lk, int key_bytes);
void* mergek_fence_buffer_fg6(int64_t n, int key_bytes, int phase, hipStream_t s);
void mergek_release_fg6(hipStream_t s);
int mergek_take_error_fg6(hipStream_t s);
// The fence stride (log2 keys) the local sort of n keys uses: 6 (runsk_fg6)
// from 2^MISORT_FENCE_FG6_MIN keys (u32: never by default, u64: 29), else MERGEK_FENCE_LOG2.
int mergek_fence_log2(int64_t n, int key_bytes);
int merge_levelk_lw_min(int key_bytes);   // shortest input runs (log2) of a multi-way pass
int merge_levelk_lwk_max(int key_bytes);  // largest output runs (log2)

// psort.cc:88-101 lower_bound on a sorted device run: *d_out = first i with
// x <= a[i], or n.
template <typename K>
hipError_t lower_bound(const K* a, int64_t n, K x, int64_t* d_out, hipStream_t s);

// lb[v] / ub[v] = first index with a[i] >= vals[v] / a[i] > vals[v] in a
// sorted run (device arrays of nv entries).
template <typename K>
hipError_t bounds(const K* a, int64_t n, const K* vals, int nv, int64_t* lb, int64_t* ub, hipStream_t s);

// Local descents a[i] > a[i+1] (psort.cc:497-501), compared as T
// (uint32_t, uint64_t or double); result added to *count (device u64).
template <typename T>
hipError_t count_descents(const T* a, int64_t n, unsigned long long* count, hipStream_t s);

// out[c] = a[min(c*stride, n-1)] for c in [0, count): the splitter samples of a
// sorted block used to bracket the compare-split crossing point.
template <typename K>
hipError_t gather_samples(const K* a, int64_t n, int64_t stride, K* out, int64_t count, hipStream_t s);

// The compare-split bracket on the device: from the partners' samples (sa of
// the keep-min side's na keys, sb of the keep-max side's nb keys, as
// gather_samples takes them) run[0..1] = {send offset, k} of this rank's
// message (keep_max: its bottom k keys; else its top k of nloc).
template <typename K>
hipError_t exchange_count(const K* sa, int64_t na, const K* sb, int64_t nb, int keep_max, int64_t nloc,
                          int64_t* run, hipStream_t s);

// IEEE double bits <-> order-preserving u64, in place.
hipError_t f64_to_ord(uint64_t* a, int64_t n, hipStream_t s);
hipError_t ord_to_f64(uint64_t* a, int64_t n, hipStream_t s);
hipError_t ord_to_f64_copy(const uint64_t* a, uint64_t* b, int64_t n, hipStream_t s);  // b = f64 bits of a

// Counter-based SplitMix64 keys for global indices [g0, g0+n) (bench/test input).
hipError_t fill_splitmix_u32(uint32_t* out, int64_t n, uint64_t seed, int64_t g0, hipStream_t s);
hipError_t fill_splitmix_u64(uint64_t* out, int64_t n, uint64_t seed, int64_t g0, hipStream_t s);

// Lossless delta coding of a sorted run (codec.hip), for the compare-split
// exchange: blocks of 1024 keys, first key + gaps packed at the block's width.
// codec_encode writes the stream to `out` (<= codec_max_words(n) u32 words)
// and sizes[0..1] = {coded words, raw words} (device int64); scratch holds
// codec_scratch_bytes(n) bytes.  codec_encode_dev does the same for the run
// base + run[0] of run[1] keys, both device int64, run[1] <= n_max.
// codec_decode restores the n keys.
int64_t codec_blocks(int64_t n);
size_t codec_scratch_bytes(int64_t n);
int64_t codec_max_words(int64_t n, int key_bytes);
template <typename K>
hipError_t codec_encode(const K* keys, int64_t n, uint32_t* out, void* scratch, size_t scratch_bytes,
                        int64_t* sizes, hipStream_t s);
template <typename K>
hipError_t codec_encode_dev(const K* base, const int64_t* run, int64_t n_max, uint32_t* out, void* scratch,
                            size_t scratch_bytes, int64_t* sizes, hipStream_t s);
template <typename K>
hipError_t codec_decode(const uint32_t* in, int64_t n, K* keys, hipStream_t s);

// Tile geometry per key type (exported for documentation/tests).
int tile_log2(int key_bytes);

// The HBM pass plan local_sort runs for n keys of key_bytes (4 or 8): writes
// up to max passes as 4 ints each (kind, hi, R, flip) and returns the count.
int plan_passes(int64_t n, int key_bytes, int* out, int max);

}  // namespace misort
