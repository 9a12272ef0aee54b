/*
 * misort.h -- C-ABI of the MI355X-native bitonic sort (libmisort.so).
 *
 * Drop-in boundary for the hot path of masrul/Parallel-Computing-MPI's
 * Parallel-Sorting/src/psort.cc.  The reference has no FFI: its swappable unit
 * is the C++ function
 *
 *     double* parallel_bitonic_sort(double* buffer, int& loc_buf_size,
 *                                   int max_size);              // psort.cc:167
 *
 * driven by the globals numprocs/myid of MPI_COMM_WORLD (psort.cc:107,535-536),
 * with compare_split_{max,min} (psort.cc:116-164) exchanging whole blocks over
 * MPI_Sendrecv.  Here ranks are GPUs (one process per GPU), the communicator is
 * RCCL over xGMI, and keys live in HBM.  All entry points are extern "C", take
 * plain pointers and sizes, return 0 on success or a negative MISORT_E_* code
 * (message via misort_last_error()), and never throw.  A context is not
 * thread-safe; use one per thread/GPU.
 *
 * Device pointers are HIP device addresses on the context's GPU.  `stream` is a
 * hipStream_t (NULL = the context's own stream); calls are asynchronous on it
 * unless stated otherwise.
 */
#ifndef MISORT_H
#define MISORT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MISORT_VERSION 1

/* Key types.  F64 keys are IEEE doubles compared as doubles (psort.cc sorts
 * double); they are sorted as order-preserving 64-bit patterns, so results are
 * bit-exact with the reference except for mixtures of -0.0/+0.0 or NaNs, whose
 * relative order std::sort leaves unspecified.  Documented deviation, measured
 * against the compiled reference (tests/golden/make_golden_f64zero.py, 1000
 * zeros of each sign among 4002 doubles, P = 1, 2, 4, 8): the reference writes
 * its zeros in an introsort-dependent sign order (487-515 sign changes), this
 * library writes -0.0 before +0.0 within each rank's block; every position is
 * equal as a double and every non-zero position is bit-exact
 * (tests/test_gpu_parity.py::test_f64_signed_zeros_vs_reference). */
enum misort_dtype { MISORT_U32 = 0, MISORT_U64 = 1, MISORT_F64 = 2 };

enum misort_status {
    MISORT_OK = 0,
    MISORT_E_INVALID = -1,   /* bad argument */
    MISORT_E_NOT_POW2 = -2,  /* psort.cc:168-172 "bitonic sort requires 2^d processors" */
    MISORT_E_HIP = -3,       /* HIP runtime error */
    MISORT_E_RCCL = -4,      /* RCCL error */
    MISORT_E_NO_COMM = -5,   /* communicator not initialised */
    MISORT_E_CAPACITY = -6,  /* a partner block exceeds max_size (MPI_Sendrecv truncation) */
    MISORT_E_INTERNAL = -7   /* a merge pass rejected its own chunk bounds (a planning bug: the
                                output is incomplete); reported by the call itself where it
                                syncs (misort_sort_host), else at the next host sync of the
                                same stream: misort_synchronize for the context's own stream,
                                misort_check_sort for the stream it is given (a sort on a
                                caller's stream is reported there, not by misort_synchronize) */
};

/* Kernel families reported by the per-launch profiler. */
enum misort_kernel_kind {
    MISORT_K_TILE_SORT = 0,   /* levels 1..LT in one LDS tile            */
    MISORT_K_GLOBAL = 1,      /* retired (round 3): network ROWS pass    */
    MISORT_K_TILE_MERGE = 2,  /* retired (round 3): network merge pass   */
    MISORT_K_MERGE_SPLIT = 3, /* device compare-split (psort.cc:116-164) */
    MISORT_K_OTHER = 4,
    MISORT_K_SPAN = 5,        /* retired (round 3): network SPAN pass    */
    MISORT_K_WIDE = 6,        /* retired (round 3): network wide pass    */
    MISORT_K_RUN_MERGE = 7,   /* one merge level: runs 2^hi -> 2^(hi+1)  */
    MISORT_K_EXCHANGE = 8,    /* compare-split exchange leg (splitter samples, RCCL
                                 send/recv, codec), device time between events */
    MISORT_K_RUN_MERGE4 = 9,  /* a multi-way pass: lk merge levels, runs 2^hi -> 2^(hi+lk) */
    MISORT_K_RUN_MERGEK_KERNEL = 10, /* the merge kernel of a multi-way pass alone (its planning
                                        kernels excluded; nested in MISORT_K_RUN_MERGE4) */
    MISORT_K_MERGE_SPLIT_TAIL = 11  /* in-place compare-split of a small bracket
                                       (misort_merge_split_tail); its bytes are an UPPER bound,
                                       2 nblock + min(nblock, nrecv) keys: the device finds the
                                       window it rewrites */
};

typedef struct misort_ctx misort_ctx;

int misort_version(void);
const char* misort_last_error(void);

/* Context on HIP device `device`: selects it, creates a non-blocking stream and
 * grows scratch buffers on demand.  Replaces MPI_Init's per-process setup. */
int misort_create(int device, misort_ctx** out);
int misort_destroy(misort_ctx* ctx);
/* hipStream_t of the context (as void*). */
void* misort_stream(misort_ctx* ctx);
/* Waits for the context's own stream (not a caller's stream) and reports a
 * merge pass's rejected chunk on it (MISORT_E_INTERNAL).  With a communicator,
 * a wait that follows transport calls is bounded by MISORT_TIMEOUT_S (default
 * 120 s; a deadline aborts the communicator, MISORT_E_RCCL); a wait on local
 * work only is not. */
int misort_synchronize(misort_ctx* ctx);

/* ---- communicator (replaces MPI_COMM_WORLD, psort.cc:107,535-536) -------- */
#define MISORT_UNIQUE_ID_BYTES 128
/* Rank 0 creates the id (ncclGetUniqueId) and ships it to all ranks by any
 * host channel (MPI_Bcast, torch.distributed, a file). */
int misort_get_unique_id(void* id /* MISORT_UNIQUE_ID_BYTES */);
/* Collective over all nranks processes: ncclCommInitRank. nranks must be a
 * power of two (else MISORT_E_NOT_POW2, the reference's abort condition). */
int misort_comm_init(misort_ctx* ctx, int nranks, int rank, const void* id);
/* In-process rank group: P ranks as P threads of one process, each with its own
 * context (on the same or different GPUs).  The exchange is a device-to-device
 * copy ordered by HIP events; the schedule, sizes and merge-split path are the
 * same as over RCCL.  Used to run the P-rank path on one GPU (tests) and to
 * drive several GPUs from one process. */
typedef struct misort_group misort_group;
int misort_group_create(int nranks, misort_group** out);
int misort_group_destroy(misort_group* g);
int misort_comm_init_group(misort_ctx* ctx, misort_group* g, int rank);
int misort_comm_size(misort_ctx* ctx);  /* numprocs */
int misort_comm_rank(misort_ctx* ctx);  /* myid */
/* psort.cc:182-196 stage schedule of `rank` in a `p`-rank hypercube: partner
 * and keep-max flag per stage (arrays of >= 64 entries); returns the stage
 * count d(d+1)/2 or a negative status.  Pure host logic. */
int misort_bitonic_schedule(int p, int rank, int* partner, int* keep_max);
/* psort.cc:556-562 block size of `rank` for n keys over p ranks. */
int64_t misort_block_size(int64_t n, int p, int rank);

/* ---- the hot path ------------------------------------------------------- */

/* psort.cc:167 parallel_bitonic_sort over the context's communicator (a
 * single rank without misort_comm_init).  d_keys holds loc_size keys of this
 * rank's block (capacity >= loc_size); on return it holds the rank's block of
 * the result -- the same block the reference leaves in its returned buffer,
 * including the reference's output for uneven blocks.  max_size bounds every
 * rank's block (psort.cc:557, the MPI_Sendrecv receive capacity); it is checked
 * collectively (every rank against the smallest max_size, so all ranks fail
 * together), and max_size <= 0 means the largest block.  Steps: local sort
 * (psort.cc:175) then d(d+1)/2 rounds of RCCL send/recv with the partner plus a
 * device merge-split.  At P = 1 everything is enqueued on `stream`; at P > 1
 * the host waits on the stream at the start (size exchange) and once per
 * stage: the exchange count k is computed on the device from the swapped
 * splitter samples, the encoder takes it from device memory, and the ranks'
 * (coded, raw) message sizes -- which carry k -- are exchanged from device
 * memory; the host reads them once to size the RCCL send/recv.  Without the
 * codec (MISORT_COMPRESS=0) k is computed on the host: two waits per stage. */
int misort_parallel_bitonic_sort(misort_ctx* ctx, int dtype, void* d_keys, int64_t loc_size,
                                 int64_t max_size, void* stream);
/* Same, out of place: d_in is left unchanged, d_out receives the block
 * (d_in == d_out allowed).
 *
 * Exchange volume: before each compare-split the partners swap splitter
 * samples (every S-th key, S = max(256, n/32768)) and both derive the same
 * lower bound of the merge-path crossing point, so each side sends only the
 * keys that can cross (the min side its top k, the max side its bottom k)
 * instead of the whole block.  The kept multisets -- hence the bytes of the
 * result -- are exactly those of the reference's whole-block MPI_Sendrecv.
 * MISORT_FULL_EXCHANGE=1 (or misort_set_full_exchange) restores whole-block
 * exchange. */
int misort_parallel_bitonic_sort_oop(misort_ctx* ctx, int dtype, const void* d_in, void* d_out,
                                     int64_t loc_size, int64_t max_size, void* stream);

/* psort.cc:175 local ascending sort of n keys on one GPU, d_in -> d_out
 * (d_in == d_out allowed). */
int misort_local_sort(misort_ctx* ctx, int dtype, const void* d_in, void* d_out, int64_t n,
                      void* stream);

/* psort.cc:377-490 parallel_quick_sort (the reference binary's shipped sort,
 * called at psort.cc:647-648): d rounds of median-of-medians pivoting over
 * shrinking hypercube sub-groups, RCCL send/recv with the partner, device merge.
 * Per-rank output sizes are data-dependent, exactly as in the reference:
 * *out_size receives this rank's count; MISORT_E_CAPACITY if it exceeds
 * out_capacity (the reference allocates (loc+1)*P).  d_in is not modified. */
int misort_parallel_quick_sort(misort_ctx* ctx, int dtype, const void* d_in, int64_t loc_size,
                               void* d_out, int64_t out_capacity, int64_t* out_size, void* stream);

/* psort.cc:203-375 parallel_sample_native_sort / parallel_sample_bitonic_sort,
 * redesigned for RCCL over xGMI: local sort, all-gathered regular samples,
 * (key, rank, position) splitters, ONE all-to-all-v (every GPU pair on its
 * own link), a device merge tree, and a rebalancing all-to-all-v into the
 * reference block layout.  Same contract as misort_parallel_bitonic_sort_oop
 * (d_out receives loc_size keys: the globally sorted sequence in the callers'
 * block sizes); d_in != d_out.  The reference's versions are not well defined
 * (an uninitialised splitter at :318, MPI_INT used for doubles at :224/:269),
 * so parity is anchored on the sorted sequence, not on their per-rank sizes. */
int misort_parallel_sample_sort(misort_ctx* ctx, int dtype, const void* d_in, void* d_out,
                                int64_t loc_size, int64_t max_size, void* stream);

/* Device half of compare_split_{max,min} (psort.cc:116-164) without the
 * exchange: d_out[0..nloc) = the nloc largest (keep_max=1) or smallest
 * (keep_max=0) keys of the sorted blocks local U recv, ascending. */
int misort_merge_split(misort_ctx* ctx, int dtype, const void* d_local, int64_t nloc,
                       const void* d_recv, int64_t nrecv, void* d_out, int keep_max,
                       void* stream);

/* The same keep-n merge IN PLACE (psort.cc:116-164, the result replaces
 * d_block): the path a hypercube stage takes when the partner's bracket k is
 * small (k <= nblock / MISORT_TAIL_DIV, default 8): only the end of the block
 * that the nrecv received keys reach is rewritten, staged through the context's
 * work buffer.  d_recv must not overlap d_block (MISORT_E_INVALID).  Exposed
 * so the path is testable on its own (extension; the reference merges the
 * whole block every stage). */
int misort_merge_split_tail(misort_ctx* ctx, int dtype, void* d_block, int64_t nblock,
                            const void* d_recv, int64_t nrecv, int keep_max, void* stream);

/* psort.cc:497-520 check_sort: local descents of this rank's block plus the
 * boundary descent against rank-1's last key, summed over the communicator.
 * Synchronous; *errors is valid on every rank. */
int misort_check_sort(misort_ctx* ctx, int dtype, const void* d_keys, int64_t n,
                      int64_t* errors, void* stream);

/* Host-buffer convenience path: h_in -> pinned staging -> device -> sort ->
 * host h_out (this rank's block, parallel sort over the communicator).
 * Synchronous. */
int misort_sort_host(misort_ctx* ctx, int dtype, const void* h_in, void* h_out, int64_t loc_size,
                     int64_t max_size);

/* ---- synthetic input ------------------------------------------------------ */
/* Counter-based SplitMix64 keys of global indices [g0, g0+n):
 * key_g = mix(seed + (g+1)*0x9E3779B97F4A7C15), u32 = top 32 bits. */
int misort_fill_splitmix(misort_ctx* ctx, int dtype, void* d_out, int64_t n, uint64_t seed,
                         int64_t g0, void* stream);

int misort_set_full_exchange(misort_ctx* ctx, int on);

/* Relay each compare-split exchange through the other GPUs (P > 2; default on,
 * env MISORT_RELAY=0 turns it off): every message is cut into P parts, 2 go
 * over the pair's own xGMI link, P-2 take two hops through the other GPUs, so
 * all P-1 links of every GPU carry the stage.  Bytes delivered are identical. */
int misort_set_relay(misort_ctx* ctx, int on);

/* Delta-code the keys of each compare-split message (default on; env
 * MISORT_COMPRESS=0 turns it off).  The k keys one side sends are a sorted
 * run: blocks of 1024 keys travel as first key + gaps packed at the block's
 * bit width (lossless; ~4x smaller for 2^27 uniform u32 keys per rank).  A
 * side whose coded message would not be smaller sends it raw; the receiver
 * tells them apart by size.  Replaces the raw MPI_Sendrecv payload of
 * psort.cc:122-123 / 146-147; the kept keys are unchanged. */
int misort_set_compress(misort_ctx* ctx, int on);

/* Tooling: encode a sorted device run of n keys with the exchange codec,
 * then decode it (into `decoded` if non-null); average ms of each over
 * `reps` launches (HIP events) and the coded size in bytes. */
int misort_codec_probe(misort_ctx* ctx, int dtype, const void* keys, int64_t n, int reps, float* enc_ms,
                       float* dec_ms, int64_t* coded_bytes, void* decoded);

/* Bytes the exchanges since the last call would have moved uncoded (sent +
 * received; the coded bytes are misort_exchange_stats' `bytes`).  Resets. */
int misort_exchange_raw_bytes(misort_ctx* ctx, int64_t* raw_bytes);
/* Host logic of the bracketed exchange (pure functions, no GPU):
 * samples of a sorted block of n keys are keys[min(c*S, n-1)], c = 0..count-1,
 * S = misort_sample_stride(n), count = misort_sample_count(n).
 * misort_exchange_count returns k, the keys each partner sends (the keep-min
 * side its top k, the keep-max side its bottom k), given both sample sets; -1
 * means whole blocks (an empty side).  u64/f64 samples are order-preserving
 * u64 patterns. */
int64_t misort_sample_stride(int64_t n);
int64_t misort_sample_count(int64_t n);
int64_t misort_exchange_count(int dtype, const void* samples_min, int64_t n_min,
                              const void* samples_max, int64_t n_max);
/* Exchange volume since the last call (then reset): compare-split stages,
 * bytes sent+received, and the bytes a whole-block exchange would have moved. */
int misort_exchange_stats(misort_ctx* ctx, int64_t* stages, int64_t* bytes, int64_t* full_bytes);

/* ---- per-launch profiling (HIP events around every kernel launch) ---------- */
int misort_profile_enable(misort_ctx* ctx, int on);
/* Reset accumulated figures. */
int misort_profile_reset(misort_ctx* ctx);
/* Synchronises the stream(s) used, then reports for one kernel kind: launches,
 * summed device time (ms) and summed algorithmic HBM bytes. */
int misort_profile_read(misort_ctx* ctx, int kind, int64_t* launches, double* total_ms,
                        double* bytes);

/* Per hypercube stage of misort_parallel_bitonic_sort (stage 0 .. d(d+1)/2-1,
 * the order of psort.cc:184-185), summed over the profiled sorts: number of
 * sorts, exchange-leg device time (ms), merge-split kernel time (ms) and the
 * bytes this rank sent plus received in the stage. */
int misort_profile_stage(misort_ctx* ctx, int stage, int64_t* count, double* exchange_ms,
                         double* merge_ms, double* exchange_bytes);

/* Every profiled record since the last reset, in completion order (a
 * multi-way pass after the k_mergek launch nested in it): kind, device ms and
 * algorithmic bytes.  Fills up to `max` entries; returns the number recorded
 * (at most 2^20 are kept).  For per-pass roofline figures. */
int misort_profile_trace(misort_ctx* ctx, int max, int* kinds, double* ms, double* bytes);

/* log2 of the LARGEST SORT tile (keys) for a key width of 4 or 8 bytes: every
 * plan's tiles divide it.  The tile a given size actually uses is chosen per
 * size (u32: 2^14 or 2^15); it is the first pass of misort_plan (hi + 1). */
int misort_tile_log2(int key_bytes);

/* The HBM pass plan of a local sort of n keys (key_bytes 4 or 8), for tools
 * and tests: writes up to max_passes entries of 4 ints (kind as
 * misort_kernel_kind, hi, R, flip) and returns the number of passes (or a
 * negative status).  Host-only; no device is touched. */
int misort_plan(int64_t n, int key_bytes, int* passes, int max_passes);

/* Tooling: average device time (ms, HIP events on the context stream) of ONE
 * HBM pass of the given shape (kind MISORT_K_TILE_SORT, MISORT_K_RUN_MERGE or
 * MISORT_K_RUN_MERGE4; hi/R as misort_plan reports them) over n keys,
 * alternating in -> out and out -> in for `reps` launches.  A merge pass
 * assumes ascending runs of 2^hi keys; other input is scrambled, not sorted. */
int misort_pass_probe(misort_ctx* ctx, int dtype, const void* in, void* out, int64_t n, int kind,
                      int hi, int r, int flip, int reps, float* ms);

#ifdef __cplusplus
}
#endif
#endif
