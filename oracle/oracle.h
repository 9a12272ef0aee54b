/*
 * oracle.h -- CPU restatement of the reference bitonic-sort hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker.
 * The product path (libmisort.so) never links or calls it.
 *
 * Every function restates a piece of /root/reference/Parallel-Sorting/src/psort.cc
 * (cited per function).  Parity of this restatement is pinned against the
 * compiled, unmodified reference (oracle/_ref, see oracle/Makefile and
 * tests/golden/make_golden.py).
 */
#ifndef MISORT_ORACLE_H
#define MISORT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_U32 = 0, ORC_U64 = 1, ORC_F64 = 2 };

/* psort.cc:556-562 -- loc_r = N/P + (r < N%P). */
void orc_block_sizes(int64_t n, int p, int64_t *sizes);

/* psort.cc:587-614 -- erand48 stream (state {0,0,1}) with the 16-bit counter
 * xi[3] and the ODD_DIST skew.  Writes keys [g0, g0+cnt) of an N-key sequence.
 * The reference's rank-to-rank seed chain makes the sequence independent of P,
 * so a block is addressed by its global offset (LCG jump-ahead). */
void orc_generate_f64(int64_t n, int64_t g0, int64_t cnt, double *out);

/* Bench / parity workload (not in the reference): counter-based SplitMix64.
 * key_g = mix(seed + (g+1)*0x9E3779B97F4A7C15); u32 keeps the top 32 bits. */
void orc_splitmix_u32(uint64_t seed, int64_t g0, int64_t cnt, uint32_t *out);
void orc_splitmix_u64(uint64_t seed, int64_t g0, int64_t cnt, uint64_t *out);

/* BASELINE config-5 key mix (not in the reference):
 * per global index g, counter-based on seed: 40 % from a 1024-value alphabet
 * (duplicate-heavy), 30 % the bit patterns of the reference's own ODD_DIST
 * doubles (psort.cc:587-609 at index g of an n-key sequence: skewed), 20 %
 * uniform, 5 % zeros, 5 % `top` (the sentinel: all-ones for the full mix;
 * 0x7FF0000000000000 for the variant the reference can carry as ordered
 * doubles, with alphabet/uniform keys then drawn below it).  Independent of
 * how the index range is split, so rank blocks can be generated alone. */
void orc_u64mix(uint64_t seed, int64_t n, int64_t g0, int64_t cnt, uint64_t top, uint64_t *out);

/* psort.cc:175 -- ascending local sort (std::sort). f64 compares as double. */
void orc_sort(int dtype, void *keys, int64_t n);

/* psort.cc:116-140 (keep_max=1) and psort.cc:142-164 (keep_max=0): keep the
 * nloc largest / smallest of local U recv by a linear merge; ties take the
 * received key exactly as the reference does. */
void orc_compare_split(int dtype, const void *local, int64_t nloc,
                       const void *recv, int64_t nrecv, void *out, int keep_max);

/* psort.cc:167-201 over P virtual ranks whose blocks are laid out contiguously
 * in rank order in keys[0..n) (block layout of psort.cc:556-562).  Returns 0,
 * or -1 when P is not a power of two (psort.cc:168-172). */
int orc_parallel_bitonic_sort(int dtype, void *keys, int64_t n, int p);

/* psort.cc:184-194 -- stage schedule for one rank: fills partner[] and
 * keep_max[] for the d(d+1)/2 stages, returns the stage count. */
int orc_bitonic_schedule(int p, int rank, int *partner, int *keep_max);

/* psort.cc:377-490 -- parallel_quick_sort over P virtual ranks (input blocks
 * in the reference layout, contiguous in rank order).  out receives the
 * rank-ordered concatenation of the final blocks (n keys), sizes[r] the final
 * block sizes (data-dependent).  Returns 0, or -1 when P is not a power of two. */
int orc_parallel_quick_sort(int dtype, const void *keys, int64_t n, int p, void *out,
                            int64_t *sizes);

/* psort.cc:497-520 -- local descents plus rank-boundary descents. */
int64_t orc_check_sort(int dtype, const void *keys, int64_t n, int p);

#ifdef __cplusplus
}
#endif
#endif
