/*
 * oracle.c -- CPU restatement of the reference bitonic-sort hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Not part of the product: the
 * HIP path in parallel-computing-mpi_amd/csrc never links this file.
 *
 * Reference: /root/reference/Parallel-Sorting/src/psort.cc (cited per function).
 * Parity pinned by tests/golden/ (fixtures produced by the compiled,
 * unmodified reference; generator script tests/golden/make_golden.py).
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ layout */

/* psort.cc:556-562: local_input_size = N/P, +1 on the first N%P ranks. */
void orc_block_sizes(int64_t n, int p, int64_t *sizes) {
    for (int r = 0; r < p; ++r)
        sizes[r] = n / p + (r < n % p ? 1 : 0);
}

/* --------------------------------------------------------------- generator */

#define LCG_A 0x5DEECE66DULL
#define LCG_C 0xBULL
#define LCG_MASK ((1ULL << 48) - 1)

/* X_k = f^k(X_0), f(X) = A X + C mod 2^48 (glibc drand48 family). */
static uint64_t lcg_skip(uint64_t x, uint64_t k) {
    uint64_t acc_a = 1, acc_c = 0, a = LCG_A, c = LCG_C;
    while (k) {
        if (k & 1) {
            acc_a = (acc_a * a) & LCG_MASK;
            acc_c = (acc_c * a + c) & LCG_MASK;
        }
        c = (c * a + c) & LCG_MASK;
        a = (a * a) & LCG_MASK;
        k >>= 1;
    }
    return (acc_a * x + acc_c) & LCG_MASK;
}

/* psort.cc:587-609.  xi = {0,0,1,0}: the erand48 state is xi[0..2] (X0 = 2^32)
 * and xi[3] is an unsigned short counter bumped before every draw.  erand48
 * advances the state, then returns X/2^48 exactly (glibc builds 1+X/2^48 in the
 * mantissa and subtracts 1).  ODD_DIST: v = pow(u, 1 + 3p)^2, p = xi[3]/N. */
void orc_generate_f64(int64_t n, int64_t g0, int64_t cnt, double *out) {
    uint64_t x = lcg_skip(1ULL << 32, (uint64_t)g0);
    for (int64_t k = 0; k < cnt; ++k) {
        int64_t g = g0 + k;
        unsigned short ctr = (unsigned short)((g + 1) & 0xFFFF);
        x = (LCG_A * x + LCG_C) & LCG_MASK;
        double val = ldexp((double)x, -48);
        double pr = (double)ctr / (double)n;
        val = pow(val, 1.0 + 3 * pr);
        val = val * val;
        out[k] = val;
    }
}

static inline uint64_t splitmix_at(uint64_t seed, int64_t g) {
    uint64_t z = seed + (uint64_t)(g + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_splitmix_u32(uint64_t seed, int64_t g0, int64_t cnt, uint32_t *out) {
    for (int64_t k = 0; k < cnt; ++k)
        out[k] = (uint32_t)(splitmix_at(seed, g0 + k) >> 32);
}

void orc_splitmix_u64(uint64_t seed, int64_t g0, int64_t cnt, uint64_t *out) {
    for (int64_t k = 0; k < cnt; ++k)
        out[k] = splitmix_at(seed, g0 + k);
}

void orc_u64mix(uint64_t seed, int64_t n, int64_t g0, int64_t cnt, uint64_t top, uint64_t *out) {
    /* draws below `top` (all-ones: the full 64-bit range below it) */
    const uint64_t lim = top;
    uint64_t x = lcg_skip(1ULL << 32, (uint64_t)g0); /* ODD_DIST stream at g0 */
    for (int64_t k = 0; k < cnt; ++k) {
        int64_t g = g0 + k;
        x = (LCG_A * x + LCG_C) & LCG_MASK;
        uint64_t h = splitmix_at(seed, g), v = splitmix_at(seed ^ 0xA5A5A5A5A5A5A5A5ULL, g);
        uint32_t c = (uint32_t)(h >> 32) % 100u;
        uint64_t key;
        if (c < 40) {
            key = splitmix_at(seed + 1, (int64_t)(v & 1023)) % lim;
        } else if (c < 70) { /* psort.cc:600-609 at index g */
            unsigned short ctr = (unsigned short)((g + 1) & 0xFFFF);
            double val = pow(ldexp((double)x, -48), 1.0 + 3 * ((double)ctr / (double)n));
            val = val * val;
            memcpy(&key, &val, 8);
        } else if (c < 90) {
            key = v % lim;
        } else if (c < 95) {
            key = 0;
        } else {
            key = top;
        }
        out[k] = key;
    }
}

/* -------------------------------------------------------------- local sort */

/* psort.cc:175 std::sort.  Keys carry no payload, so any correct ascending sort
 * gives the same bytes; LSD radix keeps the oracle fast at 10^7-10^8 keys. */
static void radix_u32(uint32_t *a, int64_t n) {
    if (n < 2) return;
    uint32_t *tmp = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    uint32_t *src = a, *dst = tmp;
    for (int shift = 0; shift < 32; shift += 8) {
        int64_t cnt[257] = {0};
        for (int64_t i = 0; i < n; ++i) cnt[((src[i] >> shift) & 0xFF) + 1]++;
        for (int b = 0; b < 256; ++b) cnt[b + 1] += cnt[b];
        for (int64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> shift) & 0xFF]++] = src[i];
        uint32_t *t = src; src = dst; dst = t;
    }
    free(tmp); /* 4 passes: result is back in a */
}

static void radix_u64(uint64_t *a, int64_t n) {
    if (n < 2) return;
    uint64_t *tmp = (uint64_t *)malloc((size_t)n * sizeof(uint64_t));
    uint64_t *src = a, *dst = tmp;
    for (int shift = 0; shift < 64; shift += 16) {
        int64_t *cnt = (int64_t *)calloc(65537, sizeof(int64_t));
        for (int64_t i = 0; i < n; ++i) cnt[((src[i] >> shift) & 0xFFFF) + 1]++;
        for (int b = 0; b < 65536; ++b) cnt[b + 1] += cnt[b];
        for (int64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> shift) & 0xFFFF]++] = src[i];
        free(cnt);
        uint64_t *t = src; src = dst; dst = t;
    }
    free(tmp); /* 4 passes: result is back in a */
}

/* Order-preserving map of IEEE doubles to u64 (negative: flip all bits,
 * non-negative: flip the sign bit).  Equal-comparing doubles with different bits
 * (-0.0 vs +0.0) are ordered -0 < +0 here; std::sort leaves their relative order
 * unspecified, so such mixtures are outside bit-exact parity. */
static inline uint64_t f64_to_ord(uint64_t b) {
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
static inline uint64_t ord_to_f64(uint64_t o) {
    return (o >> 63) ? (o & 0x7FFFFFFFFFFFFFFFULL) : ~o;
}

void orc_sort(int dtype, void *keys, int64_t n) {
    if (dtype == ORC_U32) {
        radix_u32((uint32_t *)keys, n);
    } else if (dtype == ORC_U64) {
        radix_u64((uint64_t *)keys, n);
    } else {
        uint64_t *k = (uint64_t *)keys;
        for (int64_t i = 0; i < n; ++i) k[i] = f64_to_ord(k[i]);
        radix_u64(k, n);
        for (int64_t i = 0; i < n; ++i) k[i] = ord_to_f64(k[i]);
    }
}

/* ----------------------------------------------------------- compare-split */

/* psort.cc:116-140 (max) / 142-164 (min).  The loop bodies restate the
 * reference's merges: strict '>' / '<' on the local key, else the received key
 * is taken (so ties take the received key). */
#define DEFINE_SPLIT(NAME, T, GT, LT)                                              \
    static void NAME(const T *loc, int64_t nloc, const T *rcv, int64_t nrcv,       \
                     T *out, int keep_max) {                                       \
        if (keep_max) {                                                            \
            int64_t ld = nloc - 1, rd = nrcv - 1;                                  \
            for (int64_t i = nloc - 1; i >= 0; --i) {                              \
                if (rd < 0) out[i] = loc[ld--];                                    \
                else if (ld < 0) out[i] = rcv[rd--];                               \
                else if (GT(loc[ld], rcv[rd])) out[i] = loc[ld--];                 \
                else out[i] = rcv[rd--];                                           \
            }                                                                      \
        } else {                                                                   \
            int64_t ld = 0, rd = 0;                                                \
            for (int64_t i = 0; i < nloc; ++i) {                                   \
                if (rd == nrcv) out[i] = loc[ld++];                                \
                else if (ld == nloc) out[i] = rcv[rd++];                           \
                else if (LT(loc[ld], rcv[rd])) out[i] = loc[ld++];                 \
                else out[i] = rcv[rd++];                                           \
            }                                                                      \
        }                                                                          \
    }

#define CMP_GT(a, b) ((a) > (b))
#define CMP_LT(a, b) ((a) < (b))
DEFINE_SPLIT(split_u32, uint32_t, CMP_GT, CMP_LT)
DEFINE_SPLIT(split_u64, uint64_t, CMP_GT, CMP_LT)
DEFINE_SPLIT(split_f64, double, CMP_GT, CMP_LT)

void orc_compare_split(int dtype, const void *local, int64_t nloc,
                       const void *recv, int64_t nrecv, void *out, int keep_max) {
    if (dtype == ORC_U32)
        split_u32((const uint32_t *)local, nloc, (const uint32_t *)recv, nrecv,
                  (uint32_t *)out, keep_max);
    else if (dtype == ORC_U64)
        split_u64((const uint64_t *)local, nloc, (const uint64_t *)recv, nrecv,
                  (uint64_t *)out, keep_max);
    else
        split_f64((const double *)local, nloc, (const double *)recv, nrecv,
                  (double *)out, keep_max);
}

/* ------------------------------------------------------- bitonic schedule */

static int ilog2(int v) { /* psort.cc:81-86 */
    int d = 0;
    for (v >>= 1; v != 0; v >>= 1) d++;
    return d;
}

/* psort.cc:182-196: for i in [0,d), j = i..0: partner = myid ^ 2^j, keep the
 * max half when bit(i+1) of myid differs from bit(j). */
int orc_bitonic_schedule(int p, int rank, int *partner, int *keep_max) {
    int d = ilog2(p), s = 0;
    for (int i = 0; i < d; ++i)
        for (int j = i; j >= 0; --j) {
            int ibit = (rank & (1 << (i + 1))) != 0;
            int jbit = (rank & (1 << j)) != 0;
            partner[s] = rank ^ (1 << j);
            keep_max[s] = ibit != jbit;
            ++s;
        }
    return s;
}

static size_t dsize(int dtype) { return dtype == ORC_U32 ? 4 : 8; }

/* psort.cc:167-201, all P ranks stepped in lockstep on host memory. */
int orc_parallel_bitonic_sort(int dtype, void *keys, int64_t n, int p) {
    if (p <= 0 || (p & (p - 1))) return -1; /* psort.cc:168-172 */
    size_t w = dsize(dtype);
    int64_t *sizes = (int64_t *)malloc(sizeof(int64_t) * p);
    int64_t *offs = (int64_t *)malloc(sizeof(int64_t) * (p + 1));
    orc_block_sizes(n, p, sizes);
    offs[0] = 0;
    for (int r = 0; r < p; ++r) offs[r + 1] = offs[r] + sizes[r];
    char *base = (char *)keys;
    for (int r = 0; r < p; ++r) orc_sort(dtype, base + offs[r] * w, sizes[r]);

    char *next = (char *)malloc((size_t)(n > 0 ? n : 1) * w);
    int d = ilog2(p);
    for (int i = 0; i < d; ++i) {
        for (int j = i; j >= 0; --j) {
            for (int r = 0; r < p; ++r) {
                int q = r ^ (1 << j);
                int ibit = (r & (1 << (i + 1))) != 0;
                int jbit = (r & (1 << j)) != 0;
                orc_compare_split(dtype, base + offs[r] * w, sizes[r],
                                  base + offs[q] * w, sizes[q],
                                  next + offs[r] * w, ibit != jbit);
            }
            memcpy(base, next, (size_t)n * w);
        }
    }
    free(next);
    free(offs);
    free(sizes);
    return 0;
}

/* psort.cc:88-101 */
static int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t x) {
    int64_t low = 0, high = n;
    while (low < high) {
        int64_t mid = (low + high) / 2;
        if (x <= a[mid]) high = mid;
        else low = mid + 1;
    }
    return low;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* psort.cc:377-490, all P ranks in lockstep with the reference's literal
 * buffer semantics: result_buffer holds (loc+1)*P keys, data beyond
 * result_size is stale, and an empty rank's median is the stale
 * result_buffer[0] (psort.cc:399; zero before anything was written).  Keys are
 * carried as unsigned 64-bit (u32 widened, f64 through the order-preserving
 * map: the same order as double compares except -0/+0 and NaN). */
int orc_parallel_quick_sort(int dtype, const void *keys, int64_t n, int p, void *out,
                            int64_t *sizes_out) {
    if (p <= 0 || (p & (p - 1))) return -1; /* psort.cc:378-382 */
    size_t w = dsize(dtype);
    int64_t *rs = (int64_t *)malloc(sizeof(int64_t) * p);
    int64_t *pi = (int64_t *)malloc(sizeof(int64_t) * p);
    uint64_t *med = (uint64_t *)malloc(sizeof(uint64_t) * p);
    uint64_t **buf = (uint64_t **)malloc(sizeof(uint64_t *) * p);
    uint64_t **snd = (uint64_t **)malloc(sizeof(uint64_t *) * p);
    int64_t *nsnd = (int64_t *)malloc(sizeof(int64_t) * p);
    orc_block_sizes(n, p, rs);
    const char *src = (const char *)keys;
    for (int r = 0; r < p; ++r) {
        int64_t cap = (rs[r] + 1) * p; /* psort.cc:385 */
        buf[r] = (uint64_t *)calloc((size_t)cap, 8);
        snd[r] = (uint64_t *)malloc((size_t)cap * 8);
        for (int64_t k = 0; k < rs[r]; ++k, src += w) {
            uint64_t v = 0;
            memcpy(&v, src, w);
            buf[r][k] = dtype == ORC_F64 ? f64_to_ord(v) : v;
        }
    }
    int d = ilog2(p);
    for (int i = 0; i < d; ++i) {
        int g = p >> i, half = g >> 1;
        for (int r = 0; r < p; ++r) {
            radix_u64(buf[r], rs[r]);      /* psort.cc:398 */
            med[r] = buf[r][rs[r] / 2];    /* psort.cc:399 */
        }
        for (int color = 0; color < p / g; ++color) { /* psort.cc:409-414 */
            uint64_t *mb = (uint64_t *)malloc(sizeof(uint64_t) * g);
            memcpy(mb, med + (size_t)color * g, sizeof(uint64_t) * g);
            qsort(mb, (size_t)g, sizeof(uint64_t), cmp_u64);
            uint64_t pivot = mb[g / 2];
            for (int r = color * g; r < color * g + g; ++r)
                pi[r] = lower_bound_u64(buf[r], rs[r], pivot); /* psort.cc:417 */
            free(mb);
        }
        for (int r = 0; r < p; ++r) { /* what each rank sends (psort.cc:431-470) */
            int low = (r % g) < half;
            int64_t off = low ? pi[r] : 0;
            nsnd[r] = low ? rs[r] - pi[r] : pi[r];
            memcpy(snd[r], buf[r] + off, (size_t)nsnd[r] * 8);
        }
        for (int r = 0; r < p; ++r) {
            int q = r ^ half, low = (r % g) < half;
            if (low) { /* receive at pivot_index (psort.cc:444-452) */
                memcpy(buf[r] + pi[r], snd[q], (size_t)nsnd[q] * 8);
                rs[r] = pi[r] + nsnd[q];
            } else { /* keep the upper part at the front, append (psort.cc:462-474) */
                int64_t keep = rs[r] - pi[r];
                memmove(buf[r], buf[r] + pi[r], (size_t)keep * 8);
                memcpy(buf[r] + keep, snd[q], (size_t)nsnd[q] * 8);
                rs[r] = keep + nsnd[q];
            }
        }
    }
    char *dst = (char *)out;
    for (int r = 0; r < p; ++r) {
        radix_u64(buf[r], rs[r]); /* psort.cc:485 */
        sizes_out[r] = rs[r];
        for (int64_t k = 0; k < rs[r]; ++k, dst += w) {
            uint64_t v = dtype == ORC_F64 ? ord_to_f64(buf[r][k]) : buf[r][k];
            memcpy(dst, &v, w);
        }
        free(buf[r]);
        free(snd[r]);
    }
    free(rs); free(pi); free(med); free(buf); free(snd); free(nsnd);
    return 0;
}

/* psort.cc:497-520.  The reference reads local_numbers[local_size-1] of an
 * empty block (UB); here an empty block contributes nothing and forwards the
 * previous boundary key. */
int64_t orc_check_sort(int dtype, const void *keys, int64_t n, int p) {
    int64_t *sizes = (int64_t *)malloc(sizeof(int64_t) * p);
    orc_block_sizes(n, p, sizes);
    int64_t errs = 0, off = 0, prev_last = -1;
    for (int r = 0; r < p; ++r) {
        for (int64_t i = off; i + 1 < off + sizes[r]; ++i) {
            int gt;
            if (dtype == ORC_U32) gt = ((const uint32_t *)keys)[i] > ((const uint32_t *)keys)[i + 1];
            else if (dtype == ORC_U64) gt = ((const uint64_t *)keys)[i] > ((const uint64_t *)keys)[i + 1];
            else gt = ((const double *)keys)[i] > ((const double *)keys)[i + 1];
            errs += gt;
        }
        if (sizes[r] > 0) {
            if (r > 0 && prev_last >= 0) {
                int gt;
                if (dtype == ORC_U32) gt = ((const uint32_t *)keys)[prev_last] > ((const uint32_t *)keys)[off];
                else if (dtype == ORC_U64) gt = ((const uint64_t *)keys)[prev_last] > ((const uint64_t *)keys)[off];
                else gt = ((const double *)keys)[prev_last] > ((const double *)keys)[off];
                errs += gt;
            }
            prev_last = off + sizes[r] - 1;
        }
        off += sizes[r];
    }
    free(sizes);
    return errs;
}
