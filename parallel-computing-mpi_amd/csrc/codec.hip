// codec.hip -- lossless delta coding of sorted key runs for the compare-split
// exchange over xGMI (gfx950).
//
// The keys a rank sends in one compare-split stage (psort.cc:116-164: the
// reference ships the whole block with MPI_Sendrecv) are a sorted run, so
// consecutive differences are small: 2^27 uniform u32 keys have a mean gap of
// 32.  The run is cut into blocks of CB keys; a block is stored as its first
// key (base) and its CB-1 gaps packed at the block's own bit width w (the
// width of its largest gap), "frame of reference" style.  Decoding is a
// block-wide prefix sum.  Every block decodes independently, so encode and
// decode are single HBM-streaming passes.
//
// Stream (u32 words): nblk headers of 4 words {base lo, base hi, payload
// offset (words, from the stream start), width}, then the payloads.
//
// The run to encode is given on the device as {offset, count} with an upper
// bound on the count on the host: the compare-split stage computes its
// exchange count on the device, and the host learns it together with the
// coded size in the stage's one size exchange.  The payload offsets are an
// exclusive scan of the per-block word counts -- chunks of SCN blocks scanned
// in LDS (k_scan_words), then the chunk totals (k_scan_chunks); no library
// scan.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kernels.h"

namespace misort {
namespace {

constexpr int CB = 1024, CT = 256, CI = CB / CT;  // keys per block, threads, keys per thread
constexpr int SCN = 1024;                         // blocks per chunk of the payload-offset scan

__device__ __forceinline__ int width_of(uint64_t d) { return d ? 64 - __builtin_clzll(d) : 0; }

// The lane's keys j0-1 .. j0+CI-1 (x[0] = the key before its run, unread at
// the block start): one 4-byte-aligned vector load of its CI keys (the run's
// start is any key offset) instead of a load per key and per predecessor.
template <typename K>
__device__ __forceinline__ void lane_keys(const K* __restrict__ keys, int64_t j0, int64_t k0, int64_t n,
                                          K (&x)[CI + 1]) {
    static_assert(CI == 4, "4-key lane runs");
    if (j0 + CI <= n) {
        if constexpr (sizeof(K) == 4) {
            typedef uint32_t v4 __attribute__((ext_vector_type(4), aligned(4)));
            const v4 v = *reinterpret_cast<const v4*>(keys + j0);
            x[1] = v.x;
            x[2] = v.y;
            x[3] = v.z;
            x[4] = v.w;
        } else {
            typedef uint64_t v2 __attribute__((ext_vector_type(2), aligned(8)));
            const v2 a = *reinterpret_cast<const v2*>(keys + j0), b = *reinterpret_cast<const v2*>(keys + j0 + 2);
            x[1] = a.x;
            x[2] = a.y;
            x[3] = b.x;
            x[4] = b.y;
        }
    } else {
#pragma unroll
        for (int i = 0; i < CI; ++i) x[i + 1] = j0 + i < n ? keys[j0 + i] : (K)0;
    }
    x[0] = j0 > k0 && j0 - 1 < n ? keys[j0 - 1] : (K)0;
}

// Per block: payload words for its gaps at the block's width.  (Lane-strided
// loads of 4 consecutive keys; measured faster here than coalesced loads with a
// cross-lane predecessor, and than packing through LDS atomics.)  The run is
// base + run[0] .. + run[1] keys; blocks past its end write no words.
template <typename K>
__global__ __launch_bounds__(CT) void k_codec_width(const K* __restrict__ base, const int64_t* __restrict__ run,
                                                    uint32_t* __restrict__ words, uint8_t* __restrict__ wid) {
    __shared__ uint64_t red[CT / 64];
    const int64_t b = blockIdx.x, k0 = b * CB;
    const int t = threadIdx.x;
    const int64_t n = run[1];
    const K* __restrict__ keys = base + run[0];
    if (k0 >= n) {
        if (t == 0) {
            words[b] = 0;
            wid[b] = 0;
        }
        return;
    }
    uint64_t mx = 0;
    K x[CI + 1];  // keys j-1 .. j+3 of the lane's 4-key run j = k0 + 4t
    lane_keys<K>(keys, k0 + (int64_t)t * CI, k0, n, x);
#pragma unroll
    for (int i = 0; i < CI; ++i) {
        const int64_t j = k0 + t * CI + i;  // gap: key j minus key j-1
        if (j > k0 && j < n) mx = max(mx, (uint64_t)(x[i + 1] - x[i]));
    }
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint64_t)__shfl_xor(mx, o));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    if (t == 0) {
        for (int i = 1; i < CT / 64; ++i) mx = max(mx, red[i]);
        const int w = width_of(mx);
        const int64_t cnt = n - k0 < CB ? n - k0 : CB;
        words[b] = (uint32_t)(((cnt - 1) * w + 31) >> 5);
        wid[b] = (uint8_t)w;
    }
}

// Inclusive scan of v over the SCN lanes of the block (16 waves of 64).
__device__ __forceinline__ uint32_t scan_block(uint32_t v, uint32_t* sw) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(v, o, 64);
        v += lane >= o ? u : 0u;
    }
    if (lane == 63) sw[wv] = v;
    __syncthreads();
    uint32_t pre = 0;
    for (int q = 0; q < wv; ++q) pre += sw[q];
    __syncthreads();
    return v + pre;
}

// Chunk c of SCN blocks: off[b] = the words of the chunk's blocks before b
// (chunk-local exclusive scan), csum[c] = the chunk's total.
__global__ __launch_bounds__(SCN) void k_scan_words(const uint32_t* __restrict__ words, int64_t nb,
                                                    uint32_t* __restrict__ off, uint32_t* __restrict__ csum) {
    __shared__ uint32_t sw[SCN / 64];
    const int64_t b = (int64_t)blockIdx.x * SCN + threadIdx.x;
    const uint32_t v = b < nb ? words[b] : 0u;
    const uint32_t inc = scan_block(v, sw);
    if (b < nb) off[b] = inc - v;
    if (threadIdx.x == SCN - 1) csum[blockIdx.x] = inc;
}

// One workgroup: the chunk totals exclusive-scanned in place (carried over
// rounds of SCN), then the message sizes sizes[0] = coded words (4 header
// words per block + the payload words), sizes[1] = raw words (count * key
// words) of the run's count run[1].
__global__ __launch_bounds__(SCN) void k_scan_chunks(uint32_t* __restrict__ csum, int64_t nc,
                                                     const int64_t* __restrict__ run, int key_words,
                                                     int64_t* __restrict__ sizes) {
    __shared__ uint32_t sw[SCN / 64];
    __shared__ uint32_t tot;
    uint32_t carry = 0;
    for (int64_t c0 = 0; c0 < nc; c0 += SCN) {
        const int64_t c = c0 + threadIdx.x;
        const uint32_t v = c < nc ? csum[c] : 0u;
        const uint32_t inc = scan_block(v, sw);
        if (c < nc) csum[c] = carry + inc - v;
        if (threadIdx.x == SCN - 1) tot = inc;
        __syncthreads();
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int64_t n = run[1];
        const int64_t nb = (n + CB - 1) / CB;
        sizes[0] = n > 0 ? 4 * nb + (int64_t)carry : 0;
        sizes[1] = n * key_words;
    }
}

// BPW consecutive blocks per workgroup, all their key loads issued before the
// first block is packed: a block alone is a short chain of dependent steps
// (loads, LDS, pack, stores), so one per workgroup left the pass latency-bound
// at eight blocks in flight per CU (CODEC_BPW; 1 = one block).
// Measured (profiles/r05/codec/ab.txt, k = 2^26 u32): encode 0.156 -> 0.141 ms,
// decode 0.122 -> 0.106 ms with 4; 8 was slower; u64 keys keep one block (the
// pack equal, the decode's 33 KB of staged payload per workgroup 1.5x slower).
constexpr int CODEC_BPW = 4;
template <typename K, int BPW>
__global__ __launch_bounds__(CT) void k_codec_pack(const K* __restrict__ kbase, const int64_t* __restrict__ run,
                                                   const uint32_t* __restrict__ off, const uint32_t* __restrict__ coff,
                                                   const uint8_t* __restrict__ wid, uint32_t* __restrict__ out) {
    typedef typename std::conditional<sizeof(K) == 4, uint32_t, uint64_t>::type G;  // a gap
    __shared__ G gap[CB];
    const int64_t bw = (int64_t)blockIdx.x * BPW;
    const int64_t n = run[1];
    if (bw * CB >= n) return;
    const K* __restrict__ keys = kbase + run[0];
    const int64_t nblk = (n + CB - 1) / CB;
    const int t = threadIdx.x;
    // the lane's runs of keys k0+4t .. k0+4t+3 and the key before each, for
    // every block of the workgroup
    K x[BPW][CI + 1];
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
        const int64_t k0 = (bw + u) * CB;
        if (k0 < n) lane_keys<K>(keys, k0 + (int64_t)t * CI, k0, n - k0 < CB ? n : k0 + CB, x[u]);
    }
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
        const int64_t b = bw + u, k0 = b * CB;
        if (k0 >= n) break;  // uniform
        const int64_t cnt = n - k0 < CB ? n - k0 : CB;
        if (u > 0) __syncthreads();  // the previous block's pack has read its gaps
        // gap j (key k0+j+1 minus key k0+j): gap 4t-1+i = x[i+1] - x[i]
#pragma unroll
        for (int i = 0; i < CI; ++i) {
            const int j = t * CI + i - 1;
            if (j >= 0) gap[j] = (j + 1 < cnt) ? (G)(x[u][i + 1] - x[u][i]) : (G)0;
        }
        if (t == CT - 1) gap[CB - 1] = 0;
        __syncthreads();
        const int w = wid[b];
        const uint32_t base_w = (uint32_t)(4 * nblk) + off[b] + coff[b / SCN];
        const int nw = (int)(((cnt - 1) * w + 31) >> 5);
        if (t == 0) {
            const uint64_t base = (uint64_t)x[u][1];  // lane 0's first key: the block's
            uint32_t* h = out + 4 * b;
            h[0] = (uint32_t)base;
            h[1] = (uint32_t)(base >> 32);
            h[2] = base_w;
            h[3] = (uint32_t)w;
        }
        for (int q = t; q < nw; q += CT) {
            // fields j overlapping bits [32q, 32q+32) (q < 2^11, so 32-bit)
            const int lo = q * 32;
            uint32_t v = 0;
            for (int j = lo / w; j * w < lo + 32 && j < cnt - 1; ++j) {
                const int sh = j * w - lo;  // field start relative to the word (may be < 0)
                const uint64_t f = gap[j];
                v |= sh >= 0 ? (uint32_t)(f << sh) : (uint32_t)(f >> (-sh));
            }
            out[base_w + q] = v;
        }
    }
}

__global__ void k_set_run(int64_t* run, int64_t offset, int64_t n) {
    run[0] = offset;
    run[1] = n;
}

// Lane t rebuilds keys 4t..4t+3 of its block: key p = base + the gaps before
// it, so the lane decodes gaps 4t-1..4t+2, a wave scan (cross-lane shuffles) and one
// LDS step across the 4 waves give the prefix, and the 4 keys leave as one
// 16-byte (u32) or two (u64) vector stores.  BPW blocks per workgroup, as in
// k_codec_pack: their headers, then their payloads, load at once.
template <typename K, int BPW>
__global__ __launch_bounds__(CT) void k_codec_unpack(const uint32_t* __restrict__ in, int64_t n,
                                                     K* __restrict__ keys) {
    static_assert(CI == 4, "one 4-key run per lane");
    constexpr int PW = (CB * 8 * (int)sizeof(K) + 31) / 32 + 2;  // a block's payload words at most, + 2
    __shared__ uint64_t wsum[BPW][CT / 64];
    // the blocks' payload words, staged by coalesced loads (each lane's bit
    // fields then read LDS instead of up to three scattered global words per
    // key); all BPW blocks' headers, then all their payloads, in flight at once
    __shared__ uint32_t pay[BPW][PW];
    const int64_t bw = (int64_t)blockIdx.x * BPW;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t base[BPW];
    uint32_t pw[BPW];
    int w[BPW], nw[BPW];
    int64_t cnt[BPW];
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
        const int64_t k0 = (bw + u) * CB;
        cnt[u] = k0 >= n ? 0 : (n - k0 < CB ? n - k0 : CB);
        const uint32_t* h = in + 4 * (bw + u);
        base[u] = cnt[u] ? (uint64_t)h[0] | ((uint64_t)h[1] << 32) : 0;
        pw[u] = cnt[u] ? h[2] : 0;
        w[u] = cnt[u] ? (int)h[3] : 0;
        nw[u] = cnt[u] ? (int)(((cnt[u] - 1) * w[u] + 31) >> 5) : 0;
    }
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
        for (int q = t; q < nw[u]; q += CT) pay[u][q] = in[pw[u] + q];
        if (t < 2) pay[u][nw[u] + t] = 0u;  // a field's read of the words past the payload
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < BPW; ++u) {
        if (cnt[u] == 0) break;  // uniform
        const int64_t k0 = (bw + u) * CB;
        const uint64_t mask = w[u] >= 64 ? ~0ull : ((1ull << w[u]) - 1);
        uint64_t g[CI], s = 0;
#pragma unroll
        for (int i = 0; i < CI; ++i) {
            const int j = t * CI + i - 1;  // the gap before key 4t+i
            uint64_t f = 0;
            if (w[u] && j >= 0 && j + 1 < cnt[u]) {
                const int bit = j * w[u];
                const uint32_t* p = pay[u] + (bit >> 5);
                const int sh = bit & 31;
                const uint64_t lo = (uint64_t)p[0] | ((uint64_t)(sh + w[u] > 32 ? p[1] : 0) << 32);
                f = lo >> sh;
                if (sh + w[u] > 64) f |= (uint64_t)p[2] << (64 - sh);
                f &= mask;
            }
            s += f;
            g[i] = s;  // inclusive prefix within the lane
        }
        uint64_t x = s;  // inclusive scan of the lane totals over the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint64_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[u][wv] = x;
        __syncthreads();
        uint64_t pre = x - s;
        for (int v = 0; v < wv; ++v) pre += wsum[u][v];
        K r[CI];
#pragma unroll
        for (int i = 0; i < CI; ++i) r[i] = (K)(base[u] + pre + g[i]);
        const int64_t p0 = k0 + (int64_t)t * CI;
        if ((int64_t)t * CI + CI <= cnt[u] && !((uintptr_t)(keys + p0) & 15)) {
            typedef uint32_t v4 __attribute__((ext_vector_type(4)));
            v4* dst = reinterpret_cast<v4*>(keys + p0);
            if constexpr (sizeof(K) == 4) {
                dst[0] = v4{(uint32_t)r[0], (uint32_t)r[1], (uint32_t)r[2], (uint32_t)r[3]};
            } else {
                dst[0] = v4{(uint32_t)r[0], (uint32_t)((uint64_t)r[0] >> 32), (uint32_t)r[1],
                            (uint32_t)((uint64_t)r[1] >> 32)};
                dst[1] = v4{(uint32_t)r[2], (uint32_t)((uint64_t)r[2] >> 32), (uint32_t)r[3],
                            (uint32_t)((uint64_t)r[3] >> 32)};
            }
        } else {
#pragma unroll
            for (int i = 0; i < CI; ++i)
                if ((int64_t)t * CI + i < cnt[u]) keys[p0 + i] = r[i];
        }
    }
}

}  // namespace

int64_t codec_blocks(int64_t n) { return (n + CB - 1) / CB; }

// words, off, wid per block and the chunk totals
static size_t arrays_bytes(int64_t n) {
    const int64_t nb = codec_blocks(n) > 0 ? codec_blocks(n) : 1;
    const int64_t nc = (nb + SCN - 1) / SCN;
    return (size_t)nb * (2 * sizeof(uint32_t) + 1) + (size_t)nc * sizeof(uint32_t);
}
// + 256 for alignment, + the {offset, count} slot codec_encode keeps at the end
size_t codec_scratch_bytes(int64_t n) { return arrays_bytes(n) + 512; }

int64_t codec_max_words(int64_t n, int key_bytes) {
    return 4 * codec_blocks(n) + (n * key_bytes * 8 + 31) / 32 + codec_blocks(n);
}

template <typename K>
hipError_t codec_encode_dev(const K* base, const int64_t* run, int64_t n_max, uint32_t* out, void* scratch,
                            size_t scratch_bytes, int64_t* sizes, hipStream_t s) {
    const int64_t nb = codec_blocks(n_max) > 0 ? codec_blocks(n_max) : 1;
    const int64_t nc = (nb + SCN - 1) / SCN;
    if (scratch_bytes < arrays_bytes(n_max) + 256) return hipErrorInvalidValue;
    char* p = (char*)(((uintptr_t)scratch + 255) & ~(uintptr_t)255);
    uint32_t* words = (uint32_t*)p;
    uint32_t* off = words + nb;
    uint32_t* csum = off + nb;
    uint8_t* wid = (uint8_t*)(csum + nc);
    k_codec_width<K><<<(unsigned)nb, CT, 0, s>>>(base, run, words, wid);
    k_scan_words<<<(unsigned)nc, SCN, 0, s>>>(words, nb, off, csum);
    k_scan_chunks<<<1, SCN, 0, s>>>(csum, nc, run, (int)(sizeof(K) / 4), sizes);
    constexpr int BPW = sizeof(K) == 4 ? CODEC_BPW : 1;  // u64: equal (pack) / slower (unpack)
    k_codec_pack<K, BPW><<<(unsigned)((nb + BPW - 1) / BPW), CT, 0, s>>>(base, run, off, csum, wid, out);
    return hipGetLastError();
}

template <typename K>
hipError_t codec_encode(const K* keys, int64_t n, uint32_t* out, void* scratch, size_t scratch_bytes,
                        int64_t* sizes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    // the {offset, count} slot at the end of the scratch
    int64_t* run = (int64_t*)(((uintptr_t)scratch + scratch_bytes - 64) & ~(uintptr_t)15);
    k_set_run<<<1, 1, 0, s>>>(run, 0, n);
    return codec_encode_dev<K>(keys, run, n, out, scratch, (size_t)((char*)run - (char*)scratch), sizes, s);
}

template <typename K>
hipError_t codec_decode(const uint32_t* in, int64_t n, K* keys, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    constexpr int BPW = sizeof(K) == 4 ? CODEC_BPW : 1;  // u64: 33 KB of payload LDS per workgroup
    k_codec_unpack<K, BPW><<<(unsigned)((codec_blocks(n) + BPW - 1) / BPW), CT, 0, s>>>(in, n, keys);
    return hipGetLastError();
}

template hipError_t codec_encode_dev<uint32_t>(const uint32_t*, const int64_t*, int64_t, uint32_t*, void*, size_t,
                                               int64_t*, hipStream_t);
template hipError_t codec_encode_dev<uint64_t>(const uint64_t*, const int64_t*, int64_t, uint32_t*, void*, size_t,
                                               int64_t*, hipStream_t);
template hipError_t codec_encode<uint32_t>(const uint32_t*, int64_t, uint32_t*, void*, size_t, int64_t*,
                                           hipStream_t);
template hipError_t codec_encode<uint64_t>(const uint64_t*, int64_t, uint32_t*, void*, size_t, int64_t*,
                                           hipStream_t);
template hipError_t codec_decode<uint32_t>(const uint32_t*, int64_t, uint32_t*, hipStream_t);
template hipError_t codec_decode<uint64_t>(const uint32_t*, int64_t, uint64_t*, hipStream_t);

}  // namespace misort
